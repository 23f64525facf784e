// sidx_chunk.hip -- gfx950 "chunkrecord" index: ~1 MiB chunks that
// end at a record boundary found by a regex in a 32 KiB window.
//
// Reference semantics (paths relative to /root/reference/shock-server/):
//   node/file/index/chunkrecord.go:41-99  curr = 0; n, er = SeekChunk(curr, true);
//       row (curr, er == EOF ? size - curr : n); curr += n; stop after the EOF row
//   node/file/format/fastq/fastq.go:216-243  window [curr + CHUNK - 32 KiB, curr + CHUNK):
//       end of the LAST match of FindAllIndex(Record) (clamped to 32767), else the FIRST match
//       of each following window; a short window read is io.EOF
//   node/file/format/fastq/fastq.go:23  Record regex, Go leftmost-first semantics
//   node/file/format/fasta/fasta.go:143-173  last (then first) "\n>", falling back to "\r>"
//
// The chunk chain is serial by definition (each window sits CHUNK past the previous chunk's
// end) and touches only 32 KiB of every CHUNK bytes, so one workgroup of 16 waves walks it:
// per step the window is staged in LDS (16-B loads), every lane evaluates the regex at the
// '@' positions of its 32 bytes (FASTQ) or the "\n>" pairs (FASTA), matches are compacted in
// window order and the FindAllIndex chain (next match = first start >= previous end) is
// resolved by pointer doubling in LDS.  The regex's only choice points are where each `.*`
// stops (the line's '\n', then each inner '\r' right to left); every other quantifier is
// forced to its maximal run because the following class is disjoint from it.
//
// Linear time per window (no retry per '\r'): what follows a `.*` depends only on the [\n\r]+
// run it stops in, so each run is evaluated once -- first the quality tail (tail_qual) of every
// run into a success bit mask, then the sequence tail (tail_seq2, whose plus-line `.*` is the
// rightmost successful run of that line: one mask lookup) into a second mask -- and a match
// at '@' is the rightmost successful run of its header line (one lookup).  Word tables give the
// next '\n' word and the previous success word in O(1).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned int u32;

constexpr int WIN = 32768;
constexpr int NT = 1024;
constexpr int PER = WIN / NT;     // 32 window bytes per lane
constexpr int MAXM = 2048;       // compacted match starts per window (more: serial walk)

__device__ __forceinline__ bool is_nl(u32 c) { return c == '\n' || c == '\r'; }
__device__ __forceinline__ bool is_sp(u32 c) { return c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '; }
__device__ __forceinline__ bool is_l(u32 c) { return ((c | 32) >= 'a' && (c | 32) <= 'z') || c == '-'; }

// Window class masks in LDS (bit j of word j>>6 = window byte j): '\n', '\r', [A-Za-z-],
// RE2 \s.  Every run the regex walks is found 64 bytes at a time from these words.
constexpr int NW = WIN / 64;
struct Masks {
  u64 nl[NW], cr[NW], let[NW], sp[NW];
  u64 okq[NW], okt[NW];             // run positions whose quality / sequence tail matches
  short nxn[NW + 1];                // first word >= w holding a '\n' (NW: none)
  short pvq[NW], pvt[NW];           // last word <= w holding an okq / okt bit (-1: none)
};
enum { M_NL, M_CR, M_NLR, M_LET, M_SP };

__device__ __forceinline__ u64 mword(const Masks &m, int k, int w) {
  switch (k) {
    case M_NL: return m.nl[w];
    case M_CR: return m.cr[w];
    case M_NLR: return m.nl[w] | m.cr[w];
    case M_LET: return m.let[w];
    default: return m.sp[w];
  }
}
// first position >= p whose class bit equals `set` (WIN if none)
__device__ __forceinline__ int next_bit(const Masks &m, int k, bool set, int p) {
  if (p >= WIN) return WIN;
  int w = p >> 6;
  u64 x = mword(m, k, w);
  if (!set) x = ~x;
  x &= ~0ull << (p & 63);
  while (!x) {
    if (++w == NW) return WIN;
    x = mword(m, k, w);
    if (!set) x = ~x;
  }
  return (w << 6) + __builtin_ctzll(x);
}
// NL+ S+ NL+ from a (the plus-line `.*` end, a NL byte); returns the match end or -1
__device__ __forceinline__ int tail_qual(const Masks &m, int a) {
  const int p = next_bit(m, M_NLR, false, a);
  if (p >= WIN) return -1;
  const int q = next_bit(m, M_SP, true, p);
  if (q == p || q >= WIN || !((mword(m, M_NLR, q >> 6) >> (q & 63)) & 1)) return -1;
  return next_bit(m, M_NLR, false, q);
}

// first '\n' at a position >= p (WIN if none): O(1) with the word table
__device__ __forceinline__ int next_nl(const Masks &m, int p) {
  if (p >= WIN) return WIN;
  int w = p >> 6;
  const u64 x = m.nl[w] & (~0ull << (p & 63));
  if (x) return (w << 6) + __builtin_ctzll(x);
  w = m.nxn[w + 1];
  return w >= NW ? WIN : (w << 6) + __builtin_ctzll(m.nl[w]);
}
// last position in [lo, p] whose bit is set in ok (with its word table pv); -1 if none
__device__ __forceinline__ int prev_ok(const u64 *ok, const short *pv, int lo, int p) {
  if (p < lo || p < 0) return -1;
  if (p >= WIN) p = WIN - 1;
  int w = p >> 6;
  u64 x = ok[w] & ((p & 63) == 63 ? ~0ull : ((2ull << (p & 63)) - 1));
  if (!x) {
    w = w > 0 ? pv[w - 1] : -1;
    if (w < 0) return -1;
    x = ok[w];
  }
  const int r = (w << 6) + 63 - __builtin_clzll(x);
  return r >= lo ? r : -1;
}

// NL+ L+ NL+ '+' .* NL+ S+ NL+ from a (the header `.*` end, a NL byte); the plus line's `.*`
// stops at the rightmost run of [q + 1, its '\n'] whose quality tail matches (okq)
__device__ __forceinline__ int tail_seq2(const uint8_t *b, const Masks &m, int a) {
  const int p = next_bit(m, M_NLR, false, a);
  if (p >= WIN) return -1;
  int q = next_bit(m, M_LET, false, p);
  if (q == p || q >= WIN || !is_nl(b[q])) return -1;
  q = next_bit(m, M_NLR, false, q);
  if (q >= WIN || b[q] != '+') return -1;
  const int c = prev_ok(m.okq, m.pvq, q + 1, next_nl(m, q + 1));
  return c >= 0 ? tail_qual(m, c) : -1;
}

// leftmost-first Record match anchored at s (b[s] == '@'); end or -1: the header `.*` stops
// at the rightmost run of [s + 2, the line's '\n'] whose sequence tail matches (okt)
__device__ __forceinline__ int record_at(const uint8_t *b, const Masks &m, int s) {
  if (s + 1 >= WIN || is_sp(b[s + 1])) return -1;
  const int c = prev_ok(m.okt, m.pvt, s + 2, next_nl(m, s + 2));
  return c >= 0 ? tail_seq2(b, m, c) : -1;
}

// the [\n\r]+ runs that start in [j0, j0 + PER): evaluate `tail` once per run and mark the
// run's positions in ok (LDS 64-bit or)
template <class Tail>
__device__ __forceinline__ void mark_runs(const uint8_t *b, const Masks &m, u64 *ok, int j0, Tail tail) {
  for (int j = j0; j < j0 + PER; ++j) {
    if (!is_nl(b[j]) || (j > 0 && is_nl(b[j - 1]))) continue;
    if (tail(j) < 0) continue;
    const int e = next_bit(m, M_NLR, false, j);  // run [j, e)
    for (int x = j; x < e;) {
      const int w = x >> 6, lo = x & 63;
      const int hi = (e - (w << 6)) < 64 ? (e - (w << 6)) : 64;
      const u64 bits = (hi == 64 ? ~0ull : ((1ull << hi) - 1)) & (~0ull << lo);
      atomicOr((unsigned long long *)&ok[w], (unsigned long long)bits);
      x = (w + 1) << 6;
    }
  }
}

// word tables, one wave (8 words per lane, a max / min scan over the lanes): nxn[w] = first
// word >= w with a '\n' (NW: none), or pv[w] = last word <= w with a bit of ok (-1: none)
__device__ void word_tables(Masks &m, const u64 *ok, short *pv, bool nl) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x, w0 = lane * (NW / 64);
  if (nl) {
    int first = NW;
    for (int k = NW / 64 - 1; k >= 0; --k) if (m.nl[w0 + k]) first = w0 + k;
    int sfx = first;  // min over lanes >= this one
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_down(sfx, d, 64);
      if (lane + d < 64) sfx = min(sfx, y);
    }
    int run = __shfl_down(sfx, 1, 64);
    if (lane == 63) run = NW;
    for (int k = NW / 64 - 1; k >= 0; --k) {
      if (m.nl[w0 + k]) run = w0 + k;
      m.nxn[w0 + k] = (short)run;
    }
    if (lane == 63) m.nxn[NW] = NW;
  } else {
    int last = -1;
    for (int k = 0; k < NW / 64; ++k) if (ok[w0 + k]) last = w0 + k;
    int pre = last;  // max over lanes <= this one
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(pre, d, 64);
      if (lane >= d) pre = max(pre, y);
    }
    int run = __shfl_up(pre, 1, 64);
    if (lane == 0) run = -1;
    for (int k = 0; k < NW / 64; ++k) {
      if (ok[w0 + k]) run = w0 + k;
      pv[w0 + k] = (short)run;
    }
  }
}

// block-wide exclusive scan of one int per lane (LDS, Hillis-Steele over wave totals)
__device__ int block_excl_scan(int v, int *wsum, int *total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NT / 64; ++i) {
      const int t = wsum[i];
      wsum[i] = acc;
      acc += t;
    }
    *total = acc;
  }
  __syncthreads();
  return wsum[wv] + x - v;
}

struct ChunkState {
  i64 curr, off, acc;
  u64 cnt;
  int last, done, found, pos;
};

__global__ __launch_bounds__(NT) void k_chunkrecord(const uint8_t *__restrict__ d, u64 n, int fasta, i64 chunk,
                                                    u64 *__restrict__ rows, u64 row_cap, u64 *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[WIN + 32];
  __shared__ unsigned short S[MAXM], E[MAXM], F[MAXM];
  __shared__ int wsum[NT / 64], total, red[4];
  __shared__ ChunkState st;
  __shared__ Masks mk;
  const int t = threadIdx.x;
  if (t == 0) {
    st.curr = 0; st.off = 0; st.acc = 0; st.cnt = 0; st.last = 1; st.done = 0;
  }
  __syncthreads();
  while (!st.done) {
    const i64 w = st.off + chunk - WIN;
    if ((u64)w + WIN > n) { // short read: io.EOF -> row (curr, size - curr), stop
      if (t == 0) {
        if (st.cnt < row_cap) {
          rows[2 * st.cnt] = (u64)st.curr;
          rows[2 * st.cnt + 1] = n - (u64)st.curr;
        }
        st.cnt++;
        st.done = 1;
      }
      __syncthreads();
      break;
    }
    // stage [w, w + WIN) in LDS: 16-B aligned loads, window byte j at raw[sh + j]
    const u64 base = (u64)w & ~15ull;
    const int sh = (int)((u64)w - base);
    for (int i = t; i < WIN / 16 + 1; i += NT) {
      const u64 a = base + 16ull * i;
      uint4 v;
      if (a + 16 <= n) {
        v = *reinterpret_cast<const uint4 *>(d + a);
      } else {
        uint8_t tmp[16];
        for (int k = 0; k < 16; ++k) tmp[k] = a + k < n ? d[a + k] : 0;
        v = *reinterpret_cast<const uint4 *>(tmp);
      }
      *reinterpret_cast<uint4 *>(raw + 16 * i) = v;
    }
    if (t < 4) red[t] = t & 1 ? -1 : 0x7fffffff; // [0] min '\n>', [1] max '\n>', [2] min '\r>', [3] max '\r>'
    __syncthreads();
    const uint8_t *b = raw + sh;
    const int j0 = t * PER;
    const int last = st.last;
    if (fasta) {
      int mnN = 0x7fffffff, mxN = -1, mnR = 0x7fffffff, mxR = -1;
      for (int j = j0; j < j0 + PER && j + 1 < WIN; ++j) {
        if (b[j + 1] != '>') continue;
        if (b[j] == '\n') { mnN = min(mnN, j); mxN = max(mxN, j); }
        else if (b[j] == '\r') { mnR = min(mnR, j); mxR = max(mxR, j); }
      }
      if (mxN >= 0) { atomicMin(&red[0], mnN); atomicMax(&red[1], mxN); }
      if (mxR >= 0) { atomicMin(&red[2], mnR); atomicMax(&red[3], mxR); }
      __syncthreads();
      if (t == 0) {
        const int pn = last ? red[1] : (red[0] == 0x7fffffff ? -1 : red[0]);
        const int pr = last ? red[3] : (red[2] == 0x7fffffff ? -1 : red[2]);
        const int p = pn >= 0 ? pn : pr;
        st.found = p >= 0;
        st.pos = p + 1;
      }
    } else {
      { // class masks: one 64-byte word per wave iteration, one byte per lane, ballots
        const int lane = t & 63;
        for (int w = t >> 6; w < NW; w += NT / 64) {
          const u32 c = b[64 * w + lane];
          const u64 nl = __ballot(c == '\n'), cr = __ballot(c == '\r');
          const u64 le = __ballot(is_l(c)), sp = __ballot(is_sp(c));
          if (lane == 0) { mk.nl[w] = nl; mk.cr[w] = cr; mk.let[w] = le; mk.sp[w] = sp; mk.okq[w] = 0; mk.okt[w] = 0; }
        }
      }
      __syncthreads();
      word_tables(mk, nullptr, nullptr, true);
      mark_runs(b, mk, mk.okq, j0, [&](int r) { return tail_qual(mk, r); });
      __syncthreads();
      word_tables(mk, mk.okq, mk.pvq, false);
      __syncthreads();
      mark_runs(b, mk, mk.okt, j0, [&](int r) { return tail_seq2(b, mk, r); });
      __syncthreads();
      word_tables(mk, mk.okt, mk.pvt, false);
      __syncthreads();
      int ends[PER / 8 + 1];
      int starts[PER / 8 + 1];
      int m = 0;
      for (int j = j0; j < j0 + PER; ++j) {
        if (b[j] != '@') continue;
        const int e = record_at(b, mk, j);
        if (e < 0) continue;
        if (m < PER / 8 + 1) { starts[m] = j; ends[m] = e; }
        m++;
      }
      // matching starts may overlap (a run of '@'s can all match), so a lane may hold up to
      // 32: counted exactly, stored through the scan, recomputed when the registers overflow
      const int k0 = block_excl_scan(m, wsum, &total);
      if (m > PER / 8 + 1) { // dense '@' runs: recompute in order
        int k = k0;
        for (int j = j0; j < j0 + PER; ++j) {
          if (b[j] != '@') continue;
          const int e = record_at(b, mk, j);
          if (e < 0) continue;
          if (k < MAXM) { S[k] = (unsigned short)j; E[k] = (unsigned short)e; }
          k++;
        }
      } else {
        for (int i = 0; i < m && k0 + i < MAXM; ++i) {
          S[k0 + i] = (unsigned short)starts[i];
          E[k0 + i] = (unsigned short)ends[i];
        }
      }
      __syncthreads();
      const int K = total;
      if (K > MAXM) { // pathological '@' density: FindAllIndex walked serially
        if (t == 0) {
          int p = 0, le = -1;
          while (p < WIN) {
            if (b[p] != '@') { p++; continue; }
            const int e = record_at(b, mk, p);
            if (e < 0) { p++; continue; }
            le = e;
            if (!last) break;
            p = e;
          }
          st.found = 1;
          st.pos = min(le, WIN - 1);
        }
      } else if (K > 0 && !last) {
        if (t == 0) { st.found = 1; st.pos = min((int)E[0], WIN - 1); }
      } else if (K > 0) {
        // F[k] = first k' with S[k'] >= E[k] (K if none), pinned to k at the chain's end
        for (int k = t; k < K; k += NT) {
          const int e = E[k];
          int lo = k + 1, hi = K;
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (S[mid] >= e) hi = mid; else lo = mid + 1; }
          F[k] = (unsigned short)(lo < K ? lo : k);
        }
        __syncthreads();
        for (int span = 1; span < K; span <<= 1) { // pointer doubling: F <- F o F
          unsigned short nv[MAXM / NT + 1];
          int q = 0;
          for (int k = t; k < K; k += NT) nv[q++] = F[F[k]];
          __syncthreads();
          q = 0;
          for (int k = t; k < K; k += NT) F[k] = nv[q++];
          __syncthreads();
        }
        if (t == 0) { st.found = 1; st.pos = min((int)E[F[0]], WIN - 1); }
      } else if (t == 0) {
        st.found = 0;
      }
    }
    __syncthreads();
    if (t == 0) {
      if (st.found) {
        const i64 m = st.acc + chunk - WIN + st.pos;
        if (st.cnt < row_cap) {
          rows[2 * st.cnt] = (u64)st.curr;
          rows[2 * st.cnt + 1] = (u64)m;
        }
        st.cnt++;
        st.curr += m;
        st.off = st.curr;
        st.acc = 0;
        st.last = 1;
      } else { // recursion: winSize + SeekChunk(offSet + winSize, false)
        st.acc += WIN;
        st.off += WIN;
        st.last = 0;
      }
    }
    __syncthreads();
  }
  if (t == 0) out[0] = st.cnt;
}

}  // namespace

extern "C" hipError_t sidx_launch_chunkrecord(const uint8_t *d, u64 n, int fasta, long long chunk, u64 *rows,
                                              u64 row_cap, u64 *out, hipStream_t s) {
  hipLaunchKernelGGL(k_chunkrecord, dim3(1), dim3(NT), 0, s, d, n, fasta, (i64)chunk, rows, row_cap, out);
  return hipGetLastError();
}
