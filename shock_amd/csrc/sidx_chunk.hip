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
#include "sidx_scan.hpp"

#include <cstdint>

namespace {

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned int u32;

constexpr int WIN = 32768;
constexpr int NT = 1024;
constexpr int PER = WIN / NT;     // 32 window bytes per lane
static_assert(64 % PER == 0, "a lane's window bytes lie in one class word");
constexpr int MAXM = 2048;       // compacted match starts per window (more: serial walk)

__device__ __forceinline__ bool is_nl(u32 c) { return c == '\n' || c == '\r'; }
__device__ __forceinline__ bool is_sp(u32 c) { return c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '; }
__device__ __forceinline__ bool is_l(u32 c) { return ((c | 32) >= 'a' && (c | 32) <= 'z') || c == '-'; }

// Window class masks in LDS (bit j of word j>>6 = window byte j): '\n', '\r', [A-Za-z-],
// RE2 \s.  Every run the regex walks is found 64 bytes at a time from these words.
constexpr int NW = WIN / 64;
struct Masks {
  u64 nl[NW], cr[NW], let[NW], sp[NW], at[NW];
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

// the lane's PER window bits [j0, j0 + PER) of word j0 / 64 (PER divides 64)
__device__ __forceinline__ u64 lane_bits(int j0) {
  return (PER == 64 ? ~0ull : ((1ull << PER) - 1)) << (j0 & 63);
}
// the [\n\r]+ runs that start in [j0, j0 + PER): evaluate `tail` once per run and mark the
// run's positions in ok (LDS 64-bit or).  The run starts come from the class words (a set bit
// whose predecessor is clear), so a lane visits only its runs, not its bytes.
template <class Tail>
__device__ __forceinline__ void mark_runs(const Masks &m, u64 *ok, int j0, Tail tail) {
  const int w = j0 >> 6;
  const u64 x = m.nl[w] | m.cr[w];
  const u64 carry = w > 0 ? (m.nl[w - 1] | m.cr[w - 1]) >> 63 : 0ull;
  u64 st = x & ~((x << 1) | carry) & lane_bits(j0);
  while (st) {
    const int j = (w << 6) + __builtin_ctzll(st);
    st &= st - 1;
    if (tail(j) < 0) continue;
    const int e = next_bit(m, M_NLR, false, j);  // run [j, e)
    for (int x = j; x < e;) {
      const int ww = x >> 6, lo = x & 63;
      const int hi = (e - (ww << 6)) < 64 ? (e - (ww << 6)) : 64;
      const u64 bits = (hi == 64 ? ~0ull : ((1ull << hi) - 1)) & (~0ull << lo);
      atomicOr((unsigned long long *)&ok[ww], (unsigned long long)bits);
      x = (ww + 1) << 6;
    }
  }
}

// word tables, one wave (8 words per lane, a max / min scan over the lanes): nxn[w] = first
// word >= w with a '\n' (NW: none), or pv[w] = last word <= w with a bit of ok (-1: none)
__device__ __forceinline__ void word_tables(Masks &m, const u64 *ok, short *pv, bool nl) {
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
__device__ __forceinline__ int block_excl_scan(int v, int *wsum, int *total) {
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


// SWAR byte classes of a dword: 0x80 in every byte of the class, exact for all byte values
__device__ __forceinline__ u32 cr_eq4(u32 w, u32 c) {
  const u32 x = w ^ (c * 0x01010101u);
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
__device__ __forceinline__ u32 cr_let4(u32 w) {  // [A-Za-z-] (is_l): c | 0x20 in [a, z], or '-'
  const u32 y = w | 0x20202020u, l = y & 0x7F7F7F7Fu;
  return ((l + 0x1F1F1F1Fu) & ~(l + 0x05050505u) & ~y & 0x80808080u) | cr_eq4(w, '-');
}
__device__ __forceinline__ u32 cr_sp4(u32 w) {  // RE2 \s (is_sp): 9, 10, 12, 13, 32
  const u32 l = w & 0x7F7F7F7Fu;
  const u32 r = (l + 0x77777777u) & ~(l + 0x72727272u) & ~w & 0x80808080u;  // 9 <= c <= 13
  return (r & ~cr_eq4(w, 11)) | cr_eq4(w, ' ');
}
// the 0x80 flags of 16 bytes as a 16-bit mask (byte dot products, as eq16)
__device__ __forceinline__ u32 cr_pack16(u32 f0, u32 f1, u32 f2, u32 f3) {
  const u32 lo = __builtin_amdgcn_udot4(f1, 0x80402010u, __builtin_amdgcn_udot4(f0, 0x08040201u, 0u, false), false);
  const u32 hi = __builtin_amdgcn_udot4(f3, 0x80402010u, __builtin_amdgcn_udot4(f2, 0x08040201u, 0u, false), false);
  return (lo >> 7) | ((hi >> 7) << 8);
}
// bytes [sh, sh + 16) of x:y (sh < 16, uniform)
__device__ __forceinline__ uint4 cr_shift16(const uint4 x, const uint4 y, u32 sh) {
  const u32 a[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  const u32 q = sh >> 2, r = (sh & 3u) * 8u;
  u32 o[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    u32 v = a[k];
#pragma unroll
    for (int j = 1; j < 4; ++j) v = q == (u32)j ? a[j + k] : v;
    o[k] = v;
  }
  return make_uint4(__builtin_amdgcn_alignbit(o[1], o[0], r), __builtin_amdgcn_alignbit(o[2], o[1], r),
                    __builtin_amdgcn_alignbit(o[3], o[2], r), __builtin_amdgcn_alignbit(o[4], o[3], r));
}

// ---- one window, one SeekChunk step ---------------------------------------------------------

struct CrSmem {
  __attribute__((aligned(16))) uint8_t raw[WIN + 32];
  unsigned short S[MAXM], E[MAXM], F[MAXM];
  int wsum[NT / 64], total, red[4];
  int found, pos;
  Masks mk;
};

// Window [w, w + WIN) (fastq.go:222-241 / fasta.go:150-170): sm.found / sm.pos = the end of the
// last (last != 0) or first Record match, or the '>' of the last / first "\n>" (then "\r>").
// Uniform over the workgroup; ends with a barrier.
__device__ __forceinline__ void eval_window(const uint8_t *__restrict__ d, u64 n, int fasta, u64 w, int last, CrSmem &sm) {
  const int t = threadIdx.x;
  // stage [w, w + WIN) in LDS, window byte j at raw[j]: two aligned 16-byte loads and a
  // funnel shift per 16 bytes (the shift is the same for every lane); FASTQ: the class words
  // from the same registers (16 bits per lane per class, a 16-bit LDS store each)
  const u64 al0 = w & ~15ull;
  const u32 sh = (u32)(w - al0);
  Masks &mk = sm.mk;
  for (int i = t; i < WIN / 16; i += NT) {
    const u64 al = al0 + 16ull * i;
    uint4 v;
    if (al + 32 <= n) {
      const uint4 *q = reinterpret_cast<const uint4 *>(d + al);
      v = cr_shift16(q[0], q[1], sh);
    } else {
      uint8_t tmp[16];
      for (int k = 0; k < 16; ++k) tmp[k] = w + 16ull * i + k < n ? d[w + 16ull * i + k] : 0;
      v = *reinterpret_cast<const uint4 *>(tmp);
    }
    *reinterpret_cast<uint4 *>(sm.raw + 16 * i) = v;
    if (!fasta) {
      reinterpret_cast<unsigned short *>(mk.nl)[i] = cr_pack16(cr_eq4(v.x, '\n'), cr_eq4(v.y, '\n'), cr_eq4(v.z, '\n'), cr_eq4(v.w, '\n'));
      reinterpret_cast<unsigned short *>(mk.cr)[i] = cr_pack16(cr_eq4(v.x, '\r'), cr_eq4(v.y, '\r'), cr_eq4(v.z, '\r'), cr_eq4(v.w, '\r'));
      reinterpret_cast<unsigned short *>(mk.at)[i] = cr_pack16(cr_eq4(v.x, '@'), cr_eq4(v.y, '@'), cr_eq4(v.z, '@'), cr_eq4(v.w, '@'));
      reinterpret_cast<unsigned short *>(mk.let)[i] = cr_pack16(cr_let4(v.x), cr_let4(v.y), cr_let4(v.z), cr_let4(v.w));
      reinterpret_cast<unsigned short *>(mk.sp)[i] = cr_pack16(cr_sp4(v.x), cr_sp4(v.y), cr_sp4(v.z), cr_sp4(v.w));
    }
  }
  for (int i = t; i < NW; i += NT) { mk.okq[i] = 0; mk.okt[i] = 0; }
  if (t < 4) sm.red[t] = t & 1 ? -1 : 0x7fffffff;  // [0] min '\n>', [1] max '\n>', [2] min '\r>', [3] max '\r>'
  __syncthreads();
  const uint8_t *b = sm.raw;
  const int j0 = t * PER;
  if (fasta) {
    int mnN = 0x7fffffff, mxN = -1, mnR = 0x7fffffff, mxR = -1;
    for (int j = j0; j < j0 + PER && j + 1 < WIN; ++j) {
      if (b[j + 1] != '>') continue;
      if (b[j] == '\n') { mnN = min(mnN, j); mxN = max(mxN, j); }
      else if (b[j] == '\r') { mnR = min(mnR, j); mxR = max(mxR, j); }
    }
    if (mxN >= 0) { atomicMin(&sm.red[0], mnN); atomicMax(&sm.red[1], mxN); }
    if (mxR >= 0) { atomicMin(&sm.red[2], mnR); atomicMax(&sm.red[3], mxR); }
    __syncthreads();
    if (t == 0) {
      const int pn = last ? sm.red[1] : (sm.red[0] == 0x7fffffff ? -1 : sm.red[0]);
      const int pr = last ? sm.red[3] : (sm.red[2] == 0x7fffffff ? -1 : sm.red[2]);
      const int p = pn >= 0 ? pn : pr;
      sm.found = p >= 0;
      sm.pos = p + 1;
    }
    __syncthreads();
    return;
  }
  word_tables(mk, nullptr, nullptr, true);
  mark_runs(mk, mk.okq, j0, [&](int r) { return tail_qual(mk, r); });
  __syncthreads();
  word_tables(mk, mk.okq, mk.pvq, false);
  __syncthreads();
  mark_runs(mk, mk.okt, j0, [&](int r) { return tail_seq2(b, mk, r); });
  __syncthreads();
  word_tables(mk, mk.okt, mk.pvt, false);
  __syncthreads();
  // the lane's matching '@' positions as bits (matching starts may overlap: a run of '@'s can
  // all match), their count scanned, then each match's end recomputed into S / E in order --
  // about one '@' per lane in ten, so the second evaluation costs less than registers would
  const int wb = (j0 >> 6) << 6;
  u64 hit = 0;
  for (u64 a = mk.at[j0 >> 6] & lane_bits(j0); a;) {
    const int j = wb + __builtin_ctzll(a);
    a &= a - 1;
    if (record_at(b, mk, j) >= 0) hit |= 1ull << (j - wb);
  }
  const int k0 = block_excl_scan(__popcll(hit), sm.wsum, &sm.total);
  int k = k0;
  for (u64 a = hit; a && k < MAXM; ++k) {
    const int j = wb + __builtin_ctzll(a);
    a &= a - 1;
    sm.S[k] = (unsigned short)j;
    sm.E[k] = (unsigned short)record_at(b, mk, j);
  }
  __syncthreads();
  const int K = sm.total;
  if (K > MAXM) {  // pathological '@' density: FindAllIndex walked serially
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
      sm.found = 1;
      sm.pos = min(le, WIN - 1);
    }
  } else if (K > 0 && !last) {
    if (t == 0) { sm.found = 1; sm.pos = min((int)sm.E[0], WIN - 1); }
  } else if (K > 0) {
    // F[k] = first k' with S[k'] >= E[k] (K if none), pinned to k at the chain's end
    for (int k = t; k < K; k += NT) {
      const int e = sm.E[k];
      int lo = k + 1, hi = K;
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (sm.S[mid] >= e) hi = mid; else lo = mid + 1; }
      sm.F[k] = (unsigned short)(lo < K ? lo : k);
    }
    __syncthreads();
    for (int span = 1; span < K; span <<= 1) {  // pointer doubling: F <- F o F
      unsigned short nv[MAXM / NT + 1];
      int q = 0;
      for (int k = t; k < K; k += NT) nv[q++] = sm.F[sm.F[k]];
      __syncthreads();
      q = 0;
      for (int k = t; k < K; k += NT) sm.F[k] = nv[q++];
      __syncthreads();
    }
    if (t == 0) { sm.found = 1; sm.pos = min((int)sm.E[sm.F[0]], WIN - 1); }
  } else if (t == 0) {
    sm.found = 0;
  }
  __syncthreads();
}

// SeekChunk(curr, true) with its recursion into the following windows (fastq.go:216-243,
// fasta.go:143-173): the chunk length m, or -1 when a window read is short (io.EOF).
// Uniform over the workgroup.
__device__ __forceinline__ i64 seek_step(const uint8_t *__restrict__ d, u64 n, int fasta, i64 chunk, i64 curr, CrSmem &sm) {
  i64 off = curr, acc = 0;
  int last = 1;
  for (;;) {
    const i64 w = off + chunk - WIN;
    if ((u64)w + WIN > n) return -1;
    eval_window(d, n, fasta, (u64)w, last, sm);
    const int found = sm.found, pos = sm.pos;
    __syncthreads();  // every lane has read the result before the next window reuses sm
    if (found) return acc + chunk - WIN + pos;
    acc += WIN;  // recursion: winSize + SeekChunk(offSet + winSize, false)
    off += WIN;
    last = 0;
  }
}

// The serial walk (the definition, and the fallback of the speculative build): rows from
// (curr0, row cnt0) for at most max_steps chunks; out = {count, curr, done}.
__global__ __launch_bounds__(NT) void k_chunkrecord(const uint8_t *__restrict__ d, u64 n, int fasta, i64 chunk,
                                                    u64 *__restrict__ rows, u64 row_cap, u64 *__restrict__ out,
                                                    i64 curr0, u64 cnt0, u64 max_steps) {
  __shared__ CrSmem sm;
  i64 curr = curr0;
  u64 cnt = cnt0;
  int done = 0;
  for (u64 st = 0; st < max_steps; ++st) {
    const i64 m = seek_step(d, n, fasta, chunk, curr, sm);
    if (threadIdx.x == 0 && cnt < row_cap) {
      rows[2 * cnt] = (u64)curr;
      rows[2 * cnt + 1] = m < 0 ? n - (u64)curr : (u64)m;
    }
    cnt++;
    if (m < 0) { done = 1; break; }
    curr += m;
  }
  if (threadIdx.x == 0) { out[0] = cnt; out[1] = (u64)curr; out[2] = (u64)done; }
}

// ---- speculative build ----------------------------------------------------------------------
// Chunk k+1 starts at f(curr_k), f = SeekChunk.  f lands on a small set of positions: for FASTQ
// the end of a Record match, which on record-index-valid data is the next record's start
// (a match ends after its quality line's [\n\r]+ run), or window end - 1 when the window cuts
// a record's final [\n\r]+ run (the 32767 clamp); for FASTA the '>' of a "\n>".  These
// positions are the nodes of a functional graph: J1[v] = the predicted f from node v, computed
// for every node at once from the sorted node positions.  Doubling J1 gives J_L (L steps), the
// path from position 0 is walked L nodes at a time and expanded, and every chunk of the path
// is then evaluated exactly (seek_step, one workgroup per chunk, all in parallel).  The first
// chunk whose exact f differs from the path's next position is where the path is re-entered
// (or walked serially when that position is not a node), so the result is the serial walk's
// by construction; on well-formed files the first path is the answer.
//   FASTQ nodes: v = 3 i + delta -> position off[i] - delta, delta in {0, 1, 2} (off = the
//                record index's row offsets, rows valid up to the first error)
//   FASTA nodes: v -> G[v], G = {0} + every '>' preceded by '\n', ascending
constexpr u32 NODE_END = 0xFFFFFFFFu;    // f reads a short window: the chunk is the file's last
constexpr u32 NODE_IRR = 0xFFFFFFFEu;    // no prediction (long records, the table's tail, ...)
constexpr u32 NODE_NONE = 0xFFFFFFFDu;   // a position that is not a node
constexpr u64 KIND_CAP = 0xFFFFFFFCu;    // the path reached the row capacity
constexpr int CT = 16384;                // position-table tile

struct Bases {
  const u64 *p;   // ascending base positions, p[i * stride]
  u64 stride, count;
  const u64 *ft;  // ft[t] = first base index with position >= t * CT, t in [0, ntile]
  u64 ntile;
};
__device__ __forceinline__ u64 bpos(const Bases &b, u64 i) { return b.p[i * b.stride]; }
// last base index with position <= y, -1 if none
__device__ i64 last_le(const Bases &b, u64 y) {
  u64 t = y / CT;
  if (t >= b.ntile) t = b.ntile - 1;
  u64 lo = b.ft[t], hi = b.ft[t + 1];
  if (y >= (t + 1) * (u64)CT) { lo = hi; }  // past the last tile: every base <= y
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (bpos(b, mid) <= y) lo = mid + 1; else hi = mid;
  }
  return (i64)lo - 1;
}
__device__ __forceinline__ u64 node_pos(const Bases &b, int fasta, u32 v) {
  return fasta ? bpos(b, v) : bpos(b, v / 3) - v % 3;
}
__device__ u32 node_of(const Bases &b, int fasta, u64 y) {
  const i64 j = last_le(b, y);
  if (fasta) return (j >= 0 && bpos(b, (u64)j) == y) ? (u32)j : NODE_NONE;
  if (j >= 0 && bpos(b, (u64)j) == y) return 3u * (u32)j;
  const u64 i = (u64)(j + 1);
  if (i == 0 || i >= b.count) return NODE_NONE;
  const u64 dl = bpos(b, i) - y;
  return dl <= 2 ? 3u * (u32)i + (u32)dl : NODE_NONE;
}

__global__ void k_cr_ftab(Bases b, u64 *__restrict__ ft) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > b.ntile) return;
  const u64 y = t * (u64)CT;
  u64 lo = 0, hi = b.count;
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (bpos(b, mid) < y) lo = mid + 1; else hi = mid;
  }
  ft[t] = lo;
}

__device__ __forceinline__ bool nlb(uint8_t c) { return c == '\n' || c == '\r'; }

// J1 for FASTQ nodes.  From p: x = p + chunk is the window end.  j = the record holding x - 1.
// x - 1 inside record j's closing [\n\r] run (at most 2 bytes before the next record) -> the
// match of record j ends at x (clamped to x - 1); otherwise the last match is record j - 1,
// ending at off[j].  Either record must lie inside the window.
__global__ void k_cr_next_fq(Bases b, const uint8_t *__restrict__ d, u64 n, u64 chunk, u32 *__restrict__ J1) {
  // one thread per record: its three nodes' window ends are 0-2 bytes apart, so the record
  // holding x - 1 is searched once and stepped back (records are >= 8 bytes apart)
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.count) return;
  const u64 p0 = bpos(b, i);
  i64 j = -2;  // last_le(x - 1) of the previous node (-2: not searched yet)
  u32 r3[3];
#pragma unroll
  for (int dl = 0; dl < 3; ++dl) {
    u32 r = NODE_IRR;
    if (!(dl && i == 0)) {
      const u64 x = p0 - (u64)dl + chunk;
      if (x > n) {
        r = NODE_END;
      } else {
        if (j == -2) j = last_le(b, x - 1);
        else
          while (j >= 0 && bpos(b, (u64)j) > x - 1) --j;
        if (j >= 0 && (u64)j + 1 < b.count) {
          const u64 e = bpos(b, (u64)j + 1), dd = e - (x - 1), w = x - WIN;
          if (dd <= 2 && nlb(d[x - 1]) && (dd == 1 || nlb(d[x]))) {
            if (bpos(b, (u64)j) >= w) r = 3u * (u32)(j + 1) + (u32)dd;
          } else if (j >= 1 && bpos(b, (u64)j - 1) >= w) {
            r = 3u * (u32)j;
          }
        }
      }
    }
    r3[dl] = r;
  }
  J1[3 * i] = r3[0];
  J1[3 * i + 1] = r3[1];
  J1[3 * i + 2] = r3[2];
}

// J1 for FASTA nodes: the last "\n>" of [x - WIN, x), else the first one of the following
// windows (each must be a full window; a pair split across two windows is left unpredicted)
__global__ void k_cr_next_fa(Bases b, u64 n, u64 chunk, u32 *__restrict__ J1) {
  const u64 v = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= b.count) return;
  const u64 p = bpos(b, v), x = p + chunk;
  u32 r = NODE_IRR;
  if (x > n) {
    r = NODE_END;
  } else {
    const i64 j = last_le(b, x - 1);
    if (j >= 1 && bpos(b, (u64)j) >= x - WIN + 1) {
      r = (u32)j;
    } else if ((u64)(j + 1) >= b.count) {
      r = NODE_END;  // no "\n>" left: windows until a short one
    } else {
      const u64 g = bpos(b, (u64)j + 1);
      if (g > x) {
        const u64 kk = (g - 1 - x) / WIN + 1;
        if (x + kk * WIN > n) r = NODE_END;
        else if (g <= x + kk * WIN - 1) r = (u32)(j + 1);
      }
    }
  }
  J1[v] = r;
}

__device__ __forceinline__ u32 jump2(const u32 *__restrict__ Jin, u32 a) { return a >= NODE_NONE ? a : Jin[a]; }
__global__ void k_cr_double(const u32 *__restrict__ Jin, u32 *__restrict__ Jout, u64 nn) {
  const u64 v = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nn) return;
  Jout[v] = jump2(Jin, Jin[v]);
}
// four nodes per thread (16-byte aligned tables): the gathers of a thread are independent, so
// four are in flight per lane; the targets of consecutive nodes are close (successors are
// monotone in the position), so they coalesce much like the streaming part
__global__ void k_cr_double4(const u32 *__restrict__ Jin, u32 *__restrict__ Jout, u64 nn) {
  const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x, v = 4 * q;
  if (v >= nn) return;
  if (v + 4 <= nn) {
    const uint4 a = reinterpret_cast<const uint4 *>(Jin)[q];
    reinterpret_cast<uint4 *>(Jout)[q] = make_uint4(jump2(Jin, a.x), jump2(Jin, a.y), jump2(Jin, a.z), jump2(Jin, a.w));
  } else {
    for (u64 i = v; i < nn; ++i) Jout[i] = jump2(Jin, Jin[i]);
  }
}
// Jout = Jin o Jin over nn nodes
static void launch_double(const u32 *Jin, u32 *Jout, u64 nn, hipStream_t s) {
  if ((((uintptr_t)Jin | (uintptr_t)Jout) & 15) == 0)
    hipLaunchKernelGGL(k_cr_double4, dim3((u32)((nn + 1023) / 1024)), dim3(256), 0, s, Jin, Jout, nn);
  else
    hipLaunchKernelGGL(k_cr_double, dim3((u32)((nn + 255) / 256)), dim3(256), 0, s, Jin, Jout, nn);
}

// ctl: [0] K (path length), [1] terminal kind, [2] first bad path index (~0: none), [3] its
//      exact m, [4] its exact next position
// The path from y (at most cap nodes, indexed from 0): heads every L nodes (one lane), then
// expanded L nodes per lane.
__global__ void k_cr_path(Bases b, int fasta, u64 y, const u32 *__restrict__ JL, const u32 *__restrict__ J1, u32 L,
                          u64 cap, u32 *__restrict__ heads, u64 *__restrict__ pos, u64 *__restrict__ ctl) {
  __shared__ u64 sH;
  if (threadIdx.x == 0) {
    const u32 v = node_of(b, fasta, y);
    ctl[0] = 0;
    ctl[1] = v == NODE_NONE ? NODE_NONE : 0;
    ctl[2] = ~0ull;
    u64 H = 0;
    if (v != NODE_NONE) {
      u32 h = v;
      while (h < NODE_NONE && H * L < cap) {
        heads[H++] = h;
        h = JL[h];
      }
    }
    sH = H;
  }
  __syncthreads();
  const u64 H = sH;
  for (u64 hh = threadIdx.x; hh < H; hh += blockDim.x) {
    u32 v = heads[hh];
    const bool tail = hh + 1 == H;
    u64 k = hh * L;
    u64 kind = KIND_CAP;
    for (u32 u = 0; u < L; ++u, ++k) {
      if (k >= cap) break;
      pos[k] = node_pos(b, fasta, v);
      const u32 nx = J1[v];
      if (nx >= NODE_NONE) { kind = nx; ++k; break; }
      v = nx;
    }
    if (tail) { ctl[0] = k; ctl[1] = kind; }
  }
}

// Every chunk of the path evaluated exactly, one workgroup per chunk (persistent grid): rows
// written at k0 + the path index, the first chunk whose f disagrees with the path (or whose
// window is short before the path ends) recorded.
#ifndef SIDX_CR_WPE
#define SIDX_CR_WPE 8  // waves per SIMD forced on k_cr_verify: two 1024-thread workgroups per CU (64 VGPRs, 9 spilled):
                       // FASTQ chunkrecord 8.16 -> 7.24 ms per 10 GiB; 0: the compiler's choice (89 VGPRs, one per CU)
#endif
#if SIDX_CR_WPE
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(SIDX_CR_WPE, SIDX_CR_WPE))) void k_cr_verify(
#else
__global__ __launch_bounds__(NT) void k_cr_verify(
#endif
    const uint8_t *__restrict__ d, u64 n, int fasta, i64 chunk,
                                                  const u64 *__restrict__ pos, i64 *__restrict__ mres, u64 k0,
                                                  u64 *__restrict__ ctl, u64 *__restrict__ rows, u64 row_cap) {
  __shared__ CrSmem sm;
  const u64 K = ctl[0];
  for (u64 k = blockIdx.x; k < K; k += gridDim.x) {
    const i64 p = (i64)pos[k];
    const i64 m = seek_step(d, n, fasta, chunk, p, sm);
    if (threadIdx.x == 0) {
      mres[k] = m;
      if (k0 + k < row_cap) {
        rows[2 * (k0 + k)] = (u64)p;
        rows[2 * (k0 + k) + 1] = m < 0 ? n - (u64)p : (u64)m;
      }
      const bool ok = k + 1 < K ? (m >= 0 && (u64)(p + m) == pos[k + 1]) : m < 0;
      if (!ok) atomicMin((unsigned long long *)&ctl[2], (unsigned long long)k);
    }
  }
}

__global__ void k_cr_fin(const u64 *__restrict__ pos, const i64 *__restrict__ mres, u64 *__restrict__ ctl) {
  const u64 k = ctl[2];
  if (k != ~0ull) {
    ctl[3] = (u64)mres[k];
    ctl[4] = pos[k] + (u64)mres[k];
  }
}

// FASTA node positions: per CT tile the "\n>" pairs whose '>' lies in it (pass 1 counts, pass
// 2 writes at 1 + the tile's exclusive offset; G[0] = 0 is written by the host)
// 16 bytes -> 16-bit mask of the bytes equal to c (bit 7 per differing byte, packed with
// byte dot products; as sidx_device.hpp's eq16)
__device__ __forceinline__ u32 ne4(u32 w, u32 pat) {
  const u32 x = w ^ pat;
  return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
__device__ __forceinline__ u32 eq16(const uint4 v, u32 c) {
  const u32 pat = c * 0x01010101u;
  const u32 lo = __builtin_amdgcn_udot4(ne4(v.y, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(ne4(v.x, pat), 0x08040201u, 0u, false), false);
  const u32 hi = __builtin_amdgcn_udot4(ne4(v.w, pat), 0x80402010u,
                                        __builtin_amdgcn_udot4(ne4(v.z, pat), 0x08040201u, 0u, false), false);
  return ((lo >> 7) | (hi << 1)) ^ 0xFFFFu;
}

// the '>' of every "\n>" in [a, a + 64) as a bit mask (a is 64-aligned)
__device__ __forceinline__ u64 gt_pairs(const uint8_t *__restrict__ d, u64 n, u64 a) {
  u64 mgt = 0, mnl = 0;
  if (a + 64 <= n) {
    const uint4 *q = reinterpret_cast<const uint4 *>(d + a);
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = q[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mgt |= (u64)eq16(v[k], '>') << (16 * k);
      mnl |= (u64)eq16(v[k], '\n') << (16 * k);
    }
  } else {
    for (int bit = 0; bit < 64 && a + bit < n; ++bit) {
      const uint8_t c = d[a + bit];
      mgt |= (u64)(c == '>') << bit;
      mnl |= (u64)(c == '\n') << bit;
    }
  }
  const u64 prev = (a > 0 && a - 1 < n && d[a - 1] == '\n') ? 1ull : 0ull;
  return mgt & ((mnl << 1) | prev);
}

// The input is read once: pass 1 counts each tile's pairs and, when they fit, keeps their
// tile-relative positions in the tile's slot (GSLOT u16s); pass 2 places slots at the scanned
// offsets and re-reads only the tiles whose pairs did not fit (FASTA records < 256 B average).
constexpr u32 GSLOT = 64;
__device__ __forceinline__ u64 block_excl256(u64 c, u64 *ws, u64 &total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 x = c;
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y2 = __shfl_up(x, o, 64);
    if (lane >= o) x += y2;
  }
  if (lane == 63) ws[wv] = x;
  __syncthreads();
  u64 off = x - c;
  for (int i = 0; i < wv; ++i) off += ws[i];
  total = ws[0] + ws[1] + ws[2] + ws[3];
  return off;
}

__global__ __launch_bounds__(256) void k_cr_gcount(const uint8_t *__restrict__ d, u64 n, u64 *__restrict__ tcnt,
                                                   uint16_t *__restrict__ slot) {
  __shared__ u64 ws[4];
  const u64 a = (u64)blockIdx.x * CT + 64ull * threadIdx.x;
  u64 msk = a < n ? gt_pairs(d, n, a) : 0;
  u64 total = 0;
  u64 off = block_excl256((u64)__builtin_popcountll(msk), ws, total);
  if (total <= GSLOT) {
    uint16_t *sl = slot + (u64)blockIdx.x * GSLOT;
    while (msk) {
      sl[off++] = (uint16_t)(64u * threadIdx.x + (u32)__builtin_ctzll(msk));
      msk &= msk - 1;
    }
  }
  if (threadIdx.x == 0) tcnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_cr_gwrite(const uint8_t *__restrict__ d, u64 n, const u64 *__restrict__ tcnt,
                                                   const u64 *__restrict__ toff, const uint16_t *__restrict__ slot,
                                                   u64 *__restrict__ G) {
  __shared__ u64 ws[4];
  const u64 c_t = tcnt[blockIdx.x], base = 1 + toff[blockIdx.x], t0 = (u64)blockIdx.x * CT;
  if (c_t <= GSLOT) {  // from the slot: no file bytes read
    if (threadIdx.x < c_t) G[base + threadIdx.x] = t0 + slot[(u64)blockIdx.x * GSLOT + threadIdx.x];
    return;
  }
  const u64 a = t0 + 64ull * threadIdx.x;
  u64 msk = a < n ? gt_pairs(d, n, a) : 0;
  u64 total = 0;
  u64 off = base + block_excl256((u64)__builtin_popcountll(msk), ws, total);
  while (msk) {
    G[off++] = a + (u64)__builtin_ctzll(msk);
    msk &= msk - 1;
  }
}

}  // namespace

extern "C" hipError_t sidx_launch_chunkrecord(const uint8_t *d, u64 n, int fasta, long long chunk, u64 *rows,
                                              u64 row_cap, u64 *out, long long curr0, u64 cnt0, u64 max_steps,
                                              hipStream_t s) {
  hipLaunchKernelGGL(k_chunkrecord, dim3(1), dim3(NT), 0, s, d, n, fasta, (i64)chunk, rows, row_cap, out, (i64)curr0,
                     cnt0, max_steps);
  return hipGetLastError();
}

// FASTA node positions into G (G[0] = 0); tcnt/toff: ntile = ceil(n / CT) words each, slot:
// ntile * GSLOT u16s; scan_tmp null -> size query.  The caller reads |G| = 1 + toff[last] +
// tcnt[last] after the count pass.
extern "C" hipError_t sidx_cr_gpos_count(const uint8_t *d, u64 n, u64 *tcnt, u64 *toff, uint16_t *slot,
                                         void *scan_tmp, size_t *scan_bytes, hipStream_t s) {
  const u64 nt = (n + CT - 1) / CT;
  if (!scan_tmp) return sidx::dscan::run<u64, sidx::dscan::Sum, true>(nullptr, scan_bytes, tcnt, toff, nt ? nt : 1, s);
  if (!nt) return hipSuccess;
  hipLaunchKernelGGL(k_cr_gcount, dim3((u32)nt), dim3(256), 0, s, d, n, tcnt, slot);
  return sidx::dscan::run<u64, sidx::dscan::Sum, true>(scan_tmp, scan_bytes, tcnt, toff, nt, s);
}
extern "C" hipError_t sidx_cr_gpos_write(const uint8_t *d, u64 n, const u64 *tcnt, const u64 *toff,
                                         const uint16_t *slot, u64 *G, hipStream_t s) {
  const u64 nt = (n + CT - 1) / CT;
  if (nt) hipLaunchKernelGGL(k_cr_gwrite, dim3((u32)nt), dim3(256), 0, s, d, n, tcnt, toff, slot, G);
  return hipGetLastError();
}
extern "C" u32 sidx_cr_gslot() { return GSLOT; }

// Predicted-successor graph over the nodes and its L = 2^levels jump table: ft ((ntile + 1)
// words), J1 / Ja / Jb (nodes words each).  *JL receives the L-step table.
extern "C" hipError_t sidx_cr_graph(const uint8_t *d, u64 n, int fasta, u64 chunk, const u64 *base, u64 stride,
                                    u64 count, u64 *ft, u32 *J1, u32 *Ja, u32 *Jb, int levels, const u32 **JL,
                                    hipStream_t s) {
  const u64 ntile = n / CT + 1;
  Bases b{base, stride, count, ft, ntile};
  hipLaunchKernelGGL(k_cr_ftab, dim3((u32)((ntile + 256) / 256)), dim3(256), 0, s, b, ft);
  const u64 nn = fasta ? count : 3 * count;
  const u32 g = (u32)((nn + 255) / 256);
  if (fasta) hipLaunchKernelGGL(k_cr_next_fa, dim3(g), dim3(256), 0, s, b, n, chunk, J1);
  else hipLaunchKernelGGL(k_cr_next_fq, dim3((u32)((count + 255) / 256)), dim3(256), 0, s, b, d, n, chunk, J1);
  const u32 *cur = J1;
  for (int l = 0; l < levels; ++l) {
    u32 *nxt = (l & 1) ? Jb : Ja;
    launch_double(cur, nxt, nn, s);
    cur = nxt;
  }
  *JL = cur;
  return hipGetLastError();
}

// One round: the path from position y (at most cap nodes; its first chunk is row k0), every
// chunk of it evaluated exactly (verify_grid workgroups), the first disagreement into ctl[2..4].
extern "C" hipError_t sidx_cr_round(const uint8_t *d, u64 n, int fasta, u64 chunk, const u64 *base, u64 stride,
                                    u64 count, const u64 *ft, const u32 *JL, const u32 *J1, u32 L, u64 y, u64 k0,
                                    u64 cap, u32 *heads, u64 *pos, i64 *mres, u64 *ctl, u64 *rows, u64 row_cap,
                                    u32 verify_grid, hipStream_t s) {
  Bases b{base, stride, count, ft, n / CT + 1};
  hipLaunchKernelGGL(k_cr_path, dim3(1), dim3(256), 0, s, b, fasta, y, JL, J1, L, cap, heads, pos, ctl);
  hipLaunchKernelGGL(k_cr_verify, dim3(verify_grid), dim3(NT), 0, s, d, n, fasta, (i64)chunk, pos, mres, k0, ctl,
                     rows, row_cap);
  hipLaunchKernelGGL(k_cr_fin, dim3(1), dim3(1), 0, s, pos, mres, ctl);
  return hipGetLastError();
}

extern "C" int sidx_cr_verify_blocks_per_cu() {
  int nb = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_cr_verify, NT, 0) == hipSuccess ? nb : 0;
}

namespace {

// ---- chunkrecord of a subset node (index/chunkrecord.go:100-228) ----------------------------
// The subset node's record index rows are grouped into chunks of rows by a greedy loop: a row
// joins the open chunk unless the chunk's length plus the row's reaches 1 MiB (:167).  Every
// chunk begins at a "fresh start" a (the loop's acc == 0 state, or the row that did not fit,
// which behaves the same): zero-length rows there are skipped (:159-164 resets the start), a
// row >= 1 MiB is a chunk alone (:170-184), else the chunk runs to the last row whose running
// sum stays below 1 MiB.  With P = prefix sums of the lengths each fresh start's chunk and
// successor are two binary searches, so the successor graph over the R + 1 starts (R: past the
// end, absorbing) is built for every start at once and the path from row 0 found by pointer
// doubling, as for the file chunkrecord -- exact, no verification pass needed.
constexpr u64 SUB_LIMIT = 1048576;  // chunkrecord.go:167

__global__ void k_crs_len(const u64 *__restrict__ ri, u64 R, u64 *__restrict__ len) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < R) len[i] = ri[2 * i + 1];
}

// first q in [lo, hi) with P[q] >= v, hi if none
__device__ __forceinline__ u64 lower_bound_u64(const u64 *P, u64 lo, u64 hi, u64 v) {
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (P[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// fresh start a -> (first row a1 of its chunk, end e (exclusive); a1 == R: no chunk), returns
// the next fresh start (R: end)
__device__ u64 crs_step(const u64 *__restrict__ P, u64 R, u64 a, u64 &a1, u64 &e) {
  a1 = R;
  e = R;
  if (a >= R) return R;
  const u64 q = lower_bound_u64(P, a + 1, R + 1, P[a] + 1);  // first row with a nonzero length, + 1
  if (q > R) return R;                                        // only zero-length rows left: no chunk
  a1 = q - 1;
  if (P[q] - P[a1] >= SUB_LIMIT) { e = a1 + 1; return a1 + 1; }  // a row of >= 1 MiB alone
  const u64 q2 = lower_bound_u64(P, a1 + 1, R + 1, P[a1] + SUB_LIMIT);
  if (q2 > R) { e = R; return R; }                            // runs to the last row
  e = q2 - 1;                                                 // row q2 - 1 does not fit
  return q2 - 1;
}

__global__ void k_crs_next(const u64 *__restrict__ P, u64 R, u32 *__restrict__ J1) {
  const u64 a = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (a > R) return;
  u64 a1, e;
  J1[a] = (u32)crs_step(P, R, a, a1, e);
}

// The path from start 0: heads every L starts (one lane), expanded L per lane; row k = the k-th
// chunk (16 * first row, 16 * rows).  ctl[0] = rows.
__global__ void k_crs_path(const u64 *__restrict__ P, u64 R, const u32 *__restrict__ JL, const u32 *__restrict__ J1,
                           u32 L, u32 *__restrict__ heads, u64 *__restrict__ rows, u64 row_cap, u64 *__restrict__ ctl) {
  __shared__ u64 sH;
  if (threadIdx.x == 0) {
    u64 H = 0;
    u32 h = 0;
    while (h < R) {
      heads[H++] = h;
      h = JL[h];
    }
    sH = H;
    ctl[0] = 0;
  }
  __syncthreads();
  const u64 H = sH;
  for (u64 hh = threadIdx.x; hh < H; hh += blockDim.x) {
    u64 a = heads[hh], k = hh * L;
    for (u32 u = 0; u < L && a < R; ++u) {
      u64 a1, e;
      const u64 nx = crs_step(P, R, a, a1, e);
      if (a1 < R) {
        if (k < row_cap) { rows[2 * k] = 16 * a1; rows[2 * k + 1] = 16 * (e - a1); }
        ++k;
      }
      a = nx;
    }
    if (hh + 1 == H) ctl[0] = k;
  }
}

}  // namespace (subset chunkrecord)

// Subset-node chunkrecord over a device-resident record index (ri: R rows): tmp = scan
// temporaries (null -> size query into *scan_bytes); P: R + 1 words; len: R words; J1 / Ja /
// Jb: R + 1 words; heads: R / 2^levels + 2 words; ctl: 8 words.
extern "C" hipError_t sidx_crs_scan(const u64 *ri, u64 R, u64 *len, u64 *P, void *tmp, size_t *scan_bytes,
                                    hipStream_t s) {
  if (!tmp) return sidx::dscan::run<u64, sidx::dscan::Sum, false>(nullptr, scan_bytes, len, P + 1, R ? R : 1, s);
  hipError_t e = hipMemsetAsync(P, 0, 8, s);
  if (e != hipSuccess || !R) return e;
  hipLaunchKernelGGL(k_crs_len, dim3((u32)((R + 255) / 256)), dim3(256), 0, s, ri, R, len);
  return sidx::dscan::run<u64, sidx::dscan::Sum, false>(tmp, scan_bytes, len, P + 1, R, s);
}
extern "C" hipError_t sidx_crs_build(const u64 *P, u64 R, u32 *J1, u32 *Ja, u32 *Jb, int levels, u32 *heads, u64 *rows,
                                     u64 row_cap, u64 *ctl, hipStream_t s) {
  const u32 g = (u32)((R + 1 + 255) / 256);
  hipLaunchKernelGGL(k_crs_next, dim3(g), dim3(256), 0, s, P, R, J1);
  const u32 *cur = J1;
  for (int l = 0; l < levels; ++l) {
    u32 *nxt = (l & 1) ? Jb : Ja;
    launch_double(cur, nxt, R + 1, s);
    cur = nxt;
  }
  hipLaunchKernelGGL(k_crs_path, dim3(1), dim3(256), 0, s, P, R, cur, J1, 1u << levels, heads, rows, row_cap, ctl);
  return hipGetLastError();
}
