// sidx_subset.hip -- gfx950 kernels of the subset path:
// a subset node built from a sorted list of 1-based record ids over a device-resident
// record index, and the subset node's bytes gathered from the parent file.
//
// Reference semantics (paths relative to /root/reference/shock-server/):
//   node/file/index/subset.go:133-303   CreateSubsetNodeIndexes: ids read with ReadLine,
//       blank lines skipped, strconv.Atoi, strictly increasing, <= TotalUnits, parent row
//       (id-1), subset index row per id, compressed index = maximal runs of contiguous rows
//       (offset == prevOffset + prevLength), final run written only when oSize != 0
//   controller/node/single.go:500-517 + request/streamer.go:58-117: a subset node's data is
//       the concatenation of its compressed-index runs of the parent file
//
// Pipeline (device): the id text's line ends (k_idl_count -> scan -> k_idl_emit; the line count
// is the one host round trip) -> k_sub_parse (Atoi per line) -> exclusive scan of "non-blank"
// flags -> k_sub_compact -> k_sub_check (order, bounds, row gather, run starts, first failing
// line) -> scan of run starts -> k_sub_nstart (Ke, run count) -> k_sub_runs / k_sub_run_len
// (compressed rows, oSize).  Gather: k_run_lengths -> scan of run lengths -> k_gather_plan
// (byte total, first run of every 32 KiB output block) -> k_gather.
#include <hip/hip_runtime.h>
#include "sidx_scan.hpp"

#include "sidx_common.hpp"
#include "sidx_subset.hpp"

namespace sidx {

// ---- strconv.Atoi per line (subset.go:201-206) -------------------------------------------
// Go: fast path for 0 < len < 19 (optional sign, digits); else ParseInt(s, 10, 0) where the
// first syntax or overflow event scanning left to right decides, then the int64 range.
__device__ __forceinline__ u32 go_atoi(const uint8_t *s, u64 n, i64 &v) {
  if (n > 0 && n < 19) {
    u64 i = 0;
    const bool neg = s[0] == '-';
    if (s[0] == '-' || s[0] == '+') {
      i = 1;
      if (n < 2) return SUB_SYNTAX;
    }
    i64 x = 0;
    for (; i < n; ++i) {
      const u32 d = (u32)(uint8_t)(s[i] - '0');
      if (d > 9) return SUB_SYNTAX;
      x = x * 10 + d;
    }
    v = neg ? -x : x;
    return SUB_OK;
  }
  if (n == 0) return SUB_SYNTAX;
  u64 i = 0;
  bool neg = false;
  if (s[0] == '+') i = 1;
  else if (s[0] == '-') { neg = true; i = 1; }
  if (i == n) return SUB_SYNTAX;
  const u64 cutoff10 = ~0ull / 10 + 1;
  u64 u = 0;
  for (; i < n; ++i) {
    const u32 c = s[i];
    if (c < '0' || c > '9') return SUB_SYNTAX;
    if (u >= cutoff10) return SUB_RANGE;
    const u64 u1 = u * 10 + (c - '0');
    if (u1 < u * 10) return SUB_RANGE;
    u = u1;
  }
  const u64 cut = 1ull << 63;
  if ((!neg && u >= cut) || (neg && u > cut)) return SUB_RANGE;
  v = neg ? (i64)(0 - u) : (i64)u;
  return SUB_OK;
}

// ---- the id text's lines (subset.go:189-199: ReadLine = ReadBytes('\n'); the bytes after the
// last '\n' are dropped) ----------------------------------------------------------------------
// Id lines average under 16 bytes, so the line tile pass (k_line_tiles / k_line_place) would
// rescan every tile from global memory on one wave (85 us for the C4 ids, 24 workgroups busy).
// Instead: the '\n' count of every 1 KiB block (one wave, 16 bytes per lane), their exclusive
// scan, then every block's wave writes the positions of its '\n's in order: ends[k] = the
// position of the k-th '\n', line k = [ends[k - 1] + 1, ends[k]] (the first from 0).
constexpr u32 IDL_BLOCK = 1024;
__device__ __forceinline__ u32 idl_mask(const uint8_t *text, u64 n, u64 a) {  // '\n' bits of bytes [a, a + 16)
  u32 m = 0;
  if (a + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4 *>(text + a);
    const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) m |= (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == '\n' ? 1u : 0u) << i;
  } else {
    for (u64 i = a; i < n; ++i) m |= (text[i] == '\n' ? 1u : 0u) << (u32)(i - a);
  }
  return m;
}
__global__ void k_idl_count(const uint8_t *text, u64 n, u64 nblocks, u32 *cnt) {
  const u64 b = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= nblocks) return;
  const u32 c = __popc(idl_mask(text, n, b * IDL_BLOCK + 16ull * (threadIdx.x & 63)));
  u32 x = c;
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63) == 0) cnt[b] = x;
}
__global__ void k_idl_emit(const uint8_t *text, u64 n, u64 nblocks, const u64 *base, u64 *ends) {
  const u64 b = (u64)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= nblocks) return;
  const int lane = threadIdx.x & 63;
  const u64 a = b * IDL_BLOCK + 16ull * lane;
  u32 m = idl_mask(text, n, a);
  const u32 c = __popc(m);
  u32 incl = c;
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  u64 k = base[b] + incl - c;
  while (m) {
    ends[k++] = a + __builtin_ctz(m);
    m &= m - 1;
  }
}

// line j of the id text is [ends[j - 1] + 1, ends[j]] (the '\n' included; the first from 0)
__global__ void k_sub_parse(const uint8_t *text, const u64 *ends, u64 m, u32 *keep, i64 *val, u32 *st) {
  const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const u64 off = j ? ends[j - 1] + 1 : 0, len = ends[j] + 1 - off;
  keep[j] = len > 1;  // subset.go:197-199: "\n" alone is skipped
  i64 v = 0;
  u32 s = SUB_OK;
  if (len > 1) s = go_atoi(text + off, len - 1, v);  // buf[:n-1]: the '\n' dropped
  val[j] = v;
  st[j] = s;
}

__global__ void k_sub_compact(const u32 *keep, const u64 *rank, const i64 *val, const u32 *st, u64 m, i64 *cval,
                              u32 *cst, u64 *cline, u64 *ctl) {
  const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (j + 1 == m) ctl[SC_K] = rank[j] + keep[j];  // K: the non-blank ids
  if (j >= m || !keep[j]) return;
  const u64 r = rank[j];
  cval[r] = val[j];
  cst[r] = st[j];
  cline[r] = j;
}

// Checks in Go's order per id; the first failing id (min r) is the error.  Rows (those that
// fit rows_cap) and run starts are written for every id that passes; entries past the first
// failure are unused.  K comes from the device (ctl[SC_K]); the grid covers its bound m.
__global__ void k_sub_check(const i64 *cval, const u32 *cst, u64 *ctl, const u64 *parent, u64 parent_count, i64 ilength,
                            u64 *rows, u64 rows_cap, u32 *startf) {
  const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool in = r < ctl[SC_K];
  i64 v = 0, prev = 0;
  u32 code = SUB_SORT;
  if (in) {
    v = cval[r];
    prev = r ? cval[r - 1] : 0;
    code = cst[r];
    if (code == SUB_OK) {
      if (v <= prev) code = SUB_SORT;                        // :208-211
      else if (v > ilength) code = SUB_EXIST;                // :213-216
      else if ((u64)v > parent_count) code = SUB_READ;       // :218-223
    }
  }
  const bool ok = in && code == SUB_OK;
  ulonglong2 row = make_ulonglong2(0, 0);
  if (ok) row = reinterpret_cast<const ulonglong2 *>(parent)[v - 1];
  // id r - 1's row is lane - 1's when that lane accepted it (its id is prev): one random read of
  // the parent table per id instead of two
  const u32 px0 = (u32)__shfl_up((int)(u32)row.x, 1, 64), px1 = (u32)__shfl_up((int)(u32)(row.x >> 32), 1, 64);
  const u32 py0 = (u32)__shfl_up((int)(u32)row.y, 1, 64), py1 = (u32)__shfl_up((int)(u32)(row.y >> 32), 1, 64);
  const bool okprev = __shfl_up((int)ok, 1, 64) != 0;
  if (!in) return;
  u64 *firstbad = ctl + SC_FIRSTBAD;
  if (!ok) {
    atomicMin(firstbad, (r << 3) | code);
    startf[r] = 0;
    return;
  }
  if (r < rows_cap) reinterpret_cast<ulonglong2 *>(rows)[r] = row;
  u32 start = 1;
  if (r > 0 && prev >= 1 && (u64)prev <= parent_count) {  // :245 offset != prevOffset + prevLength
    ulonglong2 pr;
    if (lane > 0 && okprev) pr = make_ulonglong2((u64)px0 | ((u64)px1 << 32), (u64)py0 | ((u64)py1 << 32));
    else pr = reinterpret_cast<const ulonglong2 *>(parent)[prev - 1];
    start = row.x != pr.x + pr.y;
  }
  startf[r] = start;
}

// Ke = the ids accepted before the first failing one; a row table too short for them is
// reported (flag 1) and nothing past it is read.  Then the run count (run starts among the
// accepted ids); a short run table is flag 2.  (One thread: the scan of the run starts between
// k_sub_check and here does not need Ke.)
__global__ void k_sub_nstart(u64 *ctl, const u32 *startf, const u64 *runid, u64 rows_cap, u64 runs_cap, int has_runs) {
  const u64 fb = ctl[SC_FIRSTBAD], K = ctl[SC_K];
  const u64 Ke = fb == ~0ull ? K : (fb >> 3);
  ctl[SC_KE] = Ke;
  if (Ke > rows_cap) ctl[SC_FLAGS] |= 1;
  const u64 ns = Ke ? runid[Ke - 1] + startf[Ke - 1] : 0;
  ctl[SC_NSTART] = ns;
  if (has_runs && ns > runs_cap) ctl[SC_FLAGS] |= 2;
}

// run id of row r = runid[r] (exclusive scan of startf) + startf[r] - 1; nothing is written
// when a capacity flag is up (the host reports the counts needed).  oSize goes to slots[SC_SLOTS]
__global__ void k_sub_runs(const u64 *rows, const u32 *startf, const u64 *runid, const u64 *ctl, u64 *runs, u64 *slots) {
  const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u64 K = ctl[SC_FLAGS] ? 0 : ctl[SC_KE];
  u64 len = 0;
  if (r < K) {
    const ulonglong2 row = reinterpret_cast<const ulonglong2 *>(rows)[r];
    len = row.y;
    if (runs && startf[r]) runs[2 * runid[r]] = row.x;
  }
  // oSize: block sum then one atomic per block (integer: order-independent)
  __shared__ u64 part[4];
  u64 x = len;
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 t = 0;
    for (u32 w = 0; w < blockDim.x / 64; ++w) t += part[w];
    if (t) atomicAdd((unsigned long long *)(slots + (blockIdx.x & (SC_SLOTS - 1))), (unsigned long long)t);
  }
}

__global__ void k_sub_run_len(const u64 *rows, const u32 *startf, const u64 *runid, const u64 *ctl, u64 *runs) {
  const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u64 K = ctl[SC_FLAGS] ? 0 : ctl[SC_KE];
  if (r >= K) return;
  if (r + 1 == K || startf[r + 1]) {  // last row of its run: coLength = end - run start
    const ulonglong2 row = reinterpret_cast<const ulonglong2 *>(rows)[r];
    const u64 id = runid[r] + startf[r] - 1;
    runs[2 * id + 1] = row.x + row.y - runs[2 * id];
  }
}

// ---- Idx.Range (index/index.go:119-193) ---------------------------------------------------
// Range reads rows a-1 .. b-1 of the .idx file in order into one reused `rec` slice; a read
// past the end of the file fails and leaves rec as it was, so row i reads as rows[i] for
// i < nrows, else as the last row read (rows[nrows-1]), or zeros when even row a-1 was past
// the end.  It coalesces a row into the open run iff curLen == nextPos - curPos; by induction
// curPos + curLen is the end of the run's last row, so that is the pairwise test
// pos[j] == pos[j-1] + len[j-1] (mod 2^64): run starts = flags, run ids = their scan.
__device__ __forceinline__ ulonglong2 range_row(const u64 *rows, u64 nrows, u64 a0, u64 i) {
  if (i < nrows) return reinterpret_cast<const ulonglong2 *>(rows)[i];
  if (a0 < nrows) return reinterpret_cast<const ulonglong2 *>(rows)[nrows - 1];
  return make_ulonglong2(0, 0);
}
// j = 0 .. nr-1 over rows a0 + j
__global__ void k_range_flags(const u64 *rows, u64 nrows, u64 a0, u64 nr, u32 *flags) {
  const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nr) return;
  u32 f = 1;
  if (j > 0) {
    const ulonglong2 c = range_row(rows, nrows, a0, a0 + j), p = range_row(rows, nrows, a0, a0 + j - 1);
    f = c.x != p.x + p.y;
  }
  flags[j] = f;
}
__global__ void k_range_pos(const u64 *rows, u64 nrows, u64 a0, u64 nr, const u32 *flags, const u64 *id, u64 *recs) {
  const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nr && flags[j]) recs[2 * id[j]] = range_row(rows, nrows, a0, a0 + j).x;
}
__global__ void k_range_len(const u64 *rows, u64 nrows, u64 a0, u64 nr, const u32 *flags, const u64 *id, u64 *recs) {
  const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nr || !(j + 1 == nr || flags[j + 1])) return;  // the last row of its run
  const ulonglong2 c = range_row(rows, nrows, a0, a0 + j);
  const u64 r = id[j] + flags[j] - 1;
  recs[2 * r + 1] = c.x + c.y - recs[2 * r];  // curLen: the run's lengths summed (mod 2^64)
}

// ---- byte gather ------------------------------------------------------------------------
constexpr u32 GB_BLOCK = GATHER_BLOCK;  // output bytes per workgroup
#ifndef SIDX_GB_THREADS
#define SIDX_GB_THREADS 256
#endif
constexpr u32 GB_THREADS = SIDX_GB_THREADS;
constexpr u32 GB_RUNS = 512;     // run descriptors staged in LDS per workgroup

// the gather's counts come from the device: ctl[SC_NSTART] runs, ctl[SC_TOTAL] bytes; nothing
// is gathered after a failing id or a capacity flag
__device__ __forceinline__ bool gather_off(const u64 *ctl) { return ctl[SC_FIRSTBAD] != ~0ull || ctl[SC_FLAGS] != 0; }

// the run lengths as a u64 array (0 past the run count) for the output-offset scan
// A run the parent file does not hold (offset + len past data_len, or wrapping) or a length of
// 2^62 or more (dscan keeps its flags in the top bits) sets flag 8, which stops the gather
// before k_gather reads anything; its length counts as 0 so the scan stays exact.
__global__ void k_run_lengths(const u64 *runs, u64 bound, u64 *ctl, u64 *lens, u64 data_len) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= bound) return;
  u64 len = 0;
  if (i < ctl[SC_NSTART]) {
    const u64 off = runs[2 * i], l = runs[2 * i + 1];
    if (l >= (1ull << 62) || off > data_len || l > data_len - off) atomicOr((unsigned long long *)&ctl[SC_FLAGS], 8ull);
    else len = l;
  }
  lens[i] = len;
}
// The bytes to gather (flag 4 when they exceed out_cap, 8 when they exceed the parent file;
// thread 0 records them for k_gather, every thread works them out itself), then the first run of
// every output block: block w starts inside run i iff i's output span holds w*B
__global__ void k_gather_plan(const u64 *runs, const u64 *outoff, const u64 *lens, u64 *ctl, u64 out_cap, u64 data_len,
                              u64 *wfirst) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u64 n = ctl[SC_NSTART];
  const u64 total = n ? outoff[n - 1] + lens[n - 1] : 0;
  const bool over = total > out_cap || total > data_len;
  if (i == 0) {
    ctl[SC_TOTAL] = total;
    if (total > out_cap) ctl[SC_FLAGS] |= 4;
    if (total > data_len) ctl[SC_FLAGS] |= 8;
  }
  if (over || gather_off(ctl) || i >= n) return;
  const u64 nblocks = (total + GB_BLOCK - 1) / GB_BLOCK;
  const u64 a = outoff[i], len = runs[2 * i + 1];
  if (!len) return;
  const u64 w0 = (a + GB_BLOCK - 1) / GB_BLOCK, w1 = (a + len - 1) / GB_BLOCK;
  for (u64 w = w0; w <= w1 && w < nblocks; ++w) wfirst[w] = i;
}

__device__ __forceinline__ u32 fsh(u32 lo, u32 hi, u32 sh) {  // bytes [sh, sh+4) of hi:lo
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__device__ __forceinline__ u32 mask4(u32 b, u32 lo, u32 hi) {  // bytes [lo, hi) of dword at byte b
  const u32 l = lo > b ? (lo - b < 4 ? lo - b : 4) : 0, h = hi > b ? (hi - b < 4 ? hi - b : 4) : 0;
  const u32 mh = h >= 4 ? ~0u : ((1u << (8 * h)) - 1u), ml = l >= 4 ? ~0u : ((1u << (8 * l)) - 1u);
  return mh & ~ml;
}
__device__ __forceinline__ uint4 byte_mask16(u32 lo, u32 hi) {
  return make_uint4(mask4(0, lo, hi), mask4(4, lo, hi), mask4(8, lo, hi), mask4(12, lo, hi));
}

// bytes [sh, sh + 16) of the 32 bytes x:y, branch-free (a switch on the dword let the compiler
// split the loads into unaligned pieces under divergent branches)
__device__ __forceinline__ uint4 shift16(const uint4 x, const uint4 y, u32 sh16) {
  const bool h = (sh16 & 8u) != 0, o = (sh16 & 4u) != 0;
  const u32 sh = sh16 & 3u;
  const u32 a0 = h ? x.z : x.x, a1 = h ? x.w : x.y, a2 = h ? y.x : x.z, a3 = h ? y.y : x.w, a4 = h ? y.z : y.x,
            a5 = h ? y.w : y.y;
  const u32 b0 = o ? a1 : a0, b1 = o ? a2 : a1, b2 = o ? a3 : a2, b3 = o ? a4 : a3, b4 = o ? a5 : a4;
  return make_uint4(fsh(b0, b1, sh), fsh(b1, b2, sh), fsh(b2, b3, sh), fsh(b3, b4, sh));
}

#ifndef SIDX_GATHER_K
#define SIDX_GATHER_K 2  // chunks per thread with their loads in flight together (0: one at a time)
#endif
// for each key x[q]: the last index i < n with a[i] <= x[q] (a ascending, a[0] <= x[q],
// n <= CAP) in a fixed number of steps, so that a thread's searches overlap in LDS
template <typename T, u32 N, u32 CAP>
__device__ __forceinline__ void lds_last_le(const T *a, u32 n, const T (&x)[N], u32 (&lo)[N]) {
#pragma unroll
  for (u32 q = 0; q < N; ++q) lo[q] = 0;
#pragma unroll
  for (u32 step = CAP / 2; step; step >>= 1)
#pragma unroll
    for (u32 q = 0; q < N; ++q) {
      const u32 c = lo[q] + step;
      if (c < n && a[c] <= x[q]) lo[q] = c;
    }
}

#ifndef SIDX_GATHER_NT
#define SIDX_GATHER_NT 1  // non-temporal output stores (written once, read by no one here: 0.397 -> 0.370 ms)
#endif
__device__ __forceinline__ void st16(uint8_t *p, const uint4 v) {
#if SIDX_GATHER_NT
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(p));
#else
  *reinterpret_cast<uint4 *>(p) = v;
#endif
}

// output chunk [o, oe) the general way: every staged run overlapping it, or byte by byte
// (runs beyond the staged ones, file ends, the partial last chunk)
__device__ __forceinline__ void gather_chunk(const uint8_t *data, u64 data_len, const u64 *runs, const u64 *outoff,
                                          u64 nruns, const u64 *s_out, const u64 *s_src, u64 nb, u64 covered, u64 o,
                                          u64 oe, uint8_t *out) {
  bool slow = o >= covered || oe > covered;
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (!slow) {
    u32 lo = 0, hi = (u32)nb;  // last staged run with s_out <= o
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) >> 1;
      if (s_out[mid] <= o) lo = mid; else hi = mid;
    }
    for (u32 j = lo; j < nb && s_out[j] < oe; ++j) {
      const u64 ra = s_out[j], rb = s_out[j + 1];
      const u32 bl = (u32)((ra > o ? ra : o) - o), bh = (u32)((rb < oe ? rb : oe) - o);
      if (bh <= bl) continue;
      const u64 src0 = s_src[j];
      if (ra > o && src0 < ra - o) { slow = true; break; }  // window would start before the file
      const u64 src = src0 + o - ra;                          // (mod 2^64 when ra > o: fine)
      const u64 al = src & ~15ull;
      if (al + 32 > data_len) { slow = true; break; }
      const uint4 d = shift16(*reinterpret_cast<const uint4 *>(data + al), *reinterpret_cast<const uint4 *>(data + al + 16),
                              (u32)src & 15u);
      const uint4 m = byte_mask16(bl, bh);  // bytes [bl, bh) of the chunk come from this run
      acc.x |= d.x & m.x; acc.y |= d.y & m.y; acc.z |= d.z & m.z; acc.w |= d.w & m.w;
    }
  }
  if (!slow && oe == o + 16) {
    st16(out + o, acc);
    return;
  }
  u64 lo = 0, hi = nruns;  // last run with outoff <= o (global binary search)
  while (hi - lo > 1) {
    const u64 mid = (lo + hi) >> 1;
    if (outoff[mid] <= o) lo = mid; else hi = mid;
  }
  u64 ri = lo;
  for (u64 pos = o; pos < oe; ++pos) {
    while (ri + 1 < nruns && outoff[ri + 1] <= pos) ++ri;
    out[pos] = data[runs[2 * ri] + (pos - outoff[ri])];
  }
}

// one workgroup per 32 KiB output block (GATHER_BLOCK); the grid is a bound of the block count
// (read from the device), the workgroups past it exit at once (a persistent grid striding over
// the blocks was 45 % slower: the blocks' costs vary with the runs they hold).  Round 5, with two
// chunks' loads in flight per lane, in one process over the C4 runs (profiles/r05/calls/r05p*):
// 16 KiB / 256 threads 0.265 ms, 32 KiB / 256 0.256, 32 KiB / 128 0.260, 64 KiB / 256 0.262,
// 8 KiB / 256 0.285, 16 KiB / 512 0.296; one chunk at a time 0.294, four 0.318 (5 waves per SIMD)
__global__ __launch_bounds__(GB_THREADS) void k_gather(const uint8_t *data, u64 data_len, const u64 *runs,
                                                         const u64 *outoff, const u64 *wfirst, const u64 *ctl,
                                                         uint8_t *out) {
  __shared__ u64 s_out[GB_RUNS + 1];
  __shared__ u64 s_src[GB_RUNS];
  if (gather_off(ctl)) return;
  const u64 nruns = ctl[SC_NSTART], total = ctl[SC_TOTAL];
  const u64 nblocks = (total + GB_BLOCK - 1) / GB_BLOCK;
  const u64 b = blockIdx.x;
  if (b >= nblocks) return;
  const u64 blo = b * GB_BLOCK;
  const u64 bhi = blo + GB_BLOCK < total ? blo + GB_BLOCK : total;
  const u64 r0 = wfirst[b];
  // the runs overlapping this block: r0 .. the run holding the next block's first byte
  const u64 rl = b + 1 < nblocks ? wfirst[b + 1] + 1 : nruns;
  const u64 nr = rl - r0 < nruns - r0 ? rl - r0 : nruns - r0;
  const u64 nb = nr < GB_RUNS ? nr : GB_RUNS;
  for (u32 i = threadIdx.x; i < nb; i += GB_THREADS) {
    s_out[i] = outoff[r0 + i];
    s_src[i] = runs[2 * (r0 + i)];
  }
  if (threadIdx.x == 0) s_out[nb] = (r0 + nb < nruns) ? outoff[r0 + nb] : total;
  __syncthreads();
  const u64 covered = s_out[nb];  // output bytes the staged runs describe
  // one code path for every chunk (gather_chunk): a separate path for the chunks inside one run
  // (most of them), or a thread's chunks looked up first and their loads issued together, ran
  // 25-50 % slower -- the ~1 in 20 chunks a run boundary crosses then diverged every wave
  if (!SIDX_GATHER_K || data_len < 32) {
    for (u64 o = blo + (u64)threadIdx.x * 16; o < bhi; o += (u64)GB_THREADS * 16)
      gather_chunk(data, data_len, runs, outoff, nruns, s_out, s_src, nb, covered, o, bhi < o + 16 ? bhi : o + 16, out);
    return;
  }
  // SIDX_GATHER_K chunks of the thread at a time: their run lookups (fixed-step searches that
  // overlap in LDS), then the first piece's two loads of every chunk, then the stores -- the
  // loop above has one chunk's two loads in flight per lane, the store waiting on them before the
  // next chunk's lookup.  A chunk that its first run does not fill (about one in twenty) takes
  // the rest of its pieces one by one; anything unusual goes through gather_chunk.
  constexpr u32 K = SIDX_GATHER_K ? SIDX_GATHER_K : 1, CH = GB_BLOCK / 16 / GB_THREADS;
  static_assert(CH % K == 0, "whole batches");
#pragma unroll
  for (u32 c0 = 0; c0 < CH; c0 += K) {
    u64 o[K];
    u32 lo[K];
#pragma unroll
    for (u32 k = 0; k < K; ++k) o[k] = blo + 16ull * (threadIdx.x + (c0 + k) * GB_THREADS);
    lds_last_le<u64, K, GB_RUNS>(s_out, nb, o, lo);
    uint4 x[K], y[K];
    u32 bh[K], sh[K];
    bool fast[K];
#pragma unroll
    for (u32 k = 0; k < K; ++k) {
      const u64 ra = s_out[lo[k]], rb = s_out[lo[k] + 1];
      const u64 src = s_src[lo[k]] + (o[k] - ra);
      const u64 al = src & ~15ull;
      fast[k] = o[k] + 16 <= bhi && o[k] + 16 <= covered && al + 32 <= data_len;
      bh[k] = (u32)((rb < o[k] + 16 ? rb : o[k] + 16) - o[k]);
      sh[k] = (u32)src & 15u;
      const u64 la = fast[k] ? al : 0;  // every lane loads (the file's first words for a general chunk): a
      // load under a branch whose other side wrote the same registers waited for each load
      x[k] = *reinterpret_cast<const uint4 *>(data + la);
      y[k] = *reinterpret_cast<const uint4 *>(data + la + 16);
    }
#pragma unroll
    for (u32 k = 0; k < K; ++k) {
      if (o[k] >= bhi) continue;
      const u64 oe = bhi < o[k] + 16 ? bhi : o[k] + 16;
      bool slow = !fast[k];
      uint4 acc = make_uint4(0, 0, 0, 0);
      if (!slow) {
        const uint4 d = shift16(x[k], y[k], sh[k]);
        const uint4 m = byte_mask16(0, bh[k]);
        acc.x = d.x & m.x; acc.y = d.y & m.y; acc.z = d.z & m.z; acc.w = d.w & m.w;
        for (u32 j = lo[k] + 1; bh[k] < 16 && j < nb && s_out[j] < oe; ++j) {  // the chunk's later pieces
          const u64 ra = s_out[j], rb = s_out[j + 1];
          const u32 bl = (u32)(ra - o[k]), bj = (u32)((rb < oe ? rb : oe) - o[k]);
          if (bj <= bl) continue;
          const u64 src0 = s_src[j];
          if (src0 < ra - o[k]) { slow = true; break; }  // the window would start before the file
          const u64 src = src0 - (ra - o[k]);
          const u64 al = src & ~15ull;
          if (al + 32 > data_len) { slow = true; break; }
          const uint4 d2 = shift16(*reinterpret_cast<const uint4 *>(data + al), *reinterpret_cast<const uint4 *>(data + al + 16),
                                   (u32)src & 15u);
          const uint4 m2 = byte_mask16(bl, bj);
          acc.x |= d2.x & m2.x; acc.y |= d2.y & m2.y; acc.z |= d2.z & m2.z; acc.w |= d2.w & m2.w;
        }
      }
      if (slow) gather_chunk(data, data_len, runs, outoff, nruns, s_out, s_src, nb, covered, o[k], oe, out);
      else st16(out + o[k], acc);
    }
  }
}

}  // namespace sidx

using namespace sidx;

namespace {
inline u32 nblk(u64 n, u32 t) { return (u32)((n + t - 1) / t); }
}

extern "C" hipError_t sidx_subset_parse(const uint8_t *text, const u64 *ends, u64 m, u32 *keep, i64 *val, u32 *st,
                                        hipStream_t s) {
  if (m) hipLaunchKernelGGL(k_sub_parse, dim3(nblk(m, 256)), dim3(256), 0, s, text, ends, m, keep, val, st);
  return hipGetLastError();
}

// the line ends of the id text (k_idl_*): cnt / base hold a u32 / u64 per 1 KiB block (the
// line count is base[nb - 1] + cnt[nb - 1]).  tmp == nullptr: the scan's temp size into *tmp_bytes
extern "C" hipError_t sidx_id_lines(const uint8_t *text, u64 n, u32 *cnt, u64 *base, u64 *ends, void *tmp,
                                    size_t *tmp_bytes, hipStream_t s) {
  const u64 nb = (n + IDL_BLOCK - 1) / IDL_BLOCK;
  if (!tmp) return dscan::run<u32, dscan::Sum, true>(nullptr, tmp_bytes, cnt, base, nb ? nb : 1, s);
  if (nb) {
    const u32 grid = (u32)((nb + 3) / 4);
    hipLaunchKernelGGL(k_idl_count, dim3(grid), dim3(256), 0, s, text, n, nb, cnt);
    hipError_t e = dscan::run<u32, dscan::Sum, true>(tmp, tmp_bytes, cnt, base, nb, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_idl_emit, dim3(grid), dim3(256), 0, s, text, n, nb, base, ends);
  }
  return hipGetLastError();
}

// exclusive sums of u32 flags into u64 (temp storage grown by the caller through *tmp/*tmp_bytes)
extern "C" hipError_t sidx_scan_flags(const u32 *in, u64 *out, u64 n, void *tmp, size_t *tmp_bytes, hipStream_t s) {
  return dscan::run<u32, dscan::Sum, true>(tmp, tmp_bytes, in, out, n, s);
}
extern "C" hipError_t sidx_scan_u64(const u64 *in, u64 *out, u64 n, void *tmp, size_t *tmp_bytes, hipStream_t s) {
  return dscan::run<u64, dscan::Sum, true>(tmp, tmp_bytes, in, out, n, s);
}

extern "C" hipError_t sidx_subset_compact(const u32 *keep, const u64 *rank, const i64 *val, const u32 *st, u64 m,
                                          i64 *cval, u32 *cst, u64 *cline, u64 *ctl, hipStream_t s) {
  if (m) hipLaunchKernelGGL(k_sub_compact, dim3(nblk(m, 256)), dim3(256), 0, s, keep, rank, val, st, m, cval, cst, cline, ctl);
  return hipGetLastError();
}

// the control words: firstbad = ~0, the rest 0; SC_NSTART = nruns (a gather of host-given runs)
__global__ void k_sub_init(u64 *ctl, u64 nruns) {
  if (threadIdx.x < SC_ALLWORDS) ctl[threadIdx.x] = threadIdx.x == SC_FIRSTBAD ? ~0ull : (threadIdx.x == SC_NSTART ? nruns : 0);
}
extern "C" hipError_t sidx_subset_init(u64 *ctl, u64 nruns, hipStream_t s) {
  hipLaunchKernelGGL(k_sub_init, dim3(1), dim3(SC_ALLWORDS), 0, s, ctl, nruns);
  return hipGetLastError();
}

// m: the id lines (a bound of every count); K, Ke, the run count and oSize stay on the device
extern "C" hipError_t sidx_subset_check(const i64 *cval, const u32 *cst, u64 m, u64 *ctl, const u64 *parent,
                                        u64 parent_count, i64 ilength, u64 *rows, u64 rows_cap, u32 *startf,
                                        hipStream_t s) {
  if (m)
    hipLaunchKernelGGL(k_sub_check, dim3(nblk(m, 256)), dim3(256), 0, s, cval, cst, ctl, parent, parent_count, ilength,
                       rows, rows_cap, startf);
  return hipGetLastError();
}

extern "C" hipError_t sidx_subset_runs(const u64 *rows, const u32 *startf, const u64 *runid, u64 m, u64 *ctl,
                                       u64 *runs, u64 rows_cap, u64 runs_cap, hipStream_t s) {
  hipLaunchKernelGGL(k_sub_nstart, dim3(1), dim3(1), 0, s, ctl, startf, runid, rows_cap, runs_cap, runs ? 1 : 0);
  if (m) {  // runs == nullptr: oSize only (CreateSubsetIndex writes no compressed index)
    hipLaunchKernelGGL(k_sub_runs, dim3(nblk(m, 256)), dim3(256), 0, s, rows, startf, runid, ctl, runs, ctl + SC_NWORDS);
    if (runs) hipLaunchKernelGGL(k_sub_run_len, dim3(nblk(m, 256)), dim3(256), 0, s, rows, startf, runid, ctl, runs);
  }
  return hipGetLastError();
}

// The gather of ctl[SC_NSTART] runs (at most `bound`): lengths, their scan (tmp), the byte
// total, the block plan, the persistent gather.  No host round trip.
extern "C" hipError_t sidx_gather(const uint8_t *data, u64 data_len, const u64 *runs, u64 bound, u64 *ctl, u64 *lens,
                                  u64 *outoff, void *tmp, size_t *tmp_bytes, u64 *wfirst, uint8_t *out, u64 out_cap,
                                  hipEvent_t e0, hipEvent_t e1, hipStream_t s) {
  if (!tmp) return dscan::run<u64, dscan::Sum, true>(nullptr, tmp_bytes, lens, outoff, bound ? bound : 1, s);
  if (!bound) return hipSuccess;
  hipLaunchKernelGGL(k_run_lengths, dim3(nblk(bound, 256)), dim3(256), 0, s, runs, bound, ctl, lens, data_len);
  hipError_t e = dscan::run<u64, dscan::Sum, true>(tmp, tmp_bytes, lens, outoff, bound, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gather_plan, dim3(nblk(bound, 256)), dim3(256), 0, s, runs, outoff, lens, ctl, out_cap, data_len,
                     wfirst);
  const u64 grid = ((out_cap < data_len ? out_cap : data_len) + GB_BLOCK - 1) / GB_BLOCK;  // blocks at most
  if (e0) (void)hipEventRecord(e0, s);
  if (grid) hipLaunchKernelGGL(k_gather, dim3((u32)grid), dim3(GB_THREADS), 0, s, data, data_len, runs, outoff, wfirst, ctl, out);
  if (e1) (void)hipEventRecord(e1, s);
  return hipGetLastError();
}

extern "C" hipError_t sidx_range_flags(const u64 *rows, u64 nrows, u64 a0, u64 nr, u32 *flags, hipStream_t s) {
  if (nr) hipLaunchKernelGGL(k_range_flags, dim3(nblk(nr, 256)), dim3(256), 0, s, rows, nrows, a0, nr, flags);
  return hipGetLastError();
}
extern "C" hipError_t sidx_range_emit(const u64 *rows, u64 nrows, u64 a0, u64 nr, const u32 *flags, const u64 *id,
                                      u64 *recs, hipStream_t s) {
  if (nr) {
    hipLaunchKernelGGL(k_range_pos, dim3(nblk(nr, 256)), dim3(256), 0, s, rows, nrows, a0, nr, flags, id, recs);
    hipLaunchKernelGGL(k_range_len, dim3(nblk(nr, 256)), dim3(256), 0, s, rows, nrows, a0, nr, flags, id, recs);
  }
  return hipGetLastError();
}
