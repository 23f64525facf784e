// sidx_synth.hip -- deterministic synthetic FASTQ / FASTA generators on the device
// (benchmark + large-size parity infrastructure; not part of the index path).
//
// Specs: SURVEY.md §8(d) C2 / C3.  Every record is a pure function of (seed, record index)
// via splitmix64, so any byte window of the virtual file (e.g. one GPU's slab) can be
// generated independently, and the expected index table is known by construction:
//   rows[k] = {off[k], len[k]},  off = exclusive prefix sum of len.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

typedef unsigned long long u64;
typedef unsigned int u32;

namespace {

__device__ __forceinline__ u64 splitmix64(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ u64 h(u64 seed, u64 i, u64 k) { return splitmix64(seed ^ splitmix64(i * 0x100000001B3ull + k)); }

__device__ __forceinline__ u32 ndigits(u64 v) {
  u32 d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}
__device__ __forceinline__ u32 put_dec(uint8_t *o, u64 v) {  // returns digits written
  const u32 d = ndigits(v);
  for (u32 k = 0; k < d; ++k) { o[d - 1 - k] = (uint8_t)('0' + v % 10); v /= 10; }
  return d;
}

// ---------------------------------------------------------------------------------------
// FASTQ (C2): "@SRR000001.{i} {i} length={L}\n" + bases + "\n" + ("+\n" | "+<id>\n") + qual
// ---------------------------------------------------------------------------------------
struct FqRec {
  u32 L, idlen, plus, len;
};
__device__ __forceinline__ FqRec fq_rec(u64 seed, u64 i) {
  FqRec r;
  r.L = 50 + (u32)(h(seed, i, 0) % 201);
  r.plus = (h(seed, i, 1) % 10) == 0;
  r.idlen = 10 + ndigits(i) + 1 + ndigits(i) + 8 + ndigits(r.L);  // "SRR000001." i " " i " length=" L
  r.len = (1 + r.idlen + 1) + (r.L + 1) + (r.plus ? 1 + r.idlen + 1 : 2) + (r.L + 1);
  return r;
}

__global__ void k_fq_len(u64 first, u64 count, u64 seed, u32 *len) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < count) len[k] = fq_rec(seed, first + k).len;
}

// bytes of record i, written only where they fall in [lo, hi) of the virtual file
struct Win {
  uint8_t *out;
  u64 lo, hi;
  __device__ __forceinline__ void put(u64 pos, uint8_t c) const {
    if (pos >= lo && pos < hi) out[pos - lo] = c;
  }
};

__device__ void fq_id(const Win &w, u64 &p, u64 i, u32 L) {
  uint8_t buf[64];
  const uint8_t pre[] = "SRR000001.";
  u32 n = 0;
  for (u32 k = 0; k < 10; ++k) buf[n++] = pre[k];
  n += put_dec(buf + n, i);
  buf[n++] = ' ';
  n += put_dec(buf + n, i);
  const uint8_t len_s[] = " length=";
  for (u32 k = 0; k < 8; ++k) buf[n++] = len_s[k];
  n += put_dec(buf + n, L);
  for (u32 k = 0; k < n; ++k) w.put(p++, buf[k]);
}

__global__ void k_fq_fill(Win w, const u64 *off, u64 first, u64 count, u64 seed) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const u64 i = first + k;
  const FqRec r = fq_rec(seed, i);
  u64 p = off[k];
  if (p + r.len <= w.lo || p >= w.hi) return;
  w.put(p++, '@');
  fq_id(w, p, i, r.L);
  w.put(p++, '\n');
  const uint8_t acgt[4] = {'A', 'C', 'G', 'T'};
  for (u32 j = 0; j < r.L; j += 4) {
    const u64 x = h(seed, i, 16 + j / 4);
    for (u32 t = 0; t < 4 && j + t < r.L; ++t) {
      const u32 v = (u32)(x >> (16 * t)) & 0xFFFF;
      w.put(p++, (v % 1000) == 0 ? 'N' : acgt[v & 3]);
    }
  }
  w.put(p++, '\n');
  w.put(p++, '+');
  if (r.plus) fq_id(w, p, i, r.L);
  w.put(p++, '\n');
  for (u32 j = 0; j < r.L; j += 8) {
    const u64 x = h(seed, i, 1u << 20 | (j / 8));
    for (u32 t = 0; t < 8 && j + t < r.L; ++t) w.put(p++, (uint8_t)('!' + ((x >> (8 * t)) & 0xFF) % 42));
  }
  w.put(p++, '\n');
}

// ---------------------------------------------------------------------------------------
// FASTA (C3): ">ctg{i} len={L} desc{d}[ a>b]\n" + sequence wrapped at W in {60,70,80}
//   L ~ lognormal(median 1000, sigma 1) clamped to [30, 200000]; 1% headers embed '>'
// ---------------------------------------------------------------------------------------
struct FaRec {
  u32 L, W, gt, hdr, len;
  u64 d;
};
__device__ __forceinline__ FaRec fa_rec(u64 seed, u64 i) {
  FaRec r;
  const double u1 = ((h(seed, i, 0) >> 11) + 1) * (1.0 / 9007199254740993.0);
  const double u2 = (h(seed, i, 1) >> 11) * (1.0 / 9007199254740992.0);
  const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  double L = exp(6.907755278982137 + z);  // ln(1000)
  if (L < 30) L = 30;
  if (L > 200000) L = 200000;
  r.L = (u32)L;
  r.W = 60 + 10 * (u32)(h(seed, i, 2) % 3);
  r.gt = (h(seed, i, 3) % 100) == 0;
  r.d = h(seed, i, 4) % 1000000;
  // ">ctg" i " len=" L " desc" d [" a>b"] "\n"
  r.hdr = 4 + ndigits(i) + 5 + ndigits(r.L) + 5 + ndigits(r.d) + (r.gt ? 4 : 0) + 1;
  r.len = r.hdr + r.L + (r.L + r.W - 1) / r.W;
  return r;
}

__global__ void k_fa_len(u64 first, u64 count, u64 seed, u32 *len) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < count) len[k] = fa_rec(seed, first + k).len;
}

__global__ void k_fa_fill(Win w, const u64 *off, u64 first, u64 count, u64 seed) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const u64 i = first + k;
  const FaRec r = fa_rec(seed, i);
  u64 p = off[k];
  if (p + r.len <= w.lo || p >= w.hi) return;
  uint8_t buf[80];
  u32 n = 0;
  const uint8_t a[] = ">ctg", b[] = " len=", c[] = " desc", g[] = " a>b";
  for (u32 t = 0; t < 4; ++t) buf[n++] = a[t];
  n += put_dec(buf + n, i);
  for (u32 t = 0; t < 5; ++t) buf[n++] = b[t];
  n += put_dec(buf + n, r.L);
  for (u32 t = 0; t < 5; ++t) buf[n++] = c[t];
  n += put_dec(buf + n, r.d);
  if (r.gt) for (u32 t = 0; t < 4; ++t) buf[n++] = g[t];
  buf[n++] = '\n';
  for (u32 t = 0; t < n; ++t) w.put(p++, buf[t]);
  const uint8_t acgt[4] = {'A', 'C', 'G', 'T'};
  for (u32 j = 0; j < r.L; j += 4) {
    const u64 x = h(seed, i, 16 + j / 4);
    for (u32 t = 0; t < 4 && j + t < r.L; ++t) {
      const u32 v = (u32)(x >> (16 * t)) & 0xFFFF;
      w.put(p++, (v % 1000) == 0 ? 'N' : acgt[v & 3]);
      if ((j + t + 1) % r.W == 0 || j + t + 1 == r.L) w.put(p++, '\n');
    }
  }
}

__global__ void k_find(const u64 *off, u64 count, u64 pos, u64 *out) {
  // first k in [0, count] with off[k] > pos, minus one: the record containing pos
  if (threadIdx.x || blockIdx.x) return;
  u64 lo = 0, hi = count;  // off[count] = end
  while (lo < hi) {
    const u64 mid = (lo + hi) / 2;
    if (off[mid] > pos) hi = mid; else lo = mid + 1;
  }
  *out = lo;  // number of record starts <= pos  (record lo-1 contains pos)
}

__global__ void k_add_base(u64 *off, u64 n, u64 base) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) off[k] += base;
}

// rows[k] == {off[k], len[k]} for k < count (row_off = index of off[0] in rows) ?
__global__ void k_check_rows(const u64 *rows, const u64 *off, const u32 *len, u64 count, unsigned long long *bad) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  if (rows[2 * k] != off[k] || rows[2 * k + 1] != (u64)len[k]) atomicAdd(bad, 1ull);
}

inline unsigned blocks(u64 n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// ---------------------------------------------------------------------------------------
// Same-box streaming floor (bench context only, not the index path): the staging skeleton of
// the tile passes -- 16 KiB tiles with a 16-byte front and a 1 KiB halo, non-temporal
// buffer_load ... lds, XCD-major tile order, 7 workgroups per CU, one LDS read per thread and
// two barriers per tile -- with no parsing and no per-tile stores.  Its time is what this box's
// HBM gives the tile passes' read pattern; bench.py prints it beside the kernels.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) unsigned char lds_u8;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t fl_rsrc(const uint8_t *base, u32 n) {
  const u64 ba = (u64)base;
  const uint8_t *sb = (const uint8_t *)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)ba)) |
                                        ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(ba >> 32)) << 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)sb, (short)0, (int)__builtin_amdgcn_readfirstlane((int)n), 0x00020000);
}
__device__ __forceinline__ void fl_dma16(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen nt lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void fl_dma4(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void fl_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(256, 7) void k_stream_floor(const uint8_t *d, u64 n, u64 ntiles, u64 G, u32 *sink) {
  constexpr int TILE = 16384, HALO = 1024, FRONT = 16;
  __shared__ __attribute__((aligned(16))) uint8_t raw[FRONT + TILE + HALO];
  __shared__ u32 wt[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  u32 acc = 0;
  for (; t < ntiles; t += G) {
    const u64 tlo = t * TILE;
    const u64 lim = tlo + TILE + HALO - FRONT < n ? tlo + TILE + HALO - FRONT : n;
    const bool sh = tlo >= FRONT;
    const auto rs = fl_rsrc(d + tlo - (sh ? FRONT : 0), (u32)(lim - tlo) + (sh ? FRONT : 0));
    const u32 adj = sh ? 0u : FRONT;
    const u32 dst = (u32)(size_t)(lds_u8 *)raw;
    __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32 o = FRONT + (u32)(wid * 4 + i) * 1024u;
      fl_dma16(o + lane * 16 - adj, dst + o, rs);
    }
    if (wid == 0 && lane < 4) fl_dma4(lane * 4 - adj, dst, rs);
    fl_dma4(FRONT + TILE + wid * 256 + lane * 4 - adj, dst + FRONT + TILE + wid * 256, rs);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32 x = *reinterpret_cast<const u32 *>(raw + FRONT + tid * 64);
    if (lane == 63) wt[wid] = x;
    fl_bar();
    acc += wt[(tid + 1) & 3];
    fl_bar();
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the reads live; practically never taken
}

}  // namespace

extern "C" {

int synth_lengths(int fasta, u64 first, u64 count, u64 seed, u32 *d_len, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!count) return 0;
  if (fasta) hipLaunchKernelGGL(k_fa_len, dim3(blocks(count, 256)), dim3(256), 0, s, first, count, seed, d_len);
  else hipLaunchKernelGGL(k_fq_len, dim3(blocks(count, 256)), dim3(256), 0, s, first, count, seed, d_len);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

__global__ void k_widen(const u32 *len, u64 *out, u64 n) {
  const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = len[k];
}

// d_off[0..count] = base + exclusive prefix sums of d_len[0..count) (d_off[count] = end);
// lengths are widened to u64 first (sums exceed 2^32 for multi-GiB files)
int synth_offsets(const u32 *d_len, u64 count, u64 base, u64 *d_off, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!count) { hipMemcpyAsync(d_off, &base, 8, hipMemcpyHostToDevice, s); hipStreamSynchronize(s); return 0; }
  hipLaunchKernelGGL(k_widen, dim3(blocks(count, 256)), dim3(256), 0, s, d_len, d_off + 1, count);
  hipMemcpyAsync(d_off, &base, 8, hipMemcpyHostToDevice, s);
  size_t tmp_bytes = 0;
  void *tmp = nullptr;  // hipcub's num_items is int: inclusive-scan in chunks of 2^30
  const u64 CH = 1ull << 30;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, d_off, d_off, (int)((count + 1) < CH ? count + 1 : CH), s);
  if (e != hipSuccess) return -2;
  if (hipMalloc(&tmp, tmp_bytes + 16) != hipSuccess) return -3;
  u64 carry = 0;
  for (u64 st = 0; st < count + 1; st += CH) {
    const u64 n = count + 1 - st < CH ? count + 1 - st : CH;
    if (st) hipLaunchKernelGGL(k_add_base, dim3(1), dim3(1), 0, s, d_off + st, 1, carry);  // fold carry into first
    e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, d_off + st, d_off + st, (int)n, s);
    if (e != hipSuccess) { hipFree(tmp); return -2; }
    hipMemcpyAsync(&carry, d_off + st + n - 1, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
  }
  hipStreamSynchronize(s);
  hipFree(tmp);
  return 0;
}

int synth_fill(int fasta, uint8_t *d_out, u64 lo, u64 hi, const u64 *d_off, u64 first, u64 count, u64 seed,
               void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!count) return 0;
  Win w{d_out, lo, hi};
  if (fasta) hipLaunchKernelGGL(k_fa_fill, dim3(blocks(count, 128)), dim3(128), 0, s, w, d_off, first, count, seed);
  else hipLaunchKernelGGL(k_fq_fill, dim3(blocks(count, 128)), dim3(128), 0, s, w, d_off, first, count, seed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Test support (C4's whole-output check): a 64-bit hash of each of `nruns` byte
// runs d[runs[2i] + d_base .. + runs[2i+1]) -- the sum over the run's 8-byte words (last one
// zero-padded) of splitmix64(word ^ (index * golden)), plus the length: order-sensitive, one
// wave per run.  Hashing the parent at each run's offset and the gathered output at the runs'
// output offsets must give the same array.
__global__ void k_run_hash(const uint8_t *d, const u64 *runs, u64 nruns, u64 *out) {
  const int lane = threadIdx.x & 63;
  for (u64 i = (u64)blockIdx.x * 4 + (threadIdx.x >> 6); i < nruns; i += (u64)gridDim.x * 4) {
    const u64 off = runs[2 * i], len = runs[2 * i + 1];
    u64 h = 0;
    for (u64 w = (u64)lane; w * 8 < len; w += 64) {
      u64 v = 0;
      for (int b = 0; b < 8; ++b)
        if (w * 8 + b < len) v |= (u64)d[off + w * 8 + b] << (8 * b);
      h += splitmix64(v ^ (w * 0x9E3779B97F4A7C15ull));
    }
    for (int o = 32; o; o >>= 1) h += (u64)__shfl_xor((long long)h, o, 64);
    if (lane == 0) out[i] = h + len;
  }
}

int synth_run_hash(const uint8_t *d_data, const u64 *d_runs, u64 nruns, u64 *d_out, void *stream) {
  if (!nruns) return 0;
  const u64 g = (nruns + 3) / 4;
  hipLaunchKernelGGL(k_run_hash, dim3(g < 65536 ? g : 65536), dim3(256), 0, (hipStream_t)stream, d_data, d_runs, nruns,
                     d_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int synth_find(const u64 *d_off, u64 count, u64 pos, u64 *d_out, void *stream) {
  hipLaunchKernelGGL(k_find, dim3(1), dim3(64), 0, (hipStream_t)stream, d_off, count, pos, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int synth_check_rows(const u64 *d_rows, const u64 *d_off, const u32 *d_len, u64 count, u64 *d_bad, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!count) return 0;
  hipLaunchKernelGGL(k_check_rows, dim3(blocks(count, 256)), dim3(256), 0, s, d_rows, d_off, d_len, count,
                     (unsigned long long *)d_bad);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// k_stream_floor over d_data[0, n): reps timed launches on `stream` (after one untimed), the
// average launch time in *ms_out (HIP events on that stream).  d_sink: 4 writable bytes.
int synth_stream_floor(const uint8_t *d_data, u64 n, int reps, u32 *d_sink, float *ms_out, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!n || reps <= 0 || !ms_out) return -1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -2;
  const u64 ntiles = (n + 16383) / 16384;
  u64 G = (u64)cus * 7;
  if (G > ntiles) G = ntiles;
  if (G >= 8) G &= ~7ull;  // XCD-major order needs G % 8 == 0
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -2;
  if (hipEventCreate(&e1) != hipSuccess) { hipEventDestroy(e0); return -2; }
  hipLaunchKernelGGL(k_stream_floor, dim3((unsigned)G), dim3(256), 0, s, d_data, n, ntiles, G, d_sink);
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL(k_stream_floor, dim3((unsigned)G), dim3(256), 0, s, d_data, n, ntiles, G, d_sink);
  hipEventRecord(e1, s);
  hipError_t e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (e != hipSuccess || hipGetLastError() != hipSuccess) return -2;
  *ms_out = ms / (float)reps;
  return 0;
}

}  // extern "C"

// Translation probe (round 5 placement study): one 4-byte load per `stride` bytes over
// d_data[0, n), lanes spread over the whole buffer (every wave touches 64 different pages at
// once), reps timed launches; *ms_out = average launch time.  A buffer mapped with small
// fragments pays a translation miss per page; a large-fragment mapping almost none.
__global__ void k_page_probe(const uint8_t *d, u64 n, u64 stride, u32 *sink) {
  const u64 np = n / stride;
  u32 acc = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += (u64)gridDim.x * blockDim.x) {
    const u64 j = (i * 0x9E3779B97F4A7C15ull) % np;  // scattered page order
    acc += *(const volatile u32 *)(d + j * stride);
  }
  if (acc == 0x12345678u) *sink = acc;
}
extern "C" int synth_page_probe(const uint8_t *d_data, u64 n, u64 stride, int reps, u32 *d_sink, float *ms_out,
                                void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!n || !stride || reps <= 0 || !ms_out) return -1;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -2;
  if (hipEventCreate(&e1) != hipSuccess) { hipEventDestroy(e0); return -2; }
  hipLaunchKernelGGL(k_page_probe, dim3(1024), dim3(256), 0, s, d_data, n, stride, d_sink);
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_page_probe, dim3(1024), dim3(256), 0, s, d_data, n, stride, d_sink);
  hipEventRecord(e1, s);
  hipError_t e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (e != hipSuccess || hipGetLastError() != hipSuccess) return -2;
  *ms_out = ms / (float)reps;
  return 0;
}

