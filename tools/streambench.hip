// streambench.hip -- dev tool: read-streaming ceilings of candidate staging structures for the
// tile passes, on a 10 GiB device buffer (no parsing; each kernel only folds what it reads so
// nothing is optimised away).  Build: hipcc -O3 --offload-arch=gfx950 -o tools/streambench
// tools/streambench.hip.  Prints one line per variant: ms per pass and GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;
typedef u32 v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) unsigned char lds_u8;

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ void dma16(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ void dma4(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
template <int NT>
__device__ __forceinline__ void dma16p(u32 voff, u32 lds, __amdgpu_buffer_rsrc_t rs) {
  if (!NT) { dma16(voff, lds, rs); return; }
  u32 keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen nt lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(rs) : "memory");
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const unsigned char *base, u32 n) {
  const u64 ba = (u64)base;
  const unsigned char *sb = (const unsigned char *)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)ba)) |
                                                    ((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)(ba >> 32)) << 32));
  return __builtin_amdgcn_make_buffer_rsrc((void *)sb, (short)0, (int)__builtin_amdgcn_readfirstlane((int)n), 0x00020000);
}
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A: the current structure -- WG of 256 threads, one slot of TILE (+ HALO) bytes, DMA -> vmcnt(0)
// -> barrier -> one LDS read per thread -> barrier, grid-stride, XCD-major order (ORDER 1) or plain.
template <int TILE, int HALO, int ORDER>
__global__ __launch_bounds__(256) void k_slot(const unsigned char *d, u64 n, u64 ntiles, u64 G, u32 *sink) {
  __shared__ __attribute__((aligned(16))) unsigned char raw[TILE + HALO + 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64 t = blockIdx.x;
  if (ORDER == 1 && (G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  // ORDER 2: a contiguous run of tiles per workgroup (tile t's halo is the next one it loads)
  const u64 per = (ntiles + G - 1) / G;
  u64 tend = ntiles, step = G;
  if (ORDER == 2) { t = blockIdx.x * per; tend = t + per < ntiles ? t + per : ntiles; step = 1; }
  u32 acc = 0;
  constexpr int PER = TILE / 1024 / 4;
  for (; t < tend; t += step) {
    const u64 tlo = t * TILE;
    const u64 lim = tlo + TILE + HALO < n ? tlo + TILE + HALO : n;
    const auto rs = rsrc(d + tlo, (u32)(lim - tlo));
    const u32 dst = (u32)(size_t)(lds_u8 *)raw;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const u32 o = (u32)(wid * PER + i) * 1024u;
      dma16(o + lane * 16, dst + o, rs);
    }
    if (HALO) {
      constexpr int HP = HALO / 256;
      for (int h = wid; h < HP; h += 4) dma4(TILE + h * 256 + lane * 4, dst + TILE + h * 256, rs);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    acc += *reinterpret_cast<const u32 *>(raw + tid * (TILE / 256));
    bar();
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// A2: k_slot shaped like k_fq_tiles' skeleton: front piece (wave 0) + one halo piece per wave,
// DMA issued at priority 3, STORES tile words per tile (tid 0), BARS barriers per tile.
template <int STORES, int BARS, int PRIO, int NT = 0>
__global__ __launch_bounds__(256, 7) void k_skel(const unsigned char *d, u64 n, u64 ntiles, u64 G, u32 *tw) {
  constexpr int TILE = 16384, HALO = 1024, FRONT = 16;
  __shared__ __attribute__((aligned(16))) unsigned char raw[FRONT + TILE + HALO];
  __shared__ u32 wt[4];
  __shared__ u64 wbuf[STORES == 18 ? 512 : 1];  // (18) the tile words, stored when the workgroup is done
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const u64 t_first = t;
  u32 nbuf = 0;
  u32 acc = 0;
  for (; t < ntiles; t += G) {
    const u64 tlo = t * TILE;
    const u64 lim = tlo + TILE + HALO - FRONT < n ? tlo + TILE + HALO - FRONT : n;
    const bool sh = tlo >= FRONT;
    const auto rs = rsrc(d + tlo - (sh ? FRONT : 0), (u32)(lim - tlo) + (sh ? FRONT : 0));
    const u32 adj = sh ? 0u : FRONT;
    const u32 dst = (u32)(size_t)(lds_u8 *)raw;
    if (PRIO) __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32 o = FRONT + (u32)(wid * 4 + i) * 1024u;
      dma16p<NT>(o + lane * 16 - adj, dst + o, rs);
    }
    if (wid == 0 && lane < 4) dma4(lane * 4 - adj, dst, rs);
    dma4(FRONT + TILE + wid * 256 + lane * 4 - adj, dst + FRONT + TILE + wid * 256, rs);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32 x = *reinterpret_cast<const u32 *>(raw + FRONT + tid * 64);
    if (lane == 63) wt[wid] = x;
    bar();
    acc += wt[(tid + 1) & 3];
    if (BARS >= 3) bar();
    if (STORES == 1 && tid == 0) {  // the old layout: 5 words at a 160-byte stride + one u32
      u32 *o = tw + t * 40;
      o[0] = acc; o[1] = (u32)t; o[2] = 3; o[3] = 0; o[5] = 0;
      tw[40 * ntiles + t] = acc;
    }
    if (STORES == 2 && tid == 0) {  // a dense 32-byte record + a u64 count
      uint4 *o = reinterpret_cast<uint4 *>(tw + t * 8);
      o[0] = make_uint4(acc, (u32)t, 3, 0);
      o[1] = make_uint4(0, 1, 0, 0);
      reinterpret_cast<u64 *>(tw + 8 * ntiles)[t] = acc;
    }
    if (STORES == 3) {  // (2) + 47 provisional rows (4 bytes per lane of wave 0, 1 KiB stride)
      if (tid == 0) {
        uint4 *o = reinterpret_cast<uint4 *>(tw + t * 8);
        o[0] = make_uint4(acc, (u32)t, 3, 0);
        o[1] = make_uint4(0, 1, 0, 0);
        reinterpret_cast<u64 *>(tw + 8 * ntiles)[t] = acc;
      }
      if (tid < 47) tw[10 * ntiles + t * 256 + tid] = acc + tid;
    }
    if (STORES == 4) {  // (3) with non-temporal stores
      if (tid == 0) {
        __builtin_nontemporal_store(acc, tw + t * 8);
        __builtin_nontemporal_store((u32)t, tw + t * 8 + 1);
        __builtin_nontemporal_store(acc, reinterpret_cast<u64 *>(tw + 8 * ntiles) + t);
      }
      if (tid < 47) __builtin_nontemporal_store(acc + tid, tw + 10 * ntiles + t * 256 + tid);
    }
    if (STORES == 5 && tid < 47) tw[10 * ntiles + t * 256 + tid] = acc + tid;  // the rows alone
    if (STORES == 6 && (t & 3) == 0 && tid < 188) tw[10 * ntiles + t * 256 + tid] = acc + tid;  // 4x the rows, 1/4 as often
    if (STORES >= 7 && tid == 0) {  // one 32-byte record (the count inside it)
      uint4 *o = reinterpret_cast<uint4 *>(tw + t * 8);
      o[0] = make_uint4(acc, (u32)t, 3, 0);
      o[1] = make_uint4(0, 1, 0, 0);
    }
    if (STORES == 7 && tid < 12)  // rows as 16 bytes per lane (192 B)
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 8 && tid < 6)  // 2-byte rows as 16 bytes per lane (96 B)
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    // whole 128-byte lines only (no separate word): is the cost partial-line writes?
    if (STORES == 10 && tid < 8)  // one full line per tile, 1 KiB stride
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 11 && tid < 16)  // two full lines per tile
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 12 && tid < 8)  // one full line per tile, dense (128 B stride)
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 32)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 13 && tid < 8)  // one full line per tile, non-temporal
      __builtin_nontemporal_store((v4u){acc, (u32)tid, acc, (u32)tid}, reinterpret_cast<v4u *>(tw + 10 * ntiles + t * 256) + tid);
    if (STORES == 15 && tid < 8)  // one full line per tile into a 256 KiB ring (L2-resident)
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + (t & 2047) * 32)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 16 && tid == 0)  // the 8-byte tile word alone, dense
      reinterpret_cast<u64 *>(tw + 8 * ntiles)[t] = acc;
    if (STORES == 17 && (t & 3) == 0 && tid < 32)  // 512 B every 4th tile
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    if (STORES == 18 && tid == 0 && nbuf < 512) wbuf[nbuf] = acc;
    if (STORES == 18) ++nbuf;
    if (STORES == 14 && tid < 4)  // half a line (64 B) per tile
      reinterpret_cast<uint4 *>(tw + 10 * ntiles + t * 256)[tid] = make_uint4(acc, tid, acc, tid);
    bar();
  }
  if (STORES == 18) {
    bar();
    for (u32 i = (u32)tid; i < nbuf && i < 512; i += 256) reinterpret_cast<u64 *>(tw + 8 * ntiles)[t_first + (u64)i * G] = wbuf[i];
  }
  if (acc == 0x12345678u) tw[0] = acc;
}

// A3: (A2 with STORES 3) but each tile's stores are issued after the NEXT tile's DMA and the
// wait counts them out (vmcnt(N)), so the DMA wait no longer includes the stores' acks.
__global__ __launch_bounds__(256, 7) void k_skel_defer(const unsigned char *d, u64 n, u64 ntiles, u64 G, u32 *tw) {
  constexpr int TILE = 16384, HALO = 1024, FRONT = 16;
  __shared__ __attribute__((aligned(16))) unsigned char raw[FRONT + TILE + HALO];
  __shared__ u32 wt[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  u32 acc = 0;
  u64 pt = ~0ull;  // the tile whose stores are pending
  u32 pacc = 0;
  for (; t < ntiles; t += G) {
    const u64 tlo = t * TILE;
    const u64 lim = tlo + TILE + HALO - FRONT < n ? tlo + TILE + HALO - FRONT : n;
    const bool sh = tlo >= FRONT;
    const auto rs = rsrc(d + tlo - (sh ? FRONT : 0), (u32)(lim - tlo) + (sh ? FRONT : 0));
    const u32 adj = sh ? 0u : FRONT;
    const u32 dst = (u32)(size_t)(lds_u8 *)raw;
    __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32 o = FRONT + (u32)(wid * 4 + i) * 1024u;
      dma16(o + lane * 16 - adj, dst + o, rs);
    }
    if (wid == 0 && lane < 4) dma4(lane * 4 - adj, dst, rs);
    dma4(FRONT + TILE + wid * 256 + lane * 4 - adj, dst + FRONT + TILE + wid * 256, rs);
    __builtin_amdgcn_s_setprio(0);
    if (pt != ~0ull && wid == 0) {  // wave 0: 1 row store (lanes < 47) + 2 record stores (lane 0) + 1 count
      if (lane < 47) tw[10 * ntiles + pt * 256 + lane] = pacc + lane;
      if (lane == 0) {
        uint4 *o = reinterpret_cast<uint4 *>(tw + pt * 8);
        o[0] = make_uint4(pacc, (u32)pt, 3, 0);
        o[1] = make_uint4(0, 1, 0, 0);
        reinterpret_cast<u64 *>(tw + 8 * ntiles)[pt] = pacc;
      }
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const u32 x = *reinterpret_cast<const u32 *>(raw + FRONT + tid * 64);
    if (lane == 63) wt[wid] = x;
    bar();
    acc += wt[(tid + 1) & 3];
    bar();
    pt = t;
    pacc = acc;
    bar();
  }
  if (pt != ~0ull && wid == 0) {
    if (lane < 47) tw[10 * ntiles + pt * 256 + lane] = pacc + lane;
    if (lane == 0) reinterpret_cast<u64 *>(tw + 8 * ntiles)[pt] = pacc;
  }
}

// B: one independent slot per WAVE (no barriers): a wave stages WT bytes (+ HALO) and reads them.
template <int WT, int HALO>
__global__ __launch_bounds__(256) void k_wave(const unsigned char *d, u64 n, u64 ntiles, u64 G, u32 *sink) {
  __shared__ __attribute__((aligned(16))) unsigned char raw[4][WT + HALO];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u64 GW = G * 4;
  u64 t = (u64)blockIdx.x * 4 + wid;
  if ((G & 7) == 0) t = ((blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3)) * 4 + wid;
  u32 acc = 0;
  for (; t < ntiles; t += GW) {
    const u64 tlo = t * WT;
    const u64 lim = tlo + WT + HALO < n ? tlo + WT + HALO : n;
    const auto rs = rsrc(d + tlo, (u32)(lim - tlo));
    const u32 dst = (u32)(size_t)(lds_u8 *)raw[wid];
#pragma unroll
    for (int i = 0; i < WT / 1024; ++i) dma16((u32)i * 1024u + lane * 16, dst + i * 1024, rs);
    if (HALO)
      for (int h = 0; h < HALO / 256; ++h) dma4(WT + h * 256 + lane * 4, dst + WT + h * 256, rs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += *reinterpret_cast<const u32 *>(&raw[wid][lane * (WT / 64)]);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// C: two slots per WG (double buffer): DMA of tile k+1 issued before waiting for tile k.
template <int TILE>
__global__ __launch_bounds__(256) void k_db(const unsigned char *d, u64 n, u64 ntiles, u64 G, u32 *sink) {
  __shared__ __attribute__((aligned(16))) unsigned char raw[2][TILE];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64 t = blockIdx.x;
  if ((G & 7) == 0) t = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  constexpr int PER = TILE / 1024 / 4;
  auto issue = [&](u64 tt, int slot) {
    const u64 tlo = tt * TILE;
    const u64 lim = tlo + TILE < n ? tlo + TILE : n;
    const auto rs = rsrc(d + tlo, (u32)(lim - tlo));
    const u32 dst = (u32)(size_t)(lds_u8 *)raw[slot];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const u32 o = (u32)(wid * PER + i) * 1024u;
      dma16(o + lane * 16, dst + o, rs);
    }
  };
  u32 acc = 0;
  int slot = 0;
  if (t < ntiles) issue(t, 0);
  for (; t < ntiles; t += G) {
    if (t + G < ntiles) {
      issue(t + G, slot ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    acc += *reinterpret_cast<const u32 *>(&raw[slot][tid * (TILE / 256)]);
    bar();
    slot ^= 1;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// D: register streaming reference: 16 bytes per lane per load, UNR loads in flight per lane.
template <int UNR>
__global__ __launch_bounds__(256) void k_reg(const uint4 *d, u64 n16, u32 *sink) {
  u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  const u64 stride = (u64)gridDim.x * 256;
  u32 acc = 0;
  for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
    uint4 v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) v[k] = d[i + k * stride];
#pragma unroll
    for (int k = 0; k < UNR; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  for (; i < n16; i += stride) { const uint4 v = d[i]; acc ^= v.x ^ v.w; }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <class F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const u64 n = (argc > 1 ? strtoull(argv[1], 0, 10) : 10ull) << 30;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  unsigned char *d;
  u32 *sink;
  CHK(hipMalloc(&d, n + 4096));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(d, 0x41, n));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto rep = [&](const char *name, double ms) { printf("%-34s %8.4f ms %8.1f GB/s\n", name, ms, n / (ms * 1e-3) / 1e9); fflush(stdout); };
#define SLOT(T, H, O, W)                                                                                       \
  {                                                                                                           \
    const u64 nt = (n + T - 1) / T, G = (u64)cus * W < nt ? (u64)cus * W : nt;                                \
    rep("slot T=" #T " H=" #H " ord=" #O " wg/cu=" #W,                                                        \
        timeit([&] { hipLaunchKernelGGL((k_slot<T, H, O>), dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, sink); }, reps)); \
  }
  SLOT(16384, 1024, 1, 7)
  SLOT(16384, 0, 1, 7)
  if (getenv("SB_ORDER")) {
    SLOT(16384, 0, 2, 7)
    SLOT(16384, 1024, 2, 7)
    SLOT(16384, 0, 0, 7)
    SLOT(16384, 0, 1, 7)
    SLOT(16384, 0, 2, 7)
    return 0;
  }
  if (getenv("SB_SKEL")) {
    u32 *tw;
    const u64 nt = n / 16384;
    CHK(hipMalloc(&tw, 4 * (10 * nt + 256 * nt) + 64));
#define SKELNT(S)                                                                                               \
    {                                                                                                          \
      const u64 G = (u64)cus * 7;                                                                              \
      rep("skel nt-dma stores=" #S,                                                                             \
          timeit([&] { hipLaunchKernelGGL((k_skel<S, 3, 1, 1>), dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, tw); }, reps)); \
    }
#define SKEL(S, B, P)                                                                                           \
    {                                                                                                          \
      const u64 G = (u64)cus * 7;                                                                              \
      rep("skel stores=" #S " bars=" #B " prio=" #P,                                                           \
          timeit([&] { hipLaunchKernelGGL((k_skel<S, B, P>), dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, tw); }, reps)); \
    }
    if (getenv("SB_NT")) {
      SKEL(18, 3, 1)
      SKELNT(18)
      SKEL(0, 3, 1)
      SKELNT(0)
      SKEL(16, 3, 1)
      SKELNT(16)
      SKEL(8, 3, 1)
      SKELNT(8)
      SKELNT(10)
      SKEL(0, 3, 1)
      return 0;
    }
    SKEL(0, 3, 1)
    SKEL(1, 3, 1)
    SKEL(2, 3, 1)
    SKEL(3, 3, 1)
    SKEL(5, 3, 1)
    SKEL(7, 3, 1)
    SKEL(8, 3, 1)
    SKEL(9, 3, 1)
    SKEL(10, 3, 1)
    SKEL(11, 3, 1)
    SKEL(12, 3, 1)
    SKEL(13, 3, 1)
    SKEL(14, 3, 1)
    SKEL(15, 3, 1)
    SKEL(16, 3, 1)
    SKEL(17, 3, 1)
    SKEL(8, 3, 1)
    {
      const u64 G = (u64)cus * 7;
      rep("skel deferred stores (3)", timeit([&] { hipLaunchKernelGGL(k_skel_defer, dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, tw); }, reps));
    }
    SKEL(0, 3, 1)
    CHK(hipFree(tw));
    return 0;
  }
  SLOT(16384, 1024, 0, 7)
  SLOT(16384, 0, 0, 8)
  SLOT(8192, 0, 1, 8)
  SLOT(8192, 512, 1, 8)
  SLOT(32768, 0, 1, 4)
#define WAVE(WT, H, W)                                                                                          \
  {                                                                                                            \
    const u64 nt = (n + WT - 1) / WT, G = (u64)cus * W;                                                        \
    rep("wave WT=" #WT " H=" #H " wg/cu=" #W,                                                                  \
        timeit([&] { hipLaunchKernelGGL((k_wave<WT, H>), dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, sink); }, reps)); \
  }
  WAVE(4096, 0, 8)
  WAVE(4096, 1024, 7)
  WAVE(8192, 0, 4)
  WAVE(8192, 1024, 4)
#define DB(T, W)                                                                                                \
  {                                                                                                            \
    const u64 nt = (n + T - 1) / T, G = (u64)cus * W < nt ? (u64)cus * W : nt;                                 \
    rep("db T=" #T " wg/cu=" #W, timeit([&] { hipLaunchKernelGGL((k_db<T>), dim3((u32)G), dim3(256), 0, 0, d, n, nt, G, sink); }, reps)); \
  }
  DB(8192, 8)
  DB(16384, 4)
#define REG(U, B)                                                                                               \
  rep("reg unroll=" #U " blocks/cu=" #B,                                                                       \
      timeit([&] { hipLaunchKernelGGL((k_reg<U>), dim3((u32)(cus * B)), dim3(256), 0, 0, (const uint4 *)d, n / 16, sink); }, reps));
  REG(4, 8)
  REG(8, 8)
  REG(4, 16)
  CHK(hipFree(d));
  return 0;
}
