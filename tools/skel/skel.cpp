// skel.cpp -- streaming-ceiling microbenchmark for the FASTQ index kernel redesign (not part of
// the product).  Measures, on a 10 GiB device buffer of FASTQ-like bytes, how fast a
// persistent grid can stream 16 KiB tiles through LDS and classify them, for several
// staging schemes:
//   R  register prefetch (16 B/lane global_load_dwordx4, one tile ahead, the k_pipe scheme)
//   L  LDS-DMA ring (global_load_lds_dwordx4, D slots, D-1 tiles in flight, hand-counted vmcnt)
// and several amounts of per-tile work (MODE 0: touch, 1: '\n' masks + count, 2: + newline
// position array).  Build: hipcc -O3 --offload-arch=gfx950 tools/skel/skel.cpp -o tools/skel/skel
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;
#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int TILE = 16384;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

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

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NT>
__device__ __forceinline__ u32 block_sum(u32 c, u32 *red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += (u32)__shfl_xor((int)c, d, 64);
  if (lane == 0) red[wid] = c;
  lds_barrier();
  u32 t = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  return t;
}

// per-tile work on bytes staged at raw[0 .. TILE) (raw 16-aligned), masks into m16
template <int NT, int MODE>
__device__ __forceinline__ u32 work(const uint8_t *raw, uint16_t *m16, uint16_t *nlpos, u32 *red) {
  const int tid = threadIdx.x;
  constexpr int CPT = TILE / 16 / NT;
  u32 c = 0;
  if (MODE == 0) {
    c = *reinterpret_cast<const u32 *>(raw + tid * 4);
  } else {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const u32 ch = (u32)(k * NT + tid);
      const uint4 v = *reinterpret_cast<const uint4 *>(raw + ch * 16);
      const u32 m = eq16(v, '\n');
      m16[ch] = (uint16_t)m;
      c += __popc(m);
    }
  }
  if (MODE >= 2) {
    // each thread owns TILE/NT contiguous bytes = (TILE/NT)/64 mask words
    lds_barrier();
    constexpr int NTW = NT > 256 ? 256 : NT;  // threads owning >= 64 bytes each
    constexpr int WPT = TILE / NTW / 64;
    const u64 *m64 = reinterpret_cast<const u64 *>(m16);
    u64 w[WPT];
    u32 cnt = 0;
#pragma unroll
    for (int j = 0; j < WPT; ++j) { w[j] = tid < NTW ? m64[tid * WPT + j] : 0; cnt += __popcll(w[j]); }
    // exclusive prefix of cnt over the block
    u32 incl = cnt;
    const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { const u32 y = __shfl_up(incl, d, 64); if (lane >= d) incl += y; }
    if (lane == 63) red[8 + wid] = incl;
    lds_barrier();
    u32 o = incl - cnt;
    for (int q = 0; q < wid; ++q) o += red[8 + q];
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      u64 m = w[j];
      while (m) {
        if (o < 2048) nlpos[o] = (uint16_t)((tid * WPT + j) * 64 + __builtin_ctzll(m));
        ++o;
        m &= m - 1;
      }
    }
  }
  return c;
}

// ---- R: register prefetch (one tile ahead) --------------------------------------------
template <int NT, int MODE>
__global__ __launch_bounds__(NT) void k_reg(const uint8_t *data, u32 ntiles, u32 *out) {
  constexpr int CPT = TILE / 16 / NT;
  __shared__ __attribute__((aligned(16))) uint8_t raw[TILE];
  __shared__ uint16_t m16[TILE / 16];
  __shared__ uint16_t nlpos[2048];
  __shared__ u32 red[16];
  const int tid = threadIdx.x;
  uint4 v[CPT];
  u32 t = blockIdx.x;
  if (t < ntiles) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) v[k] = *reinterpret_cast<const uint4 *>(data + (u64)t * TILE + (k * NT + tid) * 16);
  }
  for (; t < ntiles; t += gridDim.x) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) *reinterpret_cast<uint4 *>(raw + (k * NT + tid) * 16) = v[k];
    lds_barrier();
    const u32 tn = t + gridDim.x;
    if (tn < ntiles) {
#pragma unroll
      for (int k = 0; k < CPT; ++k) v[k] = *reinterpret_cast<const uint4 *>(data + (u64)tn * TILE + (k * NT + tid) * 16);
    }
    const u32 c = block_sum<NT>(work<NT, MODE>(raw, m16, nlpos, red), red);
    if (tid == 0) out[t] = c + nlpos[5];
    lds_barrier();
  }
}

// ---- L: LDS-DMA ring -----------------------------------------------------------------
// slot = TILE (+ HALO bytes of the next tile).  Every wave issues the same number of 1 KiB
// DMA instructions per tile (TILE/1024/NW, plus one halo instruction spread over waves by
// making it part of the same per-wave quota when HALO == 1024 * NW ... here: wave 0 also
// loads the halo, so waves differ: the wait count is chosen per wave).
template <int NT, int D, int MODE, int HALO, int NTPOL>
__global__ __launch_bounds__(NT) void k_lds(const uint8_t *data, u64 n, u32 ntiles, u32 *out) {
  constexpr int NW = NT / 64;
  constexpr int SLOT = TILE + HALO;
  constexpr int PER = TILE / 1024 / NW;  // tile DMA instructions per wave
  __shared__ __attribute__((aligned(16))) uint8_t ring[D * SLOT];
  __shared__ uint16_t m16[(TILE) / 16];
  __shared__ uint16_t nlpos[2048];
  __shared__ u32 red[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u32 G = gridDim.x, b = blockIdx.x;
  const u32 ring_lds = (u32)(size_t)(lds_u8 *)ring;
  auto issue = [&](u32 t, u32 slot) {
    const u64 base = (u64)t * TILE;
    const uint8_t *src = data + base + (u64)(wid * PER) * 1024 + lane * 16;
    u32 dst = ring_lds + slot * SLOT + (u32)(wid * PER) * 1024;
    u32 keep;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (NTPOL)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src + i * 1024), "s"(dst + i * 1024) : "memory");
      else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src + i * 1024), "s"(dst + i * 1024) : "memory");
    }
    if (HALO && wid == 0) {
      // halo = first HALO bytes of the next tile (clamped to the buffer; the buffer has slack)
      const uint8_t *hs = data + base + TILE + lane * 16;
      const u32 hd = ring_lds + slot * SLOT + TILE;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(hs), "s"(hd) : "memory");
    }
  };
  // prologue: D-1 tiles in flight
  u32 k = 0;
#pragma unroll
  for (int j = 0; j < D - 1; ++j) {
    const u32 t = b + (u32)j * G;
    if (t < ntiles) issue(t, (u32)j);
  }
  for (u32 t = b; t < ntiles; t += G, ++k) {
    const u32 slot = k % D;
    // issue tile k + D - 1 into the slot freed at the end of iteration k - 1
    const u32 tn = t + (u32)(D - 1) * G;
    const bool steady = tn < ntiles;
    if (steady) issue(tn, (k + D - 1) % D);
    // wait for tile k: D-1 younger tiles' DMA per wave (steady state), else everything
    if (steady) {
      if (HALO && wid == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * (PER + 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * PER) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    const uint8_t *raw = ring + slot * SLOT;
    const u32 c = block_sum<NT>(work<NT, MODE>(raw, m16, nlpos, red), red);
    if (tid == 0) out[t] = c + nlpos[5];
    lds_barrier();
  }
}

// ---- fill: FASTQ-like bytes ('\n' roughly every 86 bytes) -----------------------------
__global__ void k_fill(uint8_t *d, u64 n) {
  for (u64 i = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < n; i += (u64)gridDim.x * blockDim.x * 16) {
    uint8_t b[16];
    for (int j = 0; j < 16; ++j) {
      u64 x = (i + j) * 0x9E3779B97F4A7C15ull;
      x ^= x >> 29;
      b[j] = ((x & 127) == 0 || ((i + j) % 97) == 0) ? '\n' : (uint8_t)('A' + (x >> 40) % 26);
    }
    *reinterpret_cast<uint4 *>(d + i) = *reinterpret_cast<uint4 *>(b);
  }
}

template <class K>
static void timeit(const char *name, K launch, u64 bytes, int reps = 10) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float m;
    CK(hipEventElapsedTime(&m, e0, e1));
    ms.push_back(m);
  }
  CK(hipGetLastError());
  float best = 1e9, sum = 0;
  for (float m : ms) { best = m < best ? m : best; sum += m; }
  const float avg = sum / ms.size();
  printf("%-40s avg %7.3f ms  best %7.3f ms  %7.0f GB/s avg  frac(8TB/s) %.3f\n", name, avg, best, bytes / (avg * 1e-3) / 1e9,
         bytes / (avg * 1e-3) / 8e12);
  fflush(stdout);
}

template <int NT, int MODE>
static void run_reg(const uint8_t *d, u64 n, u32 *out, int cus, int per) {
  const u32 nt = (u32)(n / TILE);
  char name[64];
  snprintf(name, sizeof name, "R nt=%d mode=%d per_cu=%d", NT, MODE, per);
  timeit(name, [&] { hipLaunchKernelGGL((k_reg<NT, MODE>), dim3(cus * per), dim3(NT), 0, 0, d, nt, out); }, n);
}
template <int NT, int D, int MODE, int HALO, int NTP>
static void run_lds(const uint8_t *d, u64 n, u32 *out, int cus, int per) {
  const u32 nt = (u32)(n / TILE);
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lds<NT, D, MODE, HALO, NTP>, NT, 0));
  if (per > occ) per = occ;
  char name[80];
  snprintf(name, sizeof name, "L nt=%d D=%d mode=%d halo=%d ntpol=%d per_cu=%d(occ %d)", NT, D, MODE, HALO, NTP, per, occ);
  timeit(name, [&] { hipLaunchKernelGGL((k_lds<NT, D, MODE, HALO, NTP>), dim3(cus * per), dim3(NT), 0, 0, d, n, nt, out); }, n);
}

int main(int argc, char **argv) {
  const u64 n = (argc > 1 ? strtoull(argv[1], 0, 10) : 10ull) << 30;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *d;
  u32 *out;
  CK(hipMalloc(&d, n + (1 << 20)));
  CK(hipMalloc(&out, (n / TILE + 1) * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, d, n + (1 << 20));
  CK(hipDeviceSynchronize());
  printf("bytes %llu, CUs %d\n", (unsigned long long)n, cus);
  const int sweep = argc > 2 ? atoi(argv[2]) : 1;
  if (sweep == 1) {
    // A: pure DMA streaming
    run_lds<256, 2, 0, 0, 0>(d, n, out, cus, 4);
    run_lds<256, 2, 0, 0, 0>(d, n, out, cus, 3);
    run_lds<256, 3, 0, 0, 0>(d, n, out, cus, 2);
    run_lds<256, 4, 0, 0, 0>(d, n, out, cus, 2);
    run_lds<512, 2, 0, 0, 0>(d, n, out, cus, 2);
    run_lds<512, 4, 0, 0, 0>(d, n, out, cus, 2);
    run_lds<512, 4, 0, 0, 0>(d, n, out, cus, 1);
    run_lds<512, 8, 0, 0, 0>(d, n, out, cus, 1);
    run_lds<128, 2, 0, 0, 0>(d, n, out, cus, 4);
    run_lds<128, 4, 0, 0, 0>(d, n, out, cus, 2);
    run_lds<1024, 4, 0, 0, 0>(d, n, out, cus, 1);
    run_lds<1024, 8, 0, 0, 0>(d, n, out, cus, 1);
    // B: work
    run_lds<512, 8, 2, 0, 0>(d, n, out, cus, 1);
    run_lds<512, 8, 1, 1024, 0>(d, n, out, cus, 1);
    run_lds<512, 4, 2, 1024, 0>(d, n, out, cus, 1);
    run_lds<256, 2, 2, 1024, 0>(d, n, out, cus, 4);
    run_lds<256, 2, 2, 1024, 0>(d, n, out, cus, 3);
    run_lds<1024, 8, 1, 0, 0>(d, n, out, cus, 1);
    run_lds<1024, 8, 2, 1024, 0>(d, n, out, cus, 1);
  }
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
