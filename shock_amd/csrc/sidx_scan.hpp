// sidx_scan.hpp -- the device-wide scans of the subset, filter and chunkrecord paths: one
// single-pass decoupled look-back kernel (the same scheme as k_scan_excl on the index path,
// sidx_kernels.hip) for large inputs, three plain launches for inputs of at most 2048 blocks
// (run() picks), templated on the input word (u32 flags / u64 lengths), the operator (sum or
// max over u64) and exclusive / inclusive output.  Each is the parallel form of a serial
// running total in the reference: subset.go:245-291's run offsets (oSize), the filters'
// output positions (fq2fa.go / anonymize.go write records back to back), chunkrecord.go:64-93's
// chunk offsets.
//
// API (two-phase, like the library scans it replaces): dscan(nullptr, &bytes, ...) returns
// the workspace size; dscan(tmp, &bytes, ...) clears the workspace's look-back words and
// launches one kernel.  Workgroups take their block number from a ticket in the workspace,
// so a block only ever waits on blocks that were already running (no residency assumption).
#pragma once
#include <hip/hip_runtime.h>

#include "sidx_common.hpp"

namespace sidx {
namespace dscan {

constexpr int T = 256, ITEMS = 8, BLOCK = T * ITEMS;
constexpr u64 F_AGG = 1ull << 62, F_INC = 2ull << 62, PAY = (1ull << 62) - 1;

struct Sum {
  static __device__ __forceinline__ u64 id() { return 0; }
  static __device__ __forceinline__ u64 op(u64 a, u64 b) { return a + b; }
};
struct Max {
  static __device__ __forceinline__ u64 id() { return 0; }
  static __device__ __forceinline__ u64 op(u64 a, u64 b) { return a > b ? a : b; }
};

typedef __attribute__((address_space(1))) u64 gw64;
typedef __attribute__((address_space(1))) u32 gw32;
__device__ __forceinline__ u64 ld(u64 *p) {
  return __hip_atomic_load((gw64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(u64 *p, u64 v) {
  __hip_atomic_store((gw64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// inclusive scan over the wave's lanes (lane 0 first)
template <class M>
__device__ __forceinline__ u64 wave_incl(u64 v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u64 y = __shfl_up(v, d, 64);
    if (lane >= d) v = M::op(y, v);
  }
  return v;
}

template <class In, class M, bool EXCL>
__global__ __launch_bounds__(T) void k_dscan(const In *in, u64 *out, u64 n, u64 *look, u32 *ticket) {
  __shared__ u64 wtot[T / 64];
  __shared__ u64 bpre;
  __shared__ u32 sbid;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) sbid = __hip_atomic_fetch_add((gw32 *)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const u64 bid = sbid;
  const u64 i0 = bid * BLOCK + (u64)tid * ITEMS;
  u64 v[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) v[k] = (i0 + k < n) ? (u64)in[i0 + k] : M::id();
#pragma unroll
  for (int k = 1; k < ITEMS; ++k) v[k] = M::op(v[k - 1], v[k]);  // thread-inclusive
  const u64 tinc = wave_incl<M>(v[ITEMS - 1], lane);
  u64 texc = __shfl_up(tinc, 1, 64);
  if (lane == 0) texc = M::id();
  if (lane == 63) wtot[wid] = tinc;
  __syncthreads();
  u64 wpre = M::id(), btot = M::id();
#pragma unroll
  for (int w = 0; w < T / 64; ++w) {
    if (w < wid) wpre = M::op(wpre, wtot[w]);
    btot = M::op(btot, wtot[w]);
  }
  if (wid == 0) {
    u64 pre = M::id();
    if (bid == 0) {
      if (lane == 0) st(look, F_INC | btot);
    } else {
      if (lane == 0) st(look + bid, F_AGG | btot);
      // fold the predecessors newest first, 64 per step, back to the nearest inclusive word
      u64 acc = M::id();
      i64 hi = (i64)bid - 1;
      for (;;) {
        const i64 idx = hi - lane;
        u64 w = idx >= 0 ? ld(look + idx) : (F_INC | M::id());
        u64 incm, zm;
        for (;;) {
          const u32 f = (u32)(w >> 62);
          incm = __ballot(f == 2);
          zm = __ballot(f == 0);
          const u64 need = incm ? ((1ull << __builtin_ctzll(incm)) - 1) | (1ull << __builtin_ctzll(incm)) : ~0ull;
          if (!(zm & need)) break;  // every word up to the newest inclusive one is published
          __builtin_amdgcn_s_sleep(1);
          if (f == 0) w = ld(look + idx);
        }
        const u32 fi = incm ? (u32)__builtin_ctzll(incm) : 64u;
        u64 x = ((u32)lane <= fi) ? (w & PAY) : M::id();
        // fold lanes 0..fi (lane 0 = newest) into lane 0: order does not matter for sum / max
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x = M::op(x, __shfl_down(x, d, 64));
        acc = M::op(__shfl(x, 0, 64), acc);
        if (incm) break;
        hi -= 64;
      }
      pre = acc;
      if (lane == 0) st(look + bid, F_INC | M::op(pre, btot));
    }
    if (lane == 0) bpre = pre;
  }
  __syncthreads();
  const u64 base = M::op(bpre, M::op(wpre, texc));
#pragma unroll
  for (int k = 0; k < ITEMS; ++k)
    if (i0 + k < n) out[i0 + k] = EXCL ? (k ? M::op(base, v[k - 1]) : base) : M::op(base, v[k]);
}

// Small scans (at most SMALL_BLOCKS blocks of BLOCK items: the subset path's 1.5 M ids at C4)
// take three plain launches instead: the blocks' totals, one workgroup scanning them, then every
// block scanning its items again from its prefix.  No workspace clearing, no ticket, no look-back
// (the single-pass kernel's memset, ticket and look-back made an 18-26 us floor at that size).
#ifndef SIDX_DSCAN_SMALL
#define SIDX_DSCAN_SMALL 1
#endif
constexpr u64 SMALL_BLOCKS = SIDX_DSCAN_SMALL ? (u64)T * ITEMS : 0;

template <class In, class M>
__device__ __forceinline__ u64 block_items(const In *in, u64 n, u64 i0, u64 (&v)[ITEMS]) {  // thread-inclusive
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) v[k] = (i0 + k < n) ? (u64)in[i0 + k] : M::id();
#pragma unroll
  for (int k = 1; k < ITEMS; ++k) v[k] = M::op(v[k - 1], v[k]);
  return v[ITEMS - 1];
}
// exclusive prefix of each thread's value within the workgroup, and the workgroup's total
template <class M>
__device__ __forceinline__ u64 block_excl(u64 x, u64 *wtot, u64 &btot) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u64 tinc = wave_incl<M>(x, lane);
  u64 texc = __shfl_up(tinc, 1, 64);
  if (lane == 0) texc = M::id();
  if (lane == 63) wtot[wid] = tinc;
  __syncthreads();
  u64 wpre = M::id();
  btot = M::id();
#pragma unroll
  for (int w = 0; w < T / 64; ++w) {
    if (w < wid) wpre = M::op(wpre, wtot[w]);
    btot = M::op(btot, wtot[w]);
  }
  return M::op(wpre, texc);
}
template <class In, class M>
__global__ __launch_bounds__(T) void k_sscan_part(const In *in, u64 n, u64 *part) {
  __shared__ u64 wtot[T / 64];
  u64 v[ITEMS], btot;
  const u64 t = block_items<In, M>(in, n, (u64)blockIdx.x * BLOCK + (u64)threadIdx.x * ITEMS, v);
  (void)block_excl<M>(t, wtot, btot);
  if (threadIdx.x == 0) part[blockIdx.x] = btot;
}
template <class M>
__global__ __launch_bounds__(T) void k_sscan_top(u64 *part, u64 nb) {  // in place, exclusive
  __shared__ u64 wtot[T / 64];
  u64 v[ITEMS], btot;
  const u64 i0 = (u64)threadIdx.x * ITEMS;
  const u64 t = block_items<u64, M>(part, nb, i0, v);
  const u64 pre = block_excl<M>(t, wtot, btot);
  __syncthreads();  // (every thread read its items before any is overwritten)
#pragma unroll
  for (int k = 0; k < ITEMS; ++k)
    if (i0 + k < nb) part[i0 + k] = k ? M::op(pre, v[k - 1]) : pre;
}
template <class In, class M, bool EXCL>
__global__ __launch_bounds__(T) void k_sscan_apply(const In *in, u64 *out, u64 n, const u64 *part) {
  __shared__ u64 wtot[T / 64];
  u64 v[ITEMS], btot;
  const u64 i0 = (u64)blockIdx.x * BLOCK + (u64)threadIdx.x * ITEMS;
  const u64 t = block_items<In, M>(in, n, i0, v);
  const u64 base = M::op(part[blockIdx.x], block_excl<M>(t, wtot, btot));
#pragma unroll
  for (int k = 0; k < ITEMS; ++k)
    if (i0 + k < n) out[i0 + k] = EXCL ? (k ? M::op(base, v[k - 1]) : base) : M::op(base, v[k]);
}

// out[i] = op over in[0 .. i) (EXCL, out[0] = 0) or in[0 .. i] (inclusive).  Values (and their
// running totals) must stay below 2^62.
template <class In, class M, bool EXCL>
inline hipError_t run(void *tmp, size_t *tmp_bytes, const In *in, u64 *out, u64 n, hipStream_t s) {
  const u64 nb = (n + BLOCK - 1) / BLOCK;
  const size_t need = 16 + 8 * (size_t)(nb ? nb : 1);
  if (!tmp) {
    *tmp_bytes = need;
    return hipSuccess;
  }
  if (*tmp_bytes < need || nb > 0xFFFFFFFFull) return hipErrorInvalidValue;
  if (!n) return hipSuccess;
  if (nb <= SMALL_BLOCKS) {
    u64 *part = (u64 *)tmp + 2;
    hipLaunchKernelGGL((k_sscan_part<In, M>), dim3((u32)nb), dim3(T), 0, s, in, n, part);
    hipLaunchKernelGGL((k_sscan_top<M>), dim3(1), dim3(T), 0, s, part, nb);
    hipLaunchKernelGGL((k_sscan_apply<In, M, EXCL>), dim3((u32)nb), dim3(T), 0, s, in, out, n, (const u64 *)part);
    return hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(tmp, 0, need, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_dscan<In, M, EXCL>), dim3((u32)nb), dim3(T), 0, s, in, out, n, (u64 *)tmp + 2, (u32 *)tmp);
  return hipGetLastError();
}

}  // namespace dscan
}  // namespace sidx
