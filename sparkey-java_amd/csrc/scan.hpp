// scan.hpp -- 3-phase device exclusive scan, generic over the combine op (op(a, b) = "a then b").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"

namespace sk {

// ================================================================================================
// Scans (3-phase, generic over the combine op; op(a, b) = "a then b").
// ================================================================================================
struct OpAdd {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
  __device__ __forceinline__ uint64_t identity() const { return 0; }
};
// Carry functions f(x) = max(c, x + a) composed left to right: (f then g)(x) = g(f(x)).
struct OpMaxPlus {
  __device__ __forceinline__ MaxPlus operator()(MaxPlus f, MaxPlus g) const {
    MaxPlus r;
    r.c = max(g.c, f.c + g.a);
    r.a = f.a + g.a;
    return r;
  }
  __device__ __forceinline__ MaxPlus identity() const { return MaxPlus{0, 0}; }
};

struct OpMaxI64 {
  __device__ __forceinline__ int64_t operator()(int64_t a, int64_t b) const { return a > b ? a : b; }
  __device__ __forceinline__ int64_t identity() const { return -(1ll << 40); }
};

__device__ __forceinline__ uint64_t shfl_up_any(uint64_t v, int o) { return __shfl_up(v, o, 64); }
__device__ __forceinline__ int64_t shfl_up_any(int64_t v, int o) { return __shfl_up(v, o, 64); }
__device__ __forceinline__ uint32_t shfl_up_any(uint32_t v, int o) { return __shfl_up(v, o, 64); }
__device__ __forceinline__ MaxPlus shfl_up_any(MaxPlus v, int o) {
  MaxPlus r;
  r.c = __shfl_up(v.c, o, 64);
  r.a = __shfl_up(v.a, o, 64);
  return r;
}

// Block-wide exclusive scan (op(a, b) = "a then b"): shuffles inside each wave, one LDS round for
// the wave totals.  sh needs at least BLOCK / 64 + 1 slots.
template <class T, class Op, int BLOCK>
__device__ T block_exclusive_scan(T v, T* sh, Op op, T* total) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T t = shfl_up_any(incl, o);
    if (lane >= o) incl = op(t, incl);
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = op.identity();
    for (int i = 0; i < NW; i++) {
      const T t = sh[i];
      sh[i] = run;
      run = op(run, t);
    }
    sh[NW] = run;
  }
  __syncthreads();
  T exw = shfl_up_any(incl, 1);
  if (lane == 0) exw = op.identity();
  const T ex = op(sh[w], exw);
  if (total) *total = sh[NW];
  __syncthreads();
  return ex;
}

// Exclusive sum over a block of BLOCK threads (wave shuffles, one LDS round for the wave totals).
// sh needs BLOCK / 64 + 1 slots.
template <int BLOCK>
__device__ __forceinline__ uint64_t block_excl_sum(uint64_t v, uint64_t* sh, uint64_t* total) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int i = 0; i < NW; i++) {
      const uint64_t t = sh[i];
      sh[i] = run;
      run += t;
    }
    sh[NW] = run;
  }
  __syncthreads();
  const uint64_t ex = sh[w] + incl - v;
  if (total) *total = sh[NW];
  __syncthreads();
  return ex;
}

template <class In, class T, class Op>
__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(const In* in, T* out, T* tile_tot, uint64_t n, Op op) {
  __shared__ T sh[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  T v[kScanItems];
  T acc = op.identity();
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    const uint64_t idx = base + i;
    T x = idx < n ? (T)in[idx] : op.identity();
    v[i] = acc;  // exclusive within the thread
    acc = op(acc, x);
  }
  T tot;
  const T pre = block_exclusive_scan<T, Op, kScanBlock>(acc, sh, op, &tot);
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    const uint64_t idx = base + i;
    if (idx < n) out[idx] = op(pre, v[i]);
  }
  if (threadIdx.x == 0) tile_tot[blockIdx.x] = tot;
}

template <class T, class Op>
__global__ void k_scan_add(T* out, const T* tile_pre, uint64_t n, Op op) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t t = i / kScanTile;
  if (t == 0) return;
  out[i] = op(tile_pre[t], out[i]);
}

template <class In, class T, class Op>
inline void scan_exclusive(const In* in, T* out, uint64_t n, T* d_total, Op op, T* scratch, hipStream_t s) {
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  if (tiles <= 1) {
    hipLaunchKernelGGL((k_scan_tiles<In, T, Op>), dim3(1), dim3(kScanBlock), 0, s, in, out, d_total, n, op);
    return;
  }
  T* sums = scratch;
  hipLaunchKernelGGL((k_scan_tiles<In, T, Op>), dim3((unsigned)tiles), dim3(kScanBlock), 0, s, in, out, sums, n, op);
  scan_exclusive<T, T, Op>(sums, sums, tiles, d_total, op, scratch + tiles, s);
  hipLaunchKernelGGL((k_scan_add<T, Op>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, sums, n, op);
}

}  // namespace sk
