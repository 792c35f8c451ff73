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

template <class T, class Op, int BLOCK>
__device__ T block_exclusive_scan(T v, T* sh, Op op, T* total) {
  const int tid = threadIdx.x;
  sh[tid] = v;
  __syncthreads();
  for (int o = 1; o < BLOCK; o <<= 1) {
    T t = tid >= o ? sh[tid - o] : op.identity();
    __syncthreads();
    if (tid >= o) sh[tid] = op(t, sh[tid]);
    __syncthreads();
  }
  if (total) *total = sh[BLOCK - 1];
  T ex = tid ? sh[tid - 1] : op.identity();
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
