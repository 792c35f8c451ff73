// shard_kernels.hip -- the device steps a sharded (multi-GPU) build adds to the single-GPU path
// (DESIGN.md §6).  Each rank holds a byte range of the log; these kernels find its first record,
// count its entries per destination rank, and do the small exchanges' device work.
//
//   k_find_entry     candidate record starts at the head of the rank's byte range, walked in
//                    parallel until they all reach one common record start (the rank's entry)
//   k_dest_counts    entries per destination rank after the coarse-digit partition
//   k_apply_spill    slots another rank's placement wrote past its range
//   k_fetch_keys     key bytes of requested records (equal-hash pairs are compared by the rank
//                    that placed them, IndexHash.java:606-636)
//   k_compare_keys   the comparison itself
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"

namespace sk {

// Every plausible start in [lo, cand_end) walks its chain with the speculative rules of k_frame
// (IndexHash's iterator rules plus the header's maxKeyLen / maxValueLen) to the first record start
// >= target.  If every surviving chain reaches the same start, that start is on the true chain
// whenever the true first record survives (it does unless the header understates its maxima);
// the host verifies it against the previous rank's exact walk either way.
// out[0] = that start, or -1 when no chain survives or they do not meet.
__global__ __launch_bounds__(256) void k_find_entry(BuildParams P, int64_t lo, int64_t cand_end, int64_t target,
                                                    int64_t* out) {
  __shared__ unsigned long long s_min, s_n;
  __shared__ long long s_max;
  if (threadIdx.x == 0) {
    s_min = ~0ull;
    s_max = -1;
    s_n = 0;
  }
  __syncthreads();
  const int64_t log_len = (int64_t)P.log_len;
  auto at = [&](int64_t a) -> uint32_t { return (uint32_t)P.log[a]; };
  for (int64_t c = lo + threadIdx.x; c < cand_end; c += blockDim.x) {
    int64_t p = c;
    bool alive = true;
    while (p < target) {
      const RecHdr h = decode_header(at, p, log_len);
      if (!header_plausible(h, p, P.max_key_len, P.max_value_len, log_len) || (!h.put && P.no_deletes)) {
        alive = false;
        break;
      }
      p = record_end(h, p);
    }
    if (!alive) continue;
    const int64_t x = min(p, P.data_end);
    atomicMin(&s_min, (unsigned long long)x);
    atomicMax(&s_max, (long long)x);
    atomicAdd(&s_n, 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (s_n > 0 && (long long)s_min == s_max) ? (int64_t)s_min : -1;
}

// out[r] = first entry (in the digit-partitioned order) bound for rank r, out[world] = total.
// Rank r owns the coarse digits [nd r / world, nd (r + 1) / world) of the nd digits in use.
__global__ void k_dest_counts(BuildParams P, int world, uint32_t nd, uint64_t* out) {
  const int r = threadIdx.x;
  if (r > world) return;
  const uint32_t d = (uint32_t)(((uint64_t)nd * r) / world);
  out[r] = d < 256 ? P.p1_off[(uint64_t)d * P.p1_tiles] : P.p1_off_total[0];
}

// the pass-1 start of every coarse digit, and the total (257 values)
__global__ void k_digit_starts(BuildParams P, uint64_t* out) {
  const uint32_t d = threadIdx.x;
  if (d <= 256) out[d] = d < 256 ? P.p1_off[(uint64_t)d * P.p1_tiles] : P.p1_off_total[0];
}

__global__ void k_apply_spill(BuildParams P, const SpillEntry* in, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SpillEntry e = in[i];
  if (e.slot >= P.slot_lo && e.slot < P.slot_hi) write_slot(P, e.slot, e.hash, e.addr);
}

// rec = [u32 key length (0xffffffff: no valid record there), u32 0, key bytes, zero padding]
__global__ void k_fetch_keys(BuildParams P, const uint64_t* addrs, uint64_t n, uint8_t* rec, uint32_t rec_size) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* r = rec + i * rec_size;
  const int64_t p = (int64_t)((addrs[i] & ~kDelBit) >> P.ebb);
  const int64_t log_len = (int64_t)P.log_len;
  uint32_t klen = 0xffffffffu;
  const uint8_t* key = nullptr;
  if (p >= P.fr_entry && p < log_len) {
    auto at = [&](int64_t a) -> uint32_t { return (uint32_t)P.log[a]; };
    const RecHdr h = decode_header(at, p, log_len);
    if (header_valid(h, p, P.max_key_len, log_len) && 8u + (uint32_t)h.klen <= rec_size) {
      klen = (uint32_t)h.klen;
      key = P.log + p + h.hlen;
    }
  }
  reinterpret_cast<uint32_t*>(r)[0] = klen;
  reinterpret_cast<uint32_t*>(r)[1] = 0;
  for (uint32_t j = 0; j + 8 < rec_size; j++) r[8 + j] = (key && j < klen) ? key[j] : 0;
}

__global__ void k_compare_keys(BuildParams P, const uint8_t* rec, uint64_t npairs, uint32_t rec_size) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const uint8_t* a = rec + (2 * i) * rec_size;
  const uint8_t* b = rec + (2 * i + 1) * rec_size;
  const uint32_t ka = reinterpret_cast<const uint32_t*>(a)[0];
  const uint32_t kb = reinterpret_cast<const uint32_t*>(b)[0];
  if (ka == 0xffffffffu || kb == 0xffffffffu) {  // an address no rank could decode: never canonical
    atomicOr(&P.st->dup, 2u);
    return;
  }
  if (ka != kb) return;
  for (uint32_t j = 0; j < ka; j++)
    if (a[8 + j] != b[8 + j]) return;
  atomicOr(&P.st->dup, 1u);
}

void launch_find_entry(const BuildParams& P, hipStream_t s, int64_t lo, int64_t cand_end, int64_t target,
                       int64_t* d_out) {
  hipLaunchKernelGGL(k_find_entry, dim3(1), dim3(256), 0, s, P, lo, cand_end, target, d_out);
}

void launch_dest_counts(const BuildParams& P, hipStream_t s, int world, uint32_t nd, uint64_t* d_out) {
  hipLaunchKernelGGL(k_dest_counts, dim3(1), dim3(320), 0, s, P, world, nd, d_out);
}

void launch_digit_starts(const BuildParams& P, hipStream_t s, uint64_t* d_out) {
  hipLaunchKernelGGL(k_digit_starts, dim3(1), dim3(320), 0, s, P, d_out);
}

void launch_apply_spill(const BuildParams& P, hipStream_t s, const SpillEntry* in, uint64_t n) {
  if (n) hipLaunchKernelGGL(k_apply_spill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, in, n);
}

void launch_fetch_keys(const BuildParams& P, hipStream_t s, const uint64_t* addrs, uint64_t n, uint8_t* rec,
                       uint32_t rec_size) {
  if (n) hipLaunchKernelGGL(k_fetch_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, addrs, n, rec, rec_size);
}

void launch_compare_keys(const BuildParams& P, hipStream_t s, const uint8_t* rec, uint64_t npairs, uint32_t rec_size) {
  if (npairs)
    hipLaunchKernelGGL(k_compare_keys, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, s, P, rec, npairs, rec_size);
}

}  // namespace sk
