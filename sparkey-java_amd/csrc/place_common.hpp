// place_common.hpp -- per-bucket placement helpers (canonical Robin-Hood layout).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

// Per bucket: LDS histogram of local wanted slots and its exclusive scan; returns n.
__device__ __forceinline__ void bucket_histogram(const BuildParams& P, uint64_t b, uint32_t n, uint64_t eoff,
                                                 uint64_t start, uint32_t* cnt) {
  for (int t = threadIdx.x; t < kBucket; t += kPlaceBlock) cnt[t] = 0;
  __syncthreads();
  bool bad = false;  // (kGuardForeign: the entry is left out here and in the sort below)
  for (uint32_t i = threadIdx.x; i < n; i += kPlaceBlock) {
    const uint64_t w = fast_mod(P.ent2[eoff + i].hash, P.mod) - start;
    if (w < (uint64_t)kBucket) atomicAdd(&cnt[w], 1u);
    else bad = true;
  }
  report_foreign(P, bad);
  __syncthreads();
}

// For the bucket's bins (BINS consecutive bins per thread): exclusive base[s] and the
// inclusive prefix max M(s) of (s - base[s]) over occupied bins.
template <int BLOCK = kPlaceBlock>
__device__ __forceinline__ void bucket_scan(const uint32_t* cnt, uint32_t* base, int32_t* M, uint64_t* sh64,
                                            int64_t* shm, uint32_t* last_max) {
  constexpr int BINS = kBucket / BLOCK;
  const int tid = threadIdx.x;
  const int s0 = tid * BINS;
  uint64_t local = 0;
#pragma unroll
  for (int i = 0; i < BINS; i++) local += cnt[s0 + i];
  const uint64_t pre = block_exclusive_scan<uint64_t, OpAdd, BLOCK>(local, sh64, OpAdd(), nullptr);
  int64_t run = -(1ll << 40);
  uint64_t acc = pre;
  int64_t vals[BINS];
#pragma unroll
  for (int i = 0; i < BINS; i++) {
    base[s0 + i] = (uint32_t)acc;
    vals[i] = cnt[s0 + i] ? (int64_t)(s0 + i) - (int64_t)acc : -(1ll << 40);
    acc += cnt[s0 + i];
    run = max(run, vals[i]);
  }
  // exclusive max-scan of per-thread maxima
  int64_t all_max;
  int64_t m = block_exclusive_scan<int64_t, OpMaxI64, BLOCK>(run, shm, OpMaxI64(), &all_max);
#pragma unroll
  for (int i = 0; i < BINS; i++) {
    m = max(m, vals[i]);
    M[s0 + i] = (int32_t)max(m, (int64_t)INT32_MIN);
  }
  if (last_max) *last_max = (uint32_t)(all_max < 0 ? 0 : all_max);
}

__device__ __forceinline__ bool entry_less(const Entry& a, const Entry& b) {
  return (a.addr & ~kDelBit) < (b.addr & ~kDelBit);
}

__device__ inline void place_bucket_global(const BuildParams& P, uint64_t b, int sort_only, uint32_t* cnt,
                                           uint32_t* base, int32_t* M, int32_t* slot_of, uint64_t* sh64,
                                           int64_t* shm) {
  const uint64_t start = b << kBucketShift;
  const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - start);
  const uint32_t n = P.bcount[b];
  const uint64_t eoff = P.boff[b];
  const int tid = threadIdx.x;
  bucket_histogram(P, b, n, eoff, start, cnt);
  bucket_scan(cnt, base, M, sh64, shm, nullptr);
  // counting sort of the bucket's entries by wanted slot into ent3 (cnt reused as cursor)
  for (int t = tid; t < kBucket; t += kPlaceBlock) slot_of[t] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kPlaceBlock) {
    const Entry en = P.ent2[eoff + i];
    const uint64_t w = fast_mod(en.hash, P.mod) - start;
    if (w >= (uint64_t)kBucket) continue;  // (foreign: reported by bucket_histogram)
    const uint32_t r = atomicAdd((uint32_t*)&slot_of[w], 1u);
    P.ent3[eoff + base[w] + r] = en;
  }
  __threadfence_block();
  __syncthreads();
  // equal wanted slots: order by address (ENTRY_COMPARATOR, SortHelper.java:42); flag equal-hash
  // pairs for the duplicate-key check (IndexHash.java:606-636 replaces in place on equal keys).
  for (int i = 0; i < kBinsPerThread; i++) {
    const int s = tid * kBinsPerThread + i;
    const uint32_t g = cnt[s];
    if (g < 2) continue;
    Entry* grp = P.ent3 + eoff + base[s];
    if (sort_only && g <= kGroupMax) {
      for (uint32_t x = 1; x < g; x++) {
        const Entry v = grp[x];
        uint32_t y = x;
        while (y > 0 && entry_less(v, grp[y - 1])) { grp[y] = grp[y - 1]; y--; }
        grp[y] = v;
      }
    } else if (g <= kGroupMax) {
      for (uint32_t x = 1; x < g; x++) {
        const Entry v = grp[x];
        uint32_t y = x;
        while (y > 0 && entry_less(v, grp[y - 1])) { grp[y] = grp[y - 1]; y--; }
        grp[y] = v;
      }
      for (uint32_t x = 0; x < g; x++) {
        for (uint32_t y = x + 1; y < g; y++) {
          if (grp[x].hash == grp[y].hash && !(grp[x].addr & kDelBit) && !(grp[y].addr & kDelBit)) {
            const unsigned long long slotn = atomicAdd(&P.st->n_pairs, 1ull);
            if (slotn < P.pair_cap) {
              P.pairs[2 * slotn] = grp[x].addr;
              P.pairs[2 * slotn + 1] = grp[y].addr;
            }
          }
        }
      }
    } else {  // pathological group (massive duplicates): shell sort, defer to the exact path
      for (uint32_t gap = g / 2; gap > 0; gap /= 2) {
        for (uint32_t x = gap; x < g; x++) {
          const Entry v = grp[x];
          uint32_t y = x;
          while (y >= gap && entry_less(v, grp[y - gap])) { grp[y] = grp[y - gap]; y -= gap; }
          grp[y] = v;
        }
      }
      atomicOr(&P.st->dup_overflow, 1u);
    }
  }
  __threadfence_block();
  __syncthreads();
  if (sort_only || P.st->full) return;
  const int64_t x = P.carry[b];
  for (int t = tid; t < kBucket; t += kPlaceBlock) slot_of[t] = -1;
  __syncthreads();
  // slot of the j-th entry in (wanted, address) order: j + max(carry, M(s))
  for (int i = 0; i < kBinsPerThread; i++) {
    const int s = tid * kBinsPerThread + i;
    const uint32_t g = cnt[s];
    if (!g) continue;
    const int64_t shift = max(x, (int64_t)M[s]);
    for (uint32_t r = 0; r < g; r++) {
      const int64_t j = (int64_t)base[s] + r;
      const int64_t p = j + shift;
      if (p < bsize) {
        slot_of[p] = (int32_t)j;
      } else {
        const Entry en = P.ent3[eoff + j];
        put_slot(P, wrap_slot(start + (uint64_t)p, P.cap), en.hash, en.addr & ~kDelBit);
      }
    }
  }
  __syncthreads();
  // every slot of [x, bsize) is this bucket's: an own entry or empty (zero)
  for (int64_t t = x + tid; t < bsize; t += kPlaceBlock) {
    const int32_t j = slot_of[t];
    if (j >= 0) {
      const Entry en = P.ent3[eoff + j];
      write_slot(P, start + (uint64_t)t, en.hash, en.addr & ~kDelBit);
    } else {
      write_slot(P, start + (uint64_t)t, 0, 0);
    }
  }
}

}  // namespace sk
