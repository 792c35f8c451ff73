// build_kernels.hip -- gfx950 kernels of the Sparkey .spi build (IndexHash.createNew on MI355X).
//
// The fast path lives in fused_kernels.hip (k_frame, radix partition, k_place_reg).  This file
// holds the exact fallbacks and the shared stages:
//   k_walk(serial)  one thread walks the whole record chain (SparkeyLogIterator.java:86-138) when
//                   speculative framing disagreed with the verified chain (inconsistent headers).
//   k_emit          per chunk, one wave: hash the records of the serially framed chunk.
//   k_summary/k_carry  per bucket max-plus carry function, scan, wrap-around fixed point
//                   (DESIGN.md "canonical placement").
//   k_place         global-memory placement for buckets too big for LDS; (wantedSlot, address)
//                   order for the SORTING restatement.
//   k_verify_pairs  equal-hash PUT pairs: same key?  (IndexHash.java:606-636)
//   k_stats         calculateMaxDisplacement (IndexHash.java:195-245), header patch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"
#include "place_common.hpp"

namespace sk {

// One thread per run of unresolved chunks (or, with `serial`, one thread for the whole log):
// walks the true record chain with the reference iterator's own validity rules.
__global__ void k_walk(BuildParams P, int serial) {
  const uint64_t k = serial ? 0 : (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (serial && (blockIdx.x != 0 || threadIdx.x != 0)) return;
  const uint64_t nc = P.nchunks;
  if (k >= nc) return;
  if (!serial) {
    if (P.conv[k]) return;
    if (k > 0 && !P.conv[k - 1]) return;
  }
  int64_t p = (k == 0) ? P.fr_entry : P.exitp[k - 1];
  uint64_t m = k;
  P.G[m] = p;
  uint32_t c = 0;
  int64_t em = chunk_end(P.ch_k0 + m, P.data_end);
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  for (;;) {
    while (p >= em) {
      P.cnt[m] = c;
      c = 0;
      m++;
      if (m >= nc) {
        if (serial) P.st->exit = p;
        return;
      }
      P.G[m] = p;
      if (!serial && P.conv[m]) return;
      em = chunk_end(P.ch_k0 + m, P.data_end);
    }
    const RecHdr h = decode_header(at, p, (int64_t)P.log_len);
    if (h.rc == kEndOfLog) {  // EOF inside the first VLQ: the iteration ends here, no error
      P.cnt[m] = c;
      for (m++; m < nc; m++) {
        P.G[m] = p;
        P.cnt[m] = 0;
      }
      if (serial) P.st->exit = P.data_end;
      return;
    }
    if (!header_valid(h, p, P.max_key_len, (int64_t)P.log_len)) {
      set_error(P.st, p, header_error(h));
      for (; m < nc; m++) P.cnt[m] = 0;
      return;
    }
    c++;
    p = record_end(h, p);
  }
}

// ================================================================================================
// Hash: one wave per chunk.  Lane 0 walks the verified chain through LDS-staged bytes, then the
// wave hashes one record per lane (HashType.hash, IndexHash.java:276-286) and writes the
// (hash, address) entries in log order; address = position << entryBlockBits (entryIndex is 0 for
// NONE).  Also: bucket histogram for placement, DELETE count.
// ================================================================================================
__global__ __launch_bounds__(64) void k_emit(BuildParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kChunk + kEmitExtra];
  __shared__ uint16_t recs[kChunk / 2 + 2];
  __shared__ int32_t s_n;
  const uint64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t wb = (int64_t)((P.ch_k0 + k) << kChunkShift);
  const int64_t e = chunk_end(P.ch_k0 + k, P.data_end);
  const int wn = kChunk + P.emit_extra;
  stage_window(win, P.log, wb, wn, (int64_t)P.log_len, lane, 64);
  __syncthreads();
  const int64_t wend = min((int64_t)P.log_len, wb + wn);
  auto at = [&](int64_t a) -> uint32_t { return a < wend ? (uint32_t)win[a - wb] : (uint32_t)P.log[a]; };
  if (lane == 0) {
    int64_t p = P.G[k];
    int32_t n = 0;
    bool bad = false;
    while (p < e) {
      const RecHdr h = decode_header(at, p, (int64_t)P.log_len);
      if (h.rc == kEndOfLog) break;  // the iteration ends (k_walk ended the chain at the same byte)
      if (!header_valid(h, p, P.max_key_len, (int64_t)P.log_len)) {
        set_error(P.st, p, header_error(h));
        bad = true;
        break;
      }
      if (n > kChunk / 2) { bad = true; break; }
      recs[n++] = (uint16_t)(p - wb);
      p = record_end(h, p);
    }
    if (!bad && ((uint32_t)n != P.cnt[k] || (k + 1 < P.nchunks && p != P.G[k + 1]))) {
      atomicOr(&P.st->spec_fail, 1u);
      bad = true;
    }
    s_n = bad ? -1 : n;
  }
  __syncthreads();
  const int32_t n = s_n;
  if (n <= 0) return;
  const uint64_t base = P.off[k];
  if (base + (uint64_t)n > P.ent_cap) {
    if (lane == 0) atomicOr(&P.st->overflow, 1u);
    return;
  }
  for (int i = lane; i < n; i += 64) {
    const int64_t p = wb + recs[i];
    const RecHdr h = decode_header(at, p, (int64_t)P.log_len);
    const int64_t kp = p + h.hlen;
    uint64_t hash;
    if (kp + h.klen <= wend) hash = key_hash(P.hash_size, win + (kp - wb), h.klen, (uint32_t)P.seed);
    else hash = key_hash(P.hash_size, P.log + kp, h.klen, (uint32_t)P.seed);
    uint64_t addr = (uint64_t)p << P.ebb;
    if (!h.put) {
      addr |= kDelBit;
      atomicAdd(&P.st->n_deletes, 1ull);
    }
    Entry en;
    en.hash = hash;
    en.addr = addr;
    P.ent[base + i] = en;
  }
}

// ================================================================================================
// Placement.
// ================================================================================================
// Carry function of a bucket (DESIGN.md "canonical placement"): entries overflowing past the
// bucket end as a function of the carry-in x is out(x) = max(c, x + a), c = max(0, n + M_last - B),
// a = n - B.
__global__ __launch_bounds__(kPlaceBlock) void k_summary(BuildParams P) {
  // Only M_last = max(0, max over occupied s of s - base[s]) is needed, not base[] and M[] per slot:
  // 32-bit counts in LDS (4 KiB, was 12 KiB with the two per-slot arrays), each thread's 4 slots
  // scanned in registers, the wave prefix by DPP and one barrier for the 4 waves' totals.
  static_assert(kBucket == 4 * kPlaceBlock, "four slots per thread");
  constexpr int NW = kPlaceBlock / 64;
  constexpr int32_t kNone = INT32_MIN;
  __shared__ __attribute__((aligned(16))) uint32_t cnt[kBucket];
  __shared__ uint32_t wsum[NW];
  __shared__ int32_t wmx[NW];
  if (build_aborted(P)) return;
  if (P.p2_sorted && !P.st->need_summary) return;  // k_part2s left every carry function
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t b = P.b_lo + blockIdx.x;
  const uint64_t start = b << kBucketShift;
  const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - start);
  const uint32_t n = P.bcount[b];
  // (the framing's bucket regions: bucket b at b * kPlaceLdsMax, no offsets written)
  const uint64_t eoff = P.p1_bucket ? (b - P.b_lo) * (uint64_t)kPlaceLdsMax : P.boff[b];
  reinterpret_cast<uint4*>(cnt)[tid] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  bool bad = false;  // (kGuardForeign)
  for (uint32_t i = tid; i < n; i += kPlaceBlock) {
    const uint64_t h = (P.compact & kCompactOut) ? load_craw(reinterpret_cast<const CEntry*>(P.ent2) + eoff + i).hash : P.ent2[eoff + i].hash;
    const uint64_t w = fast_mod(h, P.mod) - start;
    if (w < (uint64_t)kBucket) atomicAdd(&cnt[w], 1u);
    else bad = true;
  }
  report_foreign(P, bad);
  __syncthreads();
  const uint4 c = reinterpret_cast<const uint4*>(cnt)[tid];
  const uint32_t tot = c.x + c.y + c.z + c.w;
  const uint32_t incl = wave_incl_sum_u32(tot);
  // max over this thread's occupied slots of s - (wave-local base of s)
  int32_t v = kNone;
  {
    const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
    uint32_t run = incl - tot;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (cc[i]) v = max(v, (int32_t)(4 * tid + i) - (int32_t)run);
      run += cc[i];
    }
  }
  const int32_t mv = wave_max_i32(v);
  if (lane == 63) wsum[wv] = incl;
  if (lane == 0) wmx[wv] = mv;
  __syncthreads();
  if (tid == 0) {
    int64_t m = -1;  // (M_last counts only when positive)
    uint32_t off = 0;
#pragma unroll
    for (int u = 0; u < NW; u++) {
      if (wmx[u] != kNone) m = max(m, (int64_t)wmx[u] - (int64_t)off);
      off += wsum[u];
    }
    const int64_t mlast = m < 0 ? 0 : m;
    MaxPlus f;
    f.a = (int64_t)n - bsize;
    f.c = n ? max((int64_t)0, (int64_t)n + mlast - bsize) : 0;
    P.bfun[b] = f;
  }
}

// carry[b] = (F_{b-1} o ... o F_0)(x0), x0 = fixed point of the whole ring = C_total when N < cap.
// Sharded: the prefix starts at b_lo and x0 is the rank's carry-in: given, or composed here from every
// rank's carry function (the ring's fixed point (N < capacity), then the ranks before this one).
__global__ void k_carry(BuildParams P) {
  if (P.carry_funs && blockIdx.x == 0 && threadIdx.x == 0) {  // (the placement's counters, before k_place)
    P.st->n_pairs = 0;
    P.st->n_spill = 0;
    P.st->dup_overflow = 0;
  }
  if (build_aborted(P)) return;
  const uint64_t b = P.b_lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const MaxPlus tot = *P.bfun_total;
  int64_t x0 = P.carry_in;
  if (P.carry_funs) {
    const int64_t* f = P.carry_funs;
    // A rank whose function could not leave its device sent an all-ones row (HostColl): c = -1, which
    // no carry function has (c >= 0).  This rank skips its placement (build_aborted) and the failed
    // rank's finish row fails every rank.
    for (int r = 0; r < P.carry_world; r++)
      if (f[2 * r] < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&P.st->p2_overflow, 1u);
        return;
      }
    int64_t c = f[0];  // the composed function's constant: the fixed point when N < capacity
    for (int r = 1; r < P.carry_world; r++) c = max(f[2 * r], c + f[2 * r + 1]);
    x0 = c;
    for (int r = 0; r < P.carry_rank; r++) x0 = max(f[2 * r], x0 + f[2 * r + 1]);
  }
  if (!P.sharded) {
    if (tot.a >= 0) {  // N >= capacity: no empty slot, the canonical layout does not apply
      if (b == 0) atomicOr(&P.st->full, 1u);
      return;
    }
    x0 = tot.c;
  }
  if (b >= P.b_hi) return;
  const MaxPlus pre = P.bpre[b];
  P.carry[b] = max(pre.c, x0 + pre.a);
}

// Global-memory placement of every bucket (buckets too big for k_place_reg), or, with
// sort_only, the (wantedSlot, address) order of every bucket into ent3 for the SORTING restatement.
__global__ __launch_bounds__(kPlaceBlock) void k_place(BuildParams P, int sort_only, int only_big) {
  __shared__ uint32_t cnt[kBucket];
  __shared__ uint32_t base[kBucket];
  __shared__ int32_t M[kBucket];
  __shared__ int32_t slot_of[kBucket];
  __shared__ uint64_t sh64[kPlaceBlock / 64 + 1];
  __shared__ int64_t shm[kPlaceBlock / 64 + 1];
  if (build_aborted(P)) return;
  const uint64_t b = P.b_lo + blockIdx.x;
  if (only_big && P.bcount[b] <= kPlaceLdsMax) return;
  place_bucket_global(P, b, sort_only, cnt, base, M, slot_of, sh64, shm);
}

// Equal-hash pairs: do they share the key?  (the reference compares key bytes in the log,
// IndexHash.java:619-629)
__device__ void verify_pair(const BuildParams& P, uint64_t i) {
  const int64_t p1 = (int64_t)(P.pairs[2 * i] >> P.ebb);
  const int64_t p2 = (int64_t)(P.pairs[2 * i + 1] >> P.ebb);
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  const RecHdr h1 = decode_header(at, p1, (int64_t)P.log_len);
  const RecHdr h2 = decode_header(at, p2, (int64_t)P.log_len);
  if (h1.rc || h2.rc || h1.klen != h2.klen) return;
  const uint8_t* k1 = P.log + p1 + h1.hlen;
  const uint8_t* k2 = P.log + p2 + h2.hlen;
  for (int32_t j = 0; j < h1.klen; j++)
    if (k1[j] != k2[j]) return;
  atomicOr(&P.st->dup, 1u);
}

__global__ void k_verify_pairs(BuildParams P) {
  if (build_aborted(P)) return;
  const unsigned long long np = min(P.st->n_pairs, (unsigned long long)P.pair_cap);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += (uint64_t)gridDim.x * blockDim.x)
    verify_pair(P, i);
}

// ================================================================================================
// Stats: calculateMaxDisplacement (IndexHash.java:195-245).  hashCollisions compares a slot's hash
// with the previous OCCUPIED slot's hash even when the current slot is empty (its hash reads 0).
// ================================================================================================
__global__ __launch_bounds__(kStatBlock) void k_stats(BuildParams P) {
  __shared__ uint64_t sh_hash[kStatBlock];
  __shared__ uint32_t sh_occ[kStatBlock];
  __shared__ unsigned long long red_sum[kStatBlock / 64];
  __shared__ unsigned long long red_col[kStatBlock / 64];
  __shared__ long long red_max[kStatBlock / 64];
  if (build_aborted(P)) return;
  if (P.stats_if_pending && !P.st->stats_pending) return;  // (the folded stats covered every slot)
  const int tid = threadIdx.x;
  const uint64_t blk0 = P.slot_lo + (uint64_t)blockIdx.x * kStatSlotsPerBlock;
  uint64_t prev_hash = 0;
  uint32_t prev_occ = 0;
  if (blk0 == P.slot_lo && P.sharded) {  // the slot before the range lives on another rank
    prev_hash = P.prev_hash;
    prev_occ = (uint32_t)P.prev_occ;
  } else if (blk0 > 0 && blk0 < P.slot_hi) {
    uint64_t h, a;
    read_slot(P, blk0 - 1, h, a);
    prev_hash = h;
    prev_occ = a != 0;
  }
  unsigned long long sum_d = 0, col = 0;
  long long max_d = 0;
  for (int it = 0; it < kStatSlotsPerBlock / kStatBlock; it++) {
    const uint64_t slot = blk0 + (uint64_t)it * kStatBlock + tid;
    uint64_t h = 0, a = 0;
    if (slot < P.slot_hi) read_slot(P, slot, h, a);
    sh_hash[tid] = h;
    sh_occ[tid] = a != 0;
    __syncthreads();
    const uint64_t ph = tid ? sh_hash[tid - 1] : prev_hash;
    const uint32_t po = tid ? sh_occ[tid - 1] : prev_occ;
    if (slot < P.slot_hi) {
      if (po && ph == h) col++;
      if (a != 0) {
        int64_t d = (int64_t)slot - (int64_t)fast_mod(h, P.mod);
        if (d < 0) d += (int64_t)P.cap;
        sum_d += (unsigned long long)d;
        max_d = max(max_d, (long long)d);
      }
    }
    prev_hash = sh_hash[kStatBlock - 1];
    prev_occ = sh_occ[kStatBlock - 1];
    __syncthreads();
  }
  sum_d = wave_sum_u64(sum_d);
  col = wave_sum_u64(col);
  max_d = wave_max_i64(max_d);
  if ((tid & 63) == 0) {
    red_sum[tid >> 6] = sum_d;
    red_col[tid >> 6] = col;
    red_max[tid >> 6] = max_d;
  }
  __syncthreads();
  if (tid == 0) {
    StatPart sp{0, 0, 0};
    for (int w = 0; w < kStatBlock / 64; w++) {
      sp.sum_disp += red_sum[w];
      sp.collisions += red_col[w];
      sp.max_disp = max(sp.max_disp, red_max[w]);
    }
    P.parts[blockIdx.x] = sp;
  }
}

__global__ __launch_bounds__(1024) void k_stats_final(BuildParams P, uint32_t nparts, int sequential) {
  __shared__ unsigned long long s_sum[16], s_col[16];
  __shared__ long long s_max[16];
  if (P.stats_if_pending && !P.st->stats_pending) return;
  const StatPart* parts = P.parts;
  const int tid = threadIdx.x;
  unsigned long long sum = 0, col = 0;
  long long mx = 0;
  for (uint32_t i = tid; i < nparts; i += 1024) {
    const StatPart sp = parts[i];
    sum += sp.sum_disp;
    col += sp.collisions;
    mx = max(mx, sp.max_disp);
  }
  sum = wave_sum_u64(sum);
  col = wave_sum_u64(col);
  mx = wave_max_i64(mx);
  if ((tid & 63) == 0) { s_sum[tid >> 6] = sum; s_col[tid >> 6] = col; s_max[tid >> 6] = mx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 16; w++) { s_sum[0] += s_sum[w]; s_col[0] += s_col[w]; s_max[0] = max(s_max[0], s_max[w]); }
    finish_stats(P, s_sum[0], s_col[0], s_max[0], sequential);
  }
}

// The folded stats (k_place_reg fold_stats): every block left the sums over the slot range it wrote
// and where that range starts; the ranges tile the ring, so the only pairs left are each range's
// first slot with the slot before it.  One thread per bucket; the last block to finish (ticket)
// writes the header.
constexpr int kStatFoldBlock = 256;
// The status block into the host's pinned, mapped copy by one block's threads (k_status_out's work,
// done by k_stats_folded's last block: one launch and its gap fewer a build).
__device__ __forceinline__ void copy_status_out(const BuildParams& P) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(P.st);
  uint32_t* dst = reinterpret_cast<uint32_t*>(P.status_host);
  constexpr int kWords = (int)(sizeof(Status) / sizeof(uint32_t));
  __threadfence();
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
}

__global__ __launch_bounds__(kStatFoldBlock) void k_stats_folded(BuildParams P) {
  __shared__ unsigned long long s_sum[kStatFoldBlock / 64], s_col[kStatFoldBlock / 64], s_max[kStatFoldBlock / 64];
  __shared__ bool last;
  if (build_aborted(P)) {  // (the host redoes the build: block 0 hands it the status)
    if (blockIdx.x == 0 && P.status_host) copy_status_out(P);
    return;
  }
  Status* st = P.st;
  const int tid = threadIdx.x;
  if (P.fused_carry) {  // k_verify_pairs' work (no launch of its own)
    const unsigned long long np = min(st->n_pairs, (unsigned long long)P.pair_cap);
    for (uint64_t i = (uint64_t)blockIdx.x * kStatFoldBlock + tid; i < np; i += (uint64_t)gridDim.x * kStatFoldBlock)
      verify_pair(P, i);
  }
  if (st->big_buckets || st->full) {  // some slots were placed outside k_place_reg: k_stats runs (and the
    if (tid == 0) st->stats_pending = 1u;  // host reads the status again after it)
    __syncthreads();
    if (blockIdx.x == 0 && P.status_host) copy_status_out(P);
    return;
  }
  unsigned long long sum = 0, col = 0, mx = 0;
  const uint64_t b = (uint64_t)blockIdx.x * kStatFoldBlock + tid;
  if (b < P.nbuckets) {
    const StatPart sp = P.parts[b];
    sum = sp.sum_disp;
    col = sp.collisions;
    mx = (unsigned long long)sp.max_disp;
    const uint64_t gs = P.bstat_start[b];
    if (gs != ~0ull && gs != 0) {
      uint64_t hp, ap, hc, ac;
      read_slot(P, gs - 1, hp, ap);
      read_slot(P, gs, hc, ac);
      col += ap != 0 && hp == hc;
    }
  }
  sum = wave_sum_u64(sum);
  col = wave_sum_u64(col);
  mx = (unsigned long long)wave_max_i64((long long)mx);
  if ((tid & 63) == 0) { s_sum[tid >> 6] = sum; s_col[tid >> 6] = col; s_max[tid >> 6] = mx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kStatFoldBlock / 64; w++) { s_sum[0] += s_sum[w]; s_col[0] += s_col[w]; s_max[0] = max(s_max[0], s_max[w]); }
    atomicAdd(&st->acc_sum, s_sum[0]);
    atomicAdd(&st->acc_col, s_col[0]);
    atomicMax(&st->acc_max, s_max[0]);
    __threadfence();
    last = atomicAdd(&st->stats_ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && tid == 0) {
    __threadfence();
    const unsigned long long tsum = atomicAdd(&st->acc_sum, 0ull), tcol = atomicAdd(&st->acc_col, 0ull);
    const unsigned long long tmax = atomicMax(&st->acc_max, 0ull);
    finish_stats(P, tsum, tcol, (long long)tmax, 0);
  }
  if (last && P.status_host) {
    __syncthreads();
    copy_status_out(P);
  }
}

// The folded stats of a sharded rank (after its spilled-in slots were written).  Every entry's
// displacement was summed by the rank that placed it (max and sum are global); the adjacent pairs
// (s - 1, s) with s in (slot_lo, slot_hi) are: inside one block's written range (k_place_reg counted
// those whose s this rank owns), at the start gs of a block of this rank other than b_lo (read here),
// or in the spilled-in run [slot_lo, slot_lo + carry[b_lo]] (read here by block 0).  The pair at
// slot_lo and the wrap quirk are the host's (sharded.py), as with k_stats.
__global__ __launch_bounds__(kStatFoldBlock) void k_stats_folded_shard(BuildParams P) {
  __shared__ unsigned long long s_sum[kStatFoldBlock / 64], s_col[kStatFoldBlock / 64], s_max[kStatFoldBlock / 64];
  __shared__ bool last;
  if (build_aborted(P)) return;
  Status* st = P.st;
  const int tid = threadIdx.x;
  if (st->big_buckets || st->full) {  // some slots were placed outside k_place_reg: k_stats runs
    if (tid == 0) st->stats_pending = 1u;
    return;
  }
  unsigned long long sum = 0, col = 0, mx = 0;
  const uint64_t b = P.b_lo + (uint64_t)blockIdx.x * kStatFoldBlock + tid;
  if (b < P.b_hi) {
    const StatPart sp = P.parts[b];
    sum = sp.sum_disp;
    col = sp.collisions;
    mx = (unsigned long long)sp.max_disp;
    const uint64_t gs = (b << kBucketShift) + (uint64_t)P.carry[b];  // (unwrapped)
    if (b > P.b_lo && P.bstat_start[b] != ~0ull && gs < P.slot_hi) {
      uint64_t hp, ap, hc, ac;
      read_slot(P, gs - 1, hp, ap);
      read_slot(P, gs, hc, ac);
      col += ap != 0 && hp == hc;
    }
  }
  if (blockIdx.x == 0 && P.b_hi > P.b_lo) {  // the spilled-in run
    const uint64_t end = min(P.slot_lo + (uint64_t)P.carry[P.b_lo], P.slot_hi - 1);
    for (uint64_t s = P.slot_lo + 1 + tid; s <= end; s += kStatFoldBlock) {
      uint64_t hp, ap, hc, ac;
      read_slot(P, s - 1, hp, ap);
      read_slot(P, s, hc, ac);
      col += ap != 0 && hp == hc;
    }
  }
  sum = wave_sum_u64(sum);
  col = wave_sum_u64(col);
  mx = (unsigned long long)wave_max_i64((long long)mx);
  if ((tid & 63) == 0) { s_sum[tid >> 6] = sum; s_col[tid >> 6] = col; s_max[tid >> 6] = mx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kStatFoldBlock / 64; w++) { s_sum[0] += s_sum[w]; s_col[0] += s_col[w]; s_max[0] = max(s_max[0], s_max[w]); }
    atomicAdd(&st->acc_sum, s_sum[0]);
    atomicAdd(&st->acc_col, s_col[0]);
    atomicMax(&st->acc_max, s_max[0]);
    __threadfence();
    last = atomicAdd(&st->stats_ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && tid == 0) {
    __threadfence();
    const unsigned long long tsum = atomicAdd(&st->acc_sum, 0ull), tcol = atomicAdd(&st->acc_col, 0ull);
    const unsigned long long tmax = atomicMax(&st->acc_max, 0ull);
    finish_stats(P, tsum, tcol, (long long)tmax, 0);
  }
}

// ================================================================================================
// host-side launchers (called by the plan in sparkey_gpu.cpp)
// ================================================================================================
static inline unsigned grid_for(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

void launch_framing_serial(const BuildParams& P, hipStream_t s) {
  if (P.nchunks == 0) return;
  hipLaunchKernelGGL(k_walk, dim3(1), dim3(64), 0, s, P, 1);
}

void launch_emit(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.nchunks == 0) return;
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.cnt, P.off, P.nchunks, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
  hipLaunchKernelGGL(k_emit, dim3((unsigned)P.nchunks), dim3(64), 0, s, P);
  tm->mark("emit", s);
}

void launch_carry(const BuildParams& P, hipStream_t s) {
  if (P.b_hi > P.b_lo) hipLaunchKernelGGL(k_carry, dim3(grid_for(P.b_hi - P.b_lo, 256)), dim3(256), 0, s, P);
}

void launch_summary_carry(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  const uint64_t nb = P.b_hi - P.b_lo;
  if (nb == 0) return;
  // (the two-level pass 2 left every bucket's carry function: k_part2f<.., kSubIn>)
  if (!P.sub_region) hipLaunchKernelGGL(k_summary, dim3((unsigned)nb), dim3(kPlaceBlock), 0, s, P);
  scan_exclusive<MaxPlus, MaxPlus, OpMaxPlus>(P.bfun + P.b_lo, P.bpre + P.b_lo, nb, P.bfun_total, OpMaxPlus(),
                                              P.scan_scratch_mp, s);
  if (!P.sharded) launch_carry(P, s);
  tm->mark("summary", s);
}

void launch_place_global(const BuildParams& P, hipStream_t s, int sort_only, int only_big) {
  if (P.b_hi > P.b_lo)
    hipLaunchKernelGGL(k_place, dim3((unsigned)(P.b_hi - P.b_lo)), dim3(kPlaceBlock), 0, s, P, sort_only, only_big);
}

void launch_verify(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  // (grid-stride over the pairs found: a grid sized to the pair buffer launched 65K idle waves a build)
  hipLaunchKernelGGL(k_verify_pairs, dim3((unsigned)std::min<uint64_t>(grid_for(P.pair_cap, 256), 1024)), dim3(256), 0,
                     s, P);
  tm->mark("verify", s);
}

// The build's first launch: the .spi header (from the host's template), the status block reset
// (err = none) and n words of the digit regions' fill cursors cleared -- one kernel in place of two
// host-to-device copies and a memset per build.
struct BuildInit {
  uint8_t hdr[kIndexHeaderBytes];
};
__global__ __launch_bounds__(256) void k_build_init(uint8_t* out, BuildInit h, Status* st, uint32_t* fill, uint32_t n) {
  const int t = threadIdx.x;
  if (t < kIndexHeaderBytes / 4) {
    const uint32_t w = (uint32_t)h.hdr[4 * t] | ((uint32_t)h.hdr[4 * t + 1] << 8) | ((uint32_t)h.hdr[4 * t + 2] << 16) |
                       ((uint32_t)h.hdr[4 * t + 3] << 24);
    reinterpret_cast<uint32_t*>(out)[t] = w;
  }
  constexpr int kWords = (int)(sizeof(Status) / 4);
  uint32_t* sw = reinterpret_cast<uint32_t*>(st);
  for (int i = t; i < kWords; i += 256) sw[i] = i < 2 ? ~0u : 0u;  // err (the first 8 bytes) = ~0
  for (uint32_t i = t; i < n; i += 256) fill[i] = 0;
}

// The status block into the caller's pinned, device-mapped host copy: one small launch queued behind
// the build (a runtime device-to-host copy costs a blit launch with about 6 us of setup before it).
__global__ __launch_bounds__(64) void k_status_out(const Status* st, Status* host) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(st);
  uint32_t* dst = reinterpret_cast<uint32_t*>(host);
  static_assert(sizeof(Status) % sizeof(uint32_t) == 0, "whole words");
  constexpr int kWords = (int)(sizeof(Status) / sizeof(uint32_t));
  for (int i = threadIdx.x; i < kWords; i += 64) dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
}

void launch_status_out(const Status* st, Status* host, hipStream_t s) {
  hipLaunchKernelGGL(k_status_out, dim3(1), dim3(64), 0, s, st, host);
}

void launch_build_init(uint8_t* out, const uint8_t* hdr, Status* st, uint32_t* fill, uint32_t n, hipStream_t s) {
  BuildInit h;
  for (int i = 0; i < kIndexHeaderBytes; i++) h.hdr[i] = hdr[i];
  hipLaunchKernelGGL(k_build_init, dim3(1), dim3(256), 0, s, out, h, st, fill, n);
}

// Before the exact path frames a log again: the framing's status words back to their initial values
// (err = none, no failed speculation, no overflow, no DELETE counted yet).
__global__ void k_status_reframe(Status* st) {
  if (threadIdx.x == 0) {
    st->err = ~0ull;
    st->spec_fail = 0;
    st->overflow = 0;
    st->max_wave_count = 0;
    st->n_deletes = 0;
  }
}

void launch_status_reframe(Status* st, hipStream_t s) { hipLaunchKernelGGL(k_status_reframe, dim3(1), dim3(64), 0, s, st); }

// The framing's spread DELETE counters into st->n_deletes, cleared for the next framing launch.
__global__ __launch_bounds__(64) void k_sum_deletes(BuildParams P) {
  const int lane = threadIdx.x;
  unsigned long long v = 0;
  for (int i = lane; i < kDelParts; i += 64) {
    v += P.del_parts[i * 16];
    P.del_parts[i * 16] = 0;
  }
  v = wave_sum_u64(v);
  if (lane == 0 && v) atomicAdd(&P.st->n_deletes, v);
}

void launch_sum_deletes(const BuildParams& P, hipStream_t s) {
  if (P.del_parts) hipLaunchKernelGGL(k_sum_deletes, dim3(1), dim3(64), 0, s, P);
}

void launch_stats_folded(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  hipLaunchKernelGGL(k_stats_folded, dim3(grid_for(std::max<uint64_t>(P.nbuckets, 1), kStatFoldBlock)),
                     dim3(kStatFoldBlock), 0, s, P);
  tm->mark("stats", s);
}

void launch_stats_folded_shard(const BuildParams& P, hipStream_t s) {
  const uint64_t nb = P.b_hi - P.b_lo;
  hipLaunchKernelGGL(k_stats_folded_shard, dim3(grid_for(std::max<uint64_t>(nb, 1), kStatFoldBlock)),
                     dim3(kStatFoldBlock), 0, s, P);
}

void launch_stats(const BuildParams& P, hipStream_t s, int sequential, StageTimer* tm) {
  const uint64_t nparts = (P.slot_hi - P.slot_lo + kStatSlotsPerBlock - 1) / kStatSlotsPerBlock;
  if (nparts) hipLaunchKernelGGL(k_stats, dim3((unsigned)nparts), dim3(kStatBlock), 0, s, P);
  hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(1024), 0, s, P, (uint32_t)nparts, sequential);
  tm->mark("stats", s);
}

}  // namespace sk
