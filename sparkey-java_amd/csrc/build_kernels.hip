// build_kernels.hip -- gfx950 kernels of the Sparkey .spi build (IndexHash.createNew on MI355X).
//
// Pipeline (one HIP stream, all device-resident; see DESIGN.md for layouts and rooflines):
//   framing   k_speculate  per 4 KiB chunk, one wave: every plausible record start in the first
//                          maxRecLen bytes is walked to the chunk end; if all surviving chains exit
//                          at one offset the chunk's exit is known without its entry.
//             k_walk       one thread per run of unresolved chunks walks the true chain serially.
//             k_count      per resolved chunk: entry = predecessor's exit, head walk to the merge
//                          point + tail count -> records per chunk.
//             scan         record offsets per chunk.
//   hash      k_emit       per chunk, one wave: walk from the verified entry (LDS-staged bytes),
//                          MurmurHash3 every key, write (hash, address) in log order, count buckets.
//   place     scan + k_scatter (bucket = wantedSlot >> 10), k_summary (per bucket max-plus carry
//             function), scan over buckets (+ wrap-around fixed point), k_place: per bucket
//             counting sort by wantedSlot, ties by address (the canonical Robin-Hood order, see
//             DESIGN.md "canonical placement"), slot = j + max(carry, prefix-max(w_i - i)), write
//             every slot of the bucket (entries or zeros).
//   stats     k_stats + k_stats_final: calculateMaxDisplacement (IndexHash.java:195-245) with its
//             quirks, patch the 112-byte header.
//   exact     k_sequential: single-lane restatement of put/delete (IndexHash.java:454-665) for logs
//             the canonical layout does not cover (DELETEs, duplicate keys, full tables).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"
#include "device_common.hpp"

namespace sk {

// ------------------------------------------------------------------------------------------------
// small device utilities
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void set_error(Status* st, int64_t pos, int code) {
  atomicMin(&st->err, ((unsigned long long)pos << 8) | (unsigned long long)(-code));
}

__device__ __forceinline__ int64_t chunk_start(uint64_t k) { return k == 0 ? kLogHeaderSize : (int64_t)(k << kChunkShift); }
__device__ __forceinline__ int64_t chunk_end(uint64_t k, int64_t data_end) {
  const int64_t e = (int64_t)((k + 1) << kChunkShift);
  return e < data_end ? e : data_end;
}

// Stage log bytes [wb, wb + n) into LDS (bytes past log_len read as 0; they are never decoded
// because every decode is bounded by log_len).  wb is 16-byte aligned; `log` must be too.
__device__ __forceinline__ void stage_window(uint8_t* win, const uint8_t* log, int64_t wb, int n, int64_t log_len,
                                             int lane, int nthreads) {
  const int nvec = n >> 4;
  for (int v = lane; v < nvec; v += nthreads) {
    const int64_t a = wb + ((int64_t)v << 4);
    uint4 val;
    if (a + 16 <= log_len) {
      val = *reinterpret_cast<const uint4*>(log + a);
    } else {
      uint8_t tmp[16];
#pragma unroll
      for (int i = 0; i < 16; i++) tmp[i] = (a + i < log_len) ? log[a + i] : 0;
      val = *reinterpret_cast<uint4*>(tmp);
    }
    *reinterpret_cast<uint4*>(win + (v << 4)) = val;
  }
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ long long wave_max_i64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ================================================================================================
// Framing.  A record's start depends on the previous record (SparkeyLogIterator.java:86-138), so
// the log is cut into 4 KiB chunks and each chunk's entry (first record start >= chunk start) is
// recovered speculatively, then verified exactly (k_emit checks entry->exit for every chunk).
// ================================================================================================
__global__ __launch_bounds__(64) void k_speculate(BuildParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kChunk + 32];
  __shared__ unsigned long long bitmap[kChunk / 64];
  const uint64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t wb = (int64_t)(k << kChunkShift);
  const int64_t s = chunk_start(k);
  const int64_t e = chunk_end(k, P.data_end);
  // A record longer than the chunk can start before it and end after it: the chunk may hold no
  // record start at all, so its exit cannot be known without its entry.
  if (k > 0 && s + P.max_rec_len - 1 >= e) {
    if (lane == 0) P.conv[k] = 0;
    return;
  }
  stage_window(win, P.log, wb, kChunk + 32, (int64_t)P.log_len, lane, 64);
  __syncthreads();
  const int64_t avail = min((int64_t)P.log_len, wb + kChunk + 32);
  auto at = [&](int64_t a) -> uint32_t { return win[a - wb]; };
  const int64_t cand_end = (k == 0) ? s + 1 : min(e, s + P.max_rec_len);

  // Pass A: walk every candidate; record survivors (chains that never hit an implausible header).
  unsigned long long surv_mask = 0;
  unsigned long long nsurv = 0, min_exit = ~0ull, min_start = ~0ull;
  long long max_exit = -1;
  int ci = 0;
  for (int64_t c = s + lane; c < cand_end; c += 64, ci++) {
    int64_t p = c;
    bool ok = true;
    while (p < e) {
      const RecHdr h = decode_header(at, p, avail);
      if (!header_plausible(h, p, P.max_key_len, P.max_value_len, (int64_t)P.log_len)) { ok = false; break; }
      p = record_end(h, p);
    }
    if (ok) {
      surv_mask |= 1ull << ci;
      nsurv++;
      min_exit = min(min_exit, (unsigned long long)p);
      max_exit = max(max_exit, (long long)p);
      min_start = min(min_start, (unsigned long long)c);
    }
  }
  nsurv = wave_sum_u64(nsurv);
  min_exit = wave_min_u64(min_exit);
  max_exit = wave_max_i64(max_exit);
  min_start = wave_min_u64(min_start);
  const bool converged = nsurv > 0 && (long long)min_exit == max_exit;
  if (!converged) {
    if (lane == 0) P.conv[k] = 0;
    return;
  }
  // Pass B: mark the chain of the first survivor; every other survivor walks until it meets that
  // chain (or exits).  q = last merge point: from q on every survivor -- hence the true chain -- is
  // the same, so the records in [q, e) are counted here once.
  bitmap[lane] = 0;
  __syncthreads();
  if (lane == 0) {
    int64_t p = (int64_t)min_start;
    while (p < e) {
      const int64_t r = p - wb;
      bitmap[r >> 6] |= 1ull << (r & 63);
      p = record_end(decode_header(at, p, avail), p);
    }
  }
  __syncthreads();
  long long qmax = (long long)min_start;
  ci = 0;
  for (int64_t c = s + lane; c < cand_end; c += 64, ci++) {
    if (!((surv_mask >> ci) & 1)) continue;
    int64_t p = c;
    while (p < e) {
      const int64_t r = p - wb;
      if ((bitmap[r >> 6] >> (r & 63)) & 1) break;
      p = record_end(decode_header(at, p, avail), p);
    }
    qmax = max(qmax, (long long)p);
  }
  qmax = wave_max_i64(qmax);
  // tail = marked positions >= q (and < e); bitmap word `lane` covers offsets [64*lane, 64*lane+64)
  unsigned long long word = bitmap[lane];
  const int64_t qr = qmax - wb;
  const int64_t lo = (int64_t)lane * 64;
  if (qr >= lo + 64) word = 0;
  else if (qr > lo) word &= ~0ull << (qr - lo);
  const unsigned long long tail = wave_sum_u64((unsigned long long)__popcll(word));
  if (lane == 0) {
    P.conv[k] = 1;
    P.exitp[k] = (int64_t)min_exit;
    P.qpos[k] = qmax;
    P.tail[k] = (uint32_t)tail;
  }
}

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
  int64_t p = (k == 0) ? kLogHeaderSize : P.exitp[k - 1];
  uint64_t m = k;
  P.G[m] = p;
  uint32_t c = 0;
  int64_t em = chunk_end(m, P.data_end);
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  for (;;) {
    while (p >= em) {
      P.cnt[m] = c;
      c = 0;
      m++;
      if (m >= nc) return;
      P.G[m] = p;
      if (!serial && P.conv[m]) return;
      em = chunk_end(m, P.data_end);
    }
    const RecHdr h = decode_header(at, p, (int64_t)P.log_len);
    if (!header_valid(h, p, P.max_key_len, (int64_t)P.log_len)) {
      set_error(P.st, p, h.rc ? h.rc : kErrCorruptLog);
      for (; m < nc; m++) P.cnt[m] = 0;
      return;
    }
    c++;
    p = record_end(h, p);
  }
}

// Per resolved chunk: entry from the predecessor (exit if it was resolved, else the walker's G),
// head walk to the merge point q, count = head + tail.
__global__ void k_count(BuildParams P) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P.nchunks || !P.conv[k]) return;
  const int64_t g = (k == 0) ? kLogHeaderSize : (P.conv[k - 1] ? P.exitp[k - 1] : P.G[k]);
  P.G[k] = g;
  const int64_t q = P.qpos[k];
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  int64_t p = g;
  uint32_t h = 0;
  while (p < q) {
    const RecHdr r = decode_header(at, p, (int64_t)P.log_len);
    if (!header_valid(r, p, P.max_key_len, (int64_t)P.log_len)) {
      set_error(P.st, p, r.rc ? r.rc : kErrCorruptLog);
      P.cnt[k] = 0;
      return;
    }
    h++;
    p = record_end(r, p);
  }
  if (p != q) {
    atomicOr(&P.st->spec_fail, 1u);
    P.cnt[k] = 0;
    return;
  }
  P.cnt[k] = h + P.tail[k];
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
  const int64_t wb = (int64_t)(k << kChunkShift);
  const int64_t e = chunk_end(k, P.data_end);
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
      if (!header_valid(h, p, P.max_key_len, (int64_t)P.log_len)) {
        set_error(P.st, p, h.rc ? h.rc : kErrCorruptLog);
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
  if (base + (uint64_t)n > P.max_records) {
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
    const uint64_t w = fast_mod(hash, P.mod);
    atomicAdd(&P.bcount[w >> kBucketShift], 1u);
  }
}

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
static void scan_exclusive(const In* in, T* out, uint64_t n, T* d_total, Op op, T* scratch, hipStream_t s) {
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

// ================================================================================================
// Placement.
// ================================================================================================
__global__ void k_scatter(BuildParams P) {
  const uint64_t N = P.st->n_records;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N && i < P.max_records; i += stride) {
    const Entry en = P.ent[i];
    const uint64_t b = fast_mod(en.hash, P.mod) >> kBucketShift;
    const uint64_t pos = P.boff[b] + atomicAdd(&P.bcursor[b], 1u);
    P.ent2[pos] = en;
  }
}

// Per bucket: LDS histogram of local wanted slots and its exclusive scan; returns n.
__device__ __forceinline__ void bucket_histogram(const BuildParams& P, uint64_t b, uint32_t n, uint64_t eoff,
                                                 uint64_t start, uint32_t* cnt) {
  for (int t = threadIdx.x; t < kBucket; t += kPlaceBlock) cnt[t] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += kPlaceBlock) {
    const uint64_t w = fast_mod(P.ent2[eoff + i].hash, P.mod) - start;
    atomicAdd(&cnt[w], 1u);
  }
  __syncthreads();
}

// For the bucket's bins (kBinsPerThread consecutive bins per thread): exclusive base[s] and the
// inclusive prefix max M(s) of (s - base[s]) over occupied bins.
__device__ __forceinline__ void bucket_scan(const uint32_t* cnt, uint32_t* base, int32_t* M, uint64_t* sh64,
                                            int64_t* shm, uint32_t* last_max) {
  const int tid = threadIdx.x;
  const int s0 = tid * kBinsPerThread;
  uint64_t local = 0;
#pragma unroll
  for (int i = 0; i < kBinsPerThread; i++) local += cnt[s0 + i];
  const uint64_t pre = block_exclusive_scan<uint64_t, OpAdd, kPlaceBlock>(local, sh64, OpAdd(), nullptr);
  int64_t run = -(1ll << 40);
  uint64_t acc = pre;
  int64_t vals[kBinsPerThread];
#pragma unroll
  for (int i = 0; i < kBinsPerThread; i++) {
    base[s0 + i] = (uint32_t)acc;
    vals[i] = cnt[s0 + i] ? (int64_t)(s0 + i) - (int64_t)acc : -(1ll << 40);
    acc += cnt[s0 + i];
    run = max(run, vals[i]);
  }
  // exclusive max-scan of per-thread maxima
  shm[tid] = run;
  __syncthreads();
  for (int o = 1; o < kPlaceBlock; o <<= 1) {
    int64_t t = tid >= o ? shm[tid - o] : -(1ll << 40);
    __syncthreads();
    if (tid >= o) shm[tid] = max(shm[tid], t);
    __syncthreads();
  }
  int64_t m = tid ? shm[tid - 1] : -(1ll << 40);
  const int64_t all_max = shm[kPlaceBlock - 1];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kBinsPerThread; i++) {
    m = max(m, vals[i]);
    M[s0 + i] = (int32_t)max(m, (int64_t)INT32_MIN);
  }
  if (last_max) *last_max = (uint32_t)(all_max < 0 ? 0 : all_max);
}

// Carry function of a bucket (DESIGN.md "canonical placement"): entries overflowing past the
// bucket end as a function of the carry-in x is out(x) = max(c, x + a), c = max(0, n + M_last - B),
// a = n - B.
__global__ __launch_bounds__(kPlaceBlock) void k_summary(BuildParams P) {
  __shared__ uint32_t cnt[kBucket];
  __shared__ uint32_t base[kBucket];
  __shared__ int32_t M[kBucket];
  __shared__ uint64_t sh64[kPlaceBlock];
  __shared__ int64_t shm[kPlaceBlock];
  const uint64_t b = blockIdx.x;
  const uint64_t start = b << kBucketShift;
  const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - start);
  const uint32_t n = P.bcount[b];
  const uint64_t eoff = P.boff[b];
  bucket_histogram(P, b, n, eoff, start, cnt);
  uint32_t mlast = 0;
  bucket_scan(cnt, base, M, sh64, shm, &mlast);
  if (threadIdx.x == 0) {
    MaxPlus f;
    f.a = (int64_t)n - bsize;
    f.c = n ? max((int64_t)0, (int64_t)n + (int64_t)mlast - bsize) : 0;
    P.bfun[b] = f;
  }
}

// carry[b] = (F_{b-1} o ... o F_0)(x0), x0 = fixed point of the whole ring = C_total when N < cap.
__global__ void k_carry(BuildParams P) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const MaxPlus tot = *P.bfun_total;
  if (tot.a >= 0) {  // N >= capacity: no empty slot, the canonical layout does not apply
    if (b == 0) atomicOr(&P.st->full, 1u);
    return;
  }
  if (b >= P.nbuckets) return;
  const MaxPlus pre = P.bpre[b];
  P.carry[b] = max(pre.c, tot.c + pre.a);
}

__device__ __forceinline__ void write_slot(const BuildParams& P, uint64_t slot, uint64_t hash, uint64_t addr) {
  uint8_t* p = P.out + kIndexHeaderSize + slot * (uint64_t)P.slot_size;
  if (P.slot_size == 16) {
    *reinterpret_cast<uint4*>(p) = make_uint4((uint32_t)hash, (uint32_t)(hash >> 32), (uint32_t)addr, (uint32_t)(addr >> 32));
  } else if (P.slot_size == 8) {
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)hash, (uint32_t)addr);
  } else if (P.hash_size == 8) {  // 8 + 4
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = (uint32_t)hash; q[1] = (uint32_t)(hash >> 32); q[2] = (uint32_t)addr;
  } else {  // 4 + 8
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = (uint32_t)hash; q[1] = (uint32_t)addr; q[2] = (uint32_t)(addr >> 32);
  }
}

__device__ __forceinline__ uint64_t wrap_slot(uint64_t s, uint64_t cap) {
  while (s >= cap) s -= cap;
  return s;
}

__device__ __forceinline__ bool entry_less(const Entry& a, const Entry& b) {
  return (a.addr & ~kDelBit) < (b.addr & ~kDelBit);
}

__global__ __launch_bounds__(kPlaceBlock) void k_place(BuildParams P) {
  __shared__ uint32_t cnt[kBucket];
  __shared__ uint32_t base[kBucket];
  __shared__ int32_t M[kBucket];
  __shared__ int32_t slot_of[kBucket];
  __shared__ uint64_t sh64[kPlaceBlock];
  __shared__ int64_t shm[kPlaceBlock];
  const uint64_t b = blockIdx.x;
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
    if (g <= kGroupMax) {
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
  if (P.st->full) return;
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
        write_slot(P, wrap_slot(start + (uint64_t)p, P.cap), en.hash, en.addr & ~kDelBit);
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

// Equal-hash pairs: do they share the key?  (the reference compares key bytes in the log,
// IndexHash.java:619-629)
__global__ void k_verify_pairs(BuildParams P) {
  const unsigned long long np = min(P.st->n_pairs, (unsigned long long)P.pair_cap);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
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

// ================================================================================================
// Stats: calculateMaxDisplacement (IndexHash.java:195-245).  hashCollisions compares a slot's hash
// with the previous OCCUPIED slot's hash even when the current slot is empty (its hash reads 0).
// ================================================================================================
__device__ __forceinline__ void read_slot(const BuildParams& P, uint64_t slot, uint64_t& hash, uint64_t& addr) {
  const uint8_t* p = P.out + kIndexHeaderSize + slot * (uint64_t)P.slot_size;
  if (P.slot_size == 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    hash = (uint64_t)v.x | ((uint64_t)v.y << 32);
    addr = (uint64_t)v.z | ((uint64_t)v.w << 32);
  } else if (P.slot_size == 8) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    hash = v.x;
    addr = v.y;
  } else {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    if (P.hash_size == 8) { hash = (uint64_t)q[0] | ((uint64_t)q[1] << 32); addr = q[2]; }
    else { hash = q[0]; addr = (uint64_t)q[1] | ((uint64_t)q[2] << 32); }
  }
}

__global__ __launch_bounds__(kStatBlock) void k_stats(BuildParams P) {
  __shared__ uint64_t sh_hash[kStatBlock];
  __shared__ uint32_t sh_occ[kStatBlock];
  __shared__ unsigned long long red_sum[kStatBlock / 64];
  __shared__ unsigned long long red_col[kStatBlock / 64];
  __shared__ long long red_max[kStatBlock / 64];
  const int tid = threadIdx.x;
  const uint64_t blk0 = (uint64_t)blockIdx.x * kStatSlotsPerBlock;
  uint64_t prev_hash = 0;
  uint32_t prev_occ = 0;
  if (blk0 > 0 && blk0 < P.cap) {
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
    if (slot < P.cap) read_slot(P, slot, h, a);
    sh_hash[tid] = h;
    sh_occ[tid] = a != 0;
    __syncthreads();
    const uint64_t ph = tid ? sh_hash[tid - 1] : prev_hash;
    const uint32_t po = tid ? sh_occ[tid - 1] : prev_occ;
    if (slot < P.cap) {
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

__device__ __forceinline__ void put_le64(uint8_t* p, uint64_t v) {
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

__global__ __launch_bounds__(256) void k_stats_final(BuildParams P, uint32_t nparts, int sequential) {
  __shared__ unsigned long long s_sum[256], s_col[256];
  __shared__ long long s_max[256];
  const int tid = threadIdx.x;
  unsigned long long sum = 0, col = 0;
  long long mx = 0;
  for (uint32_t i = tid; i < nparts; i += 256) {
    const StatPart sp = P.parts[i];
    sum += sp.sum_disp;
    col += sp.collisions;
    mx = max(mx, sp.max_disp);
  }
  s_sum[tid] = sum; s_col[tid] = col; s_max[tid] = mx;
  __syncthreads();
  if (tid == 0) {
    sum = s_sum[0]; col = s_col[0]; mx = s_max[0];
    for (int i = 1; i < 256; i++) { sum += s_sum[i]; col += s_col[i]; mx = max(mx, s_max[i]); }
    // wrap quirk (IndexHash.java:239-241): slot 0 and slot cap-1 both occupied with equal hashes
    uint64_t h0, a0, h1, a1;
    read_slot(P, 0, h0, a0);
    read_slot(P, P.cap - 1, h1, a1);
    if (a0 != 0 && a1 != 0 && h0 == h1) col++;
    Status* st = P.st;
    long long entries, garbage;
    if (sequential) { entries = st->num_entries; garbage = st->garbage; }
    else { entries = (long long)st->n_records; garbage = 0; }
    st->max_disp = mx;
    st->collisions = (long long)col;
    st->total_disp = (long long)sum;
    st->num_entries = entries;
    st->garbage = garbage;
    uint8_t* hdr = P.out;
    put_le64(hdr + 52, (uint64_t)garbage);
    put_le64(hdr + 60, (uint64_t)entries);
    put_le64(hdr + 84, (uint64_t)mx);
    put_le64(hdr + 96, col);
    put_le64(hdr + 104, sum);
  }
}

// ================================================================================================
// Exact sequential restatement (IndexHash.put/delete, IndexHash.java:454-665) on the device table,
// one lane.  IN_MEMORY order: entries in log order (ent).  SORTING order: (wantedSlot, address)
// per bucket (ent3) -- SortHelper's comparator.  Keys are compared in the log in HBM.
// ================================================================================================
struct SeqCtx {
  const BuildParams* P;
  uint8_t* table;
  int64_t num_entries;
  int64_t garbage;
};

__device__ uint64_t seq_rd(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
__device__ void seq_wr(uint8_t* p, int n, uint64_t v) {
  for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i));
}
__device__ __forceinline__ uint64_t seq_hash(const SeqCtx& c, int64_t slot) {
  return seq_rd(c.table + slot * c.P->slot_size, c.P->hash_size);
}
__device__ __forceinline__ uint64_t seq_addr(const SeqCtx& c, int64_t slot) {
  return seq_rd(c.table + slot * c.P->slot_size + c.P->hash_size, c.P->addr_size);
}
__device__ __forceinline__ void seq_write(SeqCtx& c, int64_t slot, uint64_t h, uint64_t a) {
  uint8_t* p = c.table + slot * c.P->slot_size;
  seq_wr(p, c.P->hash_size, h);
  seq_wr(p + c.P->hash_size, c.P->addr_size, a);
}
__device__ __forceinline__ int64_t seq_disp(const SeqCtx& c, int64_t slot, uint64_t hash) {
  int64_t d = slot - (int64_t)fast_mod(hash, c.P->mod);
  return d >= 0 ? d : d + (int64_t)c.P->cap;
}
__device__ __forceinline__ int32_t vlq_size_i32(int64_t v) {
  if (v < (1 << 7)) return 1;
  if (v < (1 << 14)) return 2;
  if (v < (1 << 21)) return 3;
  if (v < (1 << 28)) return 4;
  return 5;
}
__device__ __forceinline__ int64_t garbage_of(int32_t k2, int32_t v2) {  // IndexHeader.java:221-228
  return (int32_t)((uint32_t)k2 + (uint32_t)v2 + (uint32_t)vlq_size_i32((int64_t)k2 + 1) + (uint32_t)vlq_size_i32(v2));
}

// returns 0, or an error code
__device__ int seq_put(SeqCtx& c, uint64_t hash, uint64_t address) {
  const BuildParams& P = *c.P;
  const int64_t cap = (int64_t)P.cap;
  if (c.num_entries >= cap) return kErrNoFreeSlots;
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  int64_t slot = (int64_t)fast_mod(hash, P.mod);
  int64_t displacement = 0, tries = cap;
  int64_t position = (int64_t)(address >> P.ebb);
  bool might = true;
  int32_t own_klen = -1;
  int64_t own_key = 0;
  while (--tries >= 0) {
    const uint64_t hash2 = seq_hash(c, slot);
    const uint64_t address2 = seq_addr(c, slot);
    if (address2 == 0) {
      seq_write(c, slot, hash, address);
      c.num_entries++;
      return 0;
    }
    const int64_t position2 = (int64_t)(address2 >> P.ebb);
    if (might && hash == hash2) {
      if (own_klen == -1) {
        const RecHdr h = decode_header(at, position, (int64_t)P.log_len);
        if (h.rc) return h.rc;
        if (!h.put) return kErrCorruptData;
        own_klen = h.klen;
        own_key = position + h.hlen;
      }
      const RecHdr h2 = decode_header(at, position2, (int64_t)P.log_len);
      if (h2.rc) return h2.rc;
      if (!h2.put) return kErrCorruptData;  // "Invalid data - reference to delete entry"
      if (own_klen == h2.klen) {
        bool eq = true;
        const int64_t k2 = position2 + h2.hlen;
        for (int32_t j = 0; j < own_klen && eq; j++) eq = P.log[own_key + j] == P.log[k2 + j];
        if (eq) {
          seq_write(c, slot, hash, address);
          c.garbage += garbage_of(h2.klen, h2.vlen);
          return 0;
        }
      }
    }
    const int64_t other = seq_disp(c, slot, hash2);
    if (displacement > other || (displacement == other && (int64_t)address < (int64_t)address2)) {
      seq_write(c, slot, hash, address);
      position = position2;
      address = address2;
      displacement = other;
      hash = hash2;
      might = false;
    }
    displacement++;
    slot++;
    if (slot >= cap) slot = 0;
  }
  return kErrNoFreeSlots;
}

__device__ int seq_delete(SeqCtx& c, uint64_t hash, uint64_t address) {
  const BuildParams& P = *c.P;
  const int64_t cap = (int64_t)P.cap;
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  int64_t slot = (int64_t)fast_mod(hash, P.mod);
  int64_t displacement = 0;
  const int64_t position = (int64_t)(address >> P.ebb);
  int32_t own_klen = -1;
  int64_t own_key = 0;
  for (int64_t guard = 0; guard <= cap; guard++) {
    const uint64_t hash2 = seq_hash(c, slot);
    const uint64_t address2 = seq_addr(c, slot);
    if (address2 == 0) return 0;
    const int64_t position2 = (int64_t)(address2 >> P.ebb);
    if (hash == hash2) {
      if (own_klen == -1) {
        const RecHdr h = decode_header(at, position, (int64_t)P.log_len);
        if (h.rc) return h.rc;
        if (h.put) return kErrCorruptData;
        own_klen = h.klen;
        own_key = position + h.hlen;
      }
      const RecHdr h2 = decode_header(at, position2, (int64_t)P.log_len);
      if (h2.rc) return h2.rc;
      if (!h2.put) return kErrCorruptData;
      if (own_klen == h2.klen) {
        bool eq = true;
        const int64_t k2 = position2 + h2.hlen;
        for (int32_t j = 0; j < own_klen && eq; j++) eq = P.log[own_key + j] == P.log[k2 + j];
        if (eq) {
          for (int64_t g2 = 0; g2 < cap; g2++) {  // backward shift, IndexHash.java:503-524
            int64_t next = slot + 1;
            if (next == cap) next = 0;
            const uint64_t hash3 = seq_hash(c, next);
            const uint64_t pos3 = seq_addr(c, next);
            if (pos3 == 0) break;
            if ((int64_t)fast_mod(hash3, P.mod) == next) break;
            seq_write(c, slot, hash3, pos3);
            slot = next;
          }
          seq_write(c, slot, 0, 0);
          c.garbage += garbage_of(h2.klen, h2.vlen);
          c.num_entries--;
          return 0;
        }
      }
    }
    const int64_t other = seq_disp(c, slot, hash2);
    if (displacement > other) return 0;
    displacement++;
    slot++;
    if (slot == cap) slot = 0;
  }
  return 0;
}

__global__ void k_sequential(BuildParams P, int sorted_order) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  SeqCtx c;
  c.P = &P;
  c.table = P.out + kIndexHeaderSize;
  c.num_entries = 0;
  c.garbage = 0;
  const uint64_t N = min((uint64_t)P.st->n_records, P.max_records);
  const Entry* src = sorted_order ? P.ent3 : P.ent;
  for (uint64_t i = 0; i < N; i++) {
    const Entry en = src[i];
    const uint64_t addr = en.addr & ~kDelBit;
    const int rc = (en.addr & kDelBit) ? seq_delete(c, en.hash, addr) : seq_put(c, en.hash, addr);
    if (rc) {
      set_error(P.st, (int64_t)(addr >> P.ebb), rc);
      break;
    }
  }
  P.st->num_entries = c.num_entries;
  P.st->garbage = c.garbage;
}

// ================================================================================================
// host-side launchers (called by the plan in sparkey_gpu.cpp)
// ================================================================================================
static inline unsigned grid_for(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

void launch_framing(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.nchunks == 0) return;
  hipLaunchKernelGGL(k_speculate, dim3((unsigned)P.nchunks), dim3(64), 0, s, P);
  tm->mark("speculate", s);
  hipLaunchKernelGGL(k_walk, dim3(grid_for(P.nchunks, 256)), dim3(256), 0, s, P, 0);
  tm->mark("walk", s);
  hipLaunchKernelGGL(k_count, dim3(grid_for(P.nchunks, 256)), dim3(256), 0, s, P);
  tm->mark("count", s);
}

void launch_framing_serial(const BuildParams& P, hipStream_t s) {
  if (P.nchunks == 0) return;
  hipLaunchKernelGGL(k_walk, dim3(1), dim3(64), 0, s, P, 1);
}

void launch_emit(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.nchunks == 0) return;
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.cnt, P.off, P.nchunks, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
  tm->mark("scan_chunks", s);
  hipLaunchKernelGGL(k_emit, dim3((unsigned)P.nchunks), dim3(64), 0, s, P);
  tm->mark("emit", s);
}

void launch_place(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.bcount, P.boff, P.nbuckets, P.boff + P.nbuckets, OpAdd(),
                                            P.scan_scratch_u64, s);
  tm->mark("scan_buckets", s);
  hipLaunchKernelGGL(k_scatter, dim3(2048), dim3(256), 0, s, P);
  tm->mark("scatter", s);
  hipLaunchKernelGGL(k_summary, dim3((unsigned)P.nbuckets), dim3(kPlaceBlock), 0, s, P);
  tm->mark("summary", s);
  scan_exclusive<MaxPlus, MaxPlus, OpMaxPlus>(P.bfun, P.bpre, P.nbuckets, P.bfun_total, OpMaxPlus(),
                                              P.scan_scratch_mp, s);
  hipLaunchKernelGGL(k_carry, dim3(grid_for(P.nbuckets, 256)), dim3(256), 0, s, P);
  tm->mark("carry", s);
  hipLaunchKernelGGL(k_place, dim3((unsigned)P.nbuckets), dim3(kPlaceBlock), 0, s, P);
  tm->mark("place", s);
  hipLaunchKernelGGL(k_verify_pairs, dim3(grid_for(P.pair_cap, 256)), dim3(256), 0, s, P);
  tm->mark("verify", s);
}

void launch_stats(const BuildParams& P, hipStream_t s, int sequential, StageTimer* tm) {
  const uint64_t nparts = (P.cap + kStatSlotsPerBlock - 1) / kStatSlotsPerBlock;
  hipLaunchKernelGGL(k_stats, dim3((unsigned)nparts), dim3(kStatBlock), 0, s, P);
  hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(256), 0, s, P, (uint32_t)nparts, sequential);
  tm->mark("stats", s);
}

void launch_sequential(const BuildParams& P, hipStream_t s, int sorted_order) {
  hipLaunchKernelGGL(k_sequential, dim3(1), dim3(64), 0, s, P, sorted_order);
}

}  // namespace sk
