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

// a fresh status block: no error, no exit yet, n_records given
__device__ inline void status_reset(Status* st, uint64_t n_records) {
  Status z;
  memset(&z, 0, sizeof(z));
  z.err = ~0ull;
  z.exit = -1;
  z.n_records = n_records;
  *st = z;
}

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

// Uniform framing wrote the rank's entries straight into the 256 coarse-digit regions of ent3
// (partition pass 1 inside k_frame_uniform): the send buffer is those regions back to back in digit
// order, which is destination-rank order.  out = [dest offsets (world + 1) | 64 words][digit starts
// (257)], the layout of k_dest_counts + k_digit_starts.
__global__ __launch_bounds__(256) void k_region_counts(BuildParams P, int world, uint32_t nd, uint64_t* out) {
  __shared__ uint64_t start[257];
  __shared__ uint64_t wsum[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t v = min((uint64_t)P.p1_fill[t], P.p1_region);
  uint64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0;
  for (int q = 0; q < w; q++) before += wsum[q];
  start[t] = before + incl - v;
  if (t == 255) start[256] = before + incl;
  __syncthreads();
  out[64 + t] = start[t];
  if (t == 0) out[64 + 256] = start[256];
  for (int r = t; r <= world; r += 256) {
    const uint32_t d = (uint32_t)(((uint64_t)nd * r) / world);
    out[r] = start[min(d, 256u)];
  }
}

// one workgroup per digit region: its entries to their place in the send buffer (16-byte copies),
// none past send_cap
__global__ __launch_bounds__(1024) void k_region_compact(BuildParams P, Entry* send, uint64_t send_cap) {
  __shared__ uint64_t wsum[16];
  if (build_aborted(P)) return;
  const uint32_t d = blockIdx.x;
  const int t = threadIdx.x;
  uint64_t v = t < (int)d ? min((uint64_t)P.p1_fill[t], P.p1_region) : 0;  // the regions before d
  v = wave_sum_u64(v);
  if ((t & 63) == 0) wsum[t >> 6] = v;
  __syncthreads();
  uint64_t o = 0;
  for (int q = 0; q < 16; q++) o += wsum[q];
  const uint64_t n = min((uint64_t)P.p1_fill[d], P.p1_region);
  const Entry* src = P.ent3 + (uint64_t)d * P.p1_region;
  for (uint64_t i = t; i < n && o + i < send_cap; i += blockDim.x) send[o + i] = src[i];
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

// ---- the device-resident exchange rows (no host round trip between the collectives) ----

// The rank's verification row: the frame's scalars, its entries per destination rank and per
// coarse digit, from the bin's offsets (off = [dest offsets | 64 words][digit starts (257)]).
__global__ __launch_bounds__(256) void k_shard_row(ShardScalars sc, const uint64_t* off, int world, int have,
                                                   int64_t* row) {
  const int t = threadIdx.x;
  if (t < kShardScalars) row[t] = sc.v[t];
  if (t < world) row[kShardScalars + t] = have ? (int64_t)(off[t + 1] - off[t]) : 0;
  row[kShardScalars + world + t] = have ? (int64_t)(off[65 + t] - off[64 + t]) : 0;
}

// The row after a speculative framing attempt (sparkey_shard_frame_bin_async): the scalars from the
// device status, retry = the attempt did not hold (the conditions sparkey_shard_frame retries on,
// or more entries than the send buffer holds); the counts only when the entries are usable.
__global__ __launch_bounds__(256) void k_shard_row_async(ShardScalars sc, const Status* st, int path, uint32_t slab_cap,
                                                         uint64_t max_records, uint64_t send_cap, int64_t data_end,
                                                         const uint64_t* off, int world, int64_t* row) {
  const int t = threadIdx.x;
  const unsigned long long e = st->err;
  const unsigned long long n = st->n_records, nd = st->n_deletes;  // (nd: the row's scalar 4)
  const bool spec = slab_framing(path);
  const bool retry = (spec && st->max_wave_count > slab_cap) || st->overflow || n > max_records ||
                     st->spec_fail != 0 || (path != 1 && e != ~0ull) || n > send_cap;
  const int rc = e != ~0ull ? -(int)(e & 0xff) : 0;
  const bool have = !retry && !rc && n > 0;  // (the bin skips DELETE records)
  if (t == 0) {
    row[0] = sc.v[0];
    row[1] = sc.v[1];
    row[2] = rc ? (int64_t)st->exit : min((int64_t)st->exit, data_end);
    row[3] = (int64_t)n;
    row[4] = (int64_t)nd;
    row[5] = rc;
    row[6] = rc ? (int64_t)(e >> 8) : 0;
    row[7] = retry ? 1 : 0;
  }
  if (t < world) row[kShardScalars + t] = have ? (int64_t)(off[t + 1] - off[t]) : 0;
  row[kShardScalars + world + t] = have ? (int64_t)(off[65 + t] - off[64 + t]) : 0;
}

// k_part2's run table straight from the gathered rows: for each of the rank's nk coarse digits from
// d0, one (begin, end) run per source rank in the exchange buffer (source r's block holds its
// entries for digits d0.. in digit order), then the digits' output starts (nk + 1).
// dig = &rows[0][first digit column]; source r's count of digit d is dig[r * stride + d].
// One thread per digit (nk <= 256); per source rank one block scan over the digits.
__global__ __launch_bounds__(256) void k_p2_table(const int64_t* dig, int stride, int G, uint32_t d0, uint32_t nk,
                                                  uint64_t* tab, Status* st, uint64_t n_records) {
  __shared__ uint64_t wsum[4];
  const uint32_t k = threadIdx.x;
  if (k == 0) status_reset(st, n_records);
  const int lane = k & 63, w = k >> 6;
  uint64_t* segs = tab;
  uint64_t* outs = tab + 2ull * nk * G;
  // exclusive scan over the digits of v (every thread calls it), total returned
  auto scan = [&](uint64_t v, uint64_t& excl) -> uint64_t {
    uint64_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint64_t before = 0, tot = 0;
    for (int q = 0; q < 4; q++) {
      if (q < w) before += wsum[q];
      tot += wsum[q];
    }
    excl = before + incl - v;
    return tot;
  };
  uint64_t tot_k = 0, blk = 0;  // digit k over all sources; the sources before r over all digits
  for (int r = 0; r < G; r++) {
    const uint64_t c = k < nk ? (uint64_t)dig[(int64_t)r * stride + d0 + k] : 0;
    uint64_t pre;
    const uint64_t m = scan(c, pre);
    if (k < nk) {
      segs[2 * ((uint64_t)k * G + r)] = blk + pre;
      segs[2 * ((uint64_t)k * G + r) + 1] = blk + pre + c;
    }
    blk += m;
    tot_k += c;
  }
  uint64_t o;
  const uint64_t all = scan(tot_k, o);
  if (k < nk) outs[k] = o;
  if (k == 0) outs[nk] = all;
}

// One rank (world 1): k_part2's runs are the framing's digit regions of ent3 where they lie (region d
// at d * rc, fill[d] entries), no send buffer in between.
__global__ __launch_bounds__(256) void k_p2_table_regions(const uint32_t* fill, uint64_t rc, uint32_t d0, uint32_t nk,
                                                          uint64_t* tab, Status* st, uint64_t n_records) {
  __shared__ uint64_t wsum[4];
  const uint32_t k = threadIdx.x;
  if (k == 0) status_reset(st, n_records);
  const int lane = k & 63, w = k >> 6;
  const uint64_t c = k < nk ? min((uint64_t)fill[d0 + k], rc) : 0;
  uint64_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, tot = 0;
  for (int q = 0; q < 4; q++) {
    if (q < w) before += wsum[q];
    tot += wsum[q];
  }
  uint64_t* outs = tab + 2ull * nk;
  if (k < nk) {
    tab[2 * k] = (uint64_t)(d0 + k) * rc;
    tab[2 * k + 1] = (uint64_t)(d0 + k) * rc + c;
    outs[k] = before + incl - c;
  }
  if (k == 0) outs[nk] = tot;
}

// The .spi header (rank 0) from every rank's finish row (fin: world rows, stride int64 apart =
// {4 flags, first slot hash, address, last slot hash, address, non-empty, max displacement,
// collisions, total displacement}): the sums, plus the comparisons calculateMaxDisplacement makes
// across range boundaries (IndexHash.java:195-245) and its wrap quirk (IndexHash.java:239-241).
__global__ void k_shard_header(const int64_t* fin, int stride, int world, IndexHeaderBytes tmpl, int64_t n_total,
                               uint8_t* out) {
  if (threadIdx.x != 0) return;
  long long mx = 0;
  unsigned long long col = 0, tot = 0;
  bool have_prev = false, prev_occ = false;
  uint64_t prev_hash = 0;
  int last = -1;
  for (int r = 0; r < world; r++) {
    const int64_t* f = fin + (int64_t)r * stride + kShardFlags;
    mx = max(mx, (long long)f[5]);
    col += (unsigned long long)f[6];
    tot += (unsigned long long)f[7];
    if (!f[4]) continue;
    if (have_prev && prev_occ && prev_hash == (uint64_t)f[0]) col++;
    have_prev = true;
    prev_hash = (uint64_t)f[2];
    prev_occ = f[3] != 0;
    last = r;
  }
  if (last >= 0) {
    const int64_t* f0 = fin + kShardFlags;
    const int64_t* fl = fin + (int64_t)last * stride + kShardFlags;
    if (f0[1] != 0 && fl[3] != 0 && f0[0] == fl[2]) col++;
  }
  for (int i = 0; i < kIndexHeaderBytes; i++) out[i] = tmpl.b[i];
  put_le64(out + 52, 0);
  put_le64(out + 60, (uint64_t)n_total);
  put_le64(out + 84, (uint64_t)mx);
  put_le64(out + 96, col);
  put_le64(out + 104, tot);
}

// flags = {spilled slots, equal-hash pairs, non-canonical, aborted, up to inline_cap spilled slots
// as {slot, hash, address, 0}}
__global__ __launch_bounds__(256) void k_shard_flags(BuildParams P, int64_t* flags, int inline_cap) {
  const Status* st = P.st;
  const unsigned long long ns = st->n_spill;
  const int t = threadIdx.x;
  if (t == 0) {
    flags[0] = (int64_t)ns;
    flags[1] = (int64_t)st->n_pairs;
    flags[2] = (st->dup_overflow || st->n_pairs > P.pair_cap) ? 1 : 0;
    flags[3] = build_aborted(P) ? 1 : 0;
  }
  const uint64_t n = min(min(ns, (unsigned long long)P.spill_cap), (unsigned long long)inline_cap);
  for (uint64_t i = t; i < (uint64_t)inline_cap; i += blockDim.x) {
    SpillEntry e{0, 0, 0, 0};
    if (i < n) e = P.spill[i];
    int64_t* q = flags + kShardFlags + 4 * i;
    q[0] = (int64_t)e.slot;
    q[1] = (int64_t)e.hash;
    q[2] = (int64_t)e.addr;
    q[3] = 0;
  }
}

// every rank's inline spilled slots (rows = world x stride flags rows) that fall in this rank's range;
// a rank that spilled more than inline_cap is left to the host's variable-size exchange
__global__ __launch_bounds__(64) void k_apply_spill_rows(BuildParams P, const int64_t* rows, int stride,
                                                         int inline_cap) {
  const int64_t* row = rows + (int64_t)blockIdx.x * stride;
  const int64_t n = row[0];
  if (n <= 0 || n > inline_cap) return;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t* q = row + kShardFlags + 4 * i;
    const uint64_t slot = (uint64_t)q[0];
    if (slot >= P.slot_lo && slot < P.slot_hi) write_slot(P, slot, (uint64_t)q[1], (uint64_t)q[2]);
  }
}

// out = {the rank's 4 flags, first slot hash, address, last slot hash, address, non-empty, max
// displacement, collisions, total displacement} of the rank's range (after k_stats)
__global__ void k_shard_summary_row(BuildParams P, const int64_t* flags, int64_t* out) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < kShardFlags; i++) out[i] = flags[i];
  out += kShardFlags;
  uint64_t h0 = 0, a0 = 0, h1 = 0, a1 = 0;
  const bool ne = P.slot_hi > P.slot_lo;
  if (ne) {
    read_slot(P, P.slot_lo, h0, a0);
    read_slot(P, P.slot_hi - 1, h1, a1);
  }
  out[0] = (int64_t)h0;
  out[1] = (int64_t)a0;
  out[2] = (int64_t)h1;
  out[3] = (int64_t)a1;
  out[4] = ne ? 1 : 0;
  out[5] = ne ? P.st->max_disp : 0;
  out[6] = ne ? P.st->collisions : 0;
  out[7] = ne ? P.st->total_disp : 0;
}

__global__ void k_status_reset(Status* st, uint64_t n_records, uint32_t* fill, int nfill) {
  if (threadIdx.x == 0) status_reset(st, n_records);
  for (int i = threadIdx.x; i < nfill; i += blockDim.x) fill[i] = 0;
}

void launch_shard_row(hipStream_t s, const ShardScalars& sc, const uint64_t* off, int world, int have, int64_t* row) {
  hipLaunchKernelGGL(k_shard_row, dim3(1), dim3(256), 0, s, sc, off, world, have, row);
}

void launch_shard_row_async(hipStream_t s, const ShardScalars& sc, const Status* st, int path, uint32_t slab_cap,
                            uint64_t max_records, uint64_t send_cap, int64_t data_end, const uint64_t* off, int world,
                            int64_t* row) {
  hipLaunchKernelGGL(k_shard_row_async, dim3(1), dim3(256), 0, s, sc, st, path, slab_cap, max_records, send_cap,
                     data_end, off, world, row);
}

void launch_p2_table(hipStream_t s, const int64_t* dig, int stride, int G, uint32_t d0, uint32_t nk, uint64_t* tab,
                     Status* st, uint64_t n_records) {
  hipLaunchKernelGGL(k_p2_table, dim3(1), dim3(256), 0, s, dig, stride, G, d0, nk, tab, st, n_records);
}

void launch_p2_table_regions(hipStream_t s, const uint32_t* fill, uint64_t rc, uint32_t d0, uint32_t nk, uint64_t* tab,
                             Status* st, uint64_t n_records) {
  hipLaunchKernelGGL(k_p2_table_regions, dim3(1), dim3(256), 0, s, fill, rc, d0, nk, tab, st, n_records);
}

void launch_shard_header(hipStream_t s, const int64_t* fin, int stride, int world, const IndexHeaderBytes& tmpl,
                         int64_t n_total, uint8_t* out) {
  hipLaunchKernelGGL(k_shard_header, dim3(1), dim3(64), 0, s, fin, stride, world, tmpl, n_total, out);
}

void launch_shard_flags(const BuildParams& P, hipStream_t s, int64_t* flags, int inline_cap) {
  hipLaunchKernelGGL(k_shard_flags, dim3(1), dim3(256), 0, s, P, flags, inline_cap);
}

void launch_apply_spill_rows(const BuildParams& P, hipStream_t s, const int64_t* rows, int world, int stride,
                             int inline_cap) {
  hipLaunchKernelGGL(k_apply_spill_rows, dim3((unsigned)world), dim3(64), 0, s, P, rows, stride, inline_cap);
}

void launch_shard_summary_row(const BuildParams& P, hipStream_t s, const int64_t* flags, int64_t* out) {
  hipLaunchKernelGGL(k_shard_summary_row, dim3(1), dim3(64), 0, s, P, flags, out);
}

void launch_status_reset(hipStream_t s, Status* st, uint64_t n_records, uint32_t* fill, int nfill) {
  hipLaunchKernelGGL(k_status_reset, dim3(1), dim3(256), 0, s, st, n_records, fill, nfill);
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

void launch_region_send(const BuildParams& P, hipStream_t s, int world, uint32_t nd, Entry* send, uint64_t* d_out,
                        uint64_t send_cap) {
  if (send) hipLaunchKernelGGL(k_region_compact, dim3(256), dim3(1024), 0, s, P, send, send_cap);  // (null: counts only)
  hipLaunchKernelGGL(k_region_counts, dim3(1), dim3(256), 0, s, P, world, nd, d_out);
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
