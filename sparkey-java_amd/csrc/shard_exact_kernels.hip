// shard_exact_kernels.hip -- the sharded exact path: logs with DELETE records or
// duplicate keys built across ranks without gathering the log.
//
//   k_first_empty  the first slot of the rank's range that the canonical placement of every PUT record
//                  leaves empty (IndexHash.put's probes and delete's backward shifts never cross such a
//                  slot, exact_kernels.hip): the exact ranges start there
//   k_ex_count     records per (exact owner, slab): the owner of a record is the rank whose exact range
//                  holds its wanted slot
//   k_ex_scatter   every framed record (PUT and DELETE) as an exchange record {hash, address, header
//                  VLQs + key bytes}, grouped by owner, log order kept inside each owner's run
//   k_ex_ent       the owner's entries over the received records: address = the record's offset in the
//                  receive buffer (monotone in the log address, so every address comparison of the
//                  replay -- IndexHash.java:647-650, SortHelper's order -- is the reference's)
//   k_ex_extract   the replayed slots of an exact range back to log addresses, in the .spi slot layout
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

constexpr int kExMaxWorld = 256;

__global__ __launch_bounds__(256) void k_first_empty(BuildParams P, unsigned long long* out) {
  const uint64_t slot = P.slot_lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t h, a = 1;
  if (slot < P.slot_hi) read_slot(P, slot, h, a);
  const uint64_t empty = __ballot(a == 0);  // one atomic per wave (slots rise with the lane) ...
  if (empty && (threadIdx.x & 63) == (unsigned)(__ffsll((unsigned long long)empty) - 1) &&
      slot < __hip_atomic_load(out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))  // ... and none behind a found one
    atomicMin(out, (unsigned long long)slot);
}

// the rank owning wanted slot w: the last rank whose exact range starts at or before w, else (w before
// every start: the range that wraps around the ring) the last rank with a start
__device__ __forceinline__ int exact_owner(const int64_t* starts, int world, uint64_t w) {
  int own = -1, last = -1;
  for (int r = 0; r < world; r++) {
    const int64_t e = starts[r];
    if (e < 0) continue;
    last = r;
    if ((uint64_t)e <= w) own = r;
  }
  return own >= 0 ? own : last;
}

constexpr int kExWaves = 4;  // k_ex_count / k_ex_scatter: one wave per slab, four slabs per workgroup

// one wave per slab: cnt[owner * nslabs + slab]
__global__ __launch_bounds__(64 * kExWaves) void k_ex_count(BuildParams P, const int64_t* starts, int world,
                                                            uint32_t* cnt) {
  __shared__ int64_t sE[kExMaxWorld];
  __shared__ uint32_t c[kExWaves][kExMaxWorld];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * kExWaves + wv;
  for (int r = threadIdx.x; r < world; r += blockDim.x) sE[r] = starts[r];
  for (int r = lane; r < world; r += 64) c[wv][r] = 0;
  __syncthreads();
  if (w < P.nslabs) {
    const uint32_t n = P.wcount[w];
    for (uint32_t j = lane; j < n; j += 64) {
      const Entry en = P.ent[w * P.slab_cap + j];
      atomicAdd(&c[wv][exact_owner(sE, world, fast_mod(en.hash, P.mod))], 1u);
    }
  }
  __syncthreads();
  if (w < P.nslabs)
    for (int r = lane; r < world; r += 64) cnt[(uint64_t)r * P.nslabs + w] = c[wv][r];
}

// records per owner from the scanned counts (off: world * nslabs + 1, owner-major)
__global__ void k_ex_totals(const uint64_t* off, uint64_t nslabs, int world, unsigned long long* totals) {
  for (int r = threadIdx.x; r < world; r += blockDim.x)
    totals[r] = off[(uint64_t)(r + 1) * nslabs] - off[(uint64_t)r * nslabs];
}

// little-endian word of the 8 log bytes from p (p + 8 <= the buffer's end + 16), from aligned dwords
__device__ __forceinline__ uint64_t log_word(const uint8_t* log, int64_t p) {
  const int64_t a = p & ~3ll;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(log + a);
  const uint32_t sh = (uint32_t)(p - a) * 8u;
  const uint64_t lo = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
  const uint64_t hi = q[2];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// one wave per slab: each 64-record step ranks its records per owner with ballots (log order kept),
// then every lane writes its exchange record: {hash, address, the record's header VLQs and key}
__global__ __launch_bounds__(64 * kExWaves) void k_ex_scatter(BuildParams P, const int64_t* starts, int world,
                                                              const uint64_t* off, uint8_t* send, uint32_t rs) {
  __shared__ int64_t sE[kExMaxWorld];
  __shared__ uint64_t base_all[kExWaves][kExMaxWorld];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * kExWaves + wv;
  uint64_t* base = base_all[wv];
  for (int r = threadIdx.x; r < world; r += blockDim.x) sE[r] = starts[r];
  if (w < P.nslabs)
    for (int r = lane; r < world; r += 64) base[r] = off[(uint64_t)r * P.nslabs + w];
  __syncthreads();
  if (w >= P.nslabs) return;
  const uint32_t n = P.wcount[w];
  const uint64_t lt = (1ull << lane) - 1;
  const uint32_t body = rs - 16;  // multiple of 8
  for (uint32_t j0 = 0; j0 < n; j0 += 64) {
    const uint32_t j = j0 + lane;
    const bool active = j < n;
    Entry en{0, 0};
    int d = -1;
    if (active) {
      en = P.ent[w * P.slab_cap + j];
      d = exact_owner(sE, world, fast_mod(en.hash, P.mod));
    }
    uint64_t pos = 0;
    uint64_t todo = __ballot(active);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int dd = __shfl(d, leader, 64);
      const uint64_t m = __ballot(active && d == dd);
      const uint64_t b = base[dd];
      if (active && d == dd) pos = b + (uint64_t)__popcll(m & lt);
      __builtin_amdgcn_wave_barrier();
      if (lane == leader) base[dd] = b + (uint64_t)__popcll(m);
      __builtin_amdgcn_wave_barrier();
      todo &= ~m;
    }
    if (!active) continue;
    uint64_t* r = reinterpret_cast<uint64_t*>(send + pos * rs);
    r[0] = en.hash;
    r[1] = en.addr;
    const int64_t p = (int64_t)((en.addr & ~kDelBit) >> P.ebb);
    auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
    const RecHdr h = decode_header(at, p, (int64_t)P.log_len);
    const uint32_t len = h.rc ? 0u : (uint32_t)min<int64_t>((int64_t)(h.hlen + h.klen), (int64_t)body);
    for (uint32_t q = 0; q < body; q += 8) {
      uint64_t v = 0;
      if (q < len) {
        v = p + q + 12 <= (int64_t)P.log_len ? log_word(P.log, p + q) : 0;
        if (p + q + 12 > (int64_t)P.log_len)  // (the buffer's last bytes: one at a time)
          for (uint32_t k = 0; k < 8 && q + k < len; k++) v |= (uint64_t)P.log[p + q + k] << (8 * k);
        if (len - q < 8) v &= (1ull << (8 * (len - q))) - 1;
      }
      r[2 + q / 8] = v;
    }
  }
}

// entries over the received records: record i's header at offset i * rs + 16 of the receive buffer
__global__ void k_ex_ent(const uint8_t* recv, uint64_t n, uint32_t rs, Entry* ent) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* r = reinterpret_cast<const uint64_t*>(recv + i * rs);
  Entry e;
  e.hash = r[0];
  e.addr = (i * rs + 16) | (r[1] & kDelBit);
  ent[i] = e;
}

// table slots [a, b) of the local replay (L: the window of the rank's exact range, addresses =
// receive-buffer offsets) written in the .spi layout through G (the rank's own slice, or a packed
// piece for another rank), addresses mapped back to the log's: the log address sits 8 bytes before
// the record's header
__global__ void k_ex_extract(BuildParams L, BuildParams G, const uint8_t* recv, uint64_t n, uint32_t rs, uint64_t a,
                             uint64_t b) {
  const uint64_t slot = a + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= b) return;
  uint64_t h = 0, la = 0, ga = 0;
  if (L.out) {
    const uint64_t w = table_to_window(slot, L.mod);
    if (w < L.cap) read_slot(L, w, h, la);
    else atomicOr(&L.st->guard, 4u);
  }
  if (la) {
    const uint64_t q = la - 16;
    if (la < 16 || q % rs != 0 || q / rs >= n) {
      atomicOr(&L.st->guard, 4u);
      la = 0;
    } else {
      ga = reinterpret_cast<const uint64_t*>(recv + q)[1] & ~kDelBit;
    }
  }
  if (!la) h = 0;
  write_slot(G, slot, h, ga);
}

void launch_first_empty(const BuildParams& P, hipStream_t s, unsigned long long* out) {
  if (P.slot_hi > P.slot_lo)
    hipLaunchKernelGGL(k_first_empty, dim3((unsigned)((P.slot_hi - P.slot_lo + 255) / 256)), dim3(256), 0, s, P, out);
}

void launch_ex_count(const BuildParams& P, hipStream_t s, const int64_t* starts, int world, uint32_t* cnt,
                     uint64_t* off, uint64_t* scratch, unsigned long long* totals) {
  if (!P.nslabs) return;
  hipLaunchKernelGGL(k_ex_count, dim3((unsigned)((P.nslabs + kExWaves - 1) / kExWaves)), dim3(64 * kExWaves), 0, s, P,
                     starts, world, cnt);
  const uint64_t n = (uint64_t)world * P.nslabs;
  scan_exclusive<uint32_t, uint64_t, OpAdd>(cnt, off, n, off + n, OpAdd(), scratch, s);
  hipLaunchKernelGGL(k_ex_totals, dim3(1), dim3(256), 0, s, off, P.nslabs, world, totals);
}

void launch_ex_scatter(const BuildParams& P, hipStream_t s, const int64_t* starts, int world, const uint64_t* off,
                       uint8_t* send, uint32_t rs) {
  if (P.nslabs)
    hipLaunchKernelGGL(k_ex_scatter, dim3((unsigned)((P.nslabs + kExWaves - 1) / kExWaves)), dim3(64 * kExWaves), 0, s,
                       P, starts, world, off, send, rs);
}

void launch_ex_ent(hipStream_t s, const uint8_t* recv, uint64_t n, uint32_t rs, Entry* ent) {
  if (n) hipLaunchKernelGGL(k_ex_ent, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, recv, n, rs, ent);
}

void launch_ex_extract(const BuildParams& L, const BuildParams& G, hipStream_t s, const uint8_t* recv, uint64_t n,
                       uint32_t rs, uint64_t a, uint64_t b) {
  if (b > a)
    hipLaunchKernelGGL(k_ex_extract, dim3((unsigned)((b - a + 255) / 256)), dim3(256), 0, s, L, G, recv, n, rs, a, b);
}

}  // namespace sk
