// kernel_utils.hpp -- device helpers shared by the build kernels (chunk geometry, LDS staging,
// wave reductions, slot encoding).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "build_kernels.hpp"
#include "device_common.hpp"

namespace sk {

// ------------------------------------------------------------------------------------------------
// small device utilities
// ------------------------------------------------------------------------------------------------
// The framing wrote more records than the workspace holds: every later stage of this attempt is
// skipped (its offsets would run past the buffers) and the host redoes the build with more room.
__device__ __forceinline__ bool build_aborted(const BuildParams& P) {
  // (p2_overflow: the fixed bucket regions did not hold a bucket; the host redoes the build)
  // (abort_on_fail: the single-GPU build loop, whose host discards an attempt whose framing failed or
  //  stopped early, and a sharded bin right after a speculative framing attempt that did not hold --
  //  no stage consumes a region the framing left half-written)
  return P.st->overflow != 0 || P.st->n_records > P.max_records || P.st->p2_overflow != 0 ||
         (P.abort_on_fail && (P.st->spec_fail != 0 || P.st->err != ~0ull));
}

// An entry whose bucket lies outside the buckets its workgroup owns (a digit or bucket region whose
// contents disagree with its count).  That is a bug, never a property of the input: the entry is
// dropped before any LDS or global index is formed from it, st->guard gets kGuardForeign, and the host
// fails the build with SPARKEY_E_GPU (as IndexHash.put checks its bounds before it touches the table,
// IndexHash.java:574-576).  Kernels keep a per-thread flag and report it once.
constexpr unsigned kGuardForeign = 0x100u;
__device__ __forceinline__ void report_foreign(const BuildParams& P, bool bad) {
  if (bad) atomicOr(&P.st->guard, kGuardForeign);
}

// compact entries (CEntry, BuildParams.compact): raw (addr = the record index) or with its address;
// the stores are one 3-dword store (4-byte aligned), plain or non-temporal
typedef unsigned int sk_u32x3 __attribute__((ext_vector_type(3), aligned(4)));
__device__ __forceinline__ Entry load_craw(const CEntry* s) {
  const CEntry c = *s;
  Entry e;
  e.hash = (uint64_t)c.h0 | ((uint64_t)c.h1 << 32);
  e.addr = c.idx;
  return e;
}
__device__ __forceinline__ Entry load_centry(const BuildParams& P, const CEntry* s) {
  Entry e = load_craw(s);
  e.addr = (uint64_t)(P.fr_entry + (int64_t)e.addr * P.uni_rec) << P.ebb;
  return e;
}
__device__ __forceinline__ void store_craw(CEntry* d, const Entry& e) {
  sk_u32x3 v;
  v.x = (uint32_t)e.hash;
  v.y = (uint32_t)(e.hash >> 32);
  v.z = (uint32_t)e.addr;
  *reinterpret_cast<sk_u32x3*>(d) = v;
}
__device__ __forceinline__ void store_craw_nt(CEntry* d, const Entry& e) {
  sk_u32x3 v;
  v.x = (uint32_t)e.hash;
  v.y = (uint32_t)(e.hash >> 32);
  v.z = (uint32_t)e.addr;
  __builtin_nontemporal_store(v, reinterpret_cast<sk_u32x3*>(d));
}

__device__ __forceinline__ void set_error(Status* st, int64_t pos, int code) {
  atomicMin(&st->err, ((unsigned long long)pos << 8) | (unsigned long long)(-code));
}

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
// Wave-wide sum / max of 32-bit values by DPP (row shifts, then the row broadcasts of lanes 15
// and 31), in VALU with no LDS crossbar traffic; the result is read from lane 63.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// Inclusive prefix sum over the wave's lanes by the same DPP steps (each lane keeps its prefix): a
// scan in ~12 VALU cycles, where shuffles cost six LDS-crossbar round trips (ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
// Lane i gets lane i - 1's value, lane 0 gets `first` (DPP wave_shr:1); lane i gets lane i + 1's,
// lane 63 gets `last` (wave_shl:1).  No LDS crossbar.
__device__ __forceinline__ int32_t wave_prev_i32(int32_t v, int32_t first) {
  return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int32_t wave_next_i32(int32_t v, int32_t last) {
  return __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false);
}
// Inclusive prefix max over the wave's lanes (DPP, as wave_incl_sum_u32).
__device__ __forceinline__ int32_t wave_incl_max_i32(int32_t v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return v;
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {  // (v >= 0 lanes only matter: 0 shifts in)
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT32_MIN, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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

// Slot write of the placement kernels: in a sharded build a slot outside [slot_lo, slot_hi) goes
// to the spill list for its owner.
__device__ __forceinline__ void put_slot(const BuildParams& P, uint64_t slot, uint64_t hash, uint64_t addr) {
  if (!P.sharded || (slot >= P.slot_lo && slot < P.slot_hi)) {
    write_slot(P, slot, hash, addr);
    return;
  }
  const unsigned long long i = atomicAdd(&P.st->n_spill, 1ull);
  if (i < P.spill_cap) {
    SpillEntry e;
    e.slot = slot;
    e.hash = hash;
    e.addr = addr;
    e.pad = 0;
    P.spill[i] = e;
  }
}

__device__ __forceinline__ uint64_t wrap_slot(uint64_t s, uint64_t cap) {
  while (s >= cap) s -= cap;
  return s;
}

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


__device__ __forceinline__ void put_le64(uint8_t* p, uint64_t v) {
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

// The end of calculateMaxDisplacement (IndexHash.java:195-245) from the slot sums: the wrap quirk
// (IndexHash.java:239-241: slot 0 and slot cap-1 both occupied with equal hashes count once more),
// Status, and the header fields it writes.  Sharded ranks store their partial sums only; the host
// reduces them and adds the quirk.
__device__ inline void finish_stats(const BuildParams& P, unsigned long long sum, unsigned long long col, long long mx,
                                    int sequential) {
  Status* st = P.st;
  if (P.sharded) {
    st->max_disp = mx;
    st->collisions = (long long)col;
    st->total_disp = (long long)sum;
    return;
  }
  uint64_t h0, a0, h1, a1;
  read_slot(P, 0, h0, a0);
  read_slot(P, P.cap - 1, h1, a1);
  if (a0 != 0 && a1 != 0 && h0 == h1) col++;
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

}  // namespace sk
