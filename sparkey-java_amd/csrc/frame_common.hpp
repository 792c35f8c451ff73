// frame_common.hpp -- device helpers shared by the framing kernels (fused_kernels.hip k_frame /
// k_frame_uniform, frame2_kernels.hip k_frame2): byte access into LDS-staged log regions, MurmurHash3
// over key bytes read 8 at a time, the inter-wave exit granules and the record-start screen.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"

namespace sk {

// ------------------------------------------------------------------------------------------------
// LDS byte access
// ------------------------------------------------------------------------------------------------
// 8 bytes starting at any offset of an 8-byte-aligned LDS window (two aligned 8-byte reads).
// Funnel shift of hi:lo right by sh (0..63) without a branch: (hi << 1) << (63 - sh) is hi << (64 - sh)
// for sh > 0 and 0 for sh = 0.  (`sh ? ... : lo` let the compiler sink the second load into a branch,
// an exec-mask round trip per 8 bytes read.)
__device__ __forceinline__ uint64_t funnel64(uint64_t lo, uint64_t hi, uint32_t sh) {
  return (lo >> sh) | ((hi << 1) << (63u - sh));
}
__device__ __forceinline__ uint64_t lds_u64_at(const uint8_t* win, int off) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(win + (off & ~7));
  return funnel64(w[0], w[1], (uint32_t)(off & 7) * 8u);
}

// Record header at absolute position p whose bytes lie in the LDS window starting at wb.
// Fast path: both VLQs one byte (every key < 127 bytes and value < 128 bytes); otherwise the
// generic Java-int VLQ decoder on the same bytes.
__device__ __forceinline__ RecHdr decode_lds(const uint8_t* win, int64_t wb, int64_t p, int64_t avail) {
  const uint64_t x = lds_u64_at(win, (int)(p - wb));
  RecHdr h;
  if ((x & 0x8080ull) == 0) {
    h.rc = 0;
    h.hlen = 2;
    const int32_t first = (int32_t)(x & 0xff);
    const int32_t second = (int32_t)((x >> 8) & 0xff);
    if (first == 0) { h.put = 0; h.klen = second; h.vlen = 0; }
    else { h.put = 1; h.klen = first - 1; h.vlen = second; }
  } else {
    auto at = [&](int64_t a) -> uint32_t { return win[a - wb]; };
    h = decode_header(at, p, p + 12);
  }
  if (h.rc == 0 && p + h.hlen > avail) h.rc = kErrCorruptRecord;
  return h;
}

// Key byte loaders for the hashes: u64(o) = the 8 key bytes starting at key offset o (the bytes
// past the key are read but masked off).
struct LdsKey {  // key in an 8-byte aligned LDS window
  const uint8_t* win;
  int base;
  __device__ __forceinline__ uint64_t u64(int o) const { return lds_u64_at(win, base + o); }
};
struct GlobalKey {  // key in global memory with at least 32 readable bytes past its end
  const uint8_t* p;
  __device__ __forceinline__ uint64_t u64(int o) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
    const uint64_t lo = q[0], hi = q[1];
    const int sh = (int)(a & 7) * 8;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
};

// MurmurHash3 x86_32 of `len` key bytes (MurmurHash3.java:18-75).
template <class Ld>
__device__ inline uint32_t murmur32_ld(const Ld& ld, int32_t len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const int32_t nblocks = len >> 2;
  auto block = [&](uint32_t k1) {
    k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
    h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
  };
  int32_t i = 0;
  for (; i + 1 < nblocks; i += 2) {
    const uint64_t x = ld.u64(4 * i);
    block((uint32_t)x);
    block((uint32_t)(x >> 32));
  }
  if (i < nblocks) block((uint32_t)ld.u64(4 * i));
  // the tail without a branch: a zero tail mixes to zero, and h1 ^= 0 leaves it (the loaders read past
  // the key's end by contract)
  const int32_t rem = len & 3;
  uint32_t k1 = (uint32_t)ld.u64(4 * nblocks) & ((1u << (8 * rem)) - 1u);
  k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
  return h1;
}

// MurmurHash3 x64_128 -> h1 of `len` key bytes (MurmurHash3.java:100-201).
template <class Ld>
__device__ inline uint64_t murmur64_ld(const Ld& ld, int32_t len, uint32_t seed) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = (uint64_t)seed, h2 = h1;
  const int32_t nblocks = len >> 4;
  for (int32_t i = 0; i < nblocks; i++) {
    uint64_t k1 = ld.u64(16 * i);
    uint64_t k2 = ld.u64(16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729ull;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5ull;
  }
  // the tail without branches: a zero half mixes to zero, and h ^= 0 leaves it (the loaders read
  // past the key's end by contract)
  const int32_t rem = len & 15;
  const int t = 16 * nblocks;
  {
    uint64_t k2 = ld.u64(t + 8) & (rem > 8 ? (1ull << (8 * (rem - 8))) - 1ull : 0ull);
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    uint64_t k1 = ld.u64(t) & (rem >= 8 ? ~0ull : (1ull << (8 * rem)) - 1ull);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// The same two hashes for a key length every lane of the wave shares (k_frame_uniform: every record
// has the header's maxKeyLen): the block loop and the tail are scalar branches, so a key without a
// tail (C2's 16 bytes) reads and mixes none.
template <class Ld>
__device__ inline uint64_t murmur64_uni(const Ld& ld, int32_t len, uint32_t seed) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = (uint64_t)seed, h2 = h1;
  const int32_t nblocks = len >> 4;
  for (int32_t i = 0; i < nblocks; i++) {
    uint64_t k1 = ld.u64(16 * i);
    uint64_t k2 = ld.u64(16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729ull;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5ull;
  }
  const int32_t rem = len & 15;
  if (rem) {
    const int t = 16 * nblocks;
    if (rem > 8) {
      uint64_t k2 = ld.u64(t + 8) & ((1ull << (8 * (rem - 8))) - 1ull);
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    uint64_t k1 = ld.u64(t) & (rem >= 8 ? ~0ull : (1ull << (8 * rem)) - 1ull);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2;
  return h1;
}
template <class Ld>
__device__ inline uint32_t murmur32_uni(const Ld& ld, int32_t len, uint32_t seed) {
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const int32_t nblocks = len >> 2;
  auto block = [&](uint32_t k1) {
    k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
    h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
  };
  int32_t i = 0;
  for (; i + 1 < nblocks; i += 2) {
    const uint64_t x = ld.u64(4 * i);
    block((uint32_t)x);
    block((uint32_t)(x >> 32));
  }
  if (i < nblocks) block((uint32_t)ld.u64(4 * i));
  const int32_t rem = len & 3;
  if (rem) {
    uint32_t k1 = (uint32_t)ld.u64(4 * nblocks) & ((1u << (8 * rem)) - 1u);
    k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
  return h1;
}

// ------------------------------------------------------------------------------------------------
// granules (8-byte {state, value} words) -- relaxed agent-scope atomics, zeroed before the launch
// ------------------------------------------------------------------------------------------------
// Placement bucket of a hash (its wanted slot >> kBucketShift) and the bucket's coarse partition digit.
__device__ __forceinline__ uint32_t bucket_of(const BuildParams& P, uint64_t hash) {
  return (uint32_t)(fast_mod(hash, P.mod) >> kBucketShift);
}
__device__ __forceinline__ uint32_t digit_of(const BuildParams& P, uint32_t bucket) {
  return (uint32_t)(((uint64_t)bucket * P.dmagic) >> 40);
}

constexpr unsigned long long kReady = 1ull << 63;   // exit granule: bit 63 = published

__device__ __forceinline__ void granule_store(unsigned long long* g, unsigned long long v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long granule_load(unsigned long long* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool screen_start(uint32_t b0, uint32_t b1, const BuildParams& P) {
  // Canonical VLQs (what LogWriter writes).  Pruning a true start only costs speed: the chunk is
  // then unresolved or disagrees with its verified walk, and is re-walked exactly.
  if (b0 == 0) return P.max_key_len >= 128 || (int64_t)b1 <= P.max_key_len;  // DELETE, VLQ(keyLen)
  if (b0 >= 0x80) return P.max_key_len + 1 >= 128;                            // multi-byte keyLen+1
  if ((int64_t)b0 - 1 > P.max_key_len) return false;
  return P.max_value_len >= 128 || (int64_t)b1 <= P.max_value_len;            // PUT, VLQ(valueLen)
}

__device__ __forceinline__ uint4 load16_guarded(const uint8_t* log, int64_t a, int64_t log_len) {
  if (a + 16 <= log_len) return *reinterpret_cast<const uint4*>(log + a);
  uint8_t tmp[16];
#pragma unroll
  for (int i = 0; i < 16; i++) tmp[i] = (a + i < log_len) ? log[a + i] : 0;
  return *reinterpret_cast<uint4*>(tmp);
}

// 8 bytes at any region offset (two aligned 8-byte reads; the region is allocated in 256 B blocks)
__device__ __forceinline__ uint64_t rgn_u64(const uint8_t* r, uint32_t o) {
  const uint32_t a = o & ~7u;
  return funnel64(*reinterpret_cast<const uint64_t*>(r + a), *reinterpret_cast<const uint64_t*>(r + a + 8), (o & 7u) * 8u);
}
struct RgnKey {
  const uint8_t* r;
  uint32_t base;
  __device__ __forceinline__ uint64_t u64(int o) const { return rgn_u64(r, base + (uint32_t)o); }
};
// The same key through aligned dwords: the loaders read at key offsets that are multiples of 8, so
// the byte shift inside a dword is one per key and each 4 bytes out is one v_alignbit of two dwords
// (the 64-bit funnel above costs five instructions per 8 bytes).
__device__ __forceinline__ uint32_t rgn_u32(const uint8_t* r, uint32_t o) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(r + (o & ~3u));
  return __builtin_amdgcn_alignbit(w[1], w[0], (o & 3u) * 8u);
}
struct RgnKey4 {
  const uint32_t* w;  // the dword holding the key's first byte
  uint32_t sh;        // 8 x the first byte's place in it
  __device__ __forceinline__ RgnKey4(const uint8_t* r, uint32_t base)
      : w(reinterpret_cast<const uint32_t*>(r + (base & ~3u))), sh((base & 3u) * 8u) {}
  __device__ __forceinline__ uint64_t u64(int o) const {
    const uint32_t* p = w + (o >> 2);
    const uint32_t a = p[0], b = p[1], c = p[2];
    return (uint64_t)__builtin_amdgcn_alignbit(b, a, sh) |
           ((uint64_t)__builtin_amdgcn_alignbit(c, b, sh) << 32);
  }
};

// Record header at absolute position p inside the region (p - R0 + 16 <= region bytes).
__device__ __forceinline__ RecHdr decode_rgn(const uint8_t* r, int64_t R0, int64_t p, int64_t avail) {
  const uint64_t x = rgn_u64(r, (uint32_t)(p - R0));
  RecHdr h;
  if ((x & 0x8080ull) == 0) {
    h.rc = 0;
    h.hlen = 2;
    const int32_t first = (int32_t)(x & 0xff);
    const int32_t second = (int32_t)((x >> 8) & 0xff);
    if (first == 0) { h.put = 0; h.klen = second; h.vlen = 0; }
    else { h.put = 1; h.klen = first - 1; h.vlen = second; }
  } else {
    auto at = [&](int64_t a) -> uint32_t { return r[(uint32_t)(a - R0)]; };
    h = decode_header(at, p, p + 12);
  }
  if (h.rc == 0 && p + h.hlen > avail) h.rc = kErrCorruptRecord;
  return h;
}


// A framing wave's DELETE count: into one of kDelParts spread counters (build_kernels.hpp) when the
// plan gives them, else straight into the status block.
__device__ __forceinline__ void add_deletes(const BuildParams& P, uint64_t wv, unsigned long long n) {
  if (P.del_parts) atomicAdd(&P.del_parts[(wv % kDelParts) * 16], n);
  else atomicAdd(&P.st->n_deletes, n);
}

// The framing kernels run several independent waves per workgroup (one log region each): their
// LDS hand-offs are between the lanes of one wave, so they synchronise the wave, not the workgroup
// (a wave may spin on another region's exit while its neighbours are elsewhere).  Every LDS access
// and LDS-DMA of the wave has completed after this.
// s_waitcnt vmcnt(n) for a run-time n (0..63; more waits for everything): gfx9 encoding, vmcnt in bits
// 3:0 and 15:14, expcnt and lgkmcnt left at their maxima
__device__ __forceinline__ void wait_vmcnt_upto(int n) {
#define SK_VMW(v) \
  case v: __builtin_amdgcn_s_waitcnt(((v) & 0xF) | (((v) >> 4) << 14) | (0x7 << 4) | (0xF << 8)); break;
  switch (n) {
    SK_VMW(0) SK_VMW(1) SK_VMW(2) SK_VMW(3) SK_VMW(4) SK_VMW(5) SK_VMW(6) SK_VMW(7) SK_VMW(8) SK_VMW(9) SK_VMW(10) SK_VMW(11) SK_VMW(12) SK_VMW(13) SK_VMW(14) SK_VMW(15) SK_VMW(16) SK_VMW(17) SK_VMW(18) SK_VMW(19) SK_VMW(20) SK_VMW(21) SK_VMW(22) SK_VMW(23) SK_VMW(24) SK_VMW(25) SK_VMW(26) SK_VMW(27) SK_VMW(28) SK_VMW(29) SK_VMW(30) SK_VMW(31) SK_VMW(32) SK_VMW(33) SK_VMW(34) SK_VMW(35) SK_VMW(36) SK_VMW(37) SK_VMW(38) SK_VMW(39) SK_VMW(40) SK_VMW(41) SK_VMW(42) SK_VMW(43) SK_VMW(44) SK_VMW(45) SK_VMW(46) SK_VMW(47) SK_VMW(48) SK_VMW(49) SK_VMW(50) SK_VMW(51) SK_VMW(52) SK_VMW(53) SK_VMW(54) SK_VMW(55) SK_VMW(56) SK_VMW(57) SK_VMW(58) SK_VMW(59) SK_VMW(60) SK_VMW(61) SK_VMW(62) SK_VMW(63)
    default: __builtin_amdgcn_s_waitcnt(0); break;
  }
#undef SK_VMW
}

__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Framing regions per workgroup: one wave each, consecutive regions, one ticket per workgroup.  A
// region waits only for lower regions' published exits; the ticket order makes every such region
// belong to a workgroup that is already resident, whatever order the dispatcher admits workgroups
// in.  One device-scope atomic per workgroup: a ticket per wave measured 88 per microsecond at
// most, which bounds a launch of 1.7M one-wave workgroups (C3) to 19 ms.
constexpr int kFrameWaves = 4;

// Workgroups of a persistent launch that the device holds resident at once (occupancy API x CUs,
// one fewer per CU as margin -- the API can answer one high, MI355X_MICROARCH.md "Residency"), at most
// `want`.  Host side.
inline uint64_t resident_grid(const void* kernel, int block, size_t lds, uint64_t want) {
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 || cus <= 0)
    return std::min<uint64_t>(want, 256);
  const uint64_t cap = (uint64_t)std::max(1, per_cu - 1) * (uint64_t)cus;
  return std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
}

// SWAR record-start screen over 8 positions (screen_start bytewise): x = the bytes at p .. p + 7,
// y = the bytes at p + 1 .. p + 8; bit i of the result = position p + i is a plausible start
// (canonical VLQs within the header's maxima; 0x00 only when the header counts DELETEs).
struct Screen8 {
  uint64_t rk, rv, rd;
  bool allk, allv, alld, no_del;
};
__device__ __forceinline__ Screen8 make_screen8(const BuildParams& P) {
  constexpr uint64_t ONES = 0x0101010101010101ull;
  Screen8 S;
  const int64_t TK = P.max_key_len + 1 >= 128 ? 127 : P.max_key_len + 1;
  S.allk = P.max_key_len + 1 >= 128;
  S.allv = P.max_value_len >= 127;
  S.alld = P.max_key_len >= 127;
  S.rk = ONES * (uint64_t)(min(TK, (int64_t)126) + 1);
  S.rv = ONES * (uint64_t)(min(P.max_value_len, (int64_t)126) + 1);
  S.rd = ONES * (uint64_t)(min(P.max_key_len, (int64_t)126) + 1);
  S.no_del = P.no_deletes != 0;
  return S;
}
__device__ __forceinline__ uint32_t screen8(uint64_t x, uint64_t y, const Screen8& S) {
  constexpr uint64_t H = 0x8080808080808080ull, L7 = 0x7f7f7f7f7f7f7f7full, ONES = 0x0101010101010101ull;
  auto le_rep = [&](uint64_t v, uint64_t rep, bool all) -> uint64_t { return all ? H : ~(v | ((v | H) - rep)) & H; };
  const uint64_t z = ~(((x & L7) + L7) | x) & H;  // zero bytes
  const uint64_t put_first = le_rep(x, S.rk, S.allk) & ~z;
  const uint64_t r = (put_first & le_rep(y, S.rv, S.allv)) | (S.no_del ? 0ull : (z & le_rep(y, S.rd, S.alld)));
  return (uint32_t)((((r >> 7) & ONES) * 0x0102040810204080ull) >> 56);  // bit 8i -> bit i
}

// ------------------------------------------------------------------------------------------------
// Records held in registers: an array of N aligned 16-byte chunks, a lane-variable byte offset
// resolved by value selects (never by indexing registers), MurmurHash3 over it.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lo64(const uint4& c) { return (uint64_t)c.x | ((uint64_t)c.y << 32); }
__device__ __forceinline__ uint64_t hi64(const uint4& c) { return (uint64_t)c.z | ((uint64_t)c.w << 32); }

// 8 bytes at byte offset o (0..15) of the 32 bytes c0 ++ c1
__device__ __forceinline__ uint64_t bytes8(const uint4& c0, const uint4& c1, int o) {
  const uint64_t w0 = (o & 8) ? hi64(c0) : lo64(c0);
  const uint64_t w1 = (o & 8) ? lo64(c1) : hi64(c0);
  const int sh = (o & 7) * 8;
  return sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
}

// half h (8 bytes) of the chunk array: chunk h / 2, low or high half (h a compile-time index once
// unrolled; clamped to the array, since the selects below also form indices the lane never uses)
template <int N>
__device__ __forceinline__ uint64_t half_of(const uint4 (&c)[N], int h) {
  h = h < 2 * N ? h : 2 * N - 1;
  return (h & 1) ? hi64(c[h >> 1]) : lo64(c[h >> 1]);
}

// The key's 8-byte word j (key bytes 8j .. 8j + 7), the key starting at byte ko (0..31) of the chunk
// array: aligned halves (ko >> 3) + j and + j + 1, funnel-shifted.  ko >> 3 is lane-variable (0..3):
// a select among four static halves.
template <int N>
__device__ __forceinline__ uint64_t key_word(const uint4 (&c)[N], int ko, int j) {
  const int q = ko >> 3;
  // (every half index below is static once j is; q picks among them by value selects, so the array
  // stays in registers)
  const uint64_t h0 = half_of(c, j), h1 = half_of(c, j + 1), h2 = half_of(c, j + 2), h3 = half_of(c, j + 3),
                 h4 = half_of(c, j + 4);
  const bool q1 = q & 1, q2 = q & 2;
  const uint64_t a = q2 ? (q1 ? h3 : h2) : (q1 ? h1 : h0);
  const uint64_t b = q2 ? (q1 ? h4 : h3) : (q1 ? h2 : h1);
  const int sh = (ko & 7) * 8;
  return sh ? (a >> sh) | (b << (64 - sh)) : a;
}

// MurmurHash3 x64_128 -> h1 (MurmurHash3.java:100-201) of a key whose bytes are in the chunk array
// from byte ko on (ko + len + 8 <= 16 N); the loops run to the static bound with the lane's own length
// as the guard, so every chunk index is static.
template <int N>
__device__ __forceinline__ uint64_t lane_murmur64(const uint4 (&c)[N], int ko, int32_t len, uint32_t seed) {
  constexpr int kMaxBlocks = N - 1;  // (len < 16 N - 8 - ko)
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = (uint64_t)seed, h2 = h1;
  const int32_t nblocks = len >> 4;
#pragma unroll
  for (int i = 0; i < kMaxBlocks; i++) {
    if (i < nblocks) {
      uint64_t k1 = key_word(c, ko, 2 * i);
      uint64_t k2 = key_word(c, ko, 2 * i + 1);
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
      h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729ull;
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5ull;
    }
  }
  const int32_t rem = len & 15;
  uint64_t t1 = 0, t2 = 0;  // the tail's two words: word 2 * nblocks and the next (lane-variable block)
#pragma unroll
  for (int i = 0; i <= kMaxBlocks; i++) {
    if (i == nblocks) {
      t1 = key_word(c, ko, 2 * i);
      t2 = key_word(c, ko, 2 * i + 1);
    }
  }
  if (rem > 8) {
    uint64_t k2 = t2 & ((1ull << (8 * (rem - 8))) - 1ull);
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
  }
  if (rem > 0) {
    uint64_t k1 = t1;
    if (rem < 8) k1 &= (1ull << (8 * rem)) - 1ull;
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// MurmurHash3 x86_32 (MurmurHash3.java:18-75), same conventions.
template <int N>
__device__ __forceinline__ uint32_t lane_murmur32(const uint4 (&c)[N], int ko, int32_t len, uint32_t seed) {
  constexpr int kMaxWords = 2 * N - 1;  // 8-byte words the key (and its tail word) can span
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  uint32_t h1 = seed;
  const int32_t nblocks = len >> 2;
  auto block = [&](uint32_t k1) {
    k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
    h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
  };
  uint32_t tail = 0;
#pragma unroll
  for (int j = 0; j < kMaxWords; j++) {
    if (2 * j < nblocks || 2 * j == nblocks) {
      const uint64_t w = key_word(c, ko, j);
      if (2 * j < nblocks) block((uint32_t)w);
      if (2 * j + 1 < nblocks) block((uint32_t)(w >> 32));
      if (2 * j == nblocks) tail = (uint32_t)w;
      if (2 * j + 1 == nblocks) tail = (uint32_t)(w >> 32);
    }
  }
  const int32_t rem = len & 3;
  if (rem) {
    uint32_t k1 = tail & ((1u << (8 * rem)) - 1u);
    k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
  return h1;
}


}  // namespace sk
