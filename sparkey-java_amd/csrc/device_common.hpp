// device_common.hpp -- integer primitives shared by the gfx950 kernels of the .spi builder.
//
// MurmurHash3 (x86_32 and x64_128->h1), Java-int VLQ record headers and an exact 64-bit
// "hash mod capacity" by multiply-high.  Every function cites the reference behaviour it
// reproduces (paths relative to spotify/sparkey-java src/main/java/com/spotify/sparkey/).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {

constexpr int64_t kLogHeaderSize = 84;     // LogHeader.java:26
constexpr int64_t kIndexHeaderSize = 112;  // IndexHeader.java:24
constexpr uint64_t kDelBit = 1ull << 63;   // marks DELETE records inside an (hash, address) entry

// Error codes (mirror include/sparkey_gpu.h).
constexpr int kErrCorruptLog = -3;
constexpr int kErrNoFreeSlots = -4;
constexpr int kErrCorruptData = -5;
constexpr int kErrVlq = -6;
constexpr int kErrCorruptRecord = -13;  // SPARKEY_E_CORRUPT_RECORD: the iterator cannot read a record
// RecHdr.rc of a record whose first VLQ runs into the end of the file: SparkeyLogIterator.hasNext
// catches that EOFException and ends the iteration without an error (SparkeyLogIterator.java:111-115).
constexpr int kEndOfLog = 1;

// ---------------------------------------------------------------------------------------------
// wantedSlot = Long.remainderUnsigned(hash, capacity)   (IndexHash.java:667-669)
// q = mulhi(x, floor(2^64 / cap)) is floor(x / cap) or one less, so one conditional subtract
// gives the exact remainder (tests/test_fastmod.py checks it against '%' on the host -- boundary values,
// random hashes, the BASELINE capacities and every odd capacity below 4096 -- and on the device).
// ---------------------------------------------------------------------------------------------
// A table window (the sharded exact path's range-local replay) sets `base`: slots
// are then numbered from `base` around the ring, local = (wanted - base) mod cap.
struct FastMod {
  uint64_t cap;   // capacity (odd, >= 1)
  uint64_t m;     // floor(2^64 / cap); 0 when cap == 1
  uint64_t base;  // first slot of the window (0: the whole table)
};

__host__ __device__ inline uint64_t mulhi_u64(uint64_t a, uint64_t b) {
  return (uint64_t)(((unsigned __int128)a * (unsigned __int128)b) >> 64);
}

__host__ __device__ inline uint64_t fast_mod(uint64_t x, FastMod f) {
  if (f.cap == 1) return 0;
  const uint64_t q = mulhi_u64(x, f.m);
  uint64_t r = x - q * f.cap;
  if (r >= f.cap) r -= f.cap;
  return r >= f.base ? r - f.base : r + f.cap - f.base;
}

// the table slot of window slot `local` (the reference's wantedSlot for an entry's local wanted slot)
__host__ __device__ inline uint64_t window_to_table(uint64_t local, FastMod f) {
  const uint64_t s = local + f.base;
  return s >= f.cap ? s - f.cap : s;
}
// the window slot of table slot `slot`
__host__ __device__ inline uint64_t table_to_window(uint64_t slot, FastMod f) {
  return slot >= f.base ? slot - f.base : slot + f.cap - f.base;
}

inline FastMod make_fastmod(uint64_t cap, uint64_t base = 0) {
  FastMod f;
  f.cap = cap;
  f.m = cap <= 1 ? 0 : (uint64_t)(((unsigned __int128)1 << 64) / cap);
  f.base = base;
  return f;
}

// ---------------------------------------------------------------------------------------------
// MurmurHash3 over `len` bytes at `p` (p may point into LDS or global memory).
// x86_32: MurmurHash3.java:18-75.  x64_64: MurmurHash3.java:100-201 (seed widened unsigned :103,
// returns h1 after the final h1 += h2).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

template <class P>
__device__ __forceinline__ uint32_t ld_u32(P p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
template <class P>
__device__ __forceinline__ uint64_t ld_u64(P p) {
  return (uint64_t)ld_u32(p) | ((uint64_t)ld_u32(p + 4) << 32);
}

template <class P>
__device__ inline uint32_t murmur3_x86_32(P data, int32_t len, uint32_t seed) {
  const int32_t nblocks = len >> 2;
  uint32_t h1 = seed;
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  for (int32_t i = 0; i < nblocks; i++) {
    uint32_t k1 = ld_u32(data + 4 * i);
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const int32_t t = nblocks << 2;
  const int32_t rem = len & 3;
  if (rem) {
    uint32_t k1 = 0;
    if (rem == 3) k1 ^= (uint32_t)data[t + 2] << 16;
    if (rem >= 2) k1 ^= (uint32_t)data[t + 1] << 8;
    k1 ^= (uint32_t)data[t];
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
  }
  h1 ^= (uint32_t)len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

template <class P>
__device__ inline uint64_t murmur3_x64_64(P data, int32_t len, uint32_t seed) {
  const int32_t nblocks = len >> 4;
  uint64_t h1 = (uint64_t)seed;
  uint64_t h2 = h1;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  for (int32_t i = 0; i < nblocks; i++) {
    uint64_t k1 = ld_u64(data + 16 * i);
    uint64_t k2 = ld_u64(data + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729ull;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5ull;
  }
  const int32_t t = nblocks << 4;
  const int32_t rem = len & 15;
  if (rem > 8) {  // bytes 8..rem-1 into k2 (fall-through cases 15..9)
    uint64_t k2 = 0;
    for (int32_t i = rem - 1; i >= 8; i--) k2 ^= (uint64_t)data[t + i] << (8 * (i - 8));
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
  }
  if (rem > 0) {  // bytes 0..min(rem,8)-1 into k1 (cases 8..1)
    uint64_t k1 = 0;
    const int32_t lim = rem < 8 ? rem : 8;
    for (int32_t i = lim - 1; i >= 0; i--) k1 ^= (uint64_t)data[t + i] << (8 * i);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// HashType.hash (HashType.java:44-46, 70-72): 32-bit hashes are the unsigned x86_32 value.
template <class P>
__device__ __forceinline__ uint64_t key_hash(int hash_size, P key, int32_t len, uint32_t seed) {
  return hash_size == 8 ? murmur3_x64_64(key, len, seed) : (uint64_t)murmur3_x86_32(key, len, seed);
}

// ---------------------------------------------------------------------------------------------
// Record header: PUT = VLQ(keyLen+1) VLQ(valueLen) key value; DELETE = 0x00 VLQ(keyLen) key
// (UncompressedBlockOutput.java:67-87), decoded with Java-int VLQ semantics: at most 5 bytes,
// `value | b << 28` may wrap negative (Util.java:146-218), as SparkeyLogIterator.hasNext does
// (SparkeyLogIterator.java:86-138).
// ---------------------------------------------------------------------------------------------
struct RecHdr {
  int32_t rc;     // 0 ok, kErrVlq, kErrCorruptRecord (EOF inside the second VLQ), kEndOfLog (EOF inside the first)
  int32_t put;    // 1 PUT, 0 DELETE
  int32_t hlen;   // header bytes
  int32_t klen;   // Java int (may be negative on corrupt input)
  int32_t vlen;   // Java int
};

// `at(i)` returns the byte at absolute offset i; bytes at >= avail are EOF.
template <class At>
__device__ __forceinline__ int32_t read_vlq(At at, int64_t& p, int64_t avail, int32_t& rc) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (p >= avail) { rc = kErrCorruptRecord; return 0; }
    const uint32_t b = at(p);
    p++;
    if (b < 0x80u) return (int32_t)(v | (b << (7 * i)));
    v |= (b & 0x7fu) << (7 * i);
  }
  rc = kErrVlq;
  return 0;
}

template <class At>
__device__ __forceinline__ RecHdr decode_header(At at, int64_t p, int64_t avail) {
  RecHdr h;
  h.rc = 0;
  int64_t q = p;
  const int32_t first = read_vlq(at, q, avail, h.rc);
  if (h.rc) {
    if (h.rc == kErrCorruptRecord) h.rc = kEndOfLog;
    return h;
  }
  const int32_t second = read_vlq(at, q, avail, h.rc);
  if (h.rc) return h;
  h.hlen = (int32_t)(q - p);
  if (first == 0) { h.put = 0; h.klen = second; h.vlen = 0; }
  else { h.put = 1; h.klen = first - 1; h.vlen = second; }
  return h;
}

// The error code of a record header the iterator rejects (kEndOfLog ends the chain instead, where the
// caller walks the verified chain; anywhere else it is a corrupt record).
__device__ __forceinline__ int32_t header_error(const RecHdr& h) { return h.rc < 0 ? h.rc : kErrCorruptRecord; }

// What the reference's iterator accepts on the real record chain (else it throws):
// key fits its keyBuf of maxKeyLen bytes and lies inside the file.
__device__ __forceinline__ bool header_valid(const RecHdr& h, int64_t p, int64_t max_key_len, int64_t log_len) {
  return h.rc == 0 && h.klen >= 0 && h.vlen >= 0 && (int64_t)h.klen <= max_key_len &&
         p + h.hlen + h.klen <= log_len;
}

// Speculative framing additionally prunes candidates whose value exceeds the header's maxValueLen.
__device__ __forceinline__ bool header_plausible(const RecHdr& h, int64_t p, int64_t max_key_len,
                                                 int64_t max_value_len, int64_t log_len) {
  return header_valid(h, p, max_key_len, log_len) && (int64_t)h.vlen <= max_value_len;
}

__device__ __forceinline__ int64_t record_end(const RecHdr& h, int64_t p) {
  return p + h.hlen + h.klen + (h.put ? h.vlen : 0);
}

}  // namespace sk
