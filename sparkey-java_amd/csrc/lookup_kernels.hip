// lookup_kernels.hip -- batched IndexHash.get (IndexHash.java:398-452) against a built .spi and its
// log, both resident in HBM: the step after the build, and an independent
// check of every table the build writes.
//
//   k_get   one lane per query: MurmurHash3 of the key, probe from the wanted slot while the
//           displacement stays <= maxDisplacement, on an equal hash compare the key bytes in the log
//           (a DELETE record there is the reference's "Invalid data - reference to delete entry").
//           Result: the value's log offset and length, or -1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "lookup.hpp"

namespace sk {

__device__ __forceinline__ uint64_t rd_le(const uint8_t* p, int n) {
  uint64_t v = 0;
  if (n == 8) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);  // slots are 4-byte aligned
    v = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
  } else {
    v = *reinterpret_cast<const uint32_t*>(p);
  }
  return v;
}

__global__ __launch_bounds__(256) void k_get(LookupParams L) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L.n) return;
  const uint64_t k0 = L.key_off[i], k1 = L.key_off[i + 1];
  const int32_t klen = (int32_t)(k1 - k0);
  const uint8_t* key = L.keys + k0;
  const uint64_t hash = key_hash(L.hash_size, key, klen, L.seed);
  uint64_t slot = fast_mod(hash, L.mod);
  int64_t vpos = -1, vlen = -1;
  auto at = [&](int64_t a) -> uint32_t { return L.log[a]; };
  for (int64_t disp = 0;; disp++) {
    const uint8_t* s = L.slots + slot * (uint64_t)L.slot_size;
    const uint64_t hash2 = rd_le(s, L.hash_size);
    const uint64_t addr2 = rd_le(s + L.hash_size, L.addr_size);
    if (addr2 == 0) break;
    if (hash2 == hash) {
      const int64_t p = (int64_t)(addr2 >> L.ebb);
      const RecHdr h = decode_header(at, p, (int64_t)L.log_len);
      if (h.rc) {
        atomicMin(L.err, ((unsigned long long)i << 8) | (unsigned long long)(-header_error(h)));
        break;
      }
      if (!h.put) {  // "Invalid data - reference to delete entry"
        atomicMin(L.err, ((unsigned long long)i << 8) | (unsigned long long)(-kErrCorruptData));
        break;
      }
      if (h.klen == klen) {
        const int64_t kp = p + h.hlen;
        bool eq = kp + klen <= (int64_t)L.log_len;
        for (int32_t j = 0; j < klen && eq; j++) eq = L.log[kp + j] == key[j];
        if (eq) {
          vpos = kp + klen;
          vlen = h.vlen;
          break;
        }
      }
    }
    if (disp + 1 > L.max_disp) break;
    slot = slot + 1 == L.cap ? 0 : slot + 1;
  }
  L.value_pos[i] = vpos;
  L.value_len[i] = vlen;
}

void launch_get(const LookupParams& L, hipStream_t s) {
  if (L.n == 0) return;
  hipLaunchKernelGGL(k_get, dim3((unsigned)((L.n + 255) / 256)), dim3(256), 0, s, L);
}

// HashType.hash + getWantedSlot per key (sparkey_hash_batch): the same key_hash / fast_mod the build
// kernels call, one lane per key.
__global__ __launch_bounds__(256) void k_hash_batch(LookupParams L, uint64_t* hash_out, uint64_t* slot_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L.n) return;
  const uint64_t k0 = L.key_off[i];
  const uint64_t h = key_hash(L.hash_size, L.keys + k0, (int32_t)(L.key_off[i + 1] - k0), L.seed);
  hash_out[i] = h;
  if (slot_out) slot_out[i] = fast_mod(h, L.mod);
}

__global__ __launch_bounds__(256) void k_slot_batch(const uint64_t* hash, uint64_t n, FastMod mod, uint64_t* slot_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) slot_out[i] = fast_mod(hash[i], mod);
}

void launch_hash_batch(const LookupParams& L, uint64_t* hash_out, uint64_t* slot_out, hipStream_t s) {
  if (L.n == 0) return;
  hipLaunchKernelGGL(k_hash_batch, dim3((unsigned)((L.n + 255) / 256)), dim3(256), 0, s, L, hash_out, slot_out);
}

void launch_slot_batch(const uint64_t* hash, uint64_t n, const FastMod& mod, uint64_t* slot_out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_slot_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hash, n, mod, slot_out);
}

}  // namespace sk
