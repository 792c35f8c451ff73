// lookup.hpp -- batched IndexHash.get on the device (lookup_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"

namespace sk {

struct LookupParams {
  const uint8_t* log;    // the .spl, device
  uint64_t log_len;
  const uint8_t* slots;  // the .spi's slots (index + 112), device
  uint64_t cap;
  FastMod mod;
  int32_t hash_size, addr_size, slot_size, ebb;
  uint32_t seed;
  int64_t max_disp;      // IndexHeader maxDisplacement: the probe bound (IndexHash.java:441-444)
  const uint8_t* keys;   // query i = keys[key_off[i] .. key_off[i + 1])
  const uint64_t* key_off;
  uint64_t n;
  int64_t* value_pos;    // out: log offset of the value, or -1
  int64_t* value_len;    // out: value length, or -1
  unsigned long long* err;  // min over (query << 8 | -code) of the queries that hit corrupt data; ~0 = none
};

void launch_get(const LookupParams& L, hipStream_t s);
// sparkey_hash_batch: L.keys / key_off / n / hash_size / seed / mod (mod.cap == 0: no slots)
void launch_hash_batch(const LookupParams& L, uint64_t* hash_out, uint64_t* slot_out, hipStream_t s);
void launch_slot_batch(const uint64_t* hash, uint64_t n, const FastMod& mod, uint64_t* slot_out, hipStream_t s);

}  // namespace sk
