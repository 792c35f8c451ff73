// append.hpp -- batched LogWriter.put / delete on the device (append_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {

struct AppendParams {
  uint64_t n;
  const uint8_t* kind;       // 1 PUT, 0 DELETE
  const uint8_t* keys;
  const uint64_t* key_off;   // n + 1
  const uint8_t* values;
  const uint64_t* val_off;   // n + 1 (PUT i's value = values[val_off[i] .. val_off[i + 1]))
  int64_t max_key_len0;      // the log header's maxKeyLen before the batch
  uint8_t* out;              // the records, from the log's current end
  // workspace
  int64_t* keymax;           // n
  int64_t* keymax_pre;       // n: exclusive prefix max of keymax
  uint32_t* sizes;           // n
  uint64_t* off;             // n: exclusive prefix of sizes
  uint64_t* total;           // 1
  int64_t* partials;         // 6 per 256 ops
  int64_t* sums;             // 16: numPuts, numDeletes, putSize, deleteSize, maxKeyLen, maxValueLen, .., [8] scan total
  uint64_t* scan_u64;
  int64_t* scan_i64;
  uint32_t* map;             // per aligned 16-byte output word: its first op
  uint64_t nwords;
  uint32_t mis;              // d_out % 16
};

void launch_append_sizes(const AppendParams& A, hipStream_t s);
void launch_append_write(const AppendParams& A, hipStream_t s);

}  // namespace sk
