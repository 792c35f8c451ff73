/* Test-only stand-in for libsparkey_gpu's file entry point: records the arguments the JNI shim passes
 * and returns the code in $FAKE_RC (with a message), so every SPARKEY_E_* code's exception mapping can
 * be checked without a GPU. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sparkey_gpu.h"

int sparkey_build_index_file(const char* log_path, const char* index_out_path, const sparkey_build_opts* o,
                             int32_t fsync, sparkey_build_stats* st, char* err, size_t err_len) {
  printf("{\"call\": {\"log\": \"%s\", \"index\": \"%s\", \"hash_size\": %d, \"hash_seed\": %d, \"sparsity\": %.17g, "
         "\"max_memory\": %lld, \"method\": %d, \"device\": %d, \"num_gpus\": %d, \"fsync\": %d}}\n",
         log_path, index_out_path, o->hash_size, o->hash_seed, o->sparsity, (long long)o->max_memory, o->method,
         o->device, o->num_gpus, fsync);
  const int rc = getenv("FAKE_RC") ? atoi(getenv("FAKE_RC")) : 0;
  if (rc) {
    snprintf(err, err_len, "fake failure %d", rc);
    return rc;
  }
  st->num_records = 11; st->num_puts = 10; st->num_deletes = 1; st->num_entries = 9; st->capacity = 13;
  st->garbage_size = 5; st->max_displacement = 2; st->hash_collisions = 1; st->total_displacement = 7;
  return 0;
}

const char* sparkey_strerror(int code) { (void)code; return "fake strerror"; }
