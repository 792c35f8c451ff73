/*
 * sparkey_gpu.h -- C-ABI of the MI355X-native Sparkey hash-file (.spi) builder.
 *
 * Drop-in boundary: these entry points replace the package-private static
 *   IndexHash.createNew(File indexFile, File logFile, HashType hashType, double sparsity,
 *                       boolean fsync, int hashSeed, long maxMemory, ConstructionMethod method)
 * (spotify/sparkey-java src/main/java/com/spotify/sparkey/IndexHash.java:131-167), whose only
 * caller is SingleThreadedSparkeyWriter.writeHash (SingleThreadedSparkeyWriter.java:89-108).
 * The JNI binding a maintainer adds at that call site is shown in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes only; 0 = success, negative = error code below, with a
 * message copied into `err` (nullable).  The library owns every device allocation it makes and
 * frees it before returning, except inside an explicit sparkey_plan (device-resident API).
 * Writers are single-threaded in the reference (Sparkey.java:36); calls on different writers or
 * plans may run concurrently.
 */
#ifndef SPARKEY_GPU_H
#define SPARKEY_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPARKEY_GPU_ABI_VERSION 1

/* Error codes -> the reference's exception (see INTEGRATION.md for the JNI mapping). */
#define SPARKEY_OK 0
#define SPARKEY_E_NOT_LOG (-1)        /* IOException "File is not a Sparkey log file" LogHeader.java:57-60 */
#define SPARKEY_E_VERSION (-2)        /* IOException "Incompatible major/minor version" LogHeader.java:61-68 */
#define SPARKEY_E_CORRUPT_LOG (-3)    /* IOException "Corrupt log file" LogHeader.java:81-83 / framing errors */
#define SPARKEY_E_NO_FREE_SLOTS (-4)  /* IOException "No free slots in the hash" IndexHash.java:574-576,664 */
#define SPARKEY_E_CORRUPT_DATA (-5)   /* RuntimeException "Corrupt data" / "reference to delete entry" IndexHash.java:484,494,613,624 */
#define SPARKEY_E_VLQ (-6)            /* RuntimeException "Too long VLQ value" Util.java:181,217 */
#define SPARKEY_E_HEADER (-7)         /* IOException "Too large max key len" CommonHeader.java:38-43 */
#define SPARKEY_E_UNSUPPORTED (-8)    /* compressed (SNAPPY/ZSTD) logs: not on this path */
#define SPARKEY_E_IO (-9)             /* IOException from file open/read/write */
#define SPARKEY_E_GPU (-10)           /* HIP runtime error or no gfx950 device */
#define SPARKEY_E_ARG (-11)           /* IllegalArgumentException (bad hash size etc.) */
#define SPARKEY_E_BUFFER (-12)        /* caller buffer too small */

/* ConstructionMethod (SparkeyWriter.java ConstructionMethod enum) */
#define SPARKEY_METHOD_AUTO 0
#define SPARKEY_METHOD_IN_MEMORY 1
#define SPARKEY_METHOD_SORTING 2

typedef struct sparkey_build_opts {
  int32_t hash_size;   /* 0 = auto (hashType == null: numPuts < 2^23 ? 4 : 8), 4 or 8 */
  int32_t hash_seed;   /* already resolved by the writer (non-zero) */
  double sparsity;     /* clamped to >= 1.3 like IndexHash.java:135-137 */
  int64_t max_memory;  /* already resolved (>= 10 MiB); only decides AUTO */
  int32_t method;      /* SPARKEY_METHOD_* */
  int32_t device;      /* HIP device ordinal */
} sparkey_build_opts;

typedef struct sparkey_build_stats {
  int64_t num_records;        /* records framed from the log (puts + deletes) */
  int64_t num_puts;
  int64_t num_deletes;
  int64_t num_entries;        /* IndexHeader.numEntries */
  int64_t capacity;           /* IndexHeader.hashCapacity */
  int64_t garbage_size;
  int64_t max_displacement;
  int64_t hash_collisions;
  int64_t total_displacement;
  int32_t hash_size;
  int32_t address_size;
  int32_t placement_path;     /* 0 = parallel canonical placement, 1 = sequential device restatement */
  int32_t framing_path;       /* 0 = speculative parallel framing, 1 = serial device walker */
  double device_ms;           /* device time of the build (HIP events), excluding copies */
} sparkey_build_stats;

/* file -> file.  What the JNI shim calls in place of IndexHash.createNew; the Java side keeps
 * the tmp-file naming and Util.renameFile.  `fsync` applies to index_out_path. */
int sparkey_build_index_file(const char* log_path, const char* index_out_path, const sparkey_build_opts* opts,
                             int32_t fsync, sparkey_build_stats* stats_out, char* err, size_t err_len);

/* host memory -> host memory (log bytes in, full .spi bytes out: 112-byte header + slots). */
int sparkey_build_index_mem(const uint8_t* log, uint64_t log_len, uint8_t* index_out, uint64_t index_cap,
                            const sparkey_build_opts* opts, sparkey_build_stats* stats_out, char* err,
                            size_t err_len);

/* .spi size for a log (needs only its 84-byte header): 112 + slotSize * capacity, or < 0. */
int64_t sparkey_index_size(const uint8_t* log_header, uint64_t header_len, const sparkey_build_opts* opts);

/* ---- device-resident API (bench / embedding): workspace kept in a plan ---- */
typedef struct sparkey_plan sparkey_plan;

/* Allocates device workspace for logs up to max_log_bytes and max_records records. */
int sparkey_plan_create(sparkey_plan** plan_out, int32_t device, uint64_t max_log_bytes, uint64_t max_records,
                        char* err, size_t err_len);
/* d_log / d_index_out are device pointers; log_header is a HOST copy of the log's first 84 bytes.
 * `stream` is a hipStream_t (NULL = the plan's own stream).  Synchronises `stream` before returning. */
int sparkey_plan_build_device(sparkey_plan* plan, const uint8_t* log_header, const uint8_t* d_log, uint64_t log_len,
                              uint8_t* d_index_out, uint64_t index_cap, const sparkey_build_opts* opts,
                              void* stream, sparkey_build_stats* stats_out, char* err, size_t err_len);
/* Per-stage device times of the last build (HIP events on the build stream); enable first. */
void sparkey_plan_set_profiling(sparkey_plan* plan, int32_t enabled);
int32_t sparkey_plan_stage_count(const sparkey_plan* plan);
const char* sparkey_plan_stage_name(const sparkey_plan* plan, int32_t i);
double sparkey_plan_stage_ms(const sparkey_plan* plan, int32_t i);
void sparkey_plan_destroy(sparkey_plan* plan);

const char* sparkey_gpu_version(void);
const char* sparkey_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif
