// shard_host.hpp -- internal interface of the sharded build's host orchestration (shard_host.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/sparkey_gpu.h"

// One rank's view of the collectives the sharded build needs.  Buffers are device memory; both calls
// are ordered on `s` (the thread transport synchronises it).  0 or a SPARKEY_E_* code with *why set.
class Coll {
 public:
  int rank = 0, world = 1;
  virtual ~Coll() = default;
  // every rank's `bytes` bytes at d_send -> d_recv (world * bytes, in rank order)
  virtual int all_gather(const void* d_send, void* d_recv, size_t bytes, hipStream_t s, std::string* why) = 0;
  // send_bytes[r] bytes to rank r (consecutive runs of d_send in rank order); recv_bytes[r] bytes from
  // rank r (consecutive runs of d_recv in rank order)
  virtual int all_to_all(const uint8_t* d_send, const uint64_t* send_bytes, uint8_t* d_recv, const uint64_t* recv_bytes,
                         hipStream_t s, std::string* why) = 0;
  // releases every rank waiting in a collective (thread transport) after a failure outside one
  virtual void abort() {}
};

// slots [lo, hi) owned by `rank` of `world` for a table of `cap` slots: an even split of the
// placement's coarse digits (sparkey_gpu.cpp)
void shard_slot_split(uint64_t cap, int world, int rank, uint64_t* lo, uint64_t* hi);

// runs fn(rank, world, device, comm, err, err_len) for every rank of opts.num_gpus on its own thread
// (devices opts.device .. + num_gpus - 1, RCCL between them; SPARKEY_SHARD_TRANSPORT=threads: the
// in-process transport; =threads-one-device: every rank on opts.device, for tests on one GPU)
// (shared_device: every rank runs on the same device, so concurrent builds share it)
using ShardRankFn = std::function<int(int rank, int world, int device, sparkey_shard_comm* comm, bool shared_device,
                                      char* err, size_t err_len)>;
int shard_run_threads(const sparkey_build_opts& o, const ShardRankFn& fn, char* err, size_t err_len);
// frees the cached communicator groups (a group in use is freed when its build ends)
void shard_release_groups();
// sparkey_shard_build with the rank's own earlier failure rc0 (!= 0: err holds it; the rank still
// meets the other ranks at the first checkpoint so that they all fail together); plan may be NULL then
int shard_build_rank(sparkey_plan* plan, sparkey_shard_comm* comm, const uint8_t* log_header, uint64_t file_len,
                     const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi, const sparkey_build_opts* opts,
                     uint8_t* d_out, uint64_t out_cap, void* stream, sparkey_build_stats* stats_out, int rc0, char* err,
                     size_t err_len);
// the plan's ranks share their device with other builds: framing takes regions by ticket (sparkey_gpu.cpp)
void sk_plan_set_shared_device(sparkey_plan* plan, bool shared);

// Sharded compressed logs (sparkey_gpu.cpp).  0 or a SPARKEY_E_* code; a log these
// steps do not take (a missed link, a record spanning two ranks' blocks, an irregular block) is
// reported through *ok / *carry / *entry and built by the gathered path instead (DELETEs and
// overwrites take the sharded exact path, with the exchange records' addresses rewritten too).
// the hop bound H of the block chain (0: a NONE log, or blocks the parallel directory does not take)
int64_t sk_cz_hop_bound(const uint8_t* log_header);
// screen and anchors of [lo, hi) from the rank's compressed bytes [buf_lo, buf_hi); *entry: its first
// anchor (84 on rank 0, dataEnd when lo >= dataEnd, -1 none)
int sk_cz_entry(sparkey_plan* pl, const uint8_t* log_header, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo,
                uint64_t buf_hi, int64_t lo, int64_t hi, int32_t rank, hipStream_t s, int64_t* entry, char* err,
                size_t err_len);
// the chain from entry through the rank's anchors to next: *ok = 1 when every link lands on its end
int sk_cz_count(sparkey_plan* pl, int64_t entry, int64_t next, hipStream_t s, int32_t* ok, uint64_t* nblk,
                uint64_t* ulen, char* err, size_t err_len);
// the counted blocks decoded into the virtual log's slice from vbase; *carry: bytes of the last record
// past the rank's last block (-1: an irregular block)
int sk_cz_decode(sparkey_plan* pl, int64_t vbase, hipStream_t s, int64_t* carry, char* err, size_t err_len);
// sparkey_shard_begin over the slice (the virtual log is vlen bytes long), the table of the compressed log
int sk_cz_shard_begin(sparkey_plan* pl, const uint8_t* log_header, uint64_t file_len, uint64_t vlen,
                      const sparkey_build_opts* opts, int32_t rank, int32_t world, char* err, size_t err_len);
// n records of rec_bytes (16: (hash, address) entries; the exact path's exchange records), address in
// their second 8-byte word: virtual offsets -> (blockPosition << entryBlockBits) | entryIndex
int sk_cz_to_real(sparkey_plan* pl, uint8_t* d_records, uint64_t n, uint32_t rec_bytes, hipStream_t s, char* err,
                  size_t err_len);
// n compressed-log addresses of this rank's blocks -> virtual offsets (sparkey_shard_fetch_keys)
int sk_cz_to_virtual(sparkey_plan* pl, uint64_t* d_addrs, uint64_t n, hipStream_t s, char* err, size_t err_len);
