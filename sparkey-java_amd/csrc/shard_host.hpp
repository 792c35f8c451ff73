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
