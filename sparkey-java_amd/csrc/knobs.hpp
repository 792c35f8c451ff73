// knobs.hpp -- the library's test and diagnostic switches, in one place.
//
// No switch changes the bytes of a build: each forces a device path, a launch shape or a geometry
// that the default choice would not take, so that the parity tests reach every path and the
// measurement tools can compare variants.  They are set through the C-ABI (sparkey_debug_set, for
// tests) or once, when the library first reads a switch, from SPARKEY_DEBUG="name=value,..." (for
// tools).  Apart from SPARKEY_DEBUG the library reads one environment variable, SPARKEY_FILE_CACHE
// (include/sparkey_gpu.h), so a JVM that loads it inherits no other build choice.
#pragma once

#include <stdint.h>

namespace sk {

enum class Knob : int {
  NoUniform,        // the uniform-record framing off (k_frame3 / k_frame frame such logs)
  NoFrame3,         // k_frame3 off (k_frame frames one-byte-VLQ logs)
  SerialFraming,    // the exact serial walk for every log
  FrameCmin,        // k_frame: smallest chunk (bytes)
  FrameRegion,      // k_frame / k_frame3: bytes of chunks per wave
  FrameLook,        // k_frame: look-ahead of the speculative walks (bytes)
  Frame3C,          // k_frame3: chunk (bytes)
  Frame3Short,      // k_frame3: steps of the short walk
  Frame3Cover,      // k_frame3: mark reached starts (0 / 1)
  Frame3Stop,       // k_frame3: stop after this phase (instruction counts by phase)
  FrameTicket,      // k_frame / k_frame3: regions by device-wide ticket, not by workgroup id
  FrameSpinTicks,   // bound on a wave's wait for its predecessor (100 MHz ticks)
  FrameDebug,       // k_frame / k_frame3 per-wave phase counters to stderr
  Part2Debug,       // k_part2s phase counters to stderr
  NoRegions,        // partition pass 1 into digit regions off (two-pass histogram partition)
  NoBuckets,        // k_frame3 into the bucket regions off (digit regions and the two-pass partition)
  RegionCap,        // digit region capacity (entries; tests force overflows)
  ExactSerial,      // the exact path on one lane over the whole table
  ExactDebug,       // exact path phase counters (2: synchronise each class)
  ExactReframe,     // sharded exact path frames again instead of reusing the slabs
  ExactFullTable,   // sharded exact path: full-capacity replay table
  SnappyLds,        // SNAPPY decode with the block in LDS (k_snappy_lds)
  SnappyDirA,       // parallel block directory: window spacing (bytes)
  SnappyDirDebug,   // parallel block directory summary to stderr
  SnappyChunk,      // serial block directory: blocks per launch
  SnappySerialDir,  // the serial block directory
  ZstdLds,          // ZSTD decode with block and frame in LDS
  ShardSyncFrame,   // sharded build: every speculative framing attempt retried synchronously
  ShardTransport,   // num_gpus > 1: 0 RCCL, 1 threads (one device each), 2 threads on one device
  ShardFailRank,    // num_gpus > 1: this rank fails its load (tests of the ranks failing together)
  FileThreads,      // file entry points: reader pool size
  FileWriteThreads, // file entry points: index writer threads
  FileDebug,        // file entry points: phase times to stderr
  ReframeSpinTicks, // FrameSpinTicks for the exact path's second framing only (tests of its fallbacks)
  ShardGatherCompressed,  // num_gpus > 1: compressed logs gathered on every rank (the sharded path off)
  InjectForeign,    // tests of the kGuardForeign check: a foreign entry in digit region 0 (1) or bucket region 0 (2)
  ShardCollFail,    // host transport (HostColl): the k-th collective of a communicator fails its device copy (tests)
  NoCompact,        // 16-byte entries on the uniform staged path too (BuildParams.compact off)
  Part2TwoLevel,    // pass 2 through sub-digit regions: 1 forces it (any table: tests), 0 keeps k_part2f_direct
  kCount
};

// The switch's value, or -1 when it is not set.
int64_t knob(Knob k);
inline bool knob_on(Knob k) { return knob(k) > 0; }
inline bool knob_set(Knob k) { return knob(k) >= 0; }

}  // namespace sk
