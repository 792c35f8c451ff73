// snappy.hpp -- SNAPPY log front end.
//
// A SNAPPY log is 84 header bytes, then blocks VLQ(compressedSize) || Snappy stream from offset 84 to
// dataEnd (CompressedOutputStream.flush, CompressedOutputStream.java:47-58).  The device front end
// turns it into the "virtual log": 84 header bytes and every block's decompressed bytes back to back,
// which is byte for byte the record stream of a NONE log (blocks split records only where the writer
// splits them, CompressedWriter.java:59-124).  The normal build runs over the virtual log; a last pass
// rewrites each slot's address from its virtual offset to the reference's
// (blockPosition << entryBlockBits) | entryIndex (IndexHash.java:270-283,
// CompressedReader.getBlockPosition CompressedReader.java:121-126).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {

struct SnappyBlock {
  int64_t file_pos;   // offset of the block's VLQ in the log file (the address's position part)
  int64_t data;       // offset of the Snappy stream
  int64_t voff;       // offset of the decompressed bytes in the virtual log
  uint32_t clen;      // Snappy stream bytes
  uint32_t ulen;      // decompressed bytes (the stream's preamble)
};

// per-block result of the decode kernel's record walk (the walk assumes the block starts a record)
struct SnappyWalk {
  uint32_t count;     // records started in the block
  uint32_t flags;     // kWalk* bits
  int64_t overflow;   // bytes of the last record past the block end
};

constexpr uint32_t kWalkBadHeader = 1u;    // a record header runs past the block end or a VLQ > 5 bytes
constexpr uint32_t kWalkTooMany = 2u;      // more records than maxEntriesPerBlock
constexpr uint32_t kWalkBadStream = 4u;    // malformed Snappy stream
constexpr uint32_t kWalkEofFirst = 8u;     // the block ends inside a record's first VLQ: the iterator ends there
                                           // when it is the log's last block (SparkeyLogIterator.java:111-115)

// The directory's state between k_snappy_dir launches (each follows the chain for up to a chunk of
// blocks, so that the decode of one chunk overlaps the walk along the next).
struct SnappyDirResult {
  uint64_t nblk;      // blocks found so far
  uint64_t total;     // their decompressed bytes
  int64_t p;          // offset of the next block header (0: not started)
  int32_t err;        // 0 ok, 1 corrupt block framing, 2 block larger than the reader's buffers,
                      // 3 the decompressed bytes exceed vcap
  int32_t done;       // the chain reached dataEnd
};

struct SnappyParams {
  const uint8_t* log;
  int64_t log_len;          // readable bytes of `log` (vector loads stay inside)
  int64_t data_end;
  int64_t win0;             // parallel directory: the first window's start (84; a rank's range start when sharded)
  int64_t max_block;        // compressionBlockSize: the reader's uncompressed buffer
  SnappyBlock* blocks;
  uint64_t blk_cap;
  uint64_t dir_limit;       // k_snappy_dir stops at this many blocks
  int64_t vcap;             // decompressed bytes the virtual log holds (< 0: unbounded)
  uint64_t blk_base;        // decode launches: first block
  SnappyDirResult* dir;
  uint8_t* vlog;            // virtual log (84 header bytes written by the host)
  int64_t vlog_len;         // bytes of vlog
  SnappyWalk* walk;
  uint32_t* rec_off;        // [block * mepb + j]: record j's offset inside block
  uint32_t mepb;            // maxEntriesPerBlock (>= 1)
  uint32_t lds_bytes;       // k_snappy_lds: staged stream + output bytes
  // address rewrite
  const uint8_t* itab;      // internal table (slot layout ihs + ias)
  uint8_t* otab;            // final table (hs + as)
  uint64_t cap;
  int32_t ihs, ias, hs, as;
  int32_t ebb;
  uint64_t nblk;
  int32_t* err;             // rewrite: virtual offset not a record start
};

void launch_snappy_dir(const SnappyParams& S, hipStream_t s);
// the parallel directory (SNAPPY): window screen, anchors, links (count, then emit)
constexpr int kSdirCand = 32;
inline size_t sdir_screen_lds(int64_t H) { return (size_t)((H + 15 + 384 + 15) & ~15LL) + 16; }  // staged window
// (codec 0 SNAPPY, 1 ZSTD)
void launch_sdir_screen(const SnappyParams& S, hipStream_t s, int codec, int64_t A, int64_t H, uint64_t nwin,
                        int64_t* cand, int32_t* ncand);
void launch_sdir_anchor(const SnappyParams& S, hipStream_t s, int codec, int64_t A, int64_t H, uint64_t nwin,
                        const int64_t* cand, const int32_t* ncand, int64_t* anchor);
void launch_sdir_link(const SnappyParams& S, hipStream_t s, int codec, const int64_t* ends, uint64_t nlinks, int emit,
                      uint64_t* cnt, uint64_t* usum, const uint64_t* boff, const uint64_t* uoff, int32_t* fail);
// ZSTD logs (zstd_kernels.hip): the same directory with sizes from the frame headers, and the decode
void launch_zstd_dir(const SnappyParams& S, hipStream_t s);
hipError_t launch_zstd_decode(const SnappyParams& S, hipStream_t s);
uint32_t zstd_lds_bytes(int64_t max_block);  // dynamic LDS of the in-LDS decode (0: too large, global)
// blocks [blk_base, blk_base + nblk), one wave per block: LDS-staged when lds_bytes > 0, else
// lane-serial in global memory
hipError_t launch_snappy_decode(const SnappyParams& S, hipStream_t s);
// blocks [0, nblk): their records
void launch_snappy_walk(const SnappyParams& S, hipStream_t s);
void launch_snappy_rewrite(const SnappyParams& S, hipStream_t s);
// sharded compressed logs: a rank's blocks [0, nblk) with virtual offsets from
// blocks[0].voff.  to_real: the address field (second word) of n records of stride_words 8-byte
// words ((hash, address) entries, or the exact path's exchange records), a virtual offset, becomes
// (blockPosition << ebb) | entryIndex, a DELETE mark kept; *err |= 1 when it is not a record start.
// to_virtual: n such compressed-log addresses back to virtual offsets (an address of no block here:
// all ones, which no rank decodes).
void launch_cz_to_real(const SnappyParams& S, hipStream_t s, uint64_t* records, uint64_t n, uint32_t stride_words,
                       int32_t* err);
void launch_cz_to_virtual(const SnappyParams& S, hipStream_t s, uint64_t* addrs, uint64_t n);

}  // namespace sk
