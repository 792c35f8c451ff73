// build_kernels.hpp -- device data layout and launchers of the .spi build pipeline.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "device_common.hpp"

namespace sk {

constexpr int kChunkShift = 12;                   // framing chunk: 4 KiB of log bytes
constexpr int kChunk = 1 << kChunkShift;
constexpr int kEmitExtra = 1024 + 16;             // bytes staged past a chunk for headers + keys
constexpr int kBucketShift = 10;                  // placement bucket: 1024 slots
constexpr int kBucket = 1 << kBucketShift;
constexpr int kPlaceBlock = 256;
constexpr int kBinsPerThread = kBucket / kPlaceBlock;
constexpr uint32_t kGroupMax = 64;                // equal-wanted-slot group sorted by insertion
constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr uint64_t kScanTile = (uint64_t)kScanBlock * kScanItems;
constexpr int kStatBlock = 256;
constexpr int kStatSlotsPerBlock = 4096;
constexpr int kPartBlock = 256;                   // radix partition of the entries by bucket
constexpr int kPartItems = 16;
constexpr int kPartTile = kPartBlock * kPartItems;
constexpr int kPart2Block = 1024;                 // k_part2: one workgroup per coarse digit
constexpr int kPart2Items = 8;                    // k_part2: entries per thread per round
constexpr uint32_t kP2SortedMaxBpp = 64;          // k_part2s: buckets per digit (16-bit counts: 2 KB each)
constexpr int kPart2MaxBits = 14;                 // fine digit of the partition (<= 16384 buckets)
constexpr uint32_t kPlaceLdsMax = 1024;           // entries of a bucket staged in LDS (load <= 1/1.3: mean 788)
constexpr uint32_t kMaxPartGroup = 64;
constexpr int kCandCap = 448;                     // k_frame balanced walk: candidates (and listed records) per wave

// One log record as the placement sees it: 16 bytes, AoS so every access is one dwordx4.
struct alignas(16) Entry {
  uint64_t hash;  // HashType.hash of the key (32-bit hashes zero-extended)
  uint64_t addr;  // position << entryBlockBits (| kDelBit for DELETE records)
};
// The entry of a uniform log between the framing and the placement (BuildParams.compact): 12 bytes,
// the record index in place of the address, which is (fr_entry + idx * uni_rec) << entryBlockBits --
// every record of such a log has the same size and none is a DELETE (k_frame_uniform's condition).
// One 3-dword access per entry (a hash array and an index array per region measured slower: the
// framing's write-out and the partition both lost more than the single stride costs,
// profiles/r06/c2/compact_soa_ab.txt).
struct CEntry {
  uint32_t h0, h1;  // the hash, low and high words
  uint32_t idx;     // record index in the log
};
static_assert(sizeof(CEntry) == 12, "12-byte compact entries");
constexpr int kCompactIn = 1, kCompactOut = 2;  // BuildParams.compact's bits
constexpr uint32_t kSub = 64;                   // two-level pass 2: sub-digit regions a coarse digit

// Carry function f(x) = max(c, x + a) of a bucket (see k_summary).
struct MaxPlus {
  int64_t c;
  int64_t a;
};

// A slot written outside the rank's slot range in a sharded build: sent to the slot's owner.
struct alignas(16) SpillEntry {
  uint64_t slot;
  uint64_t hash;
  uint64_t addr;
  uint64_t pad;
};

// sharded build rows (sharded.py): the frame's scalars {entry, frame end, exit, records, deletes, rc,
// error position, retry (a speculative attempt that must be redone synchronously)}, and the placement flags {spilled, pairs, non-canonical, aborted} before the
// inline spilled slots
constexpr int kShardScalars = 8;
constexpr int kShardFlags = 4;
struct ShardScalars {
  int64_t v[kShardScalars];
};

constexpr int kIndexHeaderBytes = 112;
struct IndexHeaderBytes {  // the .spi header template (IndexHeader.asBytes), by value into a kernel
  uint8_t b[kIndexHeaderBytes];
};

constexpr unsigned kSpecRegionFull = 8u;  // Status.spec_fail: a digit region of ent3 overflowed

struct StatPart {
  unsigned long long sum_disp;
  unsigned long long collisions;
  long long max_disp;
};

// Device-side build status, read back once per build.
struct Status {
  unsigned long long err;  // min over (position << 8 | -code); ~0 = none
  unsigned int spec_fail;  // speculative framing disagreed with the verified chain
  unsigned int dup;        // two PUTs with the same key (canonical layout does not apply)
  unsigned int dup_overflow;
  unsigned int full;       // records >= capacity
  unsigned int overflow;   // more records than workspace
  unsigned int big_buckets;  // some bucket exceeded kPlaceLdsMax (placed by the global kernel)
  unsigned long long n_records;
  unsigned long long n_deletes;
  unsigned long long n_pairs;
  long long num_entries;
  long long garbage;
  long long max_disp;
  long long collisions;
  long long total_disp;
  unsigned int max_wave_count;  // largest per-wave record count when a slab overflowed
  unsigned int pad2;
  long long exit;                // first record start >= the frame end on the framed chain
  unsigned long long n_spill;    // sharded placement: slots written outside the rank's range
  unsigned long long n_segs[4];  // exact path: segments per size class (small, mid, large, huge)
  unsigned int guard;            // exact path: bounds-check bits that tripped (a bug; fails the build)
  unsigned int need_summary;     // k_part2s left a digit unsummarised (k_summary runs)
  unsigned int p2_overflow;      // k_part2s fixed bucket regions: a bucket outgrew its region (redo dense)
  unsigned int stats_pending;    // folded stats could not cover every slot (big buckets): k_stats runs
  unsigned int stats_ticket;     // k_stats_folded: blocks done
  unsigned long long acc_sum, acc_col, acc_max;  // k_stats_folded: totals over its blocks
  unsigned int p2_ticket;        // fused_carry: k_part2s blocks done (the last composes the digits)
  unsigned int pad3;
  unsigned int seg_next[4];      // exact path: the next listed segment of each size class (work queue)
};

struct BuildParams {
  // input log (device) and its header fields (LogHeader.java:55-88)
  const uint8_t* log;
  uint64_t log_len;
  int64_t data_end;
  int64_t max_key_len;
  int64_t max_value_len;
  int64_t max_rec_len;  // longest possible record, bounds the speculative entry window
  uint64_t nchunks;
  int32_t emit_extra;
  // index parameters (IndexHash.createNew, IndexHash.java:131-150)
  int32_t hash_size;
  int32_t addr_size;
  int32_t slot_size;
  int32_t ebb;
  int32_t seed;
  FastMod mod;
  uint64_t cap;
  uint64_t nbuckets;
  uint8_t* out;  // .spi image: 112-byte header + cap slots (device)
  Status* st;
  // framing workspace (per chunk)
  uint8_t* conv;
  int64_t* exitp;
  int64_t* qpos;
  uint32_t* tail;
  int64_t* G;
  uint32_t* cnt;
  uint64_t* off;
  // entries
  Entry* ent;   // log order, in slabs: slab w holds wcount[w] entries at ent[w * slab_cap]
  Entry* ent2;  // grouped by bucket (dense)
  Entry* ent3;  // partition pass-1 output; sorted by (wanted, address) within bucket for SORTING
  uint64_t max_records;  // capacity of ent2 / ent3 (dense)
  uint64_t ent_cap;      // capacity of ent
  uint32_t* wcount;      // entries per slab
  uint64_t* woff;        // exclusive prefix of wcount (+ total at [nslabs])
  uint32_t slab_cap;
  uint32_t part_group;   // slabs per partition tile
  uint32_t p1r_group;    // k_part1_regions: slabs per tile (<= 2 kPartTile entries, taken kPartTile at a time)
  uint32_t p1r_tiles;
  uint64_t nslabs;
  // buckets
  uint32_t* bcount;
  uint32_t* bcursor;
  uint64_t* boff;  // nbuckets + 1
  MaxPlus* bfun;
  MaxPlus* bpre;
  MaxPlus* bfun_total;
  // fused_carry (single GPU, k_part2s in one pass): k_part2s leaves bpre = each bucket's exclusive
  // prefix function inside its digit and dfun = each digit's composed function; its last block
  // composes the 256 digits around the ring into dcarry (each digit's carry-in), and k_place_reg
  // takes carry = bpre[b](dcarry[digit]) -- no k_summary / scan / k_carry launches
  MaxPlus* dfun;         // (as 256 packed words, see part2_fused_carry)
  int64_t* dcarry;
  int32_t fused_carry;
  uint32_t epoch;        // fused_carry: this build's number (1 .. 2^22 - 1), tags the dfun words
  int64_t* carry;
  uint64_t* pairs;
  uint64_t pair_cap;
  StatPart* parts;
  unsigned long long* part_dbg;   // part2_debug switch: k_part2s phase cycles, 8 words per digit
  uint64_t* scan_scratch_u64;
  MaxPlus* scan_scratch_mp;
  // k_frame granules (zeroed before every launch)
  unsigned long long* exit_desc;
  unsigned int* frame_ticket;     // k_frame wave tickets (zeroed with the granules)
  // the framing kernels' DELETE counts: kDelParts counters 128 B apart (wave wv adds to wv % kDelParts),
  // summed into st->n_deletes by launch_sum_deletes -- one device-wide counter serialised 131K atomics
  // per 10M-record churn log (1.0 ms of k_frame3's 1.65)
  unsigned long long* del_parts;
  unsigned long long fr_spin_ticks;  // bound on a wave's wait for its predecessor (100 MHz ticks)
  // radix partition
  uint32_t* p1_hist;  // [256][p1_tiles]
  uint64_t* p1_off;
  uint64_t* p1_off_total;
  uint32_t p1_tiles;
  int32_t p1_hist_ready;  // the framing kernel filled p1_hist (zeroed before it): no k_part1_hist
  // k_part2 over a sharded build's exchange buffer (null: the pass-1 runs): for each of the rank's
  // p2_nd coarse digits from p2_d0, p2_nsrc (begin, end) runs of ent3, and the digit's ent2 start
  const uint64_t* p2_seg;
  const uint64_t* p2_out;  // p2_nd + 1
  uint32_t p2_nsrc, p2_d0, p2_nd;
  uint32_t bpp;       // buckets per coarse digit: digit = bucket / bpp (< 256), computed as
  uint64_t dmagic;    // (bucket * dmagic) >> 40, dmagic = ceil(2^40 / bpp), exact for bpp < 2^18
  unsigned long long* dbg;  // diagnostic phase counters (frame_debug switch), else null
  // k_frame geometry (chunk C = 2^fr_cshift bytes, fr_w chunks per wave)
  int32_t fr_cshift;
  int32_t fr_w;
  int32_t fr_look;       // speculative walks continue this many bytes past their chunk
  int32_t fr_rgn_bytes;  // LDS region per wave: W * C + fr_look + 16, rounded up to 1 KiB
  int32_t fr_mask_words;  // 64-position screen words per chunk: ceil(min(C, maxRecLen) / 64)
  uint32_t fr_wpc_magic;  // q / (8 * fr_mask_words) == (q * magic) >> 22 for every screened word q
  int32_t fr_fast;  // maxKeyLen + 1 < 128 and maxValueLen < 128: canonical headers are 2 bytes
  int32_t no_deletes;  // the log header counts no DELETE: speculation treats 0x00 as no record start
  uint64_t fr_nchunks;
  int32_t f3_short;  // k_frame3 (frame3_kernels.hip): steps of the short walk
  int32_t f3_cover;  // k_frame3: mark the starts the short walk reached (windows hold several true starts)
  int32_t f3_stop;   // frame3_stop switch: k_frame3 gives up after this phase (instruction counts by phase)
  int32_t f3_rgn;    // k_frame3: staged region bytes per wave (W * C + fr_look + 16, 16-byte multiple)
  int32_t f3_cand_cap;  // k_frame3: candidates (and records) per wave its LDS list holds (<= 512)
  int32_t f3_surv_cap;  // k_frame3: chain heads per wave after the short walk (<= 64, one long walk per lane)
  int32_t f3_lcap;      // k_frame3: record starts a head lists inside its chunk (16 .. 128)
  int32_t fr_ticket;    // k_frame / k_frame3: regions by device-wide ticket, not by workgroup id (builds that
                        // share the device, or the frame_ticket switch)
  // uniform-stride framing (k_frame_uniform): uni_n records of uni_rec bytes from fr_entry
  uint64_t uni_n;
  int64_t uni_rec;
  uint32_t uni_wbytes;    // LDS staging bytes per wave (set by the launcher)
  uint32_t uni_hist_off;  // LDS offset of the digit counts (set by the launcher)
  uint32_t uni_nt;        // framing kernels: non-temporal LDS-DMA of the log (read once)
  // k_frame_uniform as partition pass 1: digit d's entries at ent3[d * p1_region, + p1_fill[d])
  uint64_t p1_region;   // 0 = off
  int32_t p1_kernel;    // with p1_region: k_part1_regions fills the regions from the slabs (else the framing did)
  int32_t p1_pad;
  int32_t p2_sorted;    // k_part2s: per-(bucket, slot) counts in the same pass + the carry functions
  int32_t p1_bucket;    // k_frame3 writes each entry into its bucket's fixed region (no partition);
                        // bcount[] is the atomic cursor, zeroed before the framing
  int32_t p2_fixed;     // k_part2s in one pass: bucket b's entries at ent2[b * kPlaceLdsMax, + bcount[b])
  int32_t fold_stats;   // k_place_reg leaves calculateMaxDisplacement's per-bucket parts (no k_stats pass)
  Status* status_host;  // fold_stats: k_stats_folded also copies the status block here (pinned, mapped; else null)
  int32_t stats_if_pending;  // k_stats / k_stats_final only when the folded stats left stats_pending
  uint64_t* bstat_start;  // fold_stats: per bucket, the first slot of the range it wrote (~0: none)
  uint32_t* p1_fill;
  // framing window: records start at fr_entry (84 for a whole log) and are framed while they start
  // below data_end (the frame end); k_frame chunks are numbered from fr_k0 = fr_entry >> fr_cshift,
  // serial-path chunks (kChunk) from ch_k0 = fr_entry >> kChunkShift
  int64_t fr_entry;
  uint64_t fr_k0;
  uint64_t ch_k0;
  // placement range: buckets [b_lo, b_hi), slots [slot_lo, slot_hi) (the whole table unless
  // sharded); in a sharded build slots outside the range go to the spill list, the carry into
  // b_lo is carry_in, and the slot before slot_lo is (prev_hash, prev_occ)
  int32_t sharded;
  int32_t prev_occ;
  uint64_t b_lo, b_hi;
  uint64_t slot_lo, slot_hi;
  int64_t carry_in;
  int32_t abort_on_fail;        // the bin after a speculative framing attempt: skip it when the attempt failed
  // 12-byte entries (CEntry) of single-GPU uniform logs (C2's, C4's): bit 0 (kCompactIn) the digit
  // regions (ent3: k_frame_uniform -> pass 2), bit 1 (kCompactOut) the bucket regions (ent2: pass 2 ->
  // k_summary / k_place_reg); every other path keeps 16-byte Entry
  int32_t compact;
  // two-level pass 2 (k_part2_sub -> k_part2f<.., kSubIn>, tables of thousands of buckets a digit): kSub sub-digit
  // regions of sub_region entries a digit in sub_ent, their fill cursors in sub_fill (0: one level)
  uint64_t sub_region;
  uint32_t* sub_fill;
  Entry* sub_ent;
  // sharded: the carry-in composed on the device from every rank's carry function (world x {c, a});
  // k_carry then also clears the placement's status counters
  const int64_t* carry_funs;
  int32_t carry_world, carry_rank;
  uint64_t prev_hash;
  SpillEntry* spill;
  uint64_t spill_cap;
  // exact path over independent slot segments (k_seg_*): the radix partition leaves DELETE records
  // out of the canonical placement when skip_del is set
  int32_t skip_del;
  uint64_t* eseg;     // per slab entry: first slot of its segment, or kNoSeg
  uint32_t* seg_cnt;  // per slot: records of the segment starting there
  uint64_t* seg_off;  // exclusive prefix of seg_cnt (cap + 1)
  int64_t* seg_mark;  // per slot: i + 1 when empty, else 0 (cap + 1: the max at [cap])
  int64_t* seg_start; // per slot: exclusive max-scan of seg_mark (first slot of its run, 0 = wraps)
  uint32_t* seg_cls_cnt;  // segment lists: per-workgroup counts [3][blocks], and their scan
  uint64_t* seg_cls_off;
  uint32_t* seg_len;    // per slot: distinct keys wanting it; then, at a segment's start, its length
  uint64_t* seg_first;  // per segment start: the placement slot of its first placed PUT record
  MaxPlus* seg_fun;     // per slot: the distinct-key carry functions composed before it (cap + 1)
  uint32_t* seg_krep;   // per placed record: slots back to the first placed record with its key (0: itself)
  uint32_t* ecls;       // per grouped record (ent3): its key's class, the rank of that first record in its segment
};

// Per-stage HIP events on the build stream (only when profiling is enabled).
struct StageTimer {
  bool enabled = false;
  std::vector<hipEvent_t> evs;
  std::vector<const char*> names;
  size_t used = 0;
  void begin(hipStream_t s) {
    used = 0;
    mark("begin", s);
  }
  void mark(const char* name, hipStream_t s) {
    if (!enabled) return;
    if (used == evs.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      evs.push_back(e);
      names.push_back(name);
    }
    names[used] = name;
    (void)hipEventRecord(evs[used], s);
    used++;
  }
  ~StageTimer() {
    for (auto e : evs) (void)hipEventDestroy(e);
  }
};

// fast path (fused_kernels.hip)
void launch_frame_fused(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_partition(const BuildParams& P, hipStream_t s, StageTimer* tm);
bool part2f_fits(uint32_t bpp);  // k_part2f's LDS for this many buckets a digit
int part2st_per(const BuildParams& P);  // k_part2st's stage (entries a thread), 0: pass 2 is another kernel
bool part2_direct(const BuildParams& P);  // pass 2 is k_part2f_direct
void launch_partition1(const BuildParams& P, hipStream_t s);
void launch_partition2(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_part2_recv(const BuildParams& P, hipStream_t s, StageTimer* tm);  // sharded receive, fixed regions
bool part2_recv_fits(uint32_t bpp);
void launch_dense_slabs(const BuildParams& P, hipStream_t s);
void launch_frame_uniform(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_frame3(const BuildParams& P, hipStream_t s, StageTimer* tm);  // frame3_kernels.hip
bool frame3_fits(BuildParams& P, double mean_record, double pass, double mean_short);
uint32_t frame3_lds_per_wave(const BuildParams& P);
// framing paths: 0 k_frame, 1 serial walk, 2 k_frame_uniform, 4 k_frame3 (3 and 5 were the k_frame2 and
// k_frame_lane experiments, measured slower and removed); the speculative ones with per-wave slabs
__host__ __device__ inline bool slab_framing(int path) { return path == 0 || path == 4; }
void launch_place_fast(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_place_buckets(const BuildParams& P, hipStream_t s);
void launch_inject_foreign(const BuildParams& P, hipStream_t s, int where);  // (inject_foreign switch, tests)
// fallbacks and shared stages (build_kernels.hip)
void launch_framing_serial(const BuildParams& P, hipStream_t s);
void launch_emit(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_summary_carry(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_carry(const BuildParams& P, hipStream_t s);
void launch_place_global(const BuildParams& P, hipStream_t s, int sort_only, int only_big);
void launch_verify(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_stats(const BuildParams& P, hipStream_t s, int sequential, StageTimer* tm);
void launch_stats_folded(const BuildParams& P, hipStream_t s, StageTimer* tm);
void launch_build_init(uint8_t* out, const uint8_t* hdr, Status* st, uint32_t* fill, uint32_t n, hipStream_t s);
void launch_status_out(const Status* st, Status* host, hipStream_t s);  // host: pinned, device-mapped
constexpr int kDelParts = 64;
void launch_sum_deletes(const BuildParams& P, hipStream_t s);
void launch_status_reframe(Status* st, hipStream_t s);  // the framing's status words reset (exact path reframe)
void launch_stats_folded_shard(const BuildParams& P, hipStream_t s);
// exact replay (exact_kernels.hip)
void launch_sequential(const BuildParams& P, hipStream_t s, int sorted_order);
// Streams the exact path forks its independent segment classes onto (owned by the plan).
struct SideStreams {
  hipStream_t s[3];
  hipEvent_t fork;
  hipEvent_t join[3];
};
void launch_segments(const BuildParams& P, hipStream_t s, int sorted_order, StageTimer* tm, bool check_each,
                     const SideStreams* side);
constexpr unsigned kSegDebugWaves[4] = {4096, 2048, 512, 4096};   // k_seg_replay_wave grids (mid, large, huge), k_seg_lanes
constexpr unsigned kSegDebugWords = (4096 + 2048 + 512 + 4096) * 8;  // SPARKEY_EXACT_DEBUG: per-wave phase cycles
void launch_partition_quiet(const BuildParams& P, hipStream_t s);
// sharded builds (shard_kernels.hip)
void launch_dest_counts(const BuildParams& P, hipStream_t s, int world, uint32_t nd, uint64_t* d_out);
void launch_apply_spill(const BuildParams& P, hipStream_t s, const SpillEntry* in, uint64_t n);
void launch_region_send(const BuildParams& P, hipStream_t s, int world, uint32_t nd, Entry* send, uint64_t* d_out,
                        uint64_t send_cap);
void launch_digit_starts(const BuildParams& P, hipStream_t s, uint64_t* d_out);
void launch_fetch_keys(const BuildParams& P, hipStream_t s, const uint64_t* addrs, uint64_t n, uint8_t* rec,
                       uint32_t rec_size);
void launch_compare_keys(const BuildParams& P, hipStream_t s, const uint8_t* rec, uint64_t npairs, uint32_t rec_size);
void launch_find_entry(const BuildParams& P, hipStream_t s, int64_t lo, int64_t cand_end, int64_t target, int64_t* d_out);
void launch_shard_row(hipStream_t s, const ShardScalars& sc, const uint64_t* off, int world, int have, int64_t* row);
void launch_shard_row_async(hipStream_t s, const ShardScalars& sc, const Status* st, int path, uint32_t slab_cap,
                            uint64_t max_records, uint64_t send_cap, int64_t data_end, const uint64_t* off, int world,
                            int64_t* row);
void launch_p2_table(hipStream_t s, const int64_t* dig, int stride, int G, uint32_t d0, uint32_t nk, uint64_t* tab,
                     Status* st, uint64_t n_records);
void launch_shard_flags(const BuildParams& P, hipStream_t s, int64_t* flags, int inline_cap);
void launch_apply_spill_rows(const BuildParams& P, hipStream_t s, const int64_t* rows, int world, int stride,
                             int inline_cap);
void launch_shard_summary_row(const BuildParams& P, hipStream_t s, const int64_t* flags, int64_t* out);
void launch_status_reset(hipStream_t s, Status* st, uint64_t n_records, uint32_t* fill = nullptr, int nfill = 0);
void launch_p2_table_regions(hipStream_t s, const uint32_t* fill, uint64_t rc, uint32_t d0, uint32_t nk, uint64_t* tab,
                             Status* st, uint64_t n_records);
void launch_shard_header(hipStream_t s, const int64_t* fin, int stride, int world, const IndexHeaderBytes& tmpl,
                         int64_t n_total, uint8_t* out);
// sharded exact path (shard_exact_kernels.hip)
void launch_first_empty(const BuildParams& P, hipStream_t s, unsigned long long* out);
void launch_ex_count(const BuildParams& P, hipStream_t s, const int64_t* starts, int world, uint32_t* cnt,
                     uint64_t* off, uint64_t* scratch, unsigned long long* totals);
void launch_ex_scatter(const BuildParams& P, hipStream_t s, const int64_t* starts, int world, const uint64_t* off,
                       uint8_t* send, uint32_t rs);
void launch_ex_ent(hipStream_t s, const uint8_t* recv, uint64_t n, uint32_t rs, Entry* ent);
void launch_ex_extract(const BuildParams& L, const BuildParams& G, hipStream_t s, const uint8_t* recv, uint64_t n,
                       uint32_t rs, uint64_t a, uint64_t b);

}  // namespace sk
