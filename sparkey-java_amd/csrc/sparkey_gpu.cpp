// sparkey_gpu.cpp -- C-ABI (include/sparkey_gpu.h) and host orchestration of the .spi build.
//
// Host side of IndexHash.createNew (IndexHash.java:131-167): parse and validate the 84-byte log
// header (LogHeader.java:55-88, CommonHeader.java:30-44), derive the index parameters
// (addressSize :140/:247-250, hashType :141-143, capacity :145, entryBlockBits :123-129), build
// the 112-byte header template (IndexHeader.java:125-155) and drive the device pipeline in
// build_kernels.hip.  Errors map to the reference's exceptions (include/sparkey_gpu.h).
#include <errno.h>
#include <stddef.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/sparkey_gpu.h"
#include "build_kernels.hpp"
#include "lookup.hpp"
#include "append.hpp"
#include "snappy.hpp"
#include "shard_host.hpp"
#include "knobs.hpp"

using namespace sk;

namespace {

constexpr int64_t kFrameMinChunk = 512;  // k_frame chunk (one lane) lower bound
constexpr int64_t kFrameRegion = 8192;   // bytes of chunks per k_frame wave
constexpr int64_t kFrameLook = 128;      // speculative walks continue this far past their chunk

constexpr uint32_t kLogMagic = 0x49b39c95u;
constexpr uint32_t kIndexMagic = 0x9a11318fu;

void set_err(char* err, size_t err_len, const std::string& msg) {
  if (err && err_len > 0) snprintf(err, err_len, "%s", msg.c_str());
}

uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
void wr32(uint8_t* p, uint32_t v) {
  for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}
void wr64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

struct LogHdr {
  int32_t major, minor, file_id;
  int64_t num_puts, num_deletes, data_end, max_key_len, max_value_len, delete_size;
  int32_t compression_type, compression_block_size;
  int64_t put_size;
  int32_t max_entries_per_block;
};

// LogHeader.read (LogHeader.java:55-88) + CommonHeader bounds (CommonHeader.java:38-43)
int parse_log_header(const uint8_t* b, uint64_t hdr_len, uint64_t file_len, LogHdr* h, char* err, size_t err_len,
                     bool allow_snappy = false) {
  if (hdr_len < 84 || rd32(b) != kLogMagic) {
    set_err(err, err_len, "File is not a Sparkey log file");
    return SPARKEY_E_NOT_LOG;
  }
  h->major = (int32_t)rd32(b + 4);
  if (h->major != 1) {
    set_err(err, err_len, "Incompatible major version. Expected 1, but got " + std::to_string(h->major));
    return SPARKEY_E_VERSION;
  }
  h->minor = (int32_t)rd32(b + 8);
  if (h->minor > 0) {
    set_err(err, err_len, "Incompatible minor version. Can handle up to version 0, but got " + std::to_string(h->minor));
    return SPARKEY_E_VERSION;
  }
  h->file_id = (int32_t)rd32(b + 12);
  h->num_puts = (int64_t)rd64(b + 16);
  h->num_deletes = (int64_t)rd64(b + 24);
  h->data_end = (int64_t)rd64(b + 32);
  h->max_key_len = (int64_t)rd64(b + 40);
  h->max_value_len = (int64_t)rd64(b + 48);
  h->delete_size = (int64_t)rd64(b + 56);
  h->compression_type = (int32_t)rd32(b + 64);
  h->compression_block_size = (int32_t)rd32(b + 68);
  h->put_size = (int64_t)rd64(b + 72);
  h->max_entries_per_block = (int32_t)rd32(b + 80);
  if (h->data_end > (int64_t)file_len) {
    set_err(err, err_len, "Corrupt log file: expected at least " + std::to_string(h->data_end) + " size but was " +
                              std::to_string(file_len));
    return SPARKEY_E_CORRUPT_LOG;
  }
  if (h->max_key_len > 0x7fffffffLL || h->max_key_len < 0) {
    set_err(err, err_len, "Too large max key len: " + std::to_string(h->max_key_len));
    return SPARKEY_E_HEADER;
  }
  if (h->max_value_len < 0) {
    set_err(err, err_len, "Too large max value len: " + std::to_string(h->max_value_len));
    return SPARKEY_E_HEADER;
  }
  if (h->compression_type < 0 || h->compression_type > 2) {
    set_err(err, err_len, "Corrupt log file: unknown compression type " + std::to_string(h->compression_type));
    return SPARKEY_E_CORRUPT_LOG;
  }
  if (h->compression_type != 0 && !allow_snappy) {
    set_err(err, err_len, h->compression_type == 2 ? "ZSTD logs are not supported on this entry point"
                                                   : "SNAPPY logs are not supported on this entry point");
    return SPARKEY_E_UNSUPPORTED;
  }
  return SPARKEY_OK;
}

int32_t calc_entry_block_bits(int32_t max_entries_per_block) {  // IndexHash.java:123-129
  int32_t i = 0;
  while ((1 << i) < max_entries_per_block) i++;
  return i;
}

int64_t java_d2l(double d) {  // Java (long) cast: truncation, NaN -> 0, saturating
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}

int32_t vlq_size_long(int64_t v) {  // Util.java:102-128
  int32_t n = 1;
  while (n < 9 && v >= (1LL << (7 * n))) n++;
  return n;
}

struct IndexParams {
  int32_t hash_size, addr_size, slot_size, ebb;
  uint64_t cap;
  int64_t index_size;
  bool in_memory;
};

int make_index_params(const LogHdr& lh, const sparkey_build_opts& o, IndexParams* ip, char* err, size_t err_len) {
  double sparsity = o.sparsity;
  if (sparsity < 1.3) sparsity = 1.3;                                   // IndexHash.java:135-137
  ip->ebb = calc_entry_block_bits(lh.max_entries_per_block);
  ip->addr_size = lh.data_end <= (1LL << (30 - ip->ebb)) ? 4 : 8;      // :140, :247-250
  int32_t hs = o.hash_size;
  if (hs == 0) hs = lh.num_puts < (1 << 23) ? 4 : 8;                   // :141-143
  if (hs != 4 && hs != 8) {
    set_err(err, err_len, "Can't support hash size " + std::to_string(hs));
    return SPARKEY_E_ARG;
  }
  ip->hash_size = hs;
  const int64_t cap = 1LL | java_d2l((double)lh.num_puts * sparsity);  // :145 -- the only FP op
  if (cap <= 0) {
    set_err(err, err_len, "Invalid hash capacity " + std::to_string(cap));
    return SPARKEY_E_ARG;
  }
  ip->cap = (uint64_t)cap;
  ip->slot_size = ip->hash_size + ip->addr_size;
  const int64_t hash_length = (int64_t)ip->slot_size * cap;
  ip->index_size = kIndexHeaderSize + hash_length;
  ip->in_memory = o.method == SPARKEY_METHOD_AUTO ? hash_length <= o.max_memory : o.method == SPARKEY_METHOD_IN_MEMORY;
  return SPARKEY_OK;
}

// IndexHeader.asBytes (IndexHeader.java:125-155); stats fields are patched on the device.
void index_header_template(const LogHdr& lh, const IndexParams& ip, int32_t seed, uint8_t* b) {
  memset(b, 0, kIndexHeaderSize);
  wr32(b + 0, kIndexMagic);
  wr32(b + 4, 1);
  wr32(b + 8, 1);
  wr32(b + 12, (uint32_t)lh.file_id);
  wr32(b + 16, (uint32_t)seed);
  wr64(b + 20, (uint64_t)lh.data_end);
  wr64(b + 28, (uint64_t)lh.max_key_len);
  wr64(b + 36, (uint64_t)lh.max_value_len);
  wr64(b + 44, (uint64_t)lh.num_puts);
  wr32(b + 68, (uint32_t)ip.addr_size);
  wr32(b + 72, (uint32_t)ip.hash_size);
  wr64(b + 76, ip.cap);
  wr32(b + 92, (uint32_t)ip.ebb);
}

const char* code_message(int code) {
  switch (code) {
    case SPARKEY_OK: return "OK";
    case SPARKEY_E_NOT_LOG: return "File is not a Sparkey log file";
    case SPARKEY_E_VERSION: return "Incompatible version";
    case SPARKEY_E_CORRUPT_LOG: return "Corrupt log file";
    case SPARKEY_E_NO_FREE_SLOTS: return "No free slots in the hash";
    case SPARKEY_E_CORRUPT_DATA: return "Corrupt data";
    case SPARKEY_E_VLQ: return "Too long VLQ value";
    case SPARKEY_E_HEADER: return "Too large max key len";
    case SPARKEY_E_UNSUPPORTED: return "Unsupported compression type";
    case SPARKEY_E_IO: return "I/O error";
    case SPARKEY_E_GPU: return "GPU error";
    case SPARKEY_E_ARG: return "Illegal argument";
    case SPARKEY_E_BUFFER: return "Buffer too small";
    case SPARKEY_E_CORRUPT_RECORD: return "Corrupt log record";
    default: return "Unknown error";
  }
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      set_err(err, err_len, std::string("HIP error: ") + hipGetErrorString(e_) + " at " #expr); \
      return SPARKEY_E_GPU;                                                            \
    }                                                                                  \
  } while (0)

template <class T>
hipError_t grow(T** p, uint64_t& have, uint64_t want) {
  if (want <= have && *p) return hipSuccess;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  have = 0;
  const uint64_t n = std::max<uint64_t>(want, 1);
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e == hipSuccess) have = n;
  return e;
}

// grow() that keeps the first `used` elements
template <class T>
hipError_t grow_keep(T** p, uint64_t& have, uint64_t want, uint64_t used, hipStream_t s) {
  if (want <= have && *p) return hipSuccess;
  T* q = nullptr;
  hipError_t e = hipMalloc((void**)&q, std::max<uint64_t>(want, 1) * sizeof(T));
  if (e != hipSuccess) return e;
  if (*p && used) {
    e = hipMemcpyAsync(q, *p, std::min(used, have) * sizeof(T), hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      (void)hipFree(q);
      return e;
    }
  }
  if (*p) (void)hipFree(*p);
  *p = q;
  have = std::max<uint64_t>(want, 1);
  return hipSuccess;
}

constexpr int64_t kExactMaxKey = 4096;     // sharded exact path: longest key its exchange records carry
constexpr uint64_t kSnappyChunk = 1024;  // blocks per k_snappy_dir launch (swept 256-4096)

}  // namespace

// Host state of a sharded build between its steps (sparkey_shard_*).
struct ShardState {
  bool active = false;
  LogHdr lh;
  IndexParams ip;
  sparkey_build_opts opts;
  int rank = 0, world = 1;
  const uint8_t* log = nullptr;  // virtual base of global log position 0
  uint64_t buf_lo = 0, buf_hi = 0;
  uint64_t n_local = 0, n_recv = 0;
  BuildParams P;        // placement over the rank's slot range
  BuildParams P_frame;  // the rank's framing (entries in slabs)
  int local = 0;        // world 1, no send buffer: the binned entries stay in ent3 (1 digit regions, 2 dense)
  IndexHeaderBytes tmpl;  // the .spi header template
  // exact path (sparkey_shard_exact_*): the exact ranges' starts, the exchange record size, the
  // records packed, and the replay over the received records (its local table and receive buffer)
  std::vector<int64_t> ex_starts;
  // the framing's log-order slabs (P_frame) still hold [slabs_entry, slabs_end): the exact path packs
  // them without framing again (cleared by the steps that reuse the slab counts)
  bool slabs_ok = false;
  int64_t slabs_entry = 0, slabs_end = 0;
  uint32_t ex_rs = 0;
  uint64_t ex_total = 0;
  bool ex_framed = false, ex_built = false;
  BuildParams ex_L;
  const uint8_t* ex_recv = nullptr;
  uint64_t ex_n = 0;
};

struct sparkey_plan {
  int device = 0;
  bool shared_device = false;  // other builds run on this device concurrently (threads-one-device ranks)
  ShardState shard;
  uint64_t c_small = 0;
  uint64_t* small = nullptr;  // a few words of device scratch
  hipStream_t own_stream = nullptr;
  uint64_t c_conv = 0, c_exitp = 0, c_qpos = 0, c_tail = 0, c_G = 0, c_cnt = 0, c_off = 0;
  uint64_t c_ent = 0, c_ent2 = 0, c_ent3 = 0;
  uint64_t c_bcount = 0, c_bcursor = 0, c_boff = 0, c_bfun = 0, c_bpre = 0, c_carry = 0;
  uint64_t c_p1_fill = 0, c_bstat = 0;
  uint64_t* bstat_start = nullptr;  // folded stats: first slot of each bucket's written range
  uint64_t c_pairs = 0, c_parts = 0, c_su = 0, c_smp = 0, c_bft = 0;
  uint64_t c_desc = 0, c_p1h = 0, c_p1o = 0, c_dbg = 0, c_wcount = 0, c_woff = 0;
  uint64_t c_eseg = 0, c_seg_cnt = 0, c_seg_off = 0, c_seg_mark = 0, c_seg_start = 0, c_p2tab = 0;
  uint64_t* p2tab = nullptr;  // sharded receive: k_part2's run table
  unsigned long long* delp = nullptr;  // the framing kernels' spread DELETE counters (kDelParts x 128 B)
  uint64_t c_app_i64 = 0, c_app_u32 = 0, c_app_u64 = 0, c_app_scan = 0;  // sparkey_log_append workspace
  int64_t* app_i64 = nullptr;
  uint32_t* app_u32 = nullptr;
  uint64_t* app_u64 = nullptr;
  int64_t* app_scan = nullptr;
  uint64_t c_app_map = 0;
  uint32_t* app_map = nullptr;
  // SNAPPY front end (snappy.hpp): block directory, per-block walks, record offsets, virtual log,
  // internal table
  uint64_t c_sn_blocks = 0, c_sn_dir = 0, c_sn_walk = 0, c_sn_recoff = 0, c_sn_vlog = 0, c_sn_itab = 0, c_sn_err = 0;
  SnappyBlock* sn_blocks = nullptr;
  SnappyDirResult* sn_dir = nullptr;
  SnappyWalk* sn_walk = nullptr;
  uint32_t* sn_recoff = nullptr;
  uint8_t* sn_vlog = nullptr;
  uint8_t* sn_itab = nullptr;
  int32_t* sn_err = nullptr;
  uint64_t c_sn_par = 0;
  uint8_t* sn_par = nullptr;        // the parallel directory's scratch (candidates, anchors, links)
  hipStream_t sn_stream = nullptr;  // the decode of one directory chunk overlaps the next chunk
  hipEvent_t sn_ev[2] = {nullptr, nullptr};
  uint64_t c_seg_cls_cnt = 0, c_seg_cls_off = 0, c_seg_len = 0, c_seg_first = 0, c_seg_fun = 0, c_seg_krep = 0, c_ecls = 0;
  uint32_t* seg_krep = nullptr;   // exact path: per placed record, slots back to its key's first record
  uint64_t c_sub_ent = 0, c_sub_fill = 0;
  Entry* sub_ent = nullptr;       // two-level pass 2: the sub-digit regions
  uint32_t* sub_fill = nullptr;   // two-level pass 2: their fill cursors
  uint32_t* ecls = nullptr;       // exact path: per grouped record, its key's class
  uint32_t* seg_len = nullptr;    // exact path: distinct keys per wanted slot, then segment lengths
  uint64_t* seg_first = nullptr;  // exact path: per segment, the slot of its first placed PUT record
  MaxPlus* seg_fun = nullptr;     // exact path: the distinct keys' carry functions, scanned
  // sharded compressed logs (sk_cz_*): the rank's part of the block directory and its
  // slice [vbase, vend) of the virtual log, decoded into sn_vlog from global offset vlo
  struct CzState {
    LogHdr lh;
    int codec = 0;
    int64_t H = 0, A = 0;
    SnappyParams S;
    std::vector<int64_t> anchors, ends;
    std::vector<uint64_t> cnt, usum;
    int64_t vbase = 0, vlo = 0, vend = 0;
    uint64_t nblk = 0, ulen = 0;
    int32_t* flag = nullptr;  // device word: link failures, conversion errors
    int64_t* d_ends = nullptr;
    uint64_t *d_cnt = nullptr, *d_usum = nullptr, *d_boff = nullptr, *d_uoff = nullptr;
  } cz;
  // sharded exact path: the local replay table (the .spi layout with 8-byte addresses), the exact
  // ranges' starts, per-(owner, slab) record counts and their scan
  uint64_t c_xtab = 0, c_ex_starts = 0, c_ex_cnt = 0, c_ex_off = 0;
  uint8_t* xtab = nullptr;
  int64_t* ex_starts = nullptr;
  uint32_t* ex_cnt = nullptr;
  uint64_t* ex_off = nullptr;
  uint32_t* seg_cls_cnt = nullptr;
  uint64_t* seg_cls_off = nullptr;
  int64_t* seg_mark = nullptr;
  int64_t* seg_start = nullptr;
  uint64_t* eseg = nullptr;     // exact path: per slab entry, the first slot of its segment
  uint32_t* seg_cnt = nullptr;  // exact path: per slot, records of the segment starting there
  uint64_t* seg_off = nullptr;
  uint8_t* conv = nullptr;
  int64_t* exitp = nullptr;
  int64_t* qpos = nullptr;
  uint32_t* tail = nullptr;
  int64_t* G = nullptr;
  uint32_t* cnt = nullptr;
  uint64_t* off = nullptr;
  Entry* ent = nullptr;
  Entry* ent2 = nullptr;
  Entry* ent3 = nullptr;
  uint32_t* bcount = nullptr;
  uint32_t* bcursor = nullptr;
  uint64_t* boff = nullptr;
  MaxPlus* bfun = nullptr;
  MaxPlus* bpre = nullptr;
  MaxPlus* bfun_total = nullptr;
  int64_t* carry = nullptr;
  MaxPlus* dfun = nullptr;     // fused_carry: per coarse digit
  int64_t* dcarry = nullptr;
  uint64_t c_dfun = 0, c_dcarry = 0;
  uint32_t epoch = 0;          // fused_carry builds so far (tags the dfun words)
  uint64_t* pairs = nullptr;
  StatPart* parts = nullptr;
  uint32_t* p1_fill = nullptr;
  uint64_t* scan_u64 = nullptr;
  MaxPlus* scan_mp = nullptr;
  unsigned long long* desc = nullptr;  // k_frame exit granules (memset per build)
  uint32_t* wcount = nullptr;          // entries per slab
  uint64_t* woff = nullptr;
  uint32_t* p1_hist = nullptr;
  uint64_t* p1_off = nullptr;
  Status* d_status = nullptr;
  Status* h_status = nullptr;
  Status* h_status_dev = nullptr;  // h_status as the device sees it (k_status_out writes it)
  unsigned long long* dbg = nullptr;  // SPARKEY_FRAME_DEBUG=1: k_frame phase counters
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  SideStreams side{};  // exact path: concurrent segment classes (created on first use)
  bool side_ok = false;
  StageTimer timer;
  std::vector<std::string> stage_names;
  std::vector<double> stage_ms;
};

static int plan_reserve(sparkey_plan* pl, uint64_t nchunks, uint64_t nrec, uint64_t ent_cap, uint64_t nslabs,
                        uint64_t p1_tiles, uint64_t nbuckets, uint64_t cap, char* err, size_t err_len) {
  HIP_TRY(grow(&pl->conv, pl->c_conv, nchunks));
  HIP_TRY(grow(&pl->exitp, pl->c_exitp, nchunks));
  HIP_TRY(grow(&pl->qpos, pl->c_qpos, nchunks));
  HIP_TRY(grow(&pl->tail, pl->c_tail, nchunks));
  HIP_TRY(grow(&pl->G, pl->c_G, nchunks + 1));
  HIP_TRY(grow(&pl->cnt, pl->c_cnt, nchunks));
  HIP_TRY(grow(&pl->off, pl->c_off, nchunks + 1));
  HIP_TRY(grow(&pl->ent, pl->c_ent, ent_cap));
  HIP_TRY(grow(&pl->wcount, pl->c_wcount, nslabs + 1));
  HIP_TRY(grow(&pl->woff, pl->c_woff, nslabs + 1));
  HIP_TRY(grow(&pl->ent2, pl->c_ent2, nrec));
  HIP_TRY(grow(&pl->ent3, pl->c_ent3, nrec));
  HIP_TRY(grow(&pl->bcount, pl->c_bcount, nbuckets));
  HIP_TRY(grow(&pl->bcursor, pl->c_bcursor, nbuckets));
  HIP_TRY(grow(&pl->boff, pl->c_boff, nbuckets + 1));
  HIP_TRY(grow(&pl->bfun, pl->c_bfun, nbuckets));
  HIP_TRY(grow(&pl->bpre, pl->c_bpre, nbuckets));
  HIP_TRY(grow(&pl->bfun_total, pl->c_bft, 1));
  HIP_TRY(grow(&pl->carry, pl->c_carry, nbuckets));
  if (!pl->dfun) {
    HIP_TRY(grow(&pl->dfun, pl->c_dfun, 256));
    HIP_TRY(hipMemset(pl->dfun, 0, 256 * sizeof(MaxPlus)));  // epoch 0: no build's
  }
  HIP_TRY(grow(&pl->dcarry, pl->c_dcarry, 256));
  const uint64_t pair_cap = std::max<uint64_t>(1 << 16, std::min<uint64_t>(nrec, 1 << 22));
  HIP_TRY(grow(&pl->pairs, pl->c_pairs, 2 * pair_cap));
  HIP_TRY(grow(&pl->parts, pl->c_parts, std::max<uint64_t>(nbuckets, (cap + kStatSlotsPerBlock - 1) / kStatSlotsPerBlock)));
  HIP_TRY(grow(&pl->bstat_start, pl->c_bstat, nbuckets));
  HIP_TRY(grow(&pl->desc, pl->c_desc, 2 * nchunks + 2));
  HIP_TRY(grow(&pl->p1_hist, pl->c_p1h, 256 * p1_tiles));
  HIP_TRY(grow(&pl->p1_off, pl->c_p1o, 256 * p1_tiles + 1));
  const uint64_t scratch = std::max(std::max(std::max(nchunks, nbuckets), 256 * p1_tiles), nslabs) / kScanTile + 64;
  HIP_TRY(grow(&pl->scan_u64, pl->c_su, scratch + 16));
  HIP_TRY(grow(&pl->scan_mp, pl->c_smp, scratch + 16));
  return SPARKEY_OK;
}

static void fill_stats(sparkey_build_stats* s, const Status& st, const IndexParams& ip, int placement, int framing,
                       double ms, int partition_passes = 2, int entry_bytes = 16) {
  if (!s) return;
  s->partition_passes = partition_passes;
  s->entry_bytes = entry_bytes;
  s->reserved0 = 0;
  s->sharded = 0;
  s->num_records = (int64_t)st.n_records;
  s->num_deletes = (int64_t)st.n_deletes;
  s->num_puts = (int64_t)st.n_records - (int64_t)st.n_deletes;
  s->num_entries = st.num_entries;
  s->capacity = (int64_t)ip.cap;
  s->garbage_size = st.garbage;
  s->max_displacement = st.max_disp;
  s->hash_collisions = st.collisions;
  s->total_displacement = st.total_disp;
  s->hash_size = ip.hash_size;
  s->address_size = ip.addr_size;
  s->placement_path = placement;
  s->framing_path = framing;
  s->device_ms = ms;
}

static int status_error(const Status& st, char* err, size_t err_len) {
  if (st.err == ~0ull) return SPARKEY_OK;
  const int code = -(int)(st.err & 0xff);
  const unsigned long long pos = st.err >> 8;
  set_err(err, err_len, std::string(code_message(code)) + " (log offset " + std::to_string(pos) + ")");
  return code;
}

// Geometry of one build over the log bytes a device buffer holds.  `log` is the (virtual) base
// pointer of global log position 0, `log_len` the end of the bytes it holds; records are framed
// from `entry` while they start below `frame_end`.
static int setup_params(const LogHdr& lh, const IndexParams& ip, const sparkey_build_opts& o, const uint8_t* log,
                        uint64_t log_len, int64_t entry, int64_t frame_end, BuildParams* Pp, char* err,
                        size_t err_len) {
  BuildParams& P = *Pp;
  memset(&P, 0, sizeof(P));
  P.log = log;
  P.log_len = log_len;
  P.data_end = frame_end;
  P.max_key_len = lh.max_key_len;
  P.max_value_len = lh.max_value_len;
  {
    const int64_t put_len = vlq_size_long(lh.max_key_len + 1) + vlq_size_long(lh.max_value_len) + lh.max_key_len +
                            lh.max_value_len;
    const int64_t del_len = 1 + vlq_size_long(lh.max_key_len) + lh.max_key_len;
    P.max_rec_len = std::max<int64_t>(1, std::max(put_len, del_len));
  }
  const bool any = frame_end > entry;
  P.fr_entry = entry;
  P.ch_k0 = (uint64_t)entry >> kChunkShift;
  P.nchunks = any ? (uint64_t)((frame_end + kChunk - 1) / kChunk) - P.ch_k0 : 0;
  // k_frame geometry: chunk C = max(512, nextpow2(maxRecLen)) so every chunk but a short last one
  // holds a record start; 8 KiB of chunks per wave, staged contiguously with 256 bytes of
  // look-ahead (about 10 KiB of LDS: 16 waves per CU); records longer than 4 KiB -> serial framing.
  {
    // chunk >= kFrameMinChunk and >= maxRecLen; a wave stages kFrameRegion bytes of chunks
    // (SPARKEY_FRAME_CMIN / SPARKEY_FRAME_REGION override both, for tuning)
    int64_t cmin = kFrameMinChunk, region = kFrameRegion, look = kFrameLook;
    {
      // Records of mixed sizes (the header's mean record well under the largest) take 1 KiB chunks:
      // measured 7% faster framing on C3 (8-64 B keys, mean 138 B of at most 168 B), while
      // fixed-size records keep 512 (1 KiB chunks are 8% slower on C2's 118 B records).
      const int64_t nrec = std::max<int64_t>(0, lh.num_puts) + std::max<int64_t>(0, lh.num_deletes);
      const int64_t bytes = std::max<int64_t>(0, lh.put_size) + std::max<int64_t>(0, lh.delete_size);
      if (nrec > 0 && bytes > 0 && 10 * bytes < 9 * nrec * P.max_rec_len) cmin = 1024;
      // Small records (WriteHashBenchmark's key_i / value_i, 14-26 bytes) take 128-byte chunks and the
      // balanced walk: each candidate walks about 5 records instead of 25 (c1x frame 0.244 -> 0.205 ms,
      // profiles/r04/c1x/chunk_ab.txt)
      if (nrec > 0 && bytes > 0 && bytes < 64 * nrec) cmin = 128;
    }
    if (knob_set(Knob::FrameCmin)) cmin = std::max<int64_t>(128, knob(Knob::FrameCmin));
    if (knob_set(Knob::FrameRegion)) region = std::min<int64_t>(16384, std::max<int64_t>(2048, knob(Knob::FrameRegion)));
    if (knob_set(Knob::FrameLook)) look = std::min<int64_t>(4096, std::max<int64_t>(16, knob(Knob::FrameLook)));
    int cs = 7;
    while ((1ll << cs) < std::max<int64_t>(P.max_rec_len, cmin)) cs++;
    const int64_t C = 1ll << cs;
    P.fr_cshift = cs;
    P.fr_w = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, region / C));
    // Hashing runs one record per lane per round, so a wave holding 69 records pays for 128.  The
    // header's mean record size (putSize + deleteSize over the record count) picks, among regions of
    // half to all of kFrameRegion, the W whose expected records per wave (plus a small margin) fill
    // their rounds best.
    const int64_t nrec_hdr = std::max<int64_t>(0, lh.num_puts) + std::max<int64_t>(0, lh.num_deletes);
    const int64_t bytes_hdr = std::max<int64_t>(0, lh.put_size) + std::max<int64_t>(0, lh.delete_size);
    if (!knob_set(Knob::FrameRegion) && nrec_hdr > 0 && bytes_hdr > 0 && region / C >= 2) {
      const double mean = (double)bytes_hdr / (double)nrec_hdr;
      double best = -1.0;
      for (int64_t w = std::max<int64_t>(1, region / C / 2); w <= std::min<int64_t>(64, region / C); w++) {
        const double recs = (double)(w * C) / mean;
        const double eff = recs / (64.0 * std::ceil((recs + 3.0) / 64.0));
        if (eff >= best) {
          best = eff;
          P.fr_w = (int32_t)w;
        }
      }
    }
    P.fr_look = (int32_t)((look + 15) & ~15LL);
    P.fr_rgn_bytes = (int32_t)(((int64_t)P.fr_w * C + P.fr_look + 16 + 1023) & ~1023LL);  // whole glds rows
    P.fr_mask_words = (int32_t)((std::min<int64_t>(C, P.max_rec_len) + 63) / 64);
    if (P.max_rec_len <= 4096) {  // k_frame (fused framing) finds a screened word's chunk as (q * magic) >> 22
      const uint32_t wpc = 8u * (uint32_t)P.fr_mask_words;
      P.fr_wpc_magic = (uint32_t)(((1ull << 22) + wpc - 1) / wpc);
      for (uint32_t q = 0; q < (uint32_t)P.fr_w * wpc; q++)
        if ((uint32_t)(((uint64_t)q * P.fr_wpc_magic) >> 22) != q / wpc || (uint64_t)q * P.fr_wpc_magic >= (1ull << 32)) {
          set_err(err, err_len, "k_frame screen geometry out of range");
          return SPARKEY_E_ARG;
        }
    }
    P.fr_fast = lh.max_key_len + 1 < 128 && lh.max_value_len < 128;
    P.no_deletes = lh.num_deletes == 0;
    P.fr_k0 = (uint64_t)entry >> cs;
    P.fr_nchunks = any ? (uint64_t)((frame_end + C - 1) / C) - P.fr_k0 : 0;
  }
  P.emit_extra = lh.max_key_len + 32 <= kEmitExtra ? (int32_t)((lh.max_key_len + 32 + 15) & ~15LL) : 32;
  P.uni_nt = 1u;  // framing stages the log non-temporally (read once: measured 10% faster)
  P.hash_size = ip.hash_size;
  P.addr_size = ip.addr_size;
  P.slot_size = ip.slot_size;
  P.ebb = ip.ebb;
  P.seed = o.hash_seed;
  P.mod = make_fastmod(ip.cap);
  P.cap = ip.cap;
  P.nbuckets = (ip.cap + kBucket - 1) / kBucket;
  P.bpp = (uint32_t)std::max<uint64_t>(1, (P.nbuckets + 255) / 256);
  if (P.bpp > (1u << kPart2MaxBits)) {
    set_err(err, err_len, "hash capacity too large for one device: " + std::to_string(ip.cap));
    return SPARKEY_E_UNSUPPORTED;
  }
  P.dmagic = ((1ull << 40) + P.bpp - 1) / P.bpp;
  P.b_lo = 0;
  P.b_hi = P.nbuckets;
  P.slot_lo = 0;
  P.slot_hi = ip.cap;
  return SPARKEY_OK;
}

// R when the header proves that every record of the log is a PUT of exactly R bytes: no DELETE,
// one-byte VLQs, and putSize == numPuts * R == dataEnd - 84 with R the largest PUT record the header
// allows (each record is at most R bytes and together they fill putSize).  Else 0.
// SPARKEY_NO_UNIFORM disables it (tests and the bench's general-framing measurement).
// k_frame3 (frame3_kernels.hip) frames the log when its VLQs are one byte and the header's mean
// record lets a chunk's records and a wave's records fit k_frame3's lists (SPARKEY_NO_FRAME3: k_frame).
// Its chunk: the power of two >= maxRecLen of 8-16 mean records (the long walks of about ten steps
// against a wave's candidate windows and short walks, which grow with the chunk count), the frame3_c
// switch overrides; 8 KiB of chunks per wave (frame_region).  The geometry is set on P when k_frame3 is chosen (k_frame can frame
// with it too, which its fallback does).
static bool want_frame3(BuildParams& P, const LogHdr& lh, int64_t entry, int64_t frame_end) {
  if (knob_on(Knob::NoFrame3) || !P.fr_fast || P.max_rec_len > 4096) return false;
  const int64_t nr = std::max<int64_t>(0, lh.num_puts) + std::max<int64_t>(0, lh.num_deletes);
  const int64_t by = std::max<int64_t>(0, lh.put_size) + std::max<int64_t>(0, lh.delete_size);
  if (nr <= 0 || by <= 0) return false;
  const double mean = (double)by / (double)nr;
  // (8-16 mean records a chunk: C3's shape 2048 B, 0.774 ms against 1024 B's 0.815 per 10M records;
  //  C2's records 1024 B, frame 0.62-0.64 ms against 512 B's 0.72 and 2048 B's 0.68; round 5,
  //  profiles/r05/frame3/)
  int64_t want = std::max<int64_t>(std::max<int64_t>(P.max_rec_len, 128), (int64_t)std::ceil(8.0 * mean));
  if (knob_set(Knob::Frame3C)) want = std::max<int64_t>(P.max_rec_len, knob(Knob::Frame3C));
  int cs = 7;
  while ((1ll << cs) < want) cs++;
  while (!knob_set(Knob::Frame3C) && cs > 7 && (double)(1ll << cs) / mean > 16.0 && (1ll << (cs - 1)) >= P.max_rec_len) cs--;
  int64_t region = 8192;
  if (knob_set(Knob::FrameRegion)) region = std::min<int64_t>(16384, std::max<int64_t>(2048, knob(Knob::FrameRegion)));
  BuildParams Q = P;
  const int64_t C = 1ll << cs;
  Q.fr_cshift = cs;
  Q.fr_w = (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, region / C));
  Q.fr_rgn_bytes = (int32_t)(((int64_t)Q.fr_w * C + Q.fr_look + 16 + 1023) & ~1023LL);
  Q.fr_mask_words = (int32_t)((std::min<int64_t>(C, Q.max_rec_len) + 63) / 64);
  const uint32_t wpc = 8u * (uint32_t)Q.fr_mask_words;
  Q.fr_wpc_magic = (uint32_t)(((1ull << 22) + wpc - 1) / wpc);
  for (uint32_t q = 0; q < (uint32_t)Q.fr_w * wpc; q++)
    if ((uint32_t)(((uint64_t)q * Q.fr_wpc_magic) >> 22) != q / wpc || (uint64_t)q * Q.fr_wpc_magic >= (1ull << 32))
      return false;
  Q.fr_k0 = (uint64_t)entry >> cs;
  Q.fr_nchunks = frame_end > entry ? (uint64_t)((frame_end + C - 1) / C) - Q.fr_k0 : 0;
  // a random byte pair passes the screen with about p = (maxKeyLen + 1) / 256 * (maxValueLen + 1) / 256
  // (more with DELETEs); the short walk's K steps leave p^K of the false starts
  const double pk = std::min(1.0, (double)(Q.max_key_len + 1) / 256.0) * std::min(1.0, (double)(Q.max_value_len + 1) / 256.0) +
                    (Q.no_deletes ? 0.0 : std::min(1.0, (double)(Q.max_key_len + 1) / 256.0) / 256.0);
  // a candidate window (maxRecLen bytes) holds about maxRecLen / mean true starts, all on one chain:
  // when that is well above one, the starts reached by others are marked so that only chain heads
  // walk on (SPARKEY_FRAME3_COVER=0/1 forces it)
  // (also when a wave has more chunks than half the heads its lanes walk: windows that hold two true
  // starts -- a log's shorter records -- would otherwise make two heads a chunk)
  Q.f3_cover = (double)Q.max_rec_len > 1.5 * mean || 2 * Q.fr_w + 8 > 64 ? 1 : 0;
  if (knob_set(Knob::Frame3Cover)) Q.f3_cover = knob(Knob::Frame3Cover) ? 1 : 0;
  // (a chunk's list holds its records: a stretch of a log's shorter kind -- DELETEs -- packs more of
  // them than the mean says; churn's 18-byte DELETEs among 118-byte PUTs overflowed 16-start lists)
  double mean_short = mean;
  if (lh.num_deletes > 0 && lh.delete_size > 0) mean_short = std::min(mean_short, (double)lh.delete_size / (double)lh.num_deletes);
  if (lh.num_puts > 0 && lh.put_size > 0) mean_short = std::min(mean_short, (double)lh.put_size / (double)lh.num_puts);
  if (!frame3_fits(Q, mean, pk, mean_short)) return false;
  // (C3's shape, pk 0.1: K = 3 measured 0.870 ms against K = 2's 0.903 per 10M records,
  // profiles/r03/k_frame3_sweep_c3_10m.txt)
  Q.f3_short = pk < 0.05 ? 2 : pk < 0.3 ? 3 : 4;
  if (knob_set(Knob::Frame3Short)) Q.f3_short = (int32_t)std::max<int64_t>(1, std::min<int64_t>(4, knob(Knob::Frame3Short)));
  Q.f3_stop = (int32_t)knob(Knob::Frame3Stop);
  P = Q;
  return true;
}

static int64_t uniform_record_size(const LogHdr& lh) {
  const int64_t R =
      vlq_size_long(lh.max_key_len + 1) + vlq_size_long(lh.max_value_len) + lh.max_key_len + lh.max_value_len;
  if (lh.num_deletes == 0 && lh.num_puts > 0 && lh.max_key_len + 1 < 128 && lh.max_value_len < 128 && R <= 256 &&
      lh.put_size == lh.num_puts * R && lh.data_end - kLogHeaderSize == lh.put_size && !knob_on(Knob::NoUniform))
    return R;
  return 0;
}

// Wave geometry of one framing kernel: chunks of 2^cshift bytes, w per wave.
struct FrameGeom {
  int32_t cshift, w;
  uint64_t k0, nchunks;
};
static FrameGeom get_geom(const BuildParams& P) { return FrameGeom{P.fr_cshift, P.fr_w, P.fr_k0, P.fr_nchunks}; }
static void set_geom(BuildParams& P, const FrameGeom& g) {
  P.fr_cshift = g.cshift;
  P.fr_w = g.w;
  P.fr_k0 = g.k0;
  P.fr_nchunks = g.nchunks;
}

// Slab layout of the framing output and the workspace it needs (grown on demand).
static int reserve_for_framing(sparkey_plan* pl, BuildParams& P, int framing_path, uint64_t nrec, uint32_t slab_cap,
                               char* err, size_t err_len) {
  const uint64_t nwaves = P.fr_nchunks ? (P.fr_nchunks + P.fr_w - 1) / P.fr_w : 0;
  if (slab_framing(framing_path)) {
    P.slab_cap = slab_cap;
    P.nslabs = nwaves;
  } else {  // dense entries from the serial framing path, seen as slabs of kPartTile
    P.slab_cap = kPartTile;
    P.nslabs = (std::max<uint64_t>(nrec, 1) + kPartTile - 1) / kPartTile;
  }
  P.part_group = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxPartGroup, kPartTile / P.slab_cap));
  P.p1_tiles = (uint32_t)std::max<uint64_t>(1, (P.nslabs + P.part_group - 1) / P.part_group);
  // k_part1_regions' tiles: slabs of the mean count (the header's records over the slabs) to fill
  // 0.9 kPartTile, at most 2 kPartTile entries whatever the counts (its two rounds); the slabs are sized
  // for twice the mean, which left its tiles 40% full (an atomic per digit and tile on the fill cursors)
  {
    const double mean = (double)std::max<uint64_t>(nrec, 1) / (double)std::max<uint64_t>(P.nslabs, 1);
    uint64_t g = (uint64_t)std::max(1.0, 0.9 * kPartTile / std::max(1.0, mean));
    g = std::min<uint64_t>(g, std::min<uint64_t>(kMaxPartGroup, 2 * kPartTile / std::max<uint32_t>(P.slab_cap, 1)));
    P.p1r_group = (uint32_t)std::max<uint64_t>(std::max<uint64_t>(g, 1), P.part_group);
    if ((uint64_t)P.p1r_group * P.slab_cap > 2ull * kPartTile) P.p1r_group = P.part_group;
    P.p1r_tiles = (uint32_t)std::max<uint64_t>(1, (P.nslabs + P.p1r_group - 1) / P.p1r_group);
  }
  const uint64_t ent_cap = std::max<uint64_t>(1, P.nslabs * P.slab_cap);
  int rc = plan_reserve(pl, std::max<uint64_t>(P.nchunks, nwaves), std::max<uint64_t>(nrec, 1), ent_cap, P.nslabs,
                        P.p1_tiles, P.nbuckets, P.cap, err, err_len);
  if (rc) return rc;
  P.conv = pl->conv; P.exitp = pl->exitp; P.qpos = pl->qpos; P.tail = pl->tail; P.G = pl->G;
  P.cnt = pl->cnt; P.off = pl->off;
  P.ent = pl->ent; P.ent2 = pl->ent2; P.ent3 = pl->ent3; P.max_records = pl->c_ent2;
  P.ent_cap = std::min<uint64_t>(pl->c_ent, P.nslabs * P.slab_cap);
  P.wcount = pl->wcount; P.woff = pl->woff;
  P.bcount = pl->bcount; P.bcursor = pl->bcursor; P.boff = pl->boff; P.bfun = pl->bfun; P.bpre = pl->bpre;
  P.bfun_total = pl->bfun_total; P.carry = pl->carry; P.pairs = pl->pairs; P.pair_cap = pl->c_pairs / 2;
  P.parts = pl->parts; P.scan_scratch_u64 = pl->scan_u64; P.scan_scratch_mp = pl->scan_mp;
  P.bstat_start = pl->bstat_start;
  P.exit_desc = pl->desc;
  P.frame_ticket = reinterpret_cast<unsigned int*>(pl->desc + 2 * nwaves);
  if (!pl->delp) HIP_TRY(hipMalloc(&pl->delp, (size_t)kDelParts * 16 * sizeof(unsigned long long)));
  P.del_parts = pl->delp;
  // a wave waits for its predecessor's exit at most 2 s of the 100 MHz wall clock; the host then
  // redoes the framing on the serial walk (correct, slower).  With one wave per workgroup the
  // predecessor is a lower workgroup id, which the dispatcher starts first; builds that share a
  // device (fr_ticket) take regions by ticket instead, so no wave waits on one not yet started.
  P.fr_spin_ticks = knob_set(Knob::FrameSpinTicks) ? (uint64_t)knob(Knob::FrameSpinTicks) : 200000000ull;
  P.fr_ticket = pl->shared_device || knob_on(Knob::FrameTicket) ? 1 : 0;
  P.p1_hist = pl->p1_hist; P.p1_off = pl->p1_off; P.p1_off_total = pl->p1_off + 256ull * P.p1_tiles;
  return SPARKEY_OK;
}

// Framing + hashing launches (entries into the slabs), after the status block was reset.
static int launch_framing(sparkey_plan* pl, const BuildParams& P, int framing_path, hipStream_t s, char* err,
                          size_t err_len) {
  const uint64_t nwaves = P.fr_nchunks ? (P.fr_nchunks + P.fr_w - 1) / P.fr_w : 0;
  if (slab_framing(framing_path)) {
    HIP_TRY(hipMemsetAsync(pl->desc, 0, (2 * nwaves + 2) * sizeof(unsigned long long), s));
    HIP_TRY(hipMemsetAsync(pl->wcount, 0, (P.nslabs + 1) * sizeof(uint32_t), s));
    if (P.del_parts) HIP_TRY(hipMemsetAsync(P.del_parts, 0, (size_t)kDelParts * 16 * sizeof(unsigned long long), s));
    if (framing_path == 4) launch_frame3(P, s, &pl->timer);
    else launch_frame_fused(P, s, &pl->timer);
    launch_sum_deletes(P, s);  // (the spread DELETE counters into the status block)
  } else if (framing_path == 2) {
    launch_frame_uniform(P, s, &pl->timer);
    if (!P.p1_region) launch_dense_slabs(P, s);  // (with digit regions nothing reads the slab counts)
  } else {
    launch_framing_serial(P, s);
    launch_emit(P, s, &pl->timer);
    launch_dense_slabs(P, s);
  }
  return SPARKEY_OK;
}

static void print_frame_debug(sparkey_plan* pl, const BuildParams& P) {
  if (P.dbg && P.uni_n && P.p1_region) {  // k_frame_uniform: per workgroup, thread 0's phase cycles
    const uint64_t nb = (P.uni_n + kPartTile - 1) / kPartTile;
    std::vector<unsigned long long> h(16 * nb);
    if (hipMemcpy(h.data(), pl->dbg, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    double sum[4] = {0};
    for (uint64_t c = 0; c < nb; c++)
      for (int i = 0; i < 4; i++) sum[i] += (double)h[c * 16 + i];
    fprintf(stderr, "[k_frame_uniform] workgroups=%llu mean cycles: rounds %.0f runs+scan %.0f regroup %.0f "
            "write-out %.0f\n", (unsigned long long)nb, sum[0] / nb, sum[1] / nb, sum[2] / nb, sum[3] / nb);
    return;
  }
  if (!P.dbg || !P.fr_nchunks) return;
  const uint64_t nwv = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  std::vector<unsigned long long> h(16 * nwv);
  if (hipMemcpy(h.data(), pl->dbg, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  double sum[16] = {0};
  unsigned long long mx[16] = {0};
  for (uint64_t c = 0; c < nwv; c++)
    for (int i = 0; i < 16; i++) {
      sum[i] += (double)h[c * 16 + i];
      mx[i] = std::max(mx[i], h[c * 16 + i]);
    }
  const double n = (double)nwv;
  fprintf(stderr, "[k_frame] waves=%llu C=%d W=%d mean cycles: stage %.0f screen %.0f walk %.0f entry %.0f "
          "counts %.0f slab %.0f hash %.0f | max entry %llu | walk iters %.1f survivors/wave %.1f unconverged/wave "
          "%.2f | slot 7 %.0f\n",
          (unsigned long long)nwv, 1 << P.fr_cshift, P.fr_w, sum[0] / n, sum[1] / n, sum[2] / n, sum[3] / n,
          sum[4] / n, sum[5] / n, sum[6] / n, mx[3], sum[8] / n, sum[9] / n, sum[10] / n, sum[7] / n);
}

static void print_part2_debug(const BuildParams& P) {
  if (!P.part_dbg) return;
  std::vector<unsigned long long> h(8 * 256);
  if (hipMemcpy(h.data(), P.part_dbg, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  double sum[8] = {0};
  unsigned long long mx[8] = {0};
  for (int d = 0; d < 256; d++)
    for (int i = 0; i < 8; i++) {
      sum[i] += (double)h[8 * d + i];
      mx[i] = std::max(mx[i], h[8 * d + i]);
    }
  fprintf(stderr, "[k_part2s] digits=256 mean cycles: clear %.0f count+scatter %.0f barrier %.0f functions %.0f "
          "carry %.0f | max: clear %llu count+scatter %llu barrier %llu functions %llu carry %llu\n",
          sum[0] / 256, sum[1] / 256, sum[2] / 256, sum[3] / 256, sum[4] / 256, mx[0], mx[1], mx[2], mx[3], mx[4]);
}

static int plan_build(sparkey_plan* pl, const uint8_t* log_header, const uint8_t* d_log, uint64_t log_len,
                      uint8_t* d_out, uint64_t index_cap, const sparkey_build_opts* opts, hipStream_t s,
                      sparkey_build_stats* stats_out, char* err, size_t err_len);

// SNAPPY and ZSTD logs (snappy.hpp): block directory, decode into the virtual log, the
// normal build over it into an internal table, then every slot's address rewritten to
// (blockPosition << entryBlockBits) | entryIndex (IndexHash.java:270-283).  The two codecs differ only
// in the directory (a Snappy preamble / a Zstandard Frame_Content_Size gives each block's size) and
// the decode kernel (snappy_kernels.hip / zstd_kernels.hip).
// The SNAPPY block directory in parallel: windows of the longest hop every A bytes,
// their plausible block starts chained to an anchor each (the first chain position past the window,
// where the candidates agree), then every link of the chain 84 -> anchors -> dataEnd walked from its
// start at once with k_snappy_dir's checks; a link that does not land on its end, or any check that
// fails, leaves the directory to the serial chain (*ok = false), which reports errors exactly.
// The longest hop of the block chain: VLQ + the reader's compressed buffer (Snappy.maxCompressedLength,
// ZSTD_compressBound); 0 when the parallel directory does not take such blocks (over ~128 KiB: its
// screen stages a window of H bytes in LDS).
static int64_t cz_hop_bound(int codec, int64_t mb) {
  const int64_t H = 5 + (codec == 1 ? mb + (mb >> 8) + (mb < (128 << 10) ? (((128 << 10) - mb) >> 11) : 0)
                                    : 32 + mb + mb / 6);
  return mb > 0 && sdir_screen_lds(H) <= 150 * 1024 ? H : 0;
}

// LDS of the decode kernels (0: global memory)
static uint32_t cz_decode_lds(bool zstd, int64_t mb) {
  if (zstd)  // decoded straight into the virtual log (LDS for the entropy tables only: many waves per CU)
    // measured 3x faster than the block and frame in LDS (one wave per CU); SPARKEY_ZSTD_LDS=1: that
    return knob_on(Knob::ZstdLds) ? zstd_lds_bytes(mb) : 0u;
  // SNAPPY: the decoded block, then an 8 KiB window over its stream (k_snappy_lds)
  const int64_t lds = ((mb + 15) & ~15LL) + 16 + 8192 + 16;
  return lds <= 160 * 1024 ? (uint32_t)lds : 0u;
}

static int snappy_par_dir(sparkey_plan* pl, SnappyParams& S, hipStream_t s, int codec, SnappyDirResult* dir, bool* ok,
                          char* err, size_t err_len) {
  *ok = false;
  const int64_t body = S.data_end - kLogHeaderSize;
  if (body <= 0 || S.max_block <= 0) return SPARKEY_OK;
  // the longest hop: VLQ + the reader's compressed buffer (Snappy.maxCompressedLength, ZSTD_compressBound)
  const int64_t H = cz_hop_bound(codec, S.max_block);
  if (!H) return SPARKEY_OK;   // (blocks over ~128 KiB: the serial chain)
  int64_t A = std::max<int64_t>(32 * H, body / (1 << 20) + 1);  // (screen 1/32 of the log; links of ~32 blocks)
  if (knob_set(Knob::SnappyDirA)) A = std::max<int64_t>(H, knob(Knob::SnappyDirA));  // (tests, tuning)
  const uint64_t nwin = body > H ? (uint64_t)((body - H - 1) / A + 1) : 0;
  const uint64_t maxl = nwin + 1;  // links
  const uint64_t bytes = nwin * (kSdirCand * 8 + 4 + 8) + (maxl + 1) * 8 + 4 * maxl * 8 + 64;
  HIP_TRY(grow(&pl->sn_par, pl->c_sn_par, bytes));
  uint8_t* q = pl->sn_par;
  auto carve = [&](uint64_t n) { uint8_t* r = q; q += (n + 15) & ~15ull; return r; };
  int64_t* cand = (int64_t*)carve(nwin * kSdirCand * 8);
  int32_t* ncand = (int32_t*)carve(nwin * 4);
  int64_t* anchor = (int64_t*)carve(nwin * 8);
  int64_t* ends = (int64_t*)carve((maxl + 1) * 8);
  uint64_t* cnt = (uint64_t*)carve(maxl * 8);
  uint64_t* usum = (uint64_t*)carve(maxl * 8);
  uint64_t* boff = (uint64_t*)carve(maxl * 8);
  uint64_t* uoff = (uint64_t*)carve(maxl * 8);
  int32_t* fail = (int32_t*)carve(16);
  HIP_TRY(hipMemsetAsync(fail, 0, 4, s));
  launch_sdir_screen(S, s, codec, A, H, nwin, cand, ncand);
  launch_sdir_anchor(S, s, codec, A, H, nwin, cand, ncand, anchor);
  HIP_TRY(hipGetLastError());
  std::vector<int64_t> anc(nwin);
  if (nwin) HIP_TRY(hipMemcpyAsync(anc.data(), anchor, nwin * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::vector<int64_t> e;
  e.push_back(kLogHeaderSize);
  for (int64_t x : anc)
    if (x > e.back() && x < S.data_end) e.push_back(x);
  e.push_back(S.data_end);
  const uint64_t nl = e.size() - 1;
  HIP_TRY(hipMemcpyAsync(ends, e.data(), e.size() * 8, hipMemcpyHostToDevice, s));
  launch_sdir_link(S, s, codec, ends, nl, 0, cnt, usum, nullptr, nullptr, fail);
  HIP_TRY(hipGetLastError());
  std::vector<uint64_t> hc(nl), hu(nl);
  int32_t hf = 0;
  HIP_TRY(hipMemcpyAsync(hc.data(), cnt, nl * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(hu.data(), usum, nl * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&hf, fail, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (hf) return SPARKEY_OK;
  std::vector<uint64_t> bo(nl), uo(nl);
  uint64_t nb = 0, tot = 0;
  for (uint64_t i = 0; i < nl; i++) {
    bo[i] = nb;
    uo[i] = tot;
    nb += hc[i];
    tot += hu[i];
  }
  HIP_TRY(grow(&pl->sn_blocks, pl->c_sn_blocks, std::max<uint64_t>(nb, 1)));
  HIP_TRY(grow(&pl->sn_walk, pl->c_sn_walk, pl->c_sn_blocks));
  S.blocks = pl->sn_blocks;
  S.blk_cap = pl->c_sn_blocks;
  S.walk = pl->sn_walk;
  HIP_TRY(hipMemcpyAsync(boff, bo.data(), nl * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(uoff, uo.data(), nl * 8, hipMemcpyHostToDevice, s));
  launch_sdir_link(S, s, codec, ends, nl, 1, cnt, usum, boff, uoff, fail);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(&hf, fail, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (hf) return SPARKEY_OK;
  if (knob_on(Knob::SnappyDirDebug))
    fprintf(stderr, "[%s dir] parallel: %llu blocks, %llu windows, %llu links\n", codec ? "zstd" : "snappy", (unsigned long long)nb,
            (unsigned long long)nwin, (unsigned long long)nl);
  memset(dir, 0, sizeof(*dir));
  dir->nblk = nb;
  dir->total = tot;
  dir->p = S.data_end;
  dir->done = 1;
  *ok = true;
  return SPARKEY_OK;
}

static int plan_build_snappy(sparkey_plan* pl, const LogHdr& lh, const uint8_t* log_header, const uint8_t* d_log,
                             uint64_t log_len, uint8_t* d_out, uint64_t index_cap, const sparkey_build_opts* opts,
                             hipStream_t s, sparkey_build_stats* stats_out, char* err, size_t err_len) {
  IndexParams ip;
  int rc = make_index_params(lh, *opts, &ip, err, err_len);
  if (rc) return rc;
  if ((uint64_t)ip.index_size > index_cap) {
    set_err(err, err_len, "index buffer too small: need " + std::to_string(ip.index_size));
    return SPARKEY_E_BUFFER;
  }
  if (!d_log || !d_out) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  if (((uintptr_t)d_log & 15) || ((uintptr_t)d_out & 15)) {  // k_snappy_dir reads 16-byte aligned windows
    set_err(err, err_len, "device buffers must be 16-byte aligned");
    return SPARKEY_E_ARG;
  }
  if (lh.compression_block_size < 0) {  // new byte[maxBlockSize] (CompressedReader.java:40-49)
    set_err(err, err_len, "Corrupt log file: negative compression block size");
    return SPARKEY_E_CORRUPT_RECORD;
  }
  HIP_TRY(hipSetDevice(pl->device));
  if (!s) s = pl->own_stream;
  struct Events {  // destroyed on every return path
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
    ~Events() {
      for (auto& x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } evs;
  hipEvent_t* ev = evs.e;
  const bool timed = pl->timer.enabled;
  if (timed) {
    for (auto& e : evs.e) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipEventRecord(ev[0], s));
  }
  SnappyParams S;
  memset(&S, 0, sizeof(S));
  S.log = d_log;
  S.log_len = (int64_t)log_len;
  S.data_end = lh.data_end;
  S.win0 = kLogHeaderSize;
  S.max_block = lh.compression_block_size;
  const uint64_t body = (uint64_t)std::max<int64_t>(0, lh.data_end - kLogHeaderSize);
  const bool zstd = lh.compression_type == 2;
  const char* codec = zstd ? "zstd" : "snappy";
  const int64_t mb = lh.compression_block_size;
  S.lds_bytes = cz_decode_lds(zstd, mb);
  auto decode_launch = [&](hipStream_t st) { return zstd ? launch_zstd_decode(S, st) : launch_snappy_decode(S, st); };
  // Record offsets per block: maxEntriesPerBlock from the header, bounded by what a block can hold
  // (every record is at least 2 bytes), so a corrupt header cannot size a huge allocation; a block
  // with more records than the header allows is still flagged by the walk.
  const uint32_t mepb = (uint32_t)std::max<int64_t>(
      1, std::min<int64_t>(lh.max_entries_per_block, (int64_t)lh.compression_block_size / 2 + 1));
  S.mepb = mepb;
  HIP_TRY(grow(&pl->sn_dir, pl->c_sn_dir, 1));
  HIP_TRY(grow(&pl->sn_err, pl->c_sn_err, 1));
  if (pl->c_sn_blocks == 0) {
    HIP_TRY(grow(&pl->sn_blocks, pl->c_sn_blocks, std::max<uint64_t>(4096, body / (uint64_t)std::max<int64_t>(64, mb / 2))));
  }
  HIP_TRY(grow_keep(&pl->sn_walk, pl->c_sn_walk, pl->c_sn_blocks, 0, s));
  if (!pl->sn_stream) HIP_TRY(hipStreamCreateWithFlags(&pl->sn_stream, hipStreamNonBlocking));
  if (!pl->sn_ev[0]) {
    HIP_TRY(hipEventCreateWithFlags(&pl->sn_ev[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&pl->sn_ev[1], hipEventDisableTiming));
  }
  hipStream_t s2 = pl->sn_stream;
  // The block chain is followed kSnappyChunk blocks per k_snappy_dir launch on `s`; each chunk's
  // blocks are decoded on `s2` while the next chunk is followed.  vcap bounds the virtual log
  // (dir error 3 past it); decode = false only follows the chain.
  SnappyDirResult dir;
  memset(&dir, 0, sizeof(dir));
  uint64_t chunk = kSnappyChunk;
  if (knob_set(Knob::SnappyChunk)) chunk = std::max<uint64_t>(16, (uint64_t)knob(Knob::SnappyChunk));  // tuning
  auto pipeline = [&](int64_t vcap, bool decode) -> hipError_t {
    hipError_t e;
    if ((e = hipMemsetAsync(pl->sn_dir, 0, sizeof(SnappyDirResult), s)) != hipSuccess) return e;
    if ((e = hipEventRecord(pl->sn_ev[0], s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(s2, pl->sn_ev[0], 0)) != hipSuccess) return e;
    memset(&dir, 0, sizeof(dir));
    S.vcap = vcap;
    for (;;) {
      S.blocks = pl->sn_blocks;
      S.blk_cap = pl->c_sn_blocks;
      S.walk = pl->sn_walk;
      S.dir = pl->sn_dir;
      const uint64_t before = dir.nblk;
      S.dir_limit = std::min<uint64_t>(S.blk_cap, before + chunk);
      if (zstd)
        launch_zstd_dir(S, s);
      else
        launch_snappy_dir(S, s);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      if ((e = hipMemcpyAsync(&dir, pl->sn_dir, sizeof(dir), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
      if (decode && dir.nblk > before) {
        S.blk_base = before;
        S.nblk = dir.nblk - before;
        e = decode_launch(s2);
        if (e != hipSuccess && S.lds_bytes) {  // the LDS size was refused: decode in global memory
          (void)hipGetLastError();
          S.lds_bytes = 0;
          e = decode_launch(s2);
        }
        if (e != hipSuccess) return e;
      }
      if (dir.err || dir.done) break;
      if (dir.nblk >= pl->c_sn_blocks) {  // the chain outran the block arrays: grow, keeping them
        if ((e = hipStreamSynchronize(s2)) != hipSuccess) return e;
        const uint64_t want = 2 * pl->c_sn_blocks;
        if ((e = grow_keep(&pl->sn_blocks, pl->c_sn_blocks, want, dir.nblk, s)) != hipSuccess) return e;
        if ((e = grow_keep(&pl->sn_walk, pl->c_sn_walk, want, dir.nblk, s)) != hipSuccess) return e;
      }
    }
    if ((e = hipEventRecord(pl->sn_ev[1], s2)) != hipSuccess) return e;
    return hipStreamWaitEvent(s, pl->sn_ev[1], 0);
  };
  // the reference writer's logs decompress to exactly putSize + deleteSize record bytes
  // (LogHeader.put / delete, LogHeader.java:161-172); a header that understates them gets a
  // directory-only pass to size the virtual log
  // (and a header that overstates them beyond what the blocks can decompress to -- Snappy expands at
  // most 64 bytes per 3-byte copy -- is sized the same way instead of trusted with a huge allocation;
  // ZSTD logs use the same bound: one compressing better takes the directory-only pass)
  const uint64_t ps = (uint64_t)std::max<int64_t>(0, lh.put_size), ds = (uint64_t)std::max<int64_t>(0, lh.delete_size);
  const uint64_t hdr_total = ps + ds < ps ? UINT64_MAX : ps + ds;
  const int64_t vcap0 = hdr_total <= 22 * body + 4096 ? (int64_t)hdr_total : 0;
  bool par = false;  // the directory in parallel, then every block decoded in one launch
  if (!knob_on(Knob::SnappySerialDir)) {
    rc = snappy_par_dir(pl, S, s, zstd ? 1 : 0, &dir, &par, err, err_len);
    if (rc) return rc;
  }
  if (par) {
    HIP_TRY(grow(&pl->sn_vlog, pl->c_sn_vlog, dir.total + kLogHeaderSize + 4096));
    S.vlog = pl->sn_vlog;
    S.blocks = pl->sn_blocks;
    S.walk = pl->sn_walk;
    S.blk_base = 0;
    S.nblk = dir.nblk;
    hipError_t e = decode_launch(s);
    if (e != hipSuccess && S.lds_bytes) {  // the LDS size was refused: decode in global memory
      (void)hipGetLastError();
      S.lds_bytes = 0;
      e = decode_launch(s);
    }
    HIP_TRY(e);
  } else {
    HIP_TRY(grow(&pl->sn_vlog, pl->c_sn_vlog, (uint64_t)vcap0 + kLogHeaderSize + 4096));
    S.vlog = pl->sn_vlog;
    HIP_TRY(pipeline(vcap0, true));
  }
  if (!par && dir.err == 3) {  // more decompressed bytes than vcap0 (putSize = deleteSize = 0 included)
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(pipeline(-1, false));
    if (!dir.err) {
      HIP_TRY(grow(&pl->sn_vlog, pl->c_sn_vlog, dir.total + kLogHeaderSize + 4096));
      S.vlog = pl->sn_vlog;
      HIP_TRY(pipeline((int64_t)dir.total, true));
    }
  }
  if (dir.err) {
    HIP_TRY(hipStreamSynchronize(s));
    set_err(err, err_len, dir.err == 2   ? "Corrupt log file: compressed block larger than the reader's buffers"
                          : dir.err == 4 ? "ZSTD block frame without a content size (not a layout the reference writes)"
                                         : "Corrupt log file: bad compressed block header");
    if (dir.err == 4) return SPARKEY_E_UNSUPPORTED;
    return SPARKEY_E_CORRUPT_RECORD;  // (CompressedReader.fetchBlock fails inside the iterator)
  }
  const uint64_t nblk = dir.nblk;
  const uint64_t vlen = (uint64_t)kLogHeaderSize + dir.total;
  // the virtual log: a NONE header with the same counts, then the decompressed records
  uint8_t vh[kLogHeaderSize];
  memcpy(vh, log_header, kLogHeaderSize);
  wr64(vh + 32, vlen);
  wr32(vh + 64, 0u);
  wr32(vh + 80, 1u);
  HIP_TRY(hipMemcpyAsync(pl->sn_vlog, vh, kLogHeaderSize, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(pl->sn_vlog + vlen, 0, 4096, s));
  HIP_TRY(grow(&pl->sn_recoff, pl->c_sn_recoff, nblk * mepb));
  S.blocks = pl->sn_blocks;
  S.walk = pl->sn_walk;
  S.rec_off = pl->sn_recoff;
  S.vlog_len = (int64_t)vlen;
  S.blk_base = 0;
  S.nblk = nblk;
  launch_snappy_walk(S, s);
  HIP_TRY(hipGetLastError());
  // compose the block walks: a block either starts at a record (CompressedWriter flushes after a
  // spanning record, CompressedWriter.java:71-75) or lies wholly inside the record spanning into it
  std::vector<SnappyWalk> walks(nblk);
  std::vector<SnappyBlock> blocks(nblk);
  if (nblk) {
    HIP_TRY(hipMemcpyAsync(walks.data(), pl->sn_walk, nblk * sizeof(SnappyWalk), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(blocks.data(), pl->sn_blocks, nblk * sizeof(SnappyBlock), hipMemcpyDeviceToHost, s));
  }
  if (timed) HIP_TRY(hipEventRecord(ev[1], s));
  HIP_TRY(hipStreamSynchronize(s));
  int64_t carry = 0;
  for (uint64_t b = 0; b < nblk; b++) {
    const SnappyWalk& w = walks[b];
    if (w.flags & kWalkBadStream) {
      set_err(err, err_len, std::string("Corrupt log file: bad ") + codec + " stream in block at " +
                                std::to_string(blocks[b].file_pos));
      return SPARKEY_E_CORRUPT_RECORD;
    }
    const bool last = b + 1 == nblk;
    if (carry == 0) {
      if (w.flags & ~(last ? kWalkEofFirst : 0u)) {
        set_err(err, err_len, (w.flags & kWalkTooMany)
                                  ? "Corrupt log file: more entries in a block than maxEntriesPerBlock"
                                  : "Corrupt log file: bad record header in block at " +
                                        std::to_string(blocks[b].file_pos));
        return SPARKEY_E_CORRUPT_RECORD;
      }
      carry = w.overflow;
    } else if (carry >= (int64_t)blocks[b].ulen) {
      carry -= blocks[b].ulen;
    } else {
      set_err(err, err_len, "a record ends inside a later compressed block (not a layout CompressedWriter writes)");
      return SPARKEY_E_UNSUPPORTED;
    }
  }
  if (carry) {
    set_err(err, err_len, "Corrupt log file: the last record runs past dataEnd");
    return SPARKEY_E_CORRUPT_RECORD;
  }
  // the normal build over the virtual log, into an internal table
  sparkey_build_opts o2 = *opts;
  o2.method = ip.in_memory ? SPARKEY_METHOD_IN_MEMORY : SPARKEY_METHOD_SORTING;
  LogHdr vlh;
  rc = parse_log_header(vh, kLogHeaderSize, vlen, &vlh, err, err_len);
  IndexParams vip;
  if (!rc) rc = make_index_params(vlh, o2, &vip, err, err_len);
  if (rc) return rc;
  HIP_TRY(grow(&pl->sn_itab, pl->c_sn_itab, (uint64_t)vip.index_size));
  rc = plan_build(pl, vh, pl->sn_vlog, vlen, pl->sn_itab, (uint64_t)vip.index_size, &o2, s, stats_out, err, err_len);
  if (rc) return rc;
  if (timed) HIP_TRY(hipEventRecord(ev[2], s));
  uint8_t hdr[kIndexHeaderSize];
  index_header_template(lh, ip, opts->hash_seed, hdr);
  HIP_TRY(hipMemcpyAsync(d_out, hdr, kIndexHeaderSize, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(pl->sn_err, 0, sizeof(int32_t), s));
  S.itab = pl->sn_itab + kIndexHeaderSize;
  S.otab = d_out + kIndexHeaderSize;
  S.cap = ip.cap;
  S.ihs = vip.hash_size;
  S.ias = vip.addr_size;
  S.hs = ip.hash_size;
  S.as = ip.addr_size;
  S.ebb = ip.ebb;
  S.err = pl->sn_err;
  if (nblk == 0) S.nblk = 1;  // no block: every slot is empty (the search is never reached)
  launch_snappy_rewrite(S, s);
  HIP_TRY(hipGetLastError());
  int32_t rerr = 0;
  HIP_TRY(hipMemcpyAsync(&rerr, pl->sn_err, sizeof(rerr), hipMemcpyDeviceToHost, s));
  hipEvent_t ev_end = ev[3];
  if (timed) HIP_TRY(hipEventRecord(ev_end, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (timed) {  // stages of the front end and the rewrite around the inner build's own stages
    float t0 = 0.f, t1 = 0.f;
    (void)hipEventElapsedTime(&t0, ev[0], ev[1]);
    (void)hipEventElapsedTime(&t1, ev[2], ev_end);
    pl->stage_names.insert(pl->stage_names.begin(), std::string(codec) + "_decode");
    pl->stage_ms.insert(pl->stage_ms.begin(), t0);
    pl->stage_names.push_back(std::string(codec) + "_rewrite");
    pl->stage_ms.push_back(t1);
  }
  if (rerr) {
    set_err(err, err_len, "internal error: a slot's record is not a block record start");
    return SPARKEY_E_CORRUPT_LOG;
  }
  return SPARKEY_OK;
}

// The exact path's segment replay (exact_kernels.hip) after the canonical placement of the PUT
// records in P.out: segments, their records grouped, replayed per size class.  Enqueued only.
static int run_exact_segments(sparkey_plan* pl, BuildParams& P, bool in_memory, hipStream_t s, char* err,
                              size_t err_len) {
  HIP_TRY(grow(&pl->eseg, pl->c_eseg, P.nslabs * (uint64_t)P.slab_cap));
  HIP_TRY(grow(&pl->seg_cnt, pl->c_seg_cnt, P.cap));
  HIP_TRY(grow(&pl->seg_off, pl->c_seg_off, P.cap + 1));
  HIP_TRY(grow(&pl->seg_mark, pl->c_seg_mark, P.cap + 1));
  HIP_TRY(grow(&pl->seg_start, pl->c_seg_start, P.cap));
  HIP_TRY(grow(&pl->seg_cls_cnt, pl->c_seg_cls_cnt, 9 * (P.cap / 1024 + 1)));  // (k_seg_classify's 9 lists)
  HIP_TRY(grow(&pl->seg_cls_off, pl->c_seg_cls_off, 9 * (P.cap / 1024 + 1) + 1));
  HIP_TRY(grow(&pl->seg_len, pl->c_seg_len, P.cap));
  HIP_TRY(grow(&pl->seg_first, pl->c_seg_first, P.cap));
  HIP_TRY(grow(&pl->seg_fun, pl->c_seg_fun, P.cap + 1 + 2 * (P.cap / kScanTile + 64)));  // (+ the scan's scratch)
  HIP_TRY(grow(&pl->seg_krep, pl->c_seg_krep, P.cap));
  HIP_TRY(grow(&pl->ecls, pl->c_ecls, P.max_records));
  const uint64_t scratch = P.cap / kScanTile + 64;
  if (pl->c_su < scratch + 16) {
    HIP_TRY(grow(&pl->scan_u64, pl->c_su, scratch + 16));
    P.scan_scratch_u64 = pl->scan_u64;
  }
  P.eseg = pl->eseg;
  P.seg_cnt = pl->seg_cnt;
  P.seg_off = pl->seg_off;
  P.seg_mark = pl->seg_mark;
  P.seg_start = pl->seg_start;
  P.seg_cls_cnt = pl->seg_cls_cnt;
  P.seg_cls_off = pl->seg_cls_off;
  P.seg_len = pl->seg_len;
  P.seg_first = pl->seg_first;
  P.seg_fun = pl->seg_fun;
  P.seg_krep = pl->seg_krep;
  P.ecls = pl->ecls;
  HIP_TRY(hipMemsetAsync(P.seg_cnt, 0, P.cap * sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync(P.seg_len, 0, P.cap * sizeof(uint32_t), s));
  HIP_TRY(hipMemsetAsync((uint8_t*)pl->d_status + offsetof(Status, num_entries), 0, 2 * sizeof(long long), s));
  HIP_TRY(hipMemsetAsync((uint8_t*)pl->d_status + offsetof(Status, n_segs), 0, sizeof(((Status*)0)->n_segs), s));
  const int64_t dbg_level = knob(Knob::ExactDebug);
  const bool seg_dbg = dbg_level > 0;
  if (seg_dbg) {
    HIP_TRY(grow(&pl->dbg, pl->c_dbg, kSegDebugWords));
    HIP_TRY(hipMemsetAsync(pl->dbg, 0, kSegDebugWords * sizeof(unsigned long long), s));
    P.dbg = pl->dbg;
  } else {
    P.dbg = nullptr;
  }
  if (!pl->side_ok) {
    for (int i = 0; i < 3; i++) {
      HIP_TRY(hipStreamCreateWithFlags(&pl->side.s[i], hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&pl->side.join[i], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&pl->side.fork, hipEventDisableTiming));
    pl->side_ok = true;
  }
  launch_segments(P, s, in_memory ? 0 : 1, &pl->timer, dbg_level >= 2, &pl->side);
  if (seg_dbg) {
    std::vector<unsigned long long> h(kSegDebugWords);
    HIP_TRY(hipMemcpyAsync(h.data(), pl->dbg, h.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    static const char* cname[4] = {"mid", "large", "huge", "lanes (stage, rank, replay, write)"};
    for (int c = 0, b0 = 0; c < 4; b0 += kSegDebugWaves[c], c++) {
      const unsigned b1 = b0 + kSegDebugWaves[c];
      double sum[8] = {0};
      unsigned long long mx[8] = {0};
      for (unsigned b = b0; b < b1; b++)
        for (int i = 0; i < 8; i++) {
          sum[i] += (double)h[b * 8 + i];
          mx[i] = std::max(mx[i], h[b * 8 + i]);
        }
      fprintf(stderr, "[exact %s] segs %.0f recs %.0f | cycles/seg stage %.0f sort %.0f replay %.0f write %.0f | "
                      "max wave: segs %llu stage %llu sort %llu replay %llu write %llu\n",
              cname[c], sum[4], sum[5], sum[0] / std::max(1.0, sum[4]), sum[1] / std::max(1.0, sum[4]),
              sum[2] / std::max(1.0, sum[4]), sum[3] / std::max(1.0, sum[4]), mx[4], mx[0], mx[1], mx[2], mx[3]);
    }
  }
  return SPARKEY_OK;
}

static int plan_build(sparkey_plan* pl, const uint8_t* log_header, const uint8_t* d_log, uint64_t log_len,
                      uint8_t* d_out, uint64_t index_cap, const sparkey_build_opts* opts, hipStream_t s,
                      sparkey_build_stats* stats_out, char* err, size_t err_len) {
  if (!pl || !log_header || !opts) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  LogHdr lh;
  int rc = parse_log_header(log_header, 84, log_len, &lh, err, err_len, true);
  if (rc) return rc;
  if (lh.compression_type != 0)
    return plan_build_snappy(pl, lh, log_header, d_log, log_len, d_out, index_cap, opts, s, stats_out, err, err_len);
  IndexParams ip;
  rc = make_index_params(lh, *opts, &ip, err, err_len);
  if (rc) return rc;
  if ((uint64_t)ip.index_size > index_cap) {
    set_err(err, err_len, "index buffer too small: need " + std::to_string(ip.index_size));
    return SPARKEY_E_BUFFER;
  }
  if (((uintptr_t)d_log & 15) || ((uintptr_t)d_out & 15)) {
    set_err(err, err_len, "device buffers must be 16-byte aligned");
    return SPARKEY_E_ARG;
  }
  HIP_TRY(hipSetDevice(pl->device));
  if (!s) s = pl->own_stream;

  BuildParams P;
  rc = setup_params(lh, ip, *opts, d_log, log_len, kLogHeaderSize, std::max<int64_t>(lh.data_end, kLogHeaderSize),
                    &P, err, err_len);
  if (rc) return rc;
  P.out = d_out;
  P.st = pl->d_status;
  P.skip_del = 1;  // DELETEs stay out of the canonical placement (the exact path's segments)
  const bool fused_framing = P.max_rec_len <= 4096;

  uint64_t nrec = (uint64_t)std::max<int64_t>(0, lh.num_puts) + (uint64_t)std::max<int64_t>(0, lh.num_deletes);
  uint8_t hdr[kIndexHeaderSize];
  index_header_template(lh, ip, opts->hash_seed, hdr);

  // k_frame3 for one-byte-VLQ logs whose chunks hold a few records each (its lists' sizes), k_frame
  // for the rest; both fall back to the serial walk, which alone reports errors
  const bool use_frame3 = fused_framing && want_frame3(P, lh, kLogHeaderSize, std::max<int64_t>(lh.data_end, kLogHeaderSize));
  const FrameGeom geom0 = get_geom(P);
  // the serial_framing switch forces the exact serial walk (smoke() and the tests check every path)
  const bool force_serial = knob_on(Knob::SerialFraming);
  const int spec_path = fused_framing && !force_serial ? (use_frame3 ? 4 : 0) : 1;
  int framing_path = spec_path, placement_path = 0;
  if (const int64_t R = force_serial ? 0 : uniform_record_size(lh)) {  // k_frame_uniform: every record is exactly R bytes
    framing_path = 2;
    P.uni_n = (uint64_t)lh.num_puts;
    P.uni_rec = R;
  }
  float ms = 0.f;
  Status& st = *pl->h_status;
  // the framing kernels write each wave's entries into a slab sized from the header's record count
  // (twice the mean per wave + 32); a wave that holds more grows the slabs and the build is redone
  auto slab_for = [&](const FrameGeom& g) -> uint32_t {
    const uint64_t nw = std::max<uint64_t>(1, g.nchunks ? (g.nchunks + g.w - 1) / g.w : 0);
    return (uint32_t)std::min<uint64_t>(kPartTile, std::max<uint64_t>(64, 2 * ((nrec + nw - 1) / nw) + 32));
  };
  uint32_t slab_cap = slab_for(geom0);
  bool use_regions = !knob_on(Knob::NoRegions), regions_used = false, buckets_used = false;
  bool use_fixed = true;  // k_part2st / k_part2s in one pass into fixed bucket regions
  bool use_buckets = !knob_on(Knob::NoBuckets);
  for (int attempt = 0; attempt < 8; attempt++) {
    set_geom(P, geom0);
    rc = reserve_for_framing(pl, P, framing_path, nrec, slab_cap, err, err_len);
    if (rc) return rc;
    if (knob_on(Knob::FrameDebug)) {  // per-wave phase counters: 16 words per k_frame / k_frame3 wave
      const uint64_t nw = std::max<uint64_t>(std::max<uint64_t>(P.nchunks, P.fr_nchunks ? (P.fr_nchunks + P.fr_w - 1) / P.fr_w : 0), 1);
      HIP_TRY(grow(&pl->dbg, pl->c_dbg, 16 * nw));
      HIP_TRY(hipMemsetAsync(pl->dbg, 0, 16 * nw * sizeof(unsigned long long), s));
      P.dbg = pl->dbg;
    }
    if (knob_on(Knob::Part2Debug)) {
      HIP_TRY(grow(&pl->dbg, pl->c_dbg, 8 * 256));
      HIP_TRY(hipMemsetAsync(pl->dbg, 0, 8 * 256 * sizeof(unsigned long long), s));
      P.part_dbg = pl->dbg;
    }

    HIP_TRY(hipEventRecord(pl->ev0, s));
    pl->timer.begin(s);
    // k_frame_uniform's workgroups are the partition tiles: it does partition pass 1 itself into
    // digit regions of ent3 sized for the binomial spread of the digit counts (a region that fills
    // up redoes the build with the separate pass), or leaves k_part1_hist's histogram
    const bool tiles = framing_path == 2 && P.slab_cap == (uint32_t)kPartTile && P.part_group == 1;
    // the other framings' slabs: pass 1 into the same fixed digit regions by k_part1_regions (one read
    // of the entries instead of k_part1_hist + k_part1_scatter's two)
    const bool slab_regions = !tiles;
    // k_frame3: each entry straight into its placement bucket's fixed region (an atomic on the bucket's
    // count), no partition pass at all.  (k_frame_uniform keeps its pass 1 into the digit regions: its
    // per-tile digit runs beat an atomic per entry, C2 frame 0.28 against 0.62 ms, profiles/r04/)
    // A log whose header counts DELETEs goes to the exact path, which replays from the slabs: it
    // frames into them from the start (bucket regions first and slabs again cost churn 0.8 ms).
    // k_frame too, when its waves hold about one round of records (C3's shape through k_frame: build
    // 1.41 against 1.50 ms per 10M); a wave of several rounds waits out one atomic round trip each
    // (c1x's 14-26 byte records, ~300 a wave: frame 0.59 against 0.21 ms with its slabs partitioned)
    const uint64_t nwv = P.fr_nchunks ? (P.fr_nchunks + P.fr_w - 1) / P.fr_w : 1;
    const bool frame_rounds1 = framing_path == 0 && (double)nrec / (double)std::max<uint64_t>(nwv, 1) <= 64.0;
    const bool to_buckets = (framing_path == 4 || frame_rounds1) && use_buckets && use_fixed && P.b_lo == 0 &&
                            P.no_deletes;
    P.p1_bucket = to_buckets ? 1 : 0;
    P.p1_region = 0;
    P.p1_kernel = 0;
    if ((tiles || slab_regions) && use_regions && !to_buckets) {
      const double expect = (double)nrec * (double)P.bpp * (double)kBucket / (double)P.cap;
      uint64_t rc_cap = ((uint64_t)(expect + 8.0 * std::sqrt(expect) + 1024.0) + 63) & ~63ull;
      if (knob_set(Knob::RegionCap)) rc_cap = std::max<uint64_t>(1, (uint64_t)knob(Knob::RegionCap));  // (tests)
      HIP_TRY(grow(&pl->ent2, pl->c_ent2, 256 * rc_cap));
      HIP_TRY(grow(&pl->ent3, pl->c_ent3, 256 * rc_cap));
      HIP_TRY(grow(&pl->p1_fill, pl->c_p1_fill, 256));
      P.ent2 = pl->ent2;
      P.ent3 = pl->ent3;
      P.max_records = std::min(pl->c_ent2, pl->c_ent3);
      P.p1_fill = pl->p1_fill;
      P.p1_region = rc_cap;
      P.p1_kernel = tiles ? 0 : 1;
    }
    // the header, the status reset and the region cursors in one launch
    launch_build_init(d_out, hdr, pl->d_status, P.p1_region ? pl->p1_fill : nullptr, P.p1_region ? 256u : 0u, s);
    P.p1_hist_ready = tiles && !P.p1_region && !to_buckets ? 1 : 0;
    regions_used = P.p1_region != 0 && !P.p1_kernel;  // (partition passes: 1 when the framing did pass 1)
    buckets_used = to_buckets;                         // (0 when it wrote the buckets)
    // k_part2s: pass 2 also sorts each bucket by wanted slot and leaves the carry functions
    P.p2_sorted = P.bpp <= kP2SortedMaxBpp && !to_buckets && !knob_on(Knob::Part2TwoLevel) ? 1 : 0;
    // fixed bucket regions: k_part2st (fused carry) up to kP2SortedMaxBpp buckets a digit, k_part2f past
    // that (from the digit regions of pass 1)
    P.p2_fixed = use_fixed && (to_buckets || P.p2_sorted || (P.p1_region && part2f_fits(P.bpp))) ? 1 : 0;
    if (P.p2_fixed) {  // bucket b's entries at ent2[b * kPlaceLdsMax ..)
      HIP_TRY(grow(&pl->ent2, pl->c_ent2, std::max<uint64_t>(P.max_records, P.nbuckets * (uint64_t)kPlaceLdsMax)));
      P.ent2 = pl->ent2;
    }
    if (to_buckets) HIP_TRY(hipMemsetAsync(P.bcount, 0, P.nbuckets * sizeof(uint32_t), s));  // (the cursors)
    P.fold_stats = 1;  // the stats parts from the placement (k_stats only for buckets it could not place)
    // the carry composition inside k_part2st / k_part2s (their fixed-region pass), no summary / scan /
    // carry kernels
    P.fused_carry = P.p2_fixed && P.p2_sorted ? 1 : 0;
    P.dfun = pl->dfun;
    P.dcarry = pl->dcarry;
    if (P.fused_carry) {
      pl->epoch = pl->epoch % ((1u << 22) - 1) + 1;
      P.epoch = pl->epoch;
    }
    // 12-byte entries (CEntry: hash + record index) from the uniform framing through pass 2 to the
    // placement, where the record index gives the address: a quarter less of the entry round trip.
    // C4 (1B): 54.3 against 60.5 ms on one box; C2: 0-6 us a build (profiles/r06/c2/, c4/).  Only the
    // digit regions compact (kCompactIn alone) measured slower than neither.
    P.compact = framing_path == 2 && tiles && P.p1_region && !P.p1_kernel && (part2st_per(P) > 0 || part2_direct(P)) &&
                        P.uni_n < (1ull << 32) && !knob_on(Knob::NoCompact) ? (kCompactIn | kCompactOut) : 0;
    // pass 2 in two levels where it would scatter over thousands of bucket regions a digit (C4): the
    // digit regions into kSub sub-digit regions each, sized like the digit regions (expected + 8
    // sigma), then one sub-digit's buckets a workgroup (k_part2_sub, k_part2f<.., kSubIn>)
    P.sub_region = 0;
    const int64_t two_level = knob(Knob::Part2TwoLevel);
    if (part2_direct(P) && two_level != 0 && (two_level > 0 || P.bpp >= 2 * kSub)) {
      const double expect = (double)nrec * (double)((P.bpp + kSub - 1) / kSub) * (double)kBucket / (double)P.cap;
      const uint64_t sub_cap = ((uint64_t)(expect + 8.0 * std::sqrt(expect) + 1024.0) + 63) & ~63ull;
      HIP_TRY(grow(&pl->sub_ent, pl->c_sub_ent, 256ull * kSub * sub_cap));
      HIP_TRY(grow(&pl->sub_fill, pl->c_sub_fill, 256ull * kSub));
      HIP_TRY(hipMemsetAsync(pl->sub_fill, 0, 256ull * kSub * sizeof(uint32_t), s));
      P.sub_region = sub_cap;
      P.sub_ent = pl->sub_ent;
      P.sub_fill = pl->sub_fill;
    }
    // an attempt whose framing failed, stopped early or overflowed skips every later stage (the host
    // redoes it or reports the error): no stage reads a region the framing left half-written
    P.abort_on_fail = 1;
    rc = launch_framing(pl, P, framing_path, s, err, err_len);
    if (rc) return rc;
    const int64_t inject = knob(Knob::InjectForeign);
    if (inject == 1) launch_inject_foreign(P, s, 1);
    launch_partition(P, s, &pl->timer);
    if (inject == 2) launch_inject_foreign(P, s, 2);
    launch_place_fast(P, s, &pl->timer);
    // (the folded stats' last block also hands the host its status: no k_status_out launch)
    P.status_host = P.fold_stats ? pl->h_status_dev : nullptr;
    if (P.fold_stats) launch_stats_folded(P, s, &pl->timer);
    else launch_stats(P, s, 0, &pl->timer);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(pl->ev1, s));
    if (!P.fold_stats) launch_status_out(pl->d_status, pl->h_status_dev, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipEventElapsedTime(&ms, pl->ev0, pl->ev1));
    print_frame_debug(pl, P);
    print_part2_debug(P);
    if (st.guard) {  // (a bounds check tripped: a bug, never a property of the input -- no retry)
      set_err(err, err_len, "internal error: partition/placement bounds check tripped (bits " + std::to_string(st.guard) + ")");
      return SPARKEY_E_GPU;
    }
    if (slab_framing(framing_path) && st.max_wave_count > slab_cap) {  // a wave overflowed its slab
      slab_cap = (uint32_t)std::min<uint64_t>(kPartTile, ((uint64_t)st.max_wave_count + 63) & ~63ull);
      continue;
    }
    if (st.overflow || st.n_records > P.max_records) {  // header under-counts records: grow and redo
      nrec = std::max<uint64_t>(st.n_records, nrec * 2 + 1);
      continue;
    }
    if (knob_on(Knob::FrameDebug) && (st.spec_fail || st.err != ~0ull))
      fprintf(stderr, "[framing] path %d: spec_fail %u err %llx (pos %llu)\n", framing_path, st.spec_fail,
              (unsigned long long)st.err, (unsigned long long)(st.err >> 8));
    // (a digit region filled by k_part1_regions is the partition's business, not the framing's)
    const unsigned fspec = st.spec_fail & ~(P.p1_kernel ? kSpecRegionFull : 0u);
    if (framing_path == 4 && (fspec || st.err != ~0ull)) {  // k_frame3's lists or speculation: k_frame
      framing_path = 0;
      continue;
    }
    if (framing_path == 0 && (fspec || st.err != ~0ull)) {  // only the serial walk reports
      framing_path = 1;
      continue;
    }
    if (st.p2_overflow && P.p2_fixed) {  // a bucket outgrew its fixed region: dense bucket runs
      use_fixed = false;
      continue;
    }

    if ((st.spec_fail & kSpecRegionFull) && (P.p1_kernel || !(st.spec_fail & ~kSpecRegionFull))) {
      use_regions = false;  // a digit region filled up (skewed hashes): the two-pass partition
      continue;
    }
    if (framing_path == 2 && st.spec_fail) {  // a record differs from the header's uniform shape
      framing_path = spec_path;
      continue;
    }
    break;
  }
  P.abort_on_fail = 0;  // (the exact path's stages report their own errors, at the lowest log position)
  const int entry_bytes = P.compact ? 12 : 16;
  P.compact = 0;        // (and frame into 16-byte slabs)
  rc = status_error(st, err, err_len);
  if (rc) return rc;
  if (st.overflow || st.spec_fail) {
    set_err(err, err_len, "Corrupt log file: framing did not converge");
    return SPARKEY_E_CORRUPT_LOG;
  }
  if (st.stats_pending && !(st.n_deletes > 0 || st.dup || st.dup_overflow || st.full || st.n_pairs > P.pair_cap)) {
    // folded stats did not cover every slot (a bucket was placed by the global kernel): the pass.
    // The status is read again after it, which this branch needs for correctness: k_stats_folded's
    // block 0 hands the status over as soon as it sees stats_pending, while other blocks may still be
    // verifying equal-hash pairs (st->dup).
    float ms2 = 0.f;
    HIP_TRY(hipEventRecord(pl->ev0, s));
    launch_stats(P, s, 0, &pl->timer);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(pl->ev1, s));
    HIP_TRY(hipMemcpyAsync(pl->h_status, pl->d_status, sizeof(Status), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipEventElapsedTime(&ms2, pl->ev0, pl->ev1));
    ms += ms2;
  }
  // Logs outside the canonical case (DELETEs, duplicate keys) replay the reference's put/delete
  // exactly: per independent slot segment of the canonical PUT placement (placement_path 2), or,
  // when that placement left no empty slot, on one lane over the whole table (placement_path 1).
  if (st.n_deletes > 0 || st.dup || st.dup_overflow || st.full || st.n_pairs > P.pair_cap) {
    const bool serial = st.full || knob_on(Knob::ExactSerial);
    placement_path = serial ? 1 : 2;
    P.p1_hist_ready = 0;  // the exact path's partitions (DELETEs left out) count their own digits
    P.p2_sorted = 0;
    // The exact path replays the entries in log order, from the framing's slabs (`ent`).  The slab
    // framings left them there (k_part1_regions only read them); the uniform framing wrote straight
    // into the digit regions and k_frame3 into the bucket regions, so they frame again into `ent`.
    const bool reframe = (P.p1_region && !P.p1_kernel) || P.p1_bucket;  // (k_frame3 wrote the buckets only)
    P.p1_bucket = 0;
    if (reframe) {
      P.p1_region = 0;
      // Every attempt starts from reset status words (err, spec_fail, overflow, the slab high-water
      // mark, the DELETE count) and gets the main loop's checks: a slab that overflowed or more records
      // than the workspace grow and redo it; a speculative framing that fails (spec_fail, or an error
      // only the serial walk may report) goes down the framing paths like the first framing did.  The
      // DELETE count is this framing's own, and must equal the first framing's.
      const unsigned long long ndel0 = st.n_deletes;
      if (knob_set(Knob::ReframeSpinTicks)) P.fr_spin_ticks = (uint64_t)knob(Knob::ReframeSpinTicks);
      uint64_t nrec2 = std::max<uint64_t>(nrec, st.n_records);
      for (int fp = framing_path, tries = 0;; tries++) {
        if (tries >= 16) {
          set_err(err, err_len, "internal error: the exact path's framing did not settle");
          return SPARKEY_E_GPU;
        }
        set_geom(P, geom0);
        rc = reserve_for_framing(pl, P, fp, nrec2, slab_cap, err, err_len);
        if (rc) return rc;
        if (knob_set(Knob::ReframeSpinTicks)) P.fr_spin_ticks = (uint64_t)knob(Knob::ReframeSpinTicks);
        launch_status_reframe(pl->d_status, s);
        rc = launch_framing(pl, P, fp, s, err, err_len);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(pl->h_status, pl->d_status, sizeof(Status), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (slab_framing(fp) && st.max_wave_count > slab_cap) {
          slab_cap = (uint32_t)std::min<uint64_t>(kPartTile, ((uint64_t)st.max_wave_count + 63) & ~63ull);
          continue;
        }
        if (st.overflow || st.n_records > P.max_records) {
          nrec2 = std::max<uint64_t>(st.n_records, nrec2 * 2 + 1);
          continue;
        }
        if ((!st.spec_fail && st.err == ~0ull) || fp == 1) break;
        fp = fp == 4 ? 0 : 1;
      }
      if (st.err == ~0ull && st.n_deletes != ndel0) {
        set_err(err, err_len, "internal error: the second framing counted " + std::to_string(st.n_deletes) +
                                  " DELETEs, the first " + std::to_string(ndel0));
        return SPARKEY_E_GPU;
      }
    }
    P.p1_region = 0;
    P.p1_kernel = 0;
    float ms2 = 0.f;
    HIP_TRY(hipEventRecord(pl->ev0, s));
    if (serial) {
      BuildParams Pd = P;
      Pd.skip_del = 0;  // the single lane replays every record
      Pd.p1_hist_ready = 0;
      if (!ip.in_memory) {
        launch_partition_quiet(Pd, s);
        launch_place_global(Pd, s, 1, 0);  // (wantedSlot, address) order into ent3
      }
      HIP_TRY(hipMemsetAsync(d_out + kIndexHeaderSize, 0, (size_t)(ip.index_size - kIndexHeaderSize), s));
      launch_sequential(Pd, s, ip.in_memory ? 0 : 1);
    } else {
      rc = run_exact_segments(pl, P, ip.in_memory, s, err, err_len);
      if (rc) return rc;
    }
    launch_stats(P, s, 1, &pl->timer);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(pl->ev1, s));
    HIP_TRY(hipMemcpyAsync(pl->h_status, pl->d_status, sizeof(Status), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipEventElapsedTime(&ms2, pl->ev0, pl->ev1));
    ms += ms2;
    rc = status_error(st, err, err_len);
    if (rc) return rc;
    if (st.guard) {
      set_err(err, err_len, "internal error: exact-path bounds check tripped (bits " + std::to_string(st.guard) + ")");
      return SPARKEY_E_GPU;
    }
  }
  if (pl->timer.enabled) {
    pl->stage_names.clear();
    pl->stage_ms.clear();
    for (size_t i = 1; i < pl->timer.used; i++) {
      float t = 0.f;
      (void)hipEventElapsedTime(&t, pl->timer.evs[i - 1], pl->timer.evs[i]);
      pl->stage_names.push_back(pl->timer.names[i]);
      pl->stage_ms.push_back(t);
    }
  }
  fill_stats(stats_out, st, ip, placement_path, framing_path, ms, buckets_used ? 0 : regions_used ? 1 : 2,
             entry_bytes);
  return SPARKEY_OK;
}

// LogHeader.read with the file's real length (file_build.cpp): the dataEnd > file length check
// (LogHeader.java:81-83) needs it.
// Ranks of one sharded build that share a device (file_build.cpp): framing takes regions by ticket.
void sk_plan_set_shared_device(sparkey_plan* pl, bool shared) {
  if (pl) pl->shared_device = shared;
}

int sk_check_log_header(const uint8_t* b, uint64_t hdr_len, uint64_t file_len, char* err, size_t err_len) {
  LogHdr lh;
  return parse_log_header(b, hdr_len, file_len, &lh, err, err_len, true);
}

extern "C" {

const char* sparkey_gpu_version(void) { return "sparkey-mi355x 0.1 (gfx950)"; }

// Batched LogWriter.put / delete (LogWriter.java:96-115, UncompressedBlockOutput.java:34-45,
// LogHeader.java:161-172): records written from d_out on, header84 updated in place.
int sparkey_log_append(sparkey_plan* pl, uint8_t* header84, const uint8_t* d_kind, const uint8_t* d_keys,
                       const uint64_t* d_key_off, const uint8_t* d_values, const uint64_t* d_val_off, uint64_t n,
                       uint8_t* d_out, uint64_t out_cap, uint64_t* bytes_written, void* stream, char* err,
                       size_t err_len) {
  if (!pl || !header84 || (n && (!d_kind || !d_keys || !d_key_off || !d_values || !d_val_off || !d_out))) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  LogHdr lh;
  int rc = parse_log_header(header84, kLogHeaderSize, (uint64_t)INT64_MAX, &lh, err, err_len);
  if (rc) return rc;
  if (lh.compression_type != 0) {
    set_err(err, err_len, "compressed logs are not supported");
    return SPARKEY_E_UNSUPPORTED;
  }
  if (bytes_written) *bytes_written = 0;
  if (n == 0) return SPARKEY_OK;
  HIP_TRY(hipSetDevice(pl->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const uint64_t nblk = (n + 255) / 256;
  HIP_TRY(grow(&pl->app_i64, pl->c_app_i64, 2 * n + 6 * nblk + 16));
  HIP_TRY(grow(&pl->app_u32, pl->c_app_u32, n));
  HIP_TRY(grow(&pl->app_u64, pl->c_app_u64, n + 1));
  const uint64_t scratch = n / kScanTile + 64;
  HIP_TRY(grow(&pl->scan_u64, pl->c_su, scratch + 16));
  HIP_TRY(grow(&pl->app_scan, pl->c_app_scan, scratch + 16));
  AppendParams A;
  memset(&A, 0, sizeof(A));
  A.n = n;
  A.kind = d_kind;
  A.keys = d_keys;
  A.key_off = d_key_off;
  A.values = d_values;
  A.val_off = d_val_off;
  A.max_key_len0 = lh.max_key_len;
  A.out = d_out;
  A.keymax = pl->app_i64;
  A.keymax_pre = pl->app_i64 + n;
  A.partials = pl->app_i64 + 2 * n;
  A.sums = pl->app_i64 + 2 * n + 6 * nblk;
  A.sizes = pl->app_u32;
  A.off = pl->app_u64;
  A.total = pl->app_u64 + n;
  A.scan_u64 = pl->scan_u64;
  A.scan_i64 = pl->app_scan;
  // the appended bytes must fit: sizes first, then the write
  launch_append_sizes(A, s);
  HIP_TRY(hipGetLastError());
  int64_t sums[6];
  uint64_t total = 0;
  HIP_TRY(hipMemcpyAsync(sums, A.sums, sizeof(sums), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&total, A.total, sizeof(total), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (total > out_cap) {
    set_err(err, err_len, "output buffer too small: need " + std::to_string(total) + " bytes");
    return SPARKEY_E_BUFFER;
  }
  A.mis = (uint32_t)((uintptr_t)d_out & 15);
  A.nwords = total ? (total + A.mis + 15) / 16 : 0;
  HIP_TRY(grow(&pl->app_map, pl->c_app_map, A.nwords + 1));
  A.map = pl->app_map;
  launch_append_write(A, s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  // header (LogHeader.put / delete, LogWriter.writeHeader: maxEntriesPerBlock 1, dataEnd = file end)
  wr64(header84 + 16, (uint64_t)(lh.num_puts + sums[0]));
  wr64(header84 + 24, (uint64_t)(lh.num_deletes + sums[1]));
  wr64(header84 + 32, (uint64_t)(lh.data_end + (int64_t)total));
  wr64(header84 + 40, (uint64_t)std::max<int64_t>(lh.max_key_len, sums[4]));
  wr64(header84 + 48, (uint64_t)std::max<int64_t>(lh.max_value_len, sums[5]));
  wr64(header84 + 56, (uint64_t)(lh.delete_size + sums[3]));
  wr64(header84 + 72, (uint64_t)(lh.put_size + sums[2]));
  wr32(header84 + 80, 1u);
  if (bytes_written) *bytes_written = total;
  return SPARKEY_OK;
}

// Batched IndexHash.get (IndexHash.java:398-452): IndexHash.open's checks (IndexHash.java:72-80,
// 115-121, 352-356), then one lane per query.
int sparkey_get_batch(sparkey_plan* pl, const uint8_t* d_log, uint64_t log_len, const uint8_t* d_index,
                      uint64_t index_len, const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n,
                      int64_t* d_value_pos, int64_t* d_value_len, void* stream, char* err, size_t err_len) {
  if (!pl || !d_log || !d_index || (n && (!d_keys || !d_key_off || !d_value_pos || !d_value_len))) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  HIP_TRY(hipSetDevice(pl->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (index_len < kIndexHeaderSize || log_len < kLogHeaderSize) {
    set_err(err, err_len, "Corrupt index file - incorrect size");
    return SPARKEY_E_CORRUPT_DATA;
  }
  uint8_t ih[kIndexHeaderSize], lhb[kLogHeaderSize];
  HIP_TRY(hipMemcpyAsync(ih, d_index, kIndexHeaderSize, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(lhb, d_log, kLogHeaderSize, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  LogHdr lh;
  int rc = parse_log_header(lhb, kLogHeaderSize, log_len, &lh, err, err_len);
  if (rc) return rc;
  if (rd32(ih) != kIndexMagic) {
    set_err(err, err_len, "File is not a Sparkey index file");
    return SPARKEY_E_NOT_LOG;
  }
  if (rd32(ih + 4) != 1) {
    set_err(err, err_len, "Incompatible index file version");
    return SPARKEY_E_VERSION;
  }
  if ((int32_t)rd32(ih + 12) != lh.file_id) {
    set_err(err, err_len, "Log file did not match index file");
    return SPARKEY_E_ARG;
  }
  const int64_t data_end = (int64_t)rd64(ih + 20);
  if (data_end > lh.data_end) {
    set_err(err, err_len, "Corrupt index file: referencing more data than exists in the log file");
    return SPARKEY_E_CORRUPT_DATA;
  }
  LookupParams L;
  memset(&L, 0, sizeof(L));
  L.hash_size = (int32_t)rd32(ih + 72);
  L.addr_size = (int32_t)rd32(ih + 68);
  L.cap = rd64(ih + 76);
  L.ebb = (int32_t)rd32(ih + 92);
  L.seed = rd32(ih + 16);
  L.max_disp = (int64_t)rd64(ih + 84);
  if ((L.hash_size != 4 && L.hash_size != 8) || (L.addr_size != 4 && L.addr_size != 8) || L.cap == 0) {
    set_err(err, err_len, "Corrupt index header");
    return SPARKEY_E_CORRUPT_DATA;
  }
  L.slot_size = L.hash_size + L.addr_size;
  if (index_len != kIndexHeaderSize + (uint64_t)L.slot_size * L.cap) {
    set_err(err, err_len, "Corrupt index file - incorrect size. Expected " +
                              std::to_string(kIndexHeaderSize + (uint64_t)L.slot_size * L.cap) + " but was " +
                              std::to_string(index_len));
    return SPARKEY_E_CORRUPT_DATA;
  }
  if (lh.compression_type != 0) {
    set_err(err, err_len, "compressed logs are not supported");
    return SPARKEY_E_UNSUPPORTED;
  }
  L.log = d_log;
  L.log_len = log_len;
  L.slots = d_index + kIndexHeaderSize;
  L.mod = make_fastmod(L.cap);
  L.keys = d_keys;
  L.key_off = d_key_off;
  L.n = n;
  L.value_pos = d_value_pos;
  L.value_len = d_value_len;
  HIP_TRY(grow(&pl->small, pl->c_small, 512));
  L.err = (unsigned long long*)pl->small + 400;
  const unsigned long long none = ~0ull;
  HIP_TRY(hipMemcpyAsync(L.err, &none, sizeof(none), hipMemcpyHostToDevice, s));
  launch_get(L, s);
  HIP_TRY(hipGetLastError());
  unsigned long long e = 0;
  HIP_TRY(hipMemcpyAsync(&e, L.err, sizeof(e), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (e != ~0ull) {
    const int code = -(int)(e & 0xff);
    set_err(err, err_len, std::string(code == SPARKEY_E_CORRUPT_DATA ? "Invalid data - reference to delete entry"
                                                                      : code_message(code)) +
                              " (query " + std::to_string(e >> 8) + ")");
    return code;
  }
  return SPARKEY_OK;
}

// Batched HashType.hash (+ getWantedSlot) on device keys: the build kernels' own device functions.
int sparkey_hash_batch(sparkey_plan* pl, const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n,
                       int32_t hash_size, int32_t hash_seed, uint64_t capacity, uint64_t* d_hash, uint64_t* d_slot,
                       void* stream, char* err, size_t err_len) {
  if (!pl || (n && (!d_keys || !d_key_off || !d_hash))) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  if (hash_size != 4 && hash_size != 8) {
    set_err(err, err_len, "Can't support hash size " + std::to_string(hash_size));
    return SPARKEY_E_ARG;
  }
  HIP_TRY(hipSetDevice(pl->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  LookupParams L;
  memset(&L, 0, sizeof(L));
  L.keys = d_keys;
  L.key_off = d_key_off;
  L.n = n;
  L.hash_size = hash_size;
  L.seed = (uint32_t)hash_seed;
  if (capacity) L.mod = make_fastmod(capacity);
  launch_hash_batch(L, d_hash, capacity ? d_slot : nullptr, s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  return SPARKEY_OK;
}

int sparkey_wanted_slot_batch(sparkey_plan* pl, const uint64_t* d_hash, uint64_t n, uint64_t capacity,
                              uint64_t* d_slot, void* stream, char* err, size_t err_len) {
  if (!pl || capacity == 0 || (n && (!d_hash || !d_slot))) {
    set_err(err, err_len, "null argument or zero capacity");
    return SPARKEY_E_ARG;
  }
  HIP_TRY(hipSetDevice(pl->device));
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  launch_slot_batch(d_hash, n, make_fastmod(capacity), d_slot, s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  return SPARKEY_OK;
}

const char* sparkey_strerror(int code) { return code_message(code); }

int sparkey_plan_create(sparkey_plan** plan_out, int32_t device, uint64_t max_log_bytes, uint64_t max_records,
                        char* err, size_t err_len) {
  (void)max_log_bytes;
  if (!plan_out) return SPARKEY_E_ARG;
  *plan_out = nullptr;
  int ndev = 0;
  const hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= device || device < 0) {
    set_err(err, err_len, "no HIP device " + std::to_string(device) + " (" + hipGetErrorString(e) + ", " +
                              std::to_string(ndev) + " devices)");
    return SPARKEY_E_GPU;
  }
  HIP_TRY(hipSetDevice(device));
  sparkey_plan* pl = new sparkey_plan();
  pl->device = device;
  if (hipStreamCreateWithFlags(&pl->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&pl->d_status, sizeof(Status)) != hipSuccess ||
      hipHostMalloc((void**)&pl->h_status, sizeof(Status), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&pl->h_status_dev, pl->h_status, 0) != hipSuccess ||
      hipEventCreate(&pl->ev0) != hipSuccess || hipEventCreate(&pl->ev1) != hipSuccess) {
    sparkey_plan_destroy(pl);
    set_err(err, err_len, "HIP allocation failed");
    return SPARKEY_E_GPU;
  }
  if (max_records) {
    const uint64_t nchunks = max_log_bytes / kChunk + 1;
    const uint64_t cap = max_records * 2;
    const uint64_t nslabs = max_log_bytes / 8192 + 2;
    int rc = plan_reserve(pl, nchunks, max_records, nslabs * 192, nslabs, nslabs, cap / kBucket + 1, cap, err, err_len);
    if (rc) {
      sparkey_plan_destroy(pl);
      return rc;
    }
  }
  *plan_out = pl;
  return SPARKEY_OK;
}

int sparkey_plan_build_device(sparkey_plan* plan, const uint8_t* log_header, const uint8_t* d_log, uint64_t log_len,
                              uint8_t* d_index_out, uint64_t index_cap, const sparkey_build_opts* opts, void* stream,
                              sparkey_build_stats* stats_out, char* err, size_t err_len) {
  return plan_build(plan, log_header, d_log, log_len, d_index_out, index_cap, opts, (hipStream_t)stream, stats_out,
                    err, err_len);
}

void sparkey_plan_set_profiling(sparkey_plan* plan, int32_t enabled) {
  if (plan) plan->timer.enabled = enabled != 0;
  if (plan && !enabled) {
    plan->stage_names.clear();
    plan->stage_ms.clear();
  }
}

int32_t sparkey_plan_stage_count(const sparkey_plan* plan) { return plan ? (int32_t)plan->stage_names.size() : 0; }

const char* sparkey_plan_stage_name(const sparkey_plan* plan, int32_t i) {
  if (!plan || i < 0 || i >= (int32_t)plan->stage_names.size()) return "";
  return plan->stage_names[i].c_str();
}

double sparkey_plan_stage_ms(const sparkey_plan* plan, int32_t i) {
  if (!plan || i < 0 || i >= (int32_t)plan->stage_ms.size()) return 0.0;
  return plan->stage_ms[i];
}

void sparkey_plan_destroy(sparkey_plan* pl) {
  if (!pl) return;
  (void)hipSetDevice(pl->device);
  void* bufs[] = {pl->conv, pl->exitp, pl->qpos, pl->tail, pl->G, pl->cnt, pl->off, pl->ent, pl->ent2, pl->ent3,
                  pl->bcount, pl->bcursor, pl->boff, pl->bfun, pl->bpre, pl->bfun_total, pl->carry, pl->pairs,
                  pl->dfun, pl->dcarry, pl->parts, pl->p1_fill, pl->scan_u64, pl->scan_mp, pl->desc, pl->p1_hist, pl->p1_off, pl->d_status, pl->dbg, pl->wcount, pl->woff, pl->small,
                  pl->eseg, pl->seg_cnt, pl->seg_off, pl->seg_mark, pl->seg_start, pl->bstat_start,
                  pl->seg_cls_cnt, pl->seg_cls_off, pl->seg_len, pl->seg_first, pl->seg_fun, pl->seg_krep, pl->ecls, pl->sub_ent, pl->sub_fill, pl->p2tab,
                  pl->app_i64, pl->app_u32, pl->app_u64, pl->app_scan, pl->app_map,
                  pl->sn_blocks, pl->sn_dir, pl->sn_walk, pl->sn_recoff, pl->sn_vlog, pl->sn_itab, pl->sn_err,
                  pl->xtab, pl->ex_starts, pl->ex_cnt, pl->ex_off, pl->sn_par, pl->delp};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (pl->h_status) (void)hipHostFree(pl->h_status);
  if (pl->ev0) (void)hipEventDestroy(pl->ev0);
  if (pl->ev1) (void)hipEventDestroy(pl->ev1);
  if (pl->own_stream) (void)hipStreamDestroy(pl->own_stream);
  if (pl->sn_stream) (void)hipStreamDestroy(pl->sn_stream);
  for (auto& e : pl->sn_ev)
    if (e) (void)hipEventDestroy(e);
  if (pl->side_ok) {
    for (int i = 0; i < 3; i++) {
      (void)hipStreamDestroy(pl->side.s[i]);
      (void)hipEventDestroy(pl->side.join[i]);
    }
    (void)hipEventDestroy(pl->side.fork);
  }
  delete pl;
}

int64_t sparkey_index_size(const uint8_t* log_header, uint64_t header_len, const sparkey_build_opts* opts) {
  if (!log_header || !opts) return SPARKEY_E_ARG;
  LogHdr lh;
  const uint64_t data_end = header_len >= 40 ? rd64(log_header + 32) : 0;
  int rc = parse_log_header(log_header, header_len, std::max<uint64_t>(header_len, data_end), &lh, nullptr, 0, true);
  if (rc) return rc;
  IndexParams ip;
  rc = make_index_params(lh, *opts, &ip, nullptr, 0);
  if (rc) return rc;
  return ip.index_size;
}

}  // extern "C"

// ================================================================================================
// Sharded build steps.  The host orchestrator (sparkey/sharded.py) calls these in
// order on every rank and does the collectives between them.
// ================================================================================================
static int shard_check(sparkey_plan* pl, char* err, size_t err_len) {
  if (!pl || !pl->shard.active) {
    set_err(err, err_len, "sparkey_shard_begin was not called on this plan");
    return SPARKEY_E_ARG;
  }
  return SPARKEY_OK;
}

static int shard_sync_status(sparkey_plan* pl, hipStream_t s, char* err, size_t err_len) {
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(pl->h_status, pl->d_status, sizeof(Status), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return SPARKEY_OK;
}

// the nd = ceil(nbuckets / bpp) coarse digits in use split evenly: rank r owns digits
// [nd r / world, nd (r + 1) / world) -> buckets -> slots
static uint64_t used_digits(const BuildParams& P) { return (P.nbuckets + P.bpp - 1) / P.bpp; }
// buckets and slots of `rank`: an even split of the coarse digits (bucket / bpp) that hold buckets
static void digit_split(uint64_t cap, uint64_t nbuckets, uint64_t bpp, int rank, int world, uint64_t* b_lo,
                        uint64_t* b_hi, uint64_t* s_lo, uint64_t* s_hi) {
  const uint64_t nd = (nbuckets + bpp - 1) / bpp;
  const uint64_t d0 = (nd * (uint64_t)rank) / (uint64_t)world;
  const uint64_t d1 = (nd * (uint64_t)(rank + 1)) / (uint64_t)world;
  *b_lo = std::min<uint64_t>(nbuckets, d0 * bpp);
  *b_hi = std::min<uint64_t>(nbuckets, d1 * bpp);
  *s_lo = std::min<uint64_t>(cap, *b_lo << kBucketShift);
  *s_hi = std::min<uint64_t>(cap, *b_hi << kBucketShift);
}
static void shard_range(const BuildParams& P, int rank, int world, uint64_t* b_lo, uint64_t* b_hi, uint64_t* s_lo,
                        uint64_t* s_hi) {
  digit_split(P.cap, P.nbuckets, P.bpp, rank, world, b_lo, b_hi, s_lo, s_hi);
}
void shard_slot_split(uint64_t cap, int world, int rank, uint64_t* lo, uint64_t* hi) {
  const uint64_t nb = (cap + kBucket - 1) / kBucket;  // (setup_params: nbuckets, bpp)
  const uint64_t bpp = std::max<uint64_t>(1, (nb + 255) / 256);
  uint64_t b0, b1;
  digit_split(cap, nb, bpp, rank, world, &b0, &b1, lo, hi);
}

static int shard_begin_with(sparkey_plan* pl, const LogHdr& lh, const IndexParams& ip, const LogHdr& hlh,
                            const IndexParams& hip, const uint8_t* log, uint64_t buf_lo, uint64_t buf_hi,
                            const sparkey_build_opts* opts, int32_t rank, int32_t world, char* err, size_t err_len);

extern "C" {

int sparkey_shard_begin(sparkey_plan* pl, const uint8_t* log_header, uint64_t file_len, const uint8_t* d_buf,
                        uint64_t buf_lo, uint64_t buf_hi, const sparkey_build_opts* opts, int32_t rank, int32_t world,
                        char* err, size_t err_len) {
  if (!pl || !log_header || !opts || world < 1 || rank < 0 || rank >= world || world > 256 || buf_hi < buf_lo ||
      buf_hi > file_len) {
    set_err(err, err_len, "bad shard arguments");
    return SPARKEY_E_ARG;
  }
  if (((uintptr_t)d_buf & 15) || (buf_lo & 15)) {
    set_err(err, err_len, "shard buffer and buf_lo must be 16-byte aligned");
    return SPARKEY_E_ARG;
  }
  LogHdr lh;
  IndexParams ip;
  // (compressed logs: sk_cz_shard_begin takes the sharded path over their virtual log; the Python
  //  orchestrator gathers them)
  int rc = parse_log_header(log_header, 84, file_len, &lh, err, err_len, true);
  if (rc) return rc;
  rc = make_index_params(lh, *opts, &ip, err, err_len);
  if (rc) return rc;
  return shard_begin_with(pl, lh, ip, lh, ip, d_buf - buf_lo, buf_lo, buf_hi, opts, rank, world, err, err_len);
}

}  // extern "C"

// sparkey_shard_begin's state: framing over `lh` (the log the rank reads at log[p], p in
// [buf_lo, buf_hi)) with `ip`; the .spi header template from (hlh, hip)
static int shard_begin_with(sparkey_plan* pl, const LogHdr& lh, const IndexParams& ip, const LogHdr& hlh,
                            const IndexParams& hip, const uint8_t* log, uint64_t buf_lo, uint64_t buf_hi,
                            const sparkey_build_opts* opts, int32_t rank, int32_t world, char* err, size_t err_len) {
  ShardState& sh = pl->shard;
  sh.active = false;
  sh.lh = lh;
  sh.ip = ip;
  HIP_TRY(hipSetDevice(pl->device));
  sh.opts = *opts;
  sh.rank = rank;
  sh.world = world;
  sh.log = log;  // virtual base: global log position p is at log[p] for p in [buf_lo, buf_hi)
  sh.buf_lo = buf_lo;
  sh.buf_hi = buf_hi;
  sh.n_local = 0;
  sh.n_recv = 0;
  int rc = setup_params(sh.lh, sh.ip, *opts, sh.log, buf_hi, kLogHeaderSize, kLogHeaderSize, &sh.P, err, err_len);
  if (rc) return rc;
  sh.P.st = pl->d_status;
  sh.P.sharded = 1;
  shard_range(sh.P, rank, world, &sh.P.b_lo, &sh.P.b_hi, &sh.P.slot_lo, &sh.P.slot_hi);
  index_header_template(hlh, hip, opts->hash_seed, sh.tmpl.b);
  sh.local = 0;
  sh.ex_framed = sh.ex_built = false;
  sh.slabs_ok = false;
  sh.ex_recv = nullptr;
  sh.ex_n = 0;
  HIP_TRY(grow(&pl->small, pl->c_small, 512));
  sh.active = true;
  return SPARKEY_OK;
}

extern "C" {

int sparkey_shard_slot_range(const sparkey_plan* pl, int32_t rank, uint64_t* slot_lo, uint64_t* slot_hi) {
  if (!pl || !pl->shard.active || rank < 0 || rank >= pl->shard.world) return SPARKEY_E_ARG;
  uint64_t b0, b1;
  shard_range(pl->shard.P, rank, pl->shard.world, &b0, &b1, slot_lo, slot_hi);
  return SPARKEY_OK;
}

int64_t sparkey_shard_max_record_len(const sparkey_plan* pl) {
  return pl && pl->shard.active ? pl->shard.P.max_rec_len : SPARKEY_E_ARG;
}

int sparkey_shard_find_entry(sparkey_plan* pl, uint64_t lo, uint64_t window, void* stream, int64_t* entry_out,
                             char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const int64_t data_end = std::max<int64_t>(sh.lh.data_end, kLogHeaderSize);
  const int64_t L = sh.P.max_rec_len;
  const int64_t cand_end = std::min<int64_t>((int64_t)lo + L, data_end);
  const int64_t target = std::min<int64_t>((int64_t)lo + L + (int64_t)window, data_end);
  if ((int64_t)lo >= data_end) {
    *entry_out = data_end;
    return SPARKEY_OK;
  }
  if ((int64_t)lo < (int64_t)sh.buf_lo || (target + 16 > (int64_t)sh.buf_hi && (int64_t)sh.buf_hi < data_end)) {
    set_err(err, err_len, "entry window outside the shard buffer");
    return SPARKEY_E_ARG;
  }
  BuildParams P = sh.P;
  P.data_end = data_end;
  launch_find_entry(P, s, (int64_t)lo, cand_end, target, (int64_t*)pl->small);
  HIP_TRY(hipGetLastError());
  int64_t v = -1;
  HIP_TRY(hipMemcpyAsync(&v, pl->small, sizeof(v), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *entry_out = v;
  return SPARKEY_OK;
}

// One rank's framing set-up: parameters, the framing path and the first geometry (shared by the
// synchronous sparkey_shard_frame and the speculative sparkey_shard_frame_bin_async).
struct ShardFrameSetup {
  BuildParams P;
  bool fused = false, use_frame3 = false, use_regions = true;
  int spec_path() const { return fused && !knob_on(Knob::SerialFraming) ? (use_frame3 ? 4 : 0) : 1; }
  int framing_path = 1;
  uint64_t nrec = 0;
  FrameGeom geom0;
  uint32_t slab_cap = 0;
  int slab_path = 0;
};

static uint32_t shard_slab_for(const FrameGeom& g, uint64_t nrec) {
  const uint64_t nw = std::max<uint64_t>(1, g.nchunks ? (g.nchunks + g.w - 1) / g.w : 0);
  return (uint32_t)std::min<uint64_t>(kPartTile, std::max<uint64_t>(64, 2 * ((nrec + nw - 1) / nw) + 32));
}

static int shard_frame_setup(sparkey_plan* pl, int64_t entry, int64_t frame_end, ShardFrameSetup* F, char* err,
                             size_t err_len) {
  ShardState& sh = pl->shard;
  const int64_t data_end = std::max<int64_t>(sh.lh.data_end, kLogHeaderSize);
  BuildParams& P = F->P;
  int rc = setup_params(sh.lh, sh.ip, sh.opts, sh.log, sh.buf_hi, entry, frame_end, &P, err, err_len);
  if (rc) return rc;
  P.st = pl->d_status;
  P.sharded = 1;
  P.skip_del = 1;  // the bin carries PUT records only (their canonical placement); DELETEs: the exact path
  P.b_lo = sh.P.b_lo; P.b_hi = sh.P.b_hi; P.slot_lo = sh.P.slot_lo; P.slot_hi = sh.P.slot_hi;
  F->fused = P.max_rec_len <= 4096;
  const double frac = (double)(frame_end - entry) / (double)std::max<int64_t>(1, data_end - kLogHeaderSize);
  F->nrec = (uint64_t)((double)(std::max<int64_t>(0, sh.lh.num_puts) + std::max<int64_t>(0, sh.lh.num_deletes)) *
                       frac * 1.05) + 4096;
  F->use_frame3 = F->fused && want_frame3(P, sh.lh, entry, frame_end);
  F->geom0 = get_geom(P);
  F->framing_path = F->spec_path();
  const int64_t R = uniform_record_size(sh.lh);
  if (R && (entry - kLogHeaderSize) % R == 0) {  // a record start of a uniform log: frame by stride
    F->framing_path = 2;
    P.uni_n = (uint64_t)((frame_end - entry + R - 1) / R);
    P.uni_rec = R;
    F->nrec = P.uni_n;
  }
  F->slab_cap = shard_slab_for(F->geom0, F->nrec);
  F->slab_path = F->framing_path;
  F->use_regions = !knob_on(Knob::NoRegions);
  return SPARKEY_OK;
}

// Launches one framing attempt of the set-up (status reset first); no synchronisation.
static int shard_frame_launch(sparkey_plan* pl, ShardFrameSetup* F, hipStream_t s, char* err, size_t err_len) {
  BuildParams& P = F->P;
  set_geom(P, F->geom0);
  if (slab_framing(F->framing_path) && F->framing_path != F->slab_path) {
    F->slab_cap = shard_slab_for(F->geom0, F->nrec);
    F->slab_path = F->framing_path;
  }
  int rc = reserve_for_framing(pl, P, F->framing_path, F->nrec, F->slab_cap, err, err_len);
  if (rc) return rc;
  // uniform framing also does the bin's partition pass: entries into 256 coarse-digit regions of
  // ent3 (the bin then only packs them), as on one GPU
  P.p1_region = 0;
  if (F->framing_path == 2 && F->use_regions && P.slab_cap == (uint32_t)kPartTile && P.part_group == 1) {
    const double expect = (double)F->nrec * (double)P.bpp * (double)kBucket / (double)P.cap;
    const uint64_t rc_cap = ((uint64_t)(expect + 8.0 * std::sqrt(expect) + 1024.0) + 63) & ~63ull;
    HIP_TRY(grow(&pl->ent3, pl->c_ent3, 256 * rc_cap));
    HIP_TRY(grow(&pl->p1_fill, pl->c_p1_fill, 256));
    P.ent3 = pl->ent3;
    P.p1_fill = pl->p1_fill;
    P.p1_region = rc_cap;
  }
  launch_status_reset(s, pl->d_status, 0, P.p1_region ? pl->p1_fill : nullptr, P.p1_region ? 256 : 0);
  return launch_framing(pl, P, F->framing_path, s, err, err_len);
}

static int shard_frame_args(sparkey_plan* pl, int64_t entry, int64_t* frame_end, char* err, size_t err_len) {
  ShardState& sh = pl->shard;
  const int64_t data_end = std::max<int64_t>(sh.lh.data_end, kLogHeaderSize);
  *frame_end = std::min<int64_t>(*frame_end, data_end);
  if (entry < kLogHeaderSize || entry > data_end) {
    set_err(err, err_len, "shard entry outside the log data");
    return SPARKEY_E_ARG;
  }
  if (entry < *frame_end &&
      (entry < (int64_t)sh.buf_lo || ((uint64_t)*frame_end > sh.buf_hi && sh.buf_hi < (uint64_t)data_end))) {
    set_err(err, err_len, "shard frame range outside the shard buffer");
    return SPARKEY_E_ARG;
  }
  return SPARKEY_OK;
}

}  // extern "C"

// sparkey_shard_frame's body; allow_regions = false keeps the entries in slabs in log order (the
// exact path packs them from there) where uniform framing would write digit regions
static int shard_frame_sync(sparkey_plan* pl, int64_t entry, int64_t frame_end, hipStream_t s,
                            sparkey_shard_frame_result* res, bool allow_regions, char* err, size_t err_len) {
  ShardState& sh = pl->shard;
  int rc;
  const int64_t data_end = std::max<int64_t>(sh.lh.data_end, kLogHeaderSize);
  memset(res, 0, sizeof(*res));
  res->exit = entry;
  sh.n_local = 0;
  sh.slabs_ok = false;
  rc = shard_frame_args(pl, entry, &frame_end, err, err_len);
  if (rc) return rc;
  if (entry >= frame_end) return SPARKEY_OK;  // owns no record
  ShardFrameSetup F;
  rc = shard_frame_setup(pl, entry, frame_end, &F, err, err_len);
  if (rc) return rc;
  F.use_regions = F.use_regions && allow_regions;
  BuildParams& P = F.P;
  Status& st = *pl->h_status;
  for (int attempt = 0; attempt < 7; attempt++) {
    rc = shard_frame_launch(pl, &F, s, err, err_len);
    if (rc) return rc;
    rc = shard_sync_status(pl, s, err, err_len);
    if (rc) return rc;
    const int path = F.framing_path;
    if (slab_framing(path) && st.max_wave_count > F.slab_cap) {
      F.slab_cap = (uint32_t)std::min<uint64_t>(kPartTile, ((uint64_t)st.max_wave_count + 63) & ~63ull);
      continue;
    }
    if (st.overflow || st.n_records > P.max_records) {
      F.nrec = std::max<uint64_t>(st.n_records, F.nrec * 2 + 1);
      continue;
    }
    if (path == 4 && (st.spec_fail || st.err != ~0ull)) {
      F.framing_path = 0;
      continue;
    }
    if (path == 0 && (st.spec_fail || st.err != ~0ull)) {
      F.framing_path = 1;
      continue;
    }
    if (path == 2 && (st.spec_fail & kSpecRegionFull) && !(st.spec_fail & ~kSpecRegionFull)) {
      F.use_regions = false;  // a digit region filled up: slabs, and the bin's own pass
      continue;
    }
    if (path == 2 && st.spec_fail) {  // not the uniform log its header describes
      F.framing_path = F.spec_path();
      continue;
    }
    break;
  }
  res->framing_path = F.framing_path;
  if (st.err != ~0ull) {  // an invalid record on this chain: final only once the entry is verified
    res->rc = -(int)(st.err & 0xff);
    res->err_pos = (int64_t)(st.err >> 8);
    return SPARKEY_OK;
  }
  if (st.overflow || st.spec_fail) {
    set_err(err, err_len, "Corrupt log file: framing did not converge");
    return SPARKEY_E_CORRUPT_LOG;
  }
  res->exit = std::min<int64_t>(st.exit, data_end);
  res->num_records = (int64_t)st.n_records;
  res->num_deletes = (int64_t)st.n_deletes;
  sh.P_frame = P;
  sh.n_local = st.n_records;
  sh.slabs_ok = P.p1_region == 0;
  sh.slabs_entry = entry;
  sh.slabs_end = frame_end;
  return SPARKEY_OK;
}

extern "C" {

int sparkey_shard_frame(sparkey_plan* pl, int64_t entry, int64_t frame_end, void* stream,
                        sparkey_shard_frame_result* res, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  return shard_frame_sync(pl, entry, frame_end, s, res, true, err, err_len);
}

int64_t sparkey_shard_frame_capacity(sparkey_plan* pl, int64_t entry, int64_t frame_end) {
  char err[8];
  if (shard_check(pl, err, sizeof(err))) return SPARKEY_E_ARG;
  if (shard_frame_args(pl, entry, &frame_end, err, sizeof(err))) return SPARKEY_E_ARG;
  if (entry >= frame_end) return 0;
  ShardFrameSetup F;
  if (shard_frame_setup(pl, entry, frame_end, &F, err, sizeof(err))) return SPARKEY_E_ARG;
  return (int64_t)F.nrec;
}

// Frames [entry, frame_end) with the first attempt sparkey_shard_frame would make, bins the entries
// and writes the verification row, all without waiting: the row's retry flag says when the attempt
// needs sparkey_shard_frame's retries (then nothing else in the row is final).
int sparkey_shard_frame_bin_async(sparkey_plan* pl, int64_t entry, int64_t frame_end, uint8_t* d_send,
                                  uint64_t send_cap, int64_t* d_row, void* stream, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const int64_t data_end = std::max<int64_t>(sh.lh.data_end, kLogHeaderSize);
  const int64_t fe_in = frame_end;
  sh.n_local = 0;
  sh.local = 0;
  sh.slabs_ok = false;
  if (!d_row || ((uintptr_t)d_row & 7) || ((uintptr_t)d_send & 15) || (!d_send && sh.world != 1)) {
    set_err(err, err_len, "bad row or send buffer");
    return SPARKEY_E_ARG;
  }
  rc = shard_frame_args(pl, entry, &frame_end, err, err_len);
  if (rc) return rc;
  ShardScalars sc;
  for (int i = 0; i < kShardScalars; i++) sc.v[i] = 0;
  sc.v[0] = entry;
  sc.v[1] = fe_in;
  sc.v[2] = entry;
  if (entry >= frame_end) {  // owns no record
    launch_shard_row(s, sc, (const uint64_t*)pl->small, sh.world, 0, d_row);
    HIP_TRY(hipGetLastError());
    return SPARKEY_OK;
  }
  ShardFrameSetup F;
  rc = shard_frame_setup(pl, entry, frame_end, &F, err, err_len);
  if (rc) return rc;
  rc = shard_frame_launch(pl, &F, s, err, err_len);
  if (rc) return rc;
  BuildParams P = F.P;
  sh.P_frame = P;
  sh.slabs_ok = P.p1_region == 0;  // (a failed attempt is redone by sparkey_shard_frame)
  sh.slabs_entry = entry;
  sh.slabs_end = frame_end;
  P.abort_on_fail = 1;  // the bin skips an attempt that failed (its counts are not used)
  if (P.p1_region) {
    launch_region_send(P, s, sh.world, (uint32_t)used_digits(P), reinterpret_cast<Entry*>(d_send),
                       (uint64_t*)pl->small, send_cap);
    if (!d_send) sh.local = 1;
  } else {
    if (!d_send) {  // (the framing does not use ent3 here: growing it cannot disturb it)
      HIP_TRY(grow(&pl->ent3, pl->c_ent3, std::max<uint64_t>(F.nrec, 1)));
      d_send = reinterpret_cast<uint8_t*>(pl->ent3);
      send_cap = std::min<uint64_t>(send_cap, pl->c_ent3);  // (send_cap still bounds the entries taken)
      sh.local = 2;
    }
    P.ent3 = reinterpret_cast<Entry*>(d_send);
    P.max_records = send_cap;
    launch_partition1(P, s);
    launch_dest_counts(P, s, sh.world, (uint32_t)used_digits(P), (uint64_t*)pl->small);
    launch_digit_starts(P, s, (uint64_t*)pl->small + 64);
  }
  launch_shard_row_async(s, sc, pl->d_status, F.framing_path, F.slab_cap, F.P.max_records, send_cap, data_end,
                         (const uint64_t*)pl->small, sh.world, d_row);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_bin_row(sparkey_plan* pl, uint8_t* d_send, uint64_t send_cap, uint64_t n, const int64_t* scalars,
                          int64_t* d_row, void* stream, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!scalars || !d_row || ((uintptr_t)d_row & 7)) {
    set_err(err, err_len, "bad row arguments");
    return SPARKEY_E_ARG;
  }
  if (!d_send && n && sh.world != 1) {
    set_err(err, err_len, "a send buffer is needed with more than one rank");
    return SPARKEY_E_ARG;
  }
  if (n && (n != sh.n_local || (d_send && (send_cap < n || ((uintptr_t)d_send & 15))))) {
    set_err(err, err_len, "send buffer too small or misaligned, or not the framed entries: need " +
                              std::to_string(sh.n_local) + " entries");
    return SPARKEY_E_BUFFER;
  }
  sh.local = 0;
  if (n) {
    BuildParams P = sh.P_frame;
    if (P.p1_region) {  // the framing filled the digit regions: pack them (or, one rank, leave them)
      launch_region_send(P, s, sh.world, (uint32_t)used_digits(P), reinterpret_cast<Entry*>(d_send),
                         (uint64_t*)pl->small, send_cap);
      if (!d_send) sh.local = 1;
    } else {
      if (!d_send) {
        HIP_TRY(grow(&pl->ent3, pl->c_ent3, n));
        d_send = reinterpret_cast<uint8_t*>(pl->ent3);
        send_cap = pl->c_ent3;
        sh.local = 2;
      }
      P.ent3 = reinterpret_cast<Entry*>(d_send);
      P.max_records = send_cap;
      launch_partition1(P, s);
      launch_dest_counts(P, s, sh.world, (uint32_t)used_digits(P), (uint64_t*)pl->small);
      launch_digit_starts(P, s, (uint64_t*)pl->small + 64);
    }
  }
  ShardScalars sc;
  for (int i = 0; i < kShardScalars; i++) sc.v[i] = scalars[i];
  launch_shard_row(s, sc, (const uint64_t*)pl->small, sh.world, n ? 1 : 0, d_row);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_summarize_dev(sparkey_plan* pl, const uint8_t* d_recv, uint64_t n_recv, const int64_t* d_digits,
                                int32_t stride, int32_t fixed_regions, int64_t* d_fun, void* stream, char* err,
                                size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (((uintptr_t)d_recv & 15) || !d_fun || ((uintptr_t)d_fun & 7)) {
    set_err(err, err_len, "receive buffer must be 16-byte aligned");
    return SPARKEY_E_ARG;
  }
  const int local = d_recv ? 0 : sh.local;  // no receive buffer: the entries the bin left in ent3
  if (!d_recv && (n_recv ? !local || !d_digits : false)) {
    set_err(err, err_len, "no receive buffer and no entries binned in place");
    return SPARKEY_E_ARG;
  }
  if (local) d_recv = reinterpret_cast<const uint8_t*>(pl->ent3);
  BuildParams& P = sh.P;
  const bool grouped = d_digits || local == 1;
  const uint64_t nd = used_digits(P), G = (uint64_t)sh.world;
  const uint64_t d0 = (nd * (uint64_t)sh.rank) / G, d1 = (nd * (uint64_t)(sh.rank + 1)) / G;
  const uint64_t nk = d1 - d0;
  if (grouped) {  // the run table (and the status reset) first: the device starts while the host sets up
    HIP_TRY(grow(&pl->p2tab, pl->c_p2tab, 2 * nk * G + nk + 1));
    if (local == 1) launch_p2_table_regions(s, sh.P_frame.p1_fill, sh.P_frame.p1_region, (uint32_t)d0, (uint32_t)nk,
                                            pl->p2tab, pl->d_status, n_recv);
    else launch_p2_table(s, d_digits, stride, (int)G, (uint32_t)d0, (uint32_t)nk, pl->p2tab, pl->d_status, n_recv);
  }
  P.slab_cap = kPartTile;
  P.nslabs = (std::max<uint64_t>(n_recv, 1) + kPartTile - 1) / kPartTile;
  P.part_group = 1;
  P.p1_tiles = (uint32_t)P.nslabs;
  P.p1r_group = 1;
  P.p1r_tiles = P.p1_tiles;
  {
    const Entry* keep = pl->ent3;  // (ent3 holds the local entries: it must not be reallocated)
    rc = plan_reserve(pl, 1, std::max<uint64_t>(n_recv, 1), 1, P.nslabs, P.p1_tiles, P.nbuckets, P.cap, err,
                      err_len);
    if (rc) return rc;
    if (local && pl->ent3 != keep) {
      set_err(err, err_len, "internal: local entries moved");
      return SPARKEY_E_ARG;
    }
  }
  P.ent = const_cast<Entry*>(reinterpret_cast<const Entry*>(d_recv));
  P.ent_cap = n_recv;
  P.ent2 = pl->ent2; P.ent3 = pl->ent3; P.max_records = pl->c_ent2;
  P.wcount = pl->wcount; P.woff = pl->woff;
  P.bcount = pl->bcount; P.bcursor = pl->bcursor; P.boff = pl->boff; P.bfun = pl->bfun; P.bpre = pl->bpre;
  P.bfun_total = pl->bfun_total; P.carry = pl->carry; P.pairs = pl->pairs; P.pair_cap = pl->c_pairs / 2;
  P.parts = pl->parts; P.scan_scratch_u64 = pl->scan_u64; P.scan_scratch_mp = pl->scan_mp;
  P.bstat_start = pl->bstat_start;
  P.p1_hist = pl->p1_hist; P.p1_off = pl->p1_off; P.p1_off_total = pl->p1_off + 256ull * P.p1_tiles;
  P.st = pl->d_status;
  P.carry_funs = nullptr;
  sh.n_recv = n_recv;
  P.p2_seg = nullptr;
  P.p2_out = nullptr;
  if (grouped) {
    // the exchange buffer holds, per source rank in rank order, that rank's entries for this rank's
    // coarse digits in digit order (its bin output): k_part2 reads the runs in place, its run table
    // made on the device from the gathered rows (above)
    P.ent3 = const_cast<Entry*>(reinterpret_cast<const Entry*>(d_recv));
    P.p2_seg = pl->p2tab;
    P.p2_out = pl->p2tab + 2 * nk * G;
    P.p2_nsrc = (uint32_t)G;
    P.p2_d0 = (uint32_t)d0;
    P.p2_nd = (uint32_t)nk;
    // k_part2s (tables of at most kP2SortedMaxBpp buckets per digit): one pass into fixed bucket
    // regions of the rank's range, the carry functions from the same pass.  A bucket that outgrows its
    // region sets p2_overflow: every later kernel skips, the flags row says "aborted", and the host
    // redoes the step with fixed_regions = 0 (dense runs)
    // Larger tables over N > 1 ranks: k_part2_recv, several workgroups a digit, into the fixed regions
    // (k_part2 has one workgroup per digit: 256 / N of them a rank, 32 CUs busy at N = 8).  One rank
    // keeps k_part2 (125M entries: 1.89 ms against k_part2_recv's 2.41, profiles/r04/shard/).
    P.p2_sorted = P.bpp <= kP2SortedMaxBpp ? 1 : 0;
    const bool recv = !P.p2_sorted && sh.world > 1 && part2_recv_fits(P.bpp);
    P.p2_fixed = fixed_regions && (P.p2_sorted || recv) ? 1 : 0;
    if (P.p2_fixed) {
      HIP_TRY(grow(&pl->ent2, pl->c_ent2, std::max<uint64_t>(n_recv, (P.b_hi - P.b_lo) * (uint64_t)kPlaceLdsMax)));
      P.ent2 = pl->ent2;
      P.max_records = pl->c_ent2;
    }
    if (P.p2_fixed && !P.p2_sorted) {
      if (P.b_hi > P.b_lo) HIP_TRY(hipMemsetAsync(P.bcount + P.b_lo, 0, (P.b_hi - P.b_lo) * sizeof(uint32_t), s));
      launch_part2_recv(P, s, &pl->timer);
    } else {
      launch_partition2(P, s, &pl->timer);
    }
    P.ent3 = pl->ent3;  // the later steps' scratch (k_place sorts oversized buckets there)
    P.p2_seg = nullptr;
    P.p2_out = nullptr;
  } else {
    P.p2_sorted = 0;
    P.p2_fixed = 0;
    sh.slabs_ok = false;  // (the slab counts are rewritten below)
    launch_status_reset(s, pl->d_status, n_recv);
    launch_dense_slabs(P, s);
    launch_partition(P, s, &pl->timer);
  }
  if (P.b_hi > P.b_lo) {
    launch_summary_carry(P, s, &pl->timer);
    HIP_TRY(hipMemcpyAsync(d_fun, P.bfun_total, sizeof(MaxPlus), hipMemcpyDeviceToDevice, s));
  } else {  // identity carry function f(x) = max(0, x + 0) for an empty range
    HIP_TRY(hipMemsetAsync(d_fun, 0, sizeof(MaxPlus), s));
  }
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_place_dev(sparkey_plan* pl, const int64_t* d_funs, uint8_t* d_slots, uint8_t* d_spill,
                            uint64_t spill_cap, int64_t* d_flags, int32_t inline_cap, void* stream, char* err,
                            size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  BuildParams& P = sh.P;
  if (((uintptr_t)d_slots & 3) || ((uintptr_t)d_spill & 15) || !d_funs || !d_flags || ((uintptr_t)d_flags & 7) ||
      inline_cap < 0) {
    set_err(err, err_len, "slot, spill or flags buffer misaligned");
    return SPARKEY_E_ARG;
  }
  P.out = d_slots - kIndexHeaderSize - P.slot_lo * (uint64_t)P.slot_size;  // virtual .spi base
  P.spill = reinterpret_cast<SpillEntry*>(d_spill);
  P.spill_cap = spill_cap;
  P.carry_in = 0;
  P.carry_funs = d_funs;
  P.carry_world = sh.world;
  P.carry_rank = sh.rank;
  P.fold_stats = 1;  // k_place_reg leaves the stats parts
  launch_carry(P, s);  // (also clears the placement's counters)
  launch_place_buckets(P, s);
  launch_shard_flags(P, s, d_flags, inline_cap);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_finish_dev(sparkey_plan* pl, const int64_t* d_rows, int32_t stride, int32_t inline_cap,
                             int64_t* d_out, void* stream, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!d_rows || !d_out || ((uintptr_t)d_out & 7) || stride < kShardFlags + 4 * inline_cap) {
    set_err(err, err_len, "bad flags rows");
    return SPARKEY_E_ARG;
  }
  BuildParams& P = sh.P;
  launch_apply_spill_rows(P, s, d_rows, sh.world, stride, inline_cap);
  P.prev_hash = 0;
  P.prev_occ = 0;
  if (P.slot_hi > P.slot_lo) {
    if (P.fold_stats) {  // the parts k_place_reg left; k_stats only if some bucket bypassed it
      launch_stats_folded_shard(P, s);
      BuildParams Q = P;
      Q.stats_if_pending = 1;
      launch_stats(Q, s, 0, &pl->timer);
    } else {
      launch_stats(P, s, 0, &pl->timer);
    }
  }
  launch_shard_summary_row(P, s, d_rows + (int64_t)sh.rank * stride, d_out);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_header_dev(sparkey_plan* pl, const int64_t* d_fin, int32_t stride, int64_t num_entries,
                             uint8_t* d_header, void* stream, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!d_fin || !d_header || stride < kShardFlags + 8) {
    set_err(err, err_len, "bad finish rows");
    return SPARKEY_E_ARG;
  }
  launch_shard_header(s, d_fin, stride, sh.world, sh.tmpl, num_entries, d_header);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_pairs(sparkey_plan* pl, uint64_t* h_addrs, uint64_t n_pairs, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  if (n_pairs > pl->shard.P.pair_cap) {
    set_err(err, err_len, "more pairs than recorded");
    return SPARKEY_E_ARG;
  }
  if (n_pairs) HIP_TRY(hipMemcpy(h_addrs, pl->pairs, 2 * n_pairs * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return SPARKEY_OK;
}

int32_t sparkey_shard_key_record_size(const sparkey_plan* pl) {
  if (!pl || !pl->shard.active) return SPARKEY_E_ARG;
  return (int32_t)(8 + ((pl->shard.lh.max_key_len + 7) & ~7LL));
}

int sparkey_shard_fetch_keys(sparkey_plan* pl, const uint64_t* d_addrs, uint64_t n, uint8_t* d_records,
                             uint32_t rec_size, void* stream, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  BuildParams P = pl->shard.P;
  P.fr_entry = (int64_t)pl->shard.buf_lo;
  launch_fetch_keys(P, s, d_addrs, n, d_records, rec_size);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  return SPARKEY_OK;
}

int sparkey_shard_compare_keys(sparkey_plan* pl, const uint8_t* d_records, uint64_t n_pairs, uint32_t rec_size,
                               void* stream, int32_t* dup_out, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const BuildParams& P = pl->shard.P;
  HIP_TRY(hipMemsetAsync(&pl->d_status->dup, 0, sizeof(unsigned int), s));
  launch_compare_keys(P, s, d_records, n_pairs, rec_size);
  rc = shard_sync_status(pl, s, err, err_len);
  if (rc) return rc;
  *dup_out = (int32_t)pl->h_status->dup;
  return SPARKEY_OK;
}

int sparkey_shard_apply_spill(sparkey_plan* pl, const uint8_t* d_spill, uint64_t n, void* stream, char* err,
                              size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  launch_apply_spill(pl->shard.P, s, reinterpret_cast<const SpillEntry*>(d_spill), n);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

// out = {first slot hash, first slot address, last slot hash, last slot address} of the rank's range
int sparkey_shard_boundary(sparkey_plan* pl, void* stream, uint64_t* out, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const BuildParams& P = pl->shard.P;
  for (int i = 0; i < 4; i++) out[i] = 0;
  if (P.slot_hi <= P.slot_lo) return SPARKEY_OK;
  uint8_t b[32];
  const uint8_t* base = P.out + kIndexHeaderSize;
  HIP_TRY(hipMemcpyAsync(b, base + P.slot_lo * P.slot_size, P.slot_size, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(b + 16, base + (P.slot_hi - 1) * P.slot_size, P.slot_size, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int k = 0; k < 2; k++) {
    const uint8_t* q = b + 16 * k;
    uint64_t h = 0, a = 0;
    for (int i = 0; i < P.hash_size; i++) h |= (uint64_t)q[i] << (8 * i);
    for (int i = 0; i < P.addr_size; i++) a |= (uint64_t)q[P.hash_size + i] << (8 * i);
    out[2 * k] = h;
    out[2 * k + 1] = a;
  }
  return SPARKEY_OK;
}

// out = {max displacement, hash collisions, total displacement} over the rank's slots
int sparkey_shard_stats(sparkey_plan* pl, uint64_t prev_hash, int32_t prev_occ, void* stream, int64_t* out, char* err,
                        size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  BuildParams& P = pl->shard.P;
  P.prev_hash = prev_hash;
  P.prev_occ = prev_occ;
  out[0] = out[1] = out[2] = 0;
  if (P.slot_hi <= P.slot_lo) return SPARKEY_OK;
  launch_stats(P, s, 0, &pl->timer);
  rc = shard_sync_status(pl, s, err, err_len);
  if (rc) return rc;
  out[0] = pl->h_status->max_disp;
  out[1] = pl->h_status->collisions;
  out[2] = pl->h_status->total_disp;
  return SPARKEY_OK;
}

// ---- sharded exact path ----

int sparkey_shard_first_empty(sparkey_plan* pl, void* stream, int64_t* slot_out, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const BuildParams& P = pl->shard.P;
  if (!slot_out || !P.out) {
    set_err(err, err_len, "no placement to search (sparkey_shard_place_dev first)");
    return SPARKEY_E_ARG;
  }
  unsigned long long* d = reinterpret_cast<unsigned long long*>(pl->small) + 400;
  HIP_TRY(hipMemsetAsync(d, 0xff, sizeof(unsigned long long), s));
  launch_first_empty(P, s, d);
  HIP_TRY(hipGetLastError());
  unsigned long long v = ~0ull;
  HIP_TRY(hipMemcpyAsync(&v, d, sizeof(v), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *slot_out = v == ~0ull ? -1 : (int64_t)v;
  return SPARKEY_OK;
}

int32_t sparkey_shard_exact_record_size(const sparkey_plan* pl) {
  if (!pl || !pl->shard.active) return SPARKEY_E_ARG;
  const int64_t k = pl->shard.lh.max_key_len;
  if (k < 0 || k > kExactMaxKey) return 0;
  return (int32_t)(16 + ((10 + k + 7) & ~7LL));  // {hash, address} + two VLQs (<= 5 bytes each) + key
}

static int exact_count(sparkey_plan* pl, hipStream_t s, uint64_t* counts_out, char* err, size_t err_len);

int sparkey_shard_exact_frame(sparkey_plan* pl, int64_t entry, int64_t frame_end, int64_t n_records,
                              const int64_t* starts, void* stream, uint64_t* counts_out, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  const int W = sh.world;
  sh.ex_framed = false;
  sh.ex_built = false;
  if (!starts || !counts_out) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  sh.ex_rs = (uint32_t)sparkey_shard_exact_record_size(pl);
  if (!sh.ex_rs) {
    set_err(err, err_len, "keys too long for the exact exchange records");
    return SPARKEY_E_UNSUPPORTED;
  }
  sh.ex_starts.assign(starts, starts + W);
  int64_t prev = -1;
  bool any = false;
  for (int r = 0; r < W; r++) {
    const int64_t e = starts[r];
    if (e < 0) continue;
    if ((uint64_t)e >= sh.ip.cap || e <= prev) {
      set_err(err, err_len, "exact range starts must increase with the rank and lie in the table");
      return SPARKEY_E_ARG;
    }
    prev = e;
    any = true;
  }
  if (!any) {
    set_err(err, err_len, "no exact range (no empty slot)");
    return SPARKEY_E_ARG;
  }
  for (int r = 0; r < W; r++) counts_out[r] = 0;
  {
    int64_t fe = frame_end;
    rc = shard_frame_args(pl, entry, &fe, err, err_len);
    if (rc) return rc;
    frame_end = fe;
  }
  // the canonical step's framing left its slabs in place: no second framing (the counts below check it)
  bool reuse = sh.slabs_ok && n_records >= 0 && entry == sh.slabs_entry && frame_end == sh.slabs_end &&
               sh.P_frame.ent == pl->ent && sh.P_frame.wcount == pl->wcount && !knob_on(Knob::ExactReframe);
  for (int pass = 0; pass < 2; pass++) {
    if (reuse) {
      sh.n_local = entry < frame_end ? (uint64_t)n_records : 0;
    } else {
      sparkey_shard_frame_result fr;
      rc = shard_frame_sync(pl, entry, frame_end, s, &fr, false, err, err_len);
      if (rc) return rc;
      if (fr.rc) {
        set_err(err, err_len, std::string(code_message(fr.rc)) + " (log offset " + std::to_string(fr.err_pos) + ")");
        return fr.rc;
      }
    }
    rc = exact_count(pl, s, counts_out, err, err_len);
    if (rc) return rc;
    if (sh.ex_total == sh.n_local) break;
    if (!reuse) {
      set_err(err, err_len, "internal: exact counts do not cover the framed records");
      return SPARKEY_E_GPU;
    }
    reuse = false;  // the slabs did not hold the records: frame again
  }
  sh.ex_framed = true;
  return SPARKEY_OK;
}

// records per exact owner of the framed slabs (sh.P_frame), and the scanned (owner, slab) offsets
static int exact_count(sparkey_plan* pl, hipStream_t s, uint64_t* counts_out, char* err, size_t err_len) {
  ShardState& sh = pl->shard;
  const int W = sh.world;
  sh.ex_total = 0;
  for (int r = 0; r < W; r++) counts_out[r] = 0;
  if (!sh.n_local) return SPARKEY_OK;
  BuildParams& P = sh.P_frame;
  HIP_TRY(grow(&pl->ex_starts, pl->c_ex_starts, (uint64_t)W + 1));
  HIP_TRY(grow(&pl->ex_cnt, pl->c_ex_cnt, (uint64_t)W * P.nslabs));
  HIP_TRY(grow(&pl->ex_off, pl->c_ex_off, (uint64_t)W * P.nslabs + 1));
  const uint64_t scratch = ((uint64_t)W * P.nslabs) / kScanTile + 80;
  HIP_TRY(grow(&pl->scan_u64, pl->c_su, std::max<uint64_t>(pl->c_su, scratch)));
  HIP_TRY(hipMemcpyAsync(pl->ex_starts, sh.ex_starts.data(), W * sizeof(int64_t), hipMemcpyHostToDevice, s));
  unsigned long long* tot = reinterpret_cast<unsigned long long*>(pl->small);
  launch_ex_count(P, s, pl->ex_starts, W, pl->ex_cnt, pl->ex_off, pl->scan_u64, tot);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned long long> h(W);
  HIP_TRY(hipMemcpyAsync(h.data(), tot, W * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int r = 0; r < W; r++) {
    counts_out[r] = h[r];
    sh.ex_total += h[r];
  }
  return SPARKEY_OK;
}

int sparkey_shard_exact_pack(sparkey_plan* pl, uint8_t* d_send, uint64_t send_bytes, void* stream, char* err,
                             size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!sh.ex_framed) {
    set_err(err, err_len, "sparkey_shard_exact_frame first");
    return SPARKEY_E_ARG;
  }
  if (!sh.ex_total) return SPARKEY_OK;
  if (!d_send || ((uintptr_t)d_send & 15) || send_bytes < sh.ex_total * sh.ex_rs) {
    set_err(err, err_len, "send buffer too small or misaligned: need " + std::to_string(sh.ex_total * sh.ex_rs));
    return SPARKEY_E_BUFFER;
  }
  launch_ex_scatter(sh.P_frame, s, pl->ex_starts, sh.world, pl->ex_off, d_send, sh.ex_rs);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_shard_exact_build(sparkey_plan* pl, const uint8_t* d_recv, uint64_t n, void* stream,
                              sparkey_shard_exact_result* res, char* err, size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!res || (n && (!d_recv || ((uintptr_t)d_recv & 15))) || !sh.ex_rs) {
    set_err(err, err_len, "bad exact build arguments");
    return SPARKEY_E_ARG;
  }
  memset(res, 0, sizeof(*res));
  sh.ex_built = false;
  sh.ex_recv = d_recv;
  sh.ex_n = n;
  BuildParams& L = sh.ex_L;
  memset(&L, 0, sizeof(L));
  if (n) {
    // the local replay runs on a window of the table: the rank's exact range [a, b) (b the next
    // range's start around the ring; the whole ring when this is the only range), slots numbered
    // from a.  Every record received wants a slot in it and no probe leaves it (b stays empty), so
    // the window's table, segments and placement scratch are O(b - a), about cap / world.  Slots
    // carry 8-byte addresses: offsets into the receive buffer.
    const int W = sh.world;
    const int64_t a = sh.ex_starts[sh.rank];
    if (a < 0) {
      set_err(err, err_len, "records received by a rank without an exact range");
      return SPARKEY_E_GPU;
    }
    int64_t b = -1;
    for (int k = 1; k <= W && b < 0; k++) b = sh.ex_starts[(sh.rank + k) % W];
    const uint64_t cap = sh.ip.cap;
    const uint64_t len = b == a ? cap : ((uint64_t)b + cap - (uint64_t)a) % cap;
    IndexParams ipl = sh.ip;
    ipl.cap = knob_on(Knob::ExactFullTable) ? cap : len;
    ipl.addr_size = 8;
    ipl.ebb = 0;
    ipl.slot_size = ipl.hash_size + 8;
    ipl.index_size = kIndexHeaderSize + (int64_t)ipl.cap * ipl.slot_size;
    rc = setup_params(sh.lh, ipl, sh.opts, d_recv, n * (uint64_t)sh.ex_rs, kLogHeaderSize, kLogHeaderSize, &L, err,
                      err_len);
    if (rc) return rc;
    L.mod = make_fastmod(cap, ipl.cap == cap ? 0 : (uint64_t)a);
    L.slot_hi = ipl.cap;
    L.st = pl->d_status;
    rc = reserve_for_framing(pl, L, 1, n, kPartTile, err, err_len);
    if (rc) return rc;
    HIP_TRY(grow(&pl->xtab, pl->c_xtab, (uint64_t)ipl.index_size));
    L.out = pl->xtab;
    HIP_TRY(hipMemsetAsync(pl->xtab, 0, (size_t)ipl.index_size, s));
    launch_status_reset(s, pl->d_status, n);
    launch_ex_ent(s, d_recv, n, sh.ex_rs, L.ent);
    launch_dense_slabs(L, s);
    // canonical placement of the PUT records (the segments), then the replay per segment
    L.skip_del = 1;
    L.p1_region = 0;
    L.p1_hist_ready = 0;
    L.p2_sorted = 0;
    L.p2_fixed = 0;
    L.fold_stats = 0;
    L.fused_carry = 0;
    launch_partition(L, s, &pl->timer);
    launch_summary_carry(L, s, &pl->timer);
    launch_place_buckets(L, s);  // (no pair verification: the replay compares the keys itself)
    rc = run_exact_segments(pl, L, ipl.in_memory, s, err, err_len);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(pl->h_status, pl->d_status, sizeof(Status), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const Status& st = *pl->h_status;
    if (st.guard) {
      set_err(err, err_len, "internal error: exact-path bounds check tripped (bits " + std::to_string(st.guard) + ")");
      return SPARKEY_E_GPU;
    }
    if (st.err != ~0ull) {  // an error at a local record offset: report the record's log position
      const uint64_t q = (uint64_t)(st.err >> 8);
      res->rc = -(int32_t)(st.err & 0xff);
      res->err_pos = -1;
      if (q >= 16 && (q - 16) % sh.ex_rs == 0 && (q - 16) / sh.ex_rs < n) {
        uint64_t a = 0;
        HIP_TRY(hipMemcpy(&a, d_recv + (q - 16) + 8, sizeof(a), hipMemcpyDeviceToHost));
        res->err_pos = (int64_t)((a & ~kDelBit) >> sh.ip.ebb);
      }
    }
    res->num_entries = st.num_entries;
    res->garbage_size = st.garbage;
  }
  // the stats steps read the plan's workspace through sh.P: it may have moved
  sh.P.parts = pl->parts;
  sh.P.scan_scratch_u64 = pl->scan_u64;
  sh.P.scan_scratch_mp = pl->scan_mp;
  sh.P.st = pl->d_status;
  sh.ex_built = true;
  return SPARKEY_OK;
}

int sparkey_shard_exact_extract(sparkey_plan* pl, uint64_t a, uint64_t b, uint8_t* d_dst, void* stream, char* err,
                                size_t err_len) {
  int rc = shard_check(pl, err, err_len);
  if (rc) return rc;
  ShardState& sh = pl->shard;
  hipStream_t s = stream ? (hipStream_t)stream : pl->own_stream;
  if (!sh.ex_built || a > b || b > sh.ip.cap) {
    set_err(err, err_len, "bad exact extract arguments");
    return SPARKEY_E_ARG;
  }
  if (a == b) return SPARKEY_OK;
  BuildParams G = sh.P;  // the .spi slot layout
  if (d_dst) {
    if (((uintptr_t)d_dst & 3) || (G.slot_size == 16 && ((uintptr_t)d_dst & 15)) || (G.slot_size == 8 && ((uintptr_t)d_dst & 7))) {
      set_err(err, err_len, "misaligned destination");
      return SPARKEY_E_ARG;
    }
    G.out = d_dst - kIndexHeaderSize - a * (uint64_t)G.slot_size;
  } else if (!G.out || a < G.slot_lo || b > G.slot_hi) {
    set_err(err, err_len, "slots outside the rank's range (or no slice placed)");
    return SPARKEY_E_ARG;
  }
  BuildParams L = sh.ex_L;
  if (!sh.ex_n) {
    L = sh.P;
    L.out = nullptr;  // nothing received: the range is empty
  }
  launch_ex_extract(L, G, s, sh.ex_recv, sh.ex_n, sh.ex_rs, a, b);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}

int sparkey_index_header(const uint8_t* log_header, const sparkey_build_opts* opts, int64_t num_entries,
                         int64_t garbage_size, int64_t max_displacement, int64_t hash_collisions,
                         int64_t total_displacement, uint8_t* out, char* err, size_t err_len) {
  if (!log_header || !opts || !out) return SPARKEY_E_ARG;
  LogHdr lh;
  int rc = parse_log_header(log_header, 84, (uint64_t)std::max<int64_t>(rd64(log_header + 32), 84), &lh, err, err_len,
                            true);
  if (rc) return rc;
  IndexParams ip;
  rc = make_index_params(lh, *opts, &ip, err, err_len);
  if (rc) return rc;
  index_header_template(lh, ip, opts->hash_seed, out);
  wr64(out + 52, (uint64_t)garbage_size);
  wr64(out + 60, (uint64_t)num_entries);
  wr64(out + 84, (uint64_t)max_displacement);
  wr64(out + 96, (uint64_t)hash_collisions);
  wr64(out + 104, (uint64_t)total_displacement);
  return SPARKEY_OK;
}

}  // extern "C"

// ================================================================================================
// Sharded compressed logs (shard_host.cpp Rank::compressed).  Rank g holds the
// compressed bytes [lo_g, lo_{g+1}) and a tail.  The parallel directory's screen and anchors over its
// range give its entry e_g (the first anchor; 84 on rank 0); with every rank's entry all-gathered, it
// follows the chain from e_g through its anchors to e_{g+1}, each link landing exactly on the next
// anchor (so e_{g+1} is on the chain by induction from 84, as the NONE path's record chain), decodes
// its blocks into its slice [vbase_g, vbase_{g+1}) of the whole log's virtual log, and the NONE
// sharded pipeline runs over the slices with the compressed log's index parameters, the entries'
// virtual offsets rewritten to (blockPosition << entryBlockBits) | entryIndex before the exchange.
// ================================================================================================
int64_t sk_cz_hop_bound(const uint8_t* hdr) {
  const int32_t ct = (int32_t)rd32(hdr + 64);
  if (ct != 1 && ct != 2) return 0;
  return cz_hop_bound(ct == 2 ? 1 : 0, (int64_t)(int32_t)rd32(hdr + 68));
}

int sk_cz_entry(sparkey_plan* pl, const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo,
                uint64_t buf_hi, int64_t lo, int64_t hi, int32_t rank, hipStream_t s, int64_t* entry, char* err,
                size_t err_len) {
  *entry = -1;
  auto& cz = pl->cz;
  int rc = parse_log_header(hdr, 84, file_len, &cz.lh, err, err_len, true);
  if (rc) return rc;
  cz.anchors.clear();
  if (cz.lh.compression_type == 0) return SPARKEY_OK;
  cz.codec = cz.lh.compression_type == 2 ? 1 : 0;
  cz.H = cz_hop_bound(cz.codec, cz.lh.compression_block_size);
  if (!cz.H || !d_buf || ((uintptr_t)d_buf & 15) || (buf_lo & 15) || lo < (int64_t)buf_lo) return SPARKEY_OK;
  HIP_TRY(hipSetDevice(pl->device));
  const int64_t data_end = std::max<int64_t>(cz.lh.data_end, kLogHeaderSize);
  cz.A = 32 * cz.H;
  if (knob_set(Knob::SnappyDirA)) cz.A = std::max<int64_t>(cz.H, knob(Knob::SnappyDirA));  // (tests)
  memset(&cz.S, 0, sizeof(cz.S));
  SnappyParams& S = cz.S;
  S.log = d_buf - buf_lo;  // global offset p at log[p]
  S.log_len = (int64_t)buf_hi;
  S.data_end = data_end;
  S.max_block = cz.lh.compression_block_size;
  S.win0 = lo;
  if (rank == 0) *entry = kLogHeaderSize;
  if (lo >= data_end) {
    *entry = data_end;
    return SPARKEY_OK;
  }
  const int64_t end = std::min(hi, data_end);
  const uint64_t nwin = end > lo ? (uint64_t)((end - lo + cz.A - 1) / cz.A) : 0;
  if (!nwin) return SPARKEY_OK;
  HIP_TRY(grow(&pl->sn_par, pl->c_sn_par, nwin * (kSdirCand * 8 + 4 + 8) + 64));
  uint8_t* q = pl->sn_par;
  int64_t* cand = (int64_t*)q;
  int32_t* ncand = (int32_t*)(q + ((nwin * kSdirCand * 8 + 15) & ~15ull));
  int64_t* anchor = (int64_t*)((uint8_t*)ncand + ((nwin * 4 + 15) & ~15ull));
  launch_sdir_screen(S, s, cz.codec, cz.A, cz.H, nwin, cand, ncand);
  launch_sdir_anchor(S, s, cz.codec, cz.A, cz.H, nwin, cand, ncand, anchor);
  HIP_TRY(hipGetLastError());
  std::vector<int64_t> anc(nwin);
  HIP_TRY(hipMemcpyAsync(anc.data(), anchor, nwin * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int64_t x : anc)
    if (x > lo && x <= data_end && (cz.anchors.empty() || x > cz.anchors.back())) cz.anchors.push_back(x);
  if (rank != 0 && !cz.anchors.empty()) *entry = cz.anchors[0];
  return SPARKEY_OK;
}

int sk_cz_count(sparkey_plan* pl, int64_t entry, int64_t next, hipStream_t s, int32_t* ok, uint64_t* nblk,
                uint64_t* ulen, char* err, size_t err_len) {
  auto& cz = pl->cz;
  *ok = 0;
  *nblk = *ulen = 0;
  cz.nblk = cz.ulen = 0;
  cz.ends.clear();
  if (entry > next || !cz.H) return SPARKEY_OK;
  if (entry == next) {
    *ok = 1;
    return SPARKEY_OK;
  }
  cz.ends.push_back(entry);
  for (int64_t a : cz.anchors)
    if (a > entry && a < next) cz.ends.push_back(a);
  cz.ends.push_back(next);
  const uint64_t nl = cz.ends.size() - 1;
  HIP_TRY(grow(&pl->sn_par, pl->c_sn_par, (nl + 1) * 8 + 4 * nl * 8 + 256));
  uint8_t* q = pl->sn_par;
  auto carve = [&](uint64_t n) { uint8_t* r = q; q += (n + 15) & ~15ull; return r; };
  cz.d_ends = (int64_t*)carve((nl + 1) * 8);
  cz.d_cnt = (uint64_t*)carve(nl * 8);
  cz.d_usum = (uint64_t*)carve(nl * 8);
  cz.d_boff = (uint64_t*)carve(nl * 8);
  cz.d_uoff = (uint64_t*)carve(nl * 8);
  cz.flag = (int32_t*)carve(16);
  HIP_TRY(hipMemsetAsync(cz.flag, 0, 4, s));
  HIP_TRY(hipMemcpyAsync(cz.d_ends, cz.ends.data(), (nl + 1) * 8, hipMemcpyHostToDevice, s));
  launch_sdir_link(cz.S, s, cz.codec, cz.d_ends, nl, 0, cz.d_cnt, cz.d_usum, nullptr, nullptr, cz.flag);
  HIP_TRY(hipGetLastError());
  cz.cnt.assign(nl, 0);
  cz.usum.assign(nl, 0);
  int32_t f = 0;
  HIP_TRY(hipMemcpyAsync(cz.cnt.data(), cz.d_cnt, nl * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(cz.usum.data(), cz.d_usum, nl * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(&f, cz.flag, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (f) return SPARKEY_OK;  // a link missed its end (or a block is corrupt): the gathered build says which
  for (uint64_t i = 0; i < nl; i++) {
    cz.nblk += cz.cnt[i];
    cz.ulen += cz.usum[i];
  }
  *nblk = cz.nblk;
  *ulen = cz.ulen;
  *ok = 1;
  return SPARKEY_OK;
}

int sk_cz_decode(sparkey_plan* pl, int64_t vbase, hipStream_t s, int64_t* carry_out, char* err, size_t err_len) {
  auto& cz = pl->cz;
  SnappyParams& S = cz.S;
  *carry_out = -1;
  const uint64_t nblk = cz.nblk;
  cz.vbase = vbase;
  cz.vlo = vbase & ~4095LL;  // (framing chunks start at most 4 KiB before a record)
  cz.vend = vbase + (int64_t)cz.ulen;
  const uint64_t front = (uint64_t)(vbase - cz.vlo), body = cz.ulen;
  HIP_TRY(grow(&pl->sn_vlog, pl->c_sn_vlog, front + body + 4096 + 16));
  S.vlog = pl->sn_vlog - cz.vlo;
  S.vlog_len = (int64_t)body;
  S.nblk = nblk;
  S.blk_base = 0;
  S.ebb = calc_entry_block_bits(cz.lh.max_entries_per_block);
  if (front) HIP_TRY(hipMemsetAsync(pl->sn_vlog, 0, front, s));
  HIP_TRY(hipMemsetAsync(pl->sn_vlog + front + body, 0, 4096, s));
  const uint32_t mepb = (uint32_t)std::max<int64_t>(
      1, std::min<int64_t>(cz.lh.max_entries_per_block, (int64_t)cz.lh.compression_block_size / 2 + 1));
  S.mepb = mepb;
  if (nblk) {
    const uint64_t nl = cz.cnt.size();
    std::vector<uint64_t> bo(nl), uo(nl);
    uint64_t nb = 0, tot = 0;
    for (uint64_t i = 0; i < nl; i++) {
      bo[i] = nb;
      uo[i] = (uint64_t)(vbase - kLogHeaderSize) + tot;  // (k_sdir_link: voff = 84 + uoff)
      nb += cz.cnt[i];
      tot += cz.usum[i];
    }
    HIP_TRY(grow(&pl->sn_blocks, pl->c_sn_blocks, nblk));
    HIP_TRY(grow(&pl->sn_walk, pl->c_sn_walk, nblk));
    HIP_TRY(grow(&pl->sn_recoff, pl->c_sn_recoff, nblk * mepb));
    S.blocks = pl->sn_blocks;
    S.blk_cap = pl->c_sn_blocks;
    S.walk = pl->sn_walk;
    S.rec_off = pl->sn_recoff;
    HIP_TRY(hipMemcpyAsync(cz.d_boff, bo.data(), nl * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(cz.d_uoff, uo.data(), nl * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(cz.flag, 0, 4, s));
    launch_sdir_link(S, s, cz.codec, cz.d_ends, nl, 1, cz.d_cnt, cz.d_usum, cz.d_boff, cz.d_uoff, cz.flag);
    HIP_TRY(hipGetLastError());
    const bool zstd = cz.codec == 1;
    S.lds_bytes = cz_decode_lds(zstd, cz.lh.compression_block_size);
    hipError_t e = zstd ? launch_zstd_decode(S, s) : launch_snappy_decode(S, s);
    if (e != hipSuccess && S.lds_bytes) {  // the LDS size was refused: decode in global memory
      (void)hipGetLastError();
      S.lds_bytes = 0;
      e = zstd ? launch_zstd_decode(S, s) : launch_snappy_decode(S, s);
    }
    HIP_TRY(e);
    launch_snappy_walk(S, s);
    HIP_TRY(hipGetLastError());
  }
  std::vector<SnappyWalk> walks(nblk);
  std::vector<SnappyBlock> blocks(nblk);
  int32_t f = 0;
  if (nblk) {
    HIP_TRY(hipMemcpyAsync(walks.data(), pl->sn_walk, nblk * sizeof(SnappyWalk), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(blocks.data(), pl->sn_blocks, nblk * sizeof(SnappyBlock), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&f, cz.flag, 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (f) return SPARKEY_OK;
  // plan_build_snappy's composition of the block walks; any irregular block: the gathered build
  int64_t carry = 0;
  for (uint64_t b = 0; b < nblk; b++) {
    const SnappyWalk& w = walks[b];
    if (w.flags & kWalkBadStream) return SPARKEY_OK;
    if (carry == 0) {
      if (w.flags) return SPARKEY_OK;
      carry = w.overflow;
    } else if (carry >= (int64_t)blocks[b].ulen) {
      carry -= blocks[b].ulen;
    } else {
      return SPARKEY_OK;
    }
  }
  *carry_out = carry;
  return SPARKEY_OK;
}

int sk_cz_shard_begin(sparkey_plan* pl, const uint8_t* hdr, uint64_t file_len, uint64_t vlen,
                      const sparkey_build_opts* opts, int32_t rank, int32_t world, char* err, size_t err_len) {
  auto& cz = pl->cz;
  LogHdr lh;
  int rc = parse_log_header(hdr, 84, file_len, &lh, err, err_len, true);
  if (rc) return rc;
  IndexParams ip;
  rc = make_index_params(lh, *opts, &ip, err, err_len);
  if (rc) return rc;
  uint8_t vh[kLogHeaderSize];  // the virtual log's header, as plan_build_snappy writes it
  memcpy(vh, hdr, kLogHeaderSize);
  wr64(vh + 32, vlen);
  wr32(vh + 64, 0u);
  wr32(vh + 80, 1u);
  LogHdr vlh;
  rc = parse_log_header(vh, kLogHeaderSize, vlen, &vlh, err, err_len);
  if (rc) return rc;
  IndexParams fip = ip;  // the compressed log's table; entries framed with virtual offsets (ebb 0)
  fip.ebb = 0;
  return shard_begin_with(pl, vlh, fip, lh, ip, cz.S.vlog, (uint64_t)cz.vlo, (uint64_t)cz.vend, opts, rank, world, err,
                          err_len);
}

int sk_cz_to_real(sparkey_plan* pl, uint8_t* d_records, uint64_t n, uint32_t rec_bytes, hipStream_t s, char* err,
                  size_t err_len) {
  auto& cz = pl->cz;
  if (!n) return SPARKEY_OK;
  if (rec_bytes < 16 || (rec_bytes & 7)) {
    set_err(err, err_len, "bad record size");
    return SPARKEY_E_ARG;
  }
  HIP_TRY(hipMemsetAsync(cz.flag, 0, 4, s));
  launch_cz_to_real(cz.S, s, (uint64_t*)d_records, n, rec_bytes / 8, cz.flag);
  HIP_TRY(hipGetLastError());
  int32_t f = 0;
  HIP_TRY(hipMemcpyAsync(&f, cz.flag, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (f) {
    set_err(err, err_len, "internal error: a framed entry is not a record start of its block");
    return SPARKEY_E_CORRUPT_LOG;
  }
  return SPARKEY_OK;
}

int sk_cz_to_virtual(sparkey_plan* pl, uint64_t* d_addrs, uint64_t n, hipStream_t s, char* err, size_t err_len) {
  launch_cz_to_virtual(pl->cz.S, s, d_addrs, n);
  HIP_TRY(hipGetLastError());
  return SPARKEY_OK;
}
