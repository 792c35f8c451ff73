// shard_host.cpp -- the host orchestration of the sharded .spi build, in C++.
//
// The reference build is single-threaded (Sparkey.java:36; IndexHash.createNew, IndexHash.java:131-167).
// The sharded build splits the same computation at the points where ranks exchange data and runs the
// device steps of include/sparkey_gpu.h ("sharded build") in between:
//   1. entries    rank g > 0 finds a record start near the head of its byte range; the starts are
//                 all-gathered; each rank frames [c_g, c_{g+1}) and reports its exit; exit == next
//                 start proves the next start is on the record chain (induction from 84).
//   2. exchange   every (hash, address) entry to the owner of its slot range: one all-to-all.
//   3. placement  per-range carry functions all-gathered and composed in ring order; spilled slots and
//                 equal-hash pairs (IndexHash.java:606-636) resolved with small exchanges.
//   4. stats      calculateMaxDisplacement (IndexHash.java:195-245) per range plus the boundary rows;
//                 rank 0 writes the 112-byte header.
// Logs with DELETEs or duplicate keys take the sharded exact path.  Compressed logs
//  are framed as their virtual log: each rank decodes the blocks of its own byte range
// into its slice of it (Rank::compressed).  Tables the PUT records fill gather the log on every rank
// and build it whole (correct, not scaled).
//
// One rank is one sparkey_shard_build call on its own thread / process and device.  The collectives go
// through Coll: RCCL (ncclAllGather, grouped ncclSend/ncclRecv; xGMI between the GPUs of a node), or
// threads of one process sharing memory (ranks on the same or different devices; the -m gpu tests
// run 2-4 ranks on one GPU this way).  sparkey_build_index_mem / _file with opts.num_gpus > 1 run N
// ranks as threads of the caller's process (shard_run_threads below).
//
// sparkey-java_amd/sparkey/sharded.py is the same orchestration in Python over torch.distributed; the
// CPU tests run it over a simulation of the device steps (tests/shard_sim.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>  // types only: librccl is opened at run time (shared with torch's copy when loaded)

#include "../../include/sparkey_gpu.h"
#include "knobs.hpp"
#include "shard_host.hpp"

namespace {

constexpr int64_t kLogHeader = 84;
constexpr int64_t kIndexHeader = 112;
constexpr int kSpillInline = 64;  // spilled slots per rank that travel with the placement flags
constexpr int kSpillBytes = 32;
constexpr int kEntryBytes = 16;

void set_err(char* err, size_t err_len, const std::string& msg) {
  if (err && err_len > 0) snprintf(err, err_len, "%s", msg.c_str());
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* code_text(int rc) {
  switch (rc) {
    case SPARKEY_E_NOT_LOG: return "File is not a Sparkey log file";
    case SPARKEY_E_VERSION: return "Incompatible version";
    case SPARKEY_E_CORRUPT_LOG: return "Corrupt log file";
    case SPARKEY_E_NO_FREE_SLOTS: return "No free slots in the hash";
    case SPARKEY_E_CORRUPT_DATA: return "Corrupt data";
    case SPARKEY_E_VLQ: return "Too long VLQ value";
    case SPARKEY_E_HEADER: return "Too large max key len";
    case SPARKEY_E_CORRUPT_RECORD: return "Corrupt log record";
    default: return "error";
  }
}

// ---------------------------------------------------------------------------------------------
// RCCL, opened at run time
// ---------------------------------------------------------------------------------------------
struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char* (*GetErrorString)(ncclResult_t);
};

const RcclApi* rccl_api(std::string* why) {
  static std::once_flag once;
  static RcclApi api;
  static bool ok = false;
  static std::string reason;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      reason = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p) all = false;
      return p;
    };
    api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
    api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
    api.CommInitAll = (decltype(api.CommInitAll))sym("ncclCommInitAll");
    api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
    api.AllGather = (decltype(api.AllGather))sym("ncclAllGather");
    api.Send = (decltype(api.Send))sym("ncclSend");
    api.Recv = (decltype(api.Recv))sym("ncclRecv");
    api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
    api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
    api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
    if (!all) {
      reason = "librccl lacks a needed symbol";
      return;
    }
    ok = true;
  });
  if (!ok && why) *why = reason;
  return ok ? &api : nullptr;
}

class RcclColl : public Coll {
 public:
  RcclColl(const RcclApi* api, ncclComm_t c, int r, int w) : api_(api), comm_(c) {
    rank = r;
    world = w;
  }
  ~RcclColl() override {
    if (comm_) api_->CommDestroy(comm_);
  }
  int all_gather(const void* d_send, void* d_recv, size_t bytes, hipStream_t s, std::string* why) override {
    return check(api_->AllGather(d_send, d_recv, bytes, ncclUint8, comm_, s), why);
  }
  int all_to_all(const uint8_t* d_send, const uint64_t* send_bytes, uint8_t* d_recv, const uint64_t* recv_bytes,
                 hipStream_t s, std::string* why) override {
    uint64_t so = 0, ro = 0;
    std::vector<uint64_t> soff(world), roff(world);
    for (int r = 0; r < world; r++) {
      soff[r] = so;
      roff[r] = ro;
      so += send_bytes[r];
      ro += recv_bytes[r];
    }
    if (send_bytes[rank] && hipMemcpyAsync(d_recv + roff[rank], d_send + soff[rank], send_bytes[rank],
                                           hipMemcpyDeviceToDevice, s) != hipSuccess) {
      *why = "self copy failed";
      return SPARKEY_E_GPU;
    }
    int rc = check(api_->GroupStart(), why);
    for (int r = 0; r < world && !rc; r++) {
      if (r == rank) continue;
      if (send_bytes[r]) rc = check(api_->Send(d_send + soff[r], send_bytes[r], ncclUint8, r, comm_, s), why);
      if (!rc && recv_bytes[r]) rc = check(api_->Recv(d_recv + roff[r], recv_bytes[r], ncclUint8, r, comm_, s), why);
    }
    const int rc2 = check(api_->GroupEnd(), why);
    return rc ? rc : rc2;
  }

 private:
  int check(ncclResult_t r, std::string* why) {
    if (r == ncclSuccess) return SPARKEY_OK;
    *why = std::string("RCCL: ") + api_->GetErrorString(r);
    return SPARKEY_E_GPU;
  }
  const RcclApi* api_;
  ncclComm_t comm_;
};

// ---------------------------------------------------------------------------------------------
// threads of one process: every rank posts its buffers, waits for the others, copies what it needs
// (device to device on its own stream), waits for its copies, and meets the others again before
// any buffer is reused.  abort() releases every waiter (a rank that failed outside a collective).
// ---------------------------------------------------------------------------------------------
struct ThreadShared {
  explicit ThreadShared(int w) : world(w), send(w), soff(w), sbytes(w) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<const uint8_t*> send;
  std::vector<std::vector<uint64_t>> soff, sbytes;

  bool barrier() {
    std::unique_lock<std::mutex> l(mu);
    if (aborted) return false;
    const uint64_t my = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return true;
    }
    cv.wait(l, [&] { return gen != my || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> g(mu);
    aborted = true;
    cv.notify_all();
  }
};

class ThreadColl : public Coll {
 public:
  ThreadColl(std::shared_ptr<ThreadShared> sh, int r) : sh_(std::move(sh)) {
    rank = r;
    world = sh_->world;
  }
  void abort() override { sh_->abort(); }
  int all_gather(const void* d_send, void* d_recv, size_t bytes, hipStream_t s, std::string* why) override {
    std::vector<uint64_t> sb(world, bytes), rb(world, bytes);
    // every rank's block goes to every rank: the same block offset 0 of the sender for each receiver
    return exchange((const uint8_t*)d_send, sb, (uint8_t*)d_recv, rb, true, s, why);
  }
  int all_to_all(const uint8_t* d_send, const uint64_t* send_bytes, uint8_t* d_recv, const uint64_t* recv_bytes,
                 hipStream_t s, std::string* why) override {
    return exchange(d_send, std::vector<uint64_t>(send_bytes, send_bytes + world), d_recv,
                    std::vector<uint64_t>(recv_bytes, recv_bytes + world), false, s, why);
  }

 private:
  int exchange(const uint8_t* d_send, const std::vector<uint64_t>& sb, uint8_t* d_recv, const std::vector<uint64_t>& rb,
               bool gather, hipStream_t s, std::string* why) {
    if (hipStreamSynchronize(s) != hipSuccess) {  // the send buffer is complete
      *why = "stream synchronisation failed";
      sh_->abort();
      return SPARKEY_E_GPU;
    }
    std::vector<uint64_t> off(world);
    uint64_t o = 0;
    for (int r = 0; r < world; r++) {
      off[r] = gather ? 0 : o;
      o += sb[r];
    }
    sh_->send[rank] = d_send;
    sh_->soff[rank] = off;
    sh_->sbytes[rank] = sb;
    if (!sh_->barrier()) return aborted(why);
    uint64_t ro = 0;
    bool ok = true;
    for (int r = 0; r < world; r++) {
      const uint64_t n = rb[r];
      if (n != sh_->sbytes[r][rank]) ok = false;
      if (ok && n && hipMemcpyAsync(d_recv + ro, sh_->send[r] + sh_->soff[r][rank], n, hipMemcpyDeviceToDevice, s) !=
                         hipSuccess)
        ok = false;
      ro += n;
    }
    if (hipStreamSynchronize(s) != hipSuccess) ok = false;
    if (!ok) {
      *why = "in-process exchange failed (sizes disagree or copy failed)";
      sh_->abort();
      return SPARKEY_E_GPU;
    }
    if (!sh_->barrier()) return aborted(why);
    return SPARKEY_OK;
  }
  int aborted(std::string* why) {
    *why = "another rank of the sharded build failed";
    return SPARKEY_E_GPU;
  }
  std::shared_ptr<ThreadShared> sh_;
};

// ---------------------------------------------------------------------------------------------
// collectives supplied by the host program (sparkey_shard_comm_create_host): every buffer is staged
// through pinned host memory and handed to the caller's functions, which move it between the ranks
// (torch.distributed gloo for the one-GPU multi-process rehearsal, or a JVM's own transport).
// ---------------------------------------------------------------------------------------------
class HostColl : public Coll {
 public:
  HostColl(const sparkey_shard_transport& t, int r, int w) : t_(t) {
    rank = r;
    world = w;
  }
  ~HostColl() override {
    if (h_) (void)hipHostFree(h_);
  }
  int all_gather(const void* d_send, void* d_recv, size_t bytes, hipStream_t s, std::string* why) override {
    uint8_t* h = stage((uint64_t)bytes * (world + 1));
    if (!h) return err(why, "pinned staging allocation failed");
    // A rank whose own rows cannot leave the device still takes part, with all-ones rows: the peers
    // do not block in the transport, and a row whose code words read -1 fails every rank at the next
    // checkpoint (fail_together).  (A peer that never arrives is the transport's to time out.)
    const int rc = injected(why) ? SPARKEY_E_GPU : copy(h, d_send, bytes, hipMemcpyDeviceToHost, s, why);
    if (rc) memset(h, 0xff, bytes);
    if (t_.all_gather(t_.ctx, h, h + bytes, bytes) != 0) return rc ? rc : err(why, "host transport all_gather failed");
    if (rc) return rc;
    return copy(d_recv, h + bytes, (uint64_t)bytes * world, hipMemcpyHostToDevice, s, why);
  }
  int all_to_all(const uint8_t* d_send, const uint64_t* send_bytes, uint8_t* d_recv, const uint64_t* recv_bytes,
                 hipStream_t s, std::string* why) override {
    uint64_t sb = 0, rb = 0;
    for (int r = 0; r < world; r++) {
      sb += send_bytes[r];
      rb += recv_bytes[r];
    }
    uint8_t* h = stage(sb + rb);
    if (!h) return err(why, "pinned staging allocation failed");
    const int rc = injected(why) ? SPARKEY_E_GPU : copy(h, d_send, sb, hipMemcpyDeviceToHost, s, why);  // (as all_gather: take part anyway)
    if (rc) memset(h, 0xff, sb);
    if (t_.all_to_all(t_.ctx, h, send_bytes, h + sb, recv_bytes) != 0) return rc ? rc : err(why, "host transport all_to_all failed");
    if (rc) return rc;
    return copy(d_recv, h + sb, rb, hipMemcpyHostToDevice, s, why);
  }

 private:
  static int err(std::string* why, const char* m) {
    *why = m;
    return SPARKEY_E_GPU;
  }
  uint8_t* stage(uint64_t n) {
    n = std::max<uint64_t>(n, 64);
    if (h_ && cap_ >= n) return h_;
    if (h_) (void)hipHostFree(h_);
    h_ = nullptr;
    cap_ = 0;
    if (hipHostMalloc((void**)&h_, n, hipHostMallocDefault) != hipSuccess) return nullptr;
    cap_ = n;
    return h_;
  }
  static int copy(void* dst, const void* src, uint64_t n, hipMemcpyKind k, hipStream_t s, std::string* why) {
    if (n && (hipMemcpyAsync(dst, src, n, k, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess))
      return err(why, "staging copy failed");
    return SPARKEY_OK;
  }
  // (shard_coll_fail switch, tests: the k-th collective of this communicator fails its device copy,
  //  counted from 1 over its lifetime)
  bool injected(std::string* why) {
    if (sk::knob(sk::Knob::ShardCollFail) != (int64_t)++calls_) return false;
    *why = "staging copy failed (shard_coll_fail)";
    return true;
  }
  sparkey_shard_transport t_;
  uint8_t* h_ = nullptr;
  uint64_t cap_ = 0;
  uint64_t calls_ = 0;
};

// ---------------------------------------------------------------------------------------------
// log geometry (sharded.py shard_layout)
// ---------------------------------------------------------------------------------------------
uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
int64_t rd64(const uint8_t* p) {
  int64_t v;
  memcpy(&v, p, 8);
  return v;
}

int vlq_size(int64_t v) {  // Util.java:102-128
  int n = 1;
  while (n < 9 && v >= (1LL << (7 * n))) n++;
  return n;
}

struct Layout {
  int64_t num_puts, num_deletes, data_end, max_key_len, max_value_len, put_size;
  int32_t compression, mepb;
  int64_t max_rec, window;
  std::vector<int64_t> lo, hi;
  bool small;
  int64_t uni;  // uniform record size, or 0
  int64_t cz_h;  // compressed logs: the block chain's hop bound (sk_cz_hop_bound), or 0
  int world;
  // bytes past a rank's range that it loads: records crossing into the next range; compressed logs:
  // the next range's first anchor (at most 2 hops in) and the hop past it
  int64_t overlap() const { return cz_h ? 3 * cz_h + 4096 : 2 * max_rec + window + 64; }
};

Layout make_layout(const uint8_t* h, int world) {
  Layout L;
  L.num_puts = rd64(h + 16);
  L.num_deletes = rd64(h + 24);
  L.data_end = std::max<int64_t>(rd64(h + 32), kLogHeader);
  L.max_key_len = rd64(h + 40);
  L.max_value_len = rd64(h + 48);
  L.compression = (int32_t)rd32(h + 64);
  L.put_size = rd64(h + 72);
  L.mepb = (int32_t)rd32(h + 80);
  const int64_t k = std::max<int64_t>(0, L.max_key_len), v = std::max<int64_t>(0, L.max_value_len);
  const int64_t put = vlq_size(k + 1) + vlq_size(v) + k + v, del = 1 + vlq_size(k) + k;
  L.max_rec = std::max<int64_t>(1, std::max(put, del));
  L.window = std::max<int64_t>(4096, 8 * L.max_rec);
  const int64_t span = L.data_end - kLogHeader;
  L.world = world;
  for (int g = 0; g < world; g++) L.lo.push_back(kLogHeader + (int64_t)((__int128)g * span / world));
  for (int g = 0; g < world; g++) L.hi.push_back(g + 1 < world ? L.lo[g + 1] : L.data_end);
  L.cz_h = L.compression != 0 ? std::max<int64_t>(0, sk_cz_hop_bound(h)) : 0;
  L.small = world > 1 && span / world < (L.cz_h ? 2 * L.cz_h + 4096 : 2 * (L.max_rec + L.window) + 64);
  // uniform records (sparkey_gpu.cpp uniform_record_size): the shard entries are arithmetic
  const int64_t r = vlq_size(L.max_key_len + 1) + vlq_size(L.max_value_len) + L.max_key_len + L.max_value_len;
  L.uni = (L.num_deletes == 0 && L.num_puts > 0 && L.max_key_len + 1 < 128 && L.max_value_len < 128 && r <= 256 &&
           L.put_size == L.num_puts * r && L.data_end - kLogHeader == L.put_size && !sk::knob_on(sk::Knob::NoUniform))
              ? r
              : 0;
  return L;
}

void buffer_range(const Layout& L, uint64_t file_len, int rank, uint64_t* lo, uint64_t* hi) {
  if (L.small) {
    *lo = 0;
    *hi = rank == 0 ? file_len : 0;
    return;
  }
  *lo = rank == 0 ? 0 : (uint64_t)(L.lo[rank] / 4096) * 4096;
  *hi = rank == L.world - 1 ? file_len : std::min<uint64_t>(file_len, (uint64_t)(L.hi[rank] + L.overlap()));
}

int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}

struct Geo {  // IndexHash.createNew's parameters (IndexHash.java:135-150), as make_index_params
  uint64_t cap;
  int32_t hash_size, addr_size, slot, ebb;
};

Geo make_geo(const Layout& L, const uint8_t* h, const sparkey_build_opts& o) {
  Geo G;
  double sp = o.sparsity;
  if (sp < 1.3) sp = 1.3;
  G.ebb = 0;
  while ((1LL << G.ebb) < (int64_t)L.mepb) G.ebb++;
  G.addr_size = rd64(h + 32) <= (1LL << (30 - G.ebb)) ? 4 : 8;
  G.hash_size = o.hash_size ? o.hash_size : (L.num_puts < (1 << 23) ? 4 : 8);
  G.cap = (uint64_t)(1LL | java_d2l((double)L.num_puts * sp));
  G.slot = G.hash_size + G.addr_size;
  return G;
}

int64_t signed64(uint64_t v) { return (int64_t)v; }

}  // namespace

// ---------------------------------------------------------------------------------------------
// per-rank device scratch, kept across builds (every build ends synchronised)
// ---------------------------------------------------------------------------------------------
struct DBuf {
  uint8_t* p = nullptr;
  uint64_t cap = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  uint8_t* ensure(uint64_t n) {
    n = std::max<uint64_t>(16, (n + 15) & ~15ull);
    if (p && cap >= n) return p;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc((void**)&p, n) != hipSuccess) return nullptr;
    cap = n;
    return p;
  }
};

struct sparkey_shard_comm {
  std::unique_ptr<Coll> coll;
  int device = 0;
  DBuf row, rows, send, recv, fun, funs, flags, frows, fin, fins, spill, small_send, small_recv, pad, var_recv,
      var_out, exsend, exrecv, send2, recv2, req, got, rec, back, recs, glog, full;
  std::vector<std::pair<std::string, double>> phase;
};

namespace {

// one rank's build (sharded.py ShardedBuilder._build)
class Rank {
 public:
  Rank(sparkey_plan* pl, sparkey_shard_comm* cm, hipStream_t s, char* err, size_t err_len)
      : pl_(pl), cm_(cm), c_(cm->coll.get()), s_(s), err_(err), err_len_(err_len), g_(c_->rank), G_(c_->world) {}

  // rc0 != 0: this rank already failed (e.g. loading its log range); it still meets the other ranks at
  // the first checkpoint so that every rank returns the error instead of waiting for it
  int run(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi,
          const sparkey_build_opts& o, uint8_t* d_out, uint64_t out_cap, sparkey_build_stats* st, int rc0);

 private:
  // ---- helpers ----
  int fail(int rc, const std::string& msg) {
    set_err(err_, err_len_, msg);
    return rc;
  }
  // Every rank fails together: a rank whose own step failed does not return on its own,
  // it posts its code at the next exchange (a checkpoint, or a field of a row every rank gathers
  // anyway) and all ranks return from the same place.  `codes[r]` is rank r's code (0 = fine).
  int fail_together(const std::vector<int64_t>& codes, int own) {
    for (int r = 0; r < G_; r++)
      if (codes[r]) {
        if (r == g_) return own ? own : (int)codes[r];  // (its own message is in err_)
        if (own) return own;
        // (-1 from a peer is HostColl's all-ones row: its row could not leave its device.  No step after
        //  the header checks -- which every rank makes alike before any collective -- returns
        //  SPARKEY_E_NOT_LOG.)
        const int code = codes[r] == -1 ? SPARKEY_E_GPU : (int)codes[r];
        return fail(code, std::string("another rank of the sharded build failed (rank ") + std::to_string(r) + ": " +
                              (codes[r] == -1 ? "its row could not leave its device" : code_text(code)) + ")");
      }
    return SPARKEY_OK;
  }
  // a checkpoint: every rank's local code gathered; non-zero anywhere -> every rank fails
  int agree(int own) {
    if (G_ == 1) return own;
    std::vector<int64_t> codes;
    const int rc = gather_i64({own}, &codes);
    if (rc) return rc;
    return fail_together(codes, own);
  }
  int gpu(hipError_t e, const char* what) {
    if (e == hipSuccess) return SPARKEY_OK;
    return fail(SPARKEY_E_GPU, std::string(what) + ": " + hipGetErrorString(e));
  }
  int coll_rc(int rc, const std::string& why) { return rc ? fail(rc, why) : SPARKEY_OK; }
  void mark(const char* name) {
    const double t = now_ms();
    cm_->phase.emplace_back(name, t - clock_);
    clock_ = t;
  }
  // every rank's small int64 vector (same length on every rank) -> host rows.  Every such gather is
  // also a checkpoint: the row carries the rank's sticky failure (sticky_) as one more word, and a
  // nonzero word in any row -- a failure recorded since the last checkpoint, or -1 from HostColl's
  // all-ones row of a rank whose copy failed -- fails every rank here, together.
  int gather_i64(const std::vector<int64_t>& v, std::vector<int64_t>* out) {
    const size_t w = v.size() + 1;
    const uint64_t b = w * 8;
    std::vector<int64_t> row(v);
    row.push_back(sticky_);
    uint8_t* sd = cm_->small_send.ensure(b);
    uint8_t* rd = cm_->small_recv.ensure(b * G_);
    if (!sd || !rd) return fail(SPARKEY_E_GPU, "hipMalloc failed");
    int rc = gpu(hipMemcpyAsync(sd, row.data(), b, hipMemcpyHostToDevice, s_), "H2D");
    std::string why;
    if (!rc) rc = coll_rc(c_->all_gather(sd, rd, b, s_, &why), why);
    std::vector<int64_t> all(w * G_, 0);
    if (!rc) rc = gpu(hipMemcpyAsync(all.data(), rd, b * G_, hipMemcpyDeviceToHost, s_), "D2H");
    if (!rc) rc = gpu(hipStreamSynchronize(s_), "sync");
    out->assign(v.size() * G_, 0);
    if (rc) return sticky_ ? sticky_ : rc;
    std::vector<int64_t> codes(G_);
    for (int r = 0; r < G_; r++) {
      for (size_t i = 0; i + 1 < w; i++) (*out)[(size_t)r * v.size() + i] = all[(size_t)r * w + i];
      codes[r] = all[(size_t)r * w + w - 1];
    }
    return fail_together(codes, sticky_);
  }
  // a failure after which this rank still joins the collectives up to the next gather_i64 (where every
  // rank fails): it skips its device steps meanwhile (ok() false)
  int note(int rc) {
    if (rc && !sticky_) sticky_ = rc;
    return rc;
  }
  bool ok() const { return sticky_ == SPARKEY_OK; }
  int all_gather(const void* d_send, DBuf& dst, uint64_t bytes) {
    uint8_t* rd = dst.ensure(bytes * G_);
    if (!rd) return fail(SPARKEY_E_GPU, "hipMalloc failed");
    std::string why;
    return coll_rc(c_->all_gather(d_send, rd, bytes, s_, &why), why);
  }
  int to_host(void* h, const void* d, uint64_t b) {
    int rc = gpu(hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, s_), "D2H");
    return rc ? rc : gpu(hipStreamSynchronize(s_), "sync");
  }
  // every rank's first n[rank] bytes of d_src, concatenated in rank order into dst (allgather_var)
  int gather_var(const uint8_t* d_src, uint64_t n, DBuf& dst, uint64_t* total) {
    std::vector<int64_t> cnt;
    int rc = gather_i64({(int64_t)n}, &cnt);
    if (rc) return rc;
    uint64_t m = 1, tot = 0;
    for (int r = 0; r < G_; r++) {
      m = std::max<uint64_t>(m, (uint64_t)cnt[r]);
      tot += (uint64_t)cnt[r];
    }
    m = (m + 15) & ~15ull;
    uint8_t* pad = cm_->pad.ensure(m);
    uint8_t* rv = cm_->var_recv.ensure(m * G_);
    uint8_t* out = dst.ensure(tot + 16);
    // (after the count checkpoint: a failure is noted and the rank still joins the data gather; its
    //  caller's next checkpoint fails every rank)
    if (!pad || !rv || !out) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
    if (ok() && n) note(gpu(hipMemcpyAsync(pad, d_src, n, hipMemcpyDeviceToDevice, s_), "D2D"));
    std::string why;
    note(coll_rc(c_->all_gather(pad, rv, m, s_, &why), why));
    uint64_t at = 0;
    for (int r = 0; r < G_ && ok(); r++) {
      if (cnt[r]) note(gpu(hipMemcpyAsync(out + at, rv + (uint64_t)r * m, (uint64_t)cnt[r], hipMemcpyDeviceToDevice, s_), "D2D"));
      at += (uint64_t)cnt[r];
    }
    *total = tot;
    return SPARKEY_OK;  // (the count checkpoint's outcome; a later failure is sticky_)
  }
  int64_t fe(int r) const {  // sharded.py frame_end(r)
    if (r == G_ - 1) return F_.data_end;
    return valid_[r + 1] ? entries_[r + 1] : F_.hi[r];
  }

  int range_stats(uint64_t slot_lo, uint64_t slot_hi, std::vector<int64_t>* bnd);
  void combine_stats(const std::vector<int64_t>& bnd, int stride, int off, int64_t* mx, int64_t* col, int64_t* tot);
  int pairs_share_a_key(int64_t n_pairs, bool* dup);
  int exact(uint8_t* out, uint64_t hdr_off, int64_t n_records, const sparkey_build_opts& o, uint64_t slot_lo,
            uint64_t slot_hi, bool* done, sparkey_build_stats* st);
  int gathered(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo,
               const sparkey_build_opts& o, uint8_t* out, uint64_t slot_lo, uint64_t out_len, sparkey_build_stats* st);
  int compressed(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi,
                 const sparkey_build_opts& o, std::vector<int64_t>* cs, int64_t* vlen, bool* take);

  sparkey_plan* pl_;
  sparkey_shard_comm* cm_;
  Coll* c_;
  hipStream_t s_;
  char* err_;
  size_t err_len_;
  int g_, G_;
  Layout L_;
  Layout F_;    // the framed log's layout: L_, or the virtual log's (compressed logs)
  bool virt_ = false;           // compressed log framed as its virtual log (Rank::compressed)
  std::vector<int64_t> ce_;     // ... each rank's first block in the compressed log
  Geo geo_;
  std::vector<int64_t> entries_;
  std::vector<bool> valid_;
  double clock_ = 0;
  const uint8_t* hdr_ = nullptr;
  int sticky_ = SPARKEY_OK;  // this rank's failure since the last checkpoint (gather_i64)
};

int Rank::range_stats(uint64_t slot_lo, uint64_t slot_hi, std::vector<int64_t>* bnd) {
  const int nonempty = slot_hi > slot_lo ? 1 : 0;
  uint64_t b[4] = {0, 0, 0, 0};
  if (ok()) note(sparkey_shard_boundary(pl_, s_, b, err_, err_len_));
  int64_t sx[3] = {0, 0, 0};
  if (nonempty && ok()) note(sparkey_shard_stats(pl_, 0, 0, s_, sx, err_, err_len_));
  return gather_i64({signed64(b[0]), signed64(b[1]), signed64(b[2]), signed64(b[3]), nonempty, sx[0], sx[1], sx[2]}, bnd);
}

// calculateMaxDisplacement (IndexHash.java:195-245) from every rank's range row {first hash, first
// address, last hash, last address, non-empty, max, collisions, total} at bnd[r * stride + off ..]:
// the per-range sums plus the comparisons across range boundaries and the wrap quirk (:239-241).
void Rank::combine_stats(const std::vector<int64_t>& bnd, int stride, int off, int64_t* mx, int64_t* col,
                         int64_t* tot) {
  auto at = [&](int r, int k) { return bnd[(size_t)r * stride + off + k]; };
  int64_t m = 0, c = 0, t = 0;
  bool have_prev = false;
  uint64_t prev_hash = 0;
  bool prev_occ = false;
  int last = -1;
  for (int r = 0; r < G_; r++) {
    m = std::max(m, at(r, 5));
    c += at(r, 6);
    t += at(r, 7);
    if (!at(r, 4)) continue;
    if (have_prev && prev_occ && prev_hash == (uint64_t)at(r, 0)) c++;
    have_prev = true;
    prev_hash = (uint64_t)at(r, 2);
    prev_occ = at(r, 3) != 0;
    last = r;
  }
  if (last >= 0 && at(0, 1) != 0 && at(last, 3) != 0 && at(0, 0) == at(last, 2)) c++;
  *mx = m;
  *col = c;
  *tot = t;
}

// Equal-hash pairs: both keys fetched from the ranks holding the records, compared on the device
// (IndexHash.java:606-636: put compares the keys of equal hashes).
int Rank::pairs_share_a_key(int64_t n_pairs, bool* dup_any) {
  std::vector<uint64_t> addrs((size_t)(2 * n_pairs));
  if (n_pairs && note(sparkey_shard_pairs(pl_, addrs.data(), (uint64_t)n_pairs, err_, err_len_)))
    n_pairs = 0;  // (noted: the checkpoint below fails every rank)
  const int64_t n2 = 2 * n_pairs;
  std::vector<int> owner((size_t)n2);
  for (int64_t i = 0; i < n2; i++) {
    const int64_t pos = (int64_t)((addrs[i] & ~(1ull << 63)) >> geo_.ebb);
    int o = 0;
    for (int r = 0; r < G_; r++) {
      const int64_t st = virt_ ? ce_[r] : valid_[r] ? entries_[r] : L_.data_end;
      if (st <= pos) o = r;  // searchsorted(starts, pos, right) - 1, clipped
    }
    owner[i] = o;
  }
  std::vector<int64_t> order((size_t)n2);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return owner[a] < owner[b]; });
  std::vector<int64_t> req((size_t)n2), counts(G_, 0);
  for (int64_t i = 0; i < n2; i++) {
    req[i] = (int64_t)addrs[order[i]];
    counts[owner[order[i]]]++;
  }
  std::vector<int64_t> M;
  int rc = gather_i64(counts, &M);
  if (rc) return rc;
  const int32_t rs = sparkey_shard_key_record_size(pl_);
  std::vector<uint64_t> sb(G_), rb(G_), sb2(G_), rb2(G_);
  uint64_t n_req = 0;
  for (int r = 0; r < G_; r++) {
    sb[r] = (uint64_t)counts[r] * 8;
    rb[r] = (uint64_t)M[(size_t)r * G_ + g_] * 8;
    n_req += (uint64_t)M[(size_t)r * G_ + g_];
    sb2[r] = (uint64_t)M[(size_t)r * G_ + g_] * rs;
    rb2[r] = (uint64_t)counts[r] * rs;
  }
  // (from here to the closing checkpoint a failure is noted and the rank still joins both all_to_alls)
  uint8_t* dreq = cm_->req.ensure(std::max<uint64_t>(8, n2 * 8));
  uint8_t* dgot = cm_->got.ensure(std::max<uint64_t>(8, n_req * 8));
  uint8_t* drec = cm_->rec.ensure(std::max<uint64_t>(1, n_req) * rs);
  uint8_t* dback = cm_->back.ensure(std::max<int64_t>(1, n2) * rs);
  if (!dreq || !dgot || !drec || !dback) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
  if (ok() && n2) note(gpu(hipMemcpyAsync(dreq, req.data(), n2 * 8, hipMemcpyHostToDevice, s_), "H2D"));
  std::string why;
  note(coll_rc(c_->all_to_all(dreq, sb.data(), dgot, rb.data(), s_, &why), why));
  if (ok() && n_req && virt_) note(sk_cz_to_virtual(pl_, (uint64_t*)dgot, n_req, s_, err_, err_len_));
  if (ok() && n_req) note(sparkey_shard_fetch_keys(pl_, (const uint64_t*)dgot, n_req, drec, (uint32_t)rs, s_, err_, err_len_));
  note(coll_rc(c_->all_to_all(drec, sb2.data(), dback, rb2.data(), s_, &why), why));
  int32_t dup = 0;
  if (ok() && n_pairs) {  // the records back in pair order: pair i's address sits at request position inv[i]
    std::vector<uint8_t> back((size_t)(n2 * rs)), recs((size_t)(n2 * rs));
    rc = note(to_host(back.data(), dback, n2 * rs));
    for (int64_t i = 0; i < n2 && !rc; i++) memcpy(&recs[(size_t)(order[i] * rs)], &back[(size_t)(i * rs)], (size_t)rs);
    uint8_t* drecs = rc ? nullptr : cm_->recs.ensure(n2 * rs);
    if (!rc && !drecs) rc = note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
    if (!rc) rc = note(gpu(hipMemcpyAsync(drecs, recs.data(), n2 * rs, hipMemcpyHostToDevice, s_), "H2D"));
    if (!rc) note(sparkey_shard_compare_keys(pl_, drecs, (uint64_t)n_pairs, (uint32_t)rs, s_, &dup, err_, err_len_));
  }
  std::vector<int64_t> d;
  rc = gather_i64({dup != 0 ? 1 : 0}, &d);
  if (rc) return rc;
  *dup_any = std::any_of(d.begin(), d.end(), [](int64_t x) { return x != 0; });
  return SPARKEY_OK;
}

// The sharded exact path: IndexHash.put / delete (IndexHash.java:454-665) replayed
// on exact ranges.  *done = false when the log needs the gathered path (no empty slot, long keys).
int Rank::exact(uint8_t* out, uint64_t hdr_off, int64_t n_records, const sparkey_build_opts& o, uint64_t slot_lo,
                uint64_t slot_hi, bool* done, sparkey_build_stats* st) {
  *done = false;
  const uint64_t cap = geo_.cap;
  const uint64_t ss = (uint64_t)geo_.slot;
  // (a failure between two checkpoints is noted and the rank joins the collectives up to the next
  //  gather_i64, which fails every rank together)
  int64_t fe_slot = -1;
  if (note(sparkey_shard_first_empty(pl_, s_, &fe_slot, err_, err_len_))) fe_slot = -1;
  std::vector<int64_t> E;
  int rc = gather_i64({fe_slot}, &E);
  if (rc) return rc;
  std::vector<int> have;
  for (int r = 0; r < G_; r++)
    if (E[r] >= 0) have.push_back(r);
  const int32_t rs = sparkey_shard_exact_record_size(pl_);
  if (have.empty() || rs <= 0) return SPARKEY_OK;
  std::map<int, std::pair<uint64_t, uint64_t>> ranges;
  for (size_t i = 0; i < have.size(); i++) {
    const uint64_t a = (uint64_t)E[have[i]], b = (uint64_t)E[have[(i + 1) % have.size()]];
    ranges[have[i]] = {a, b <= a ? b + cap : b};
  }
  // every record (PUT and DELETE) with its header and key to the owner of its wanted slot's range
  std::vector<uint64_t> counts(G_, 0);
  if (note(sparkey_shard_exact_frame(pl_, entries_[g_], fe(g_), n_records, E.data(), s_, counts.data(), err_, err_len_)))
    std::fill(counts.begin(), counts.end(), 0);
  uint64_t n_send = 0;
  for (uint64_t v : counts) n_send += v;
  uint8_t* send = cm_->exsend.ensure(std::max<uint64_t>(1, n_send) * rs);
  if (!send) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
  if (ok()) note(sparkey_shard_exact_pack(pl_, send, cm_->exsend.cap, s_, err_, err_len_));
  // a compressed log framed as its virtual log: the records' addresses to the compressed log's (the
  // replay orders by receive-buffer offset; the address field is what the extract writes)
  if (ok() && virt_) note(sk_cz_to_real(pl_, send, n_send, (uint32_t)rs, s_, err_, err_len_));
  std::vector<int64_t> M;
  rc = gather_i64(std::vector<int64_t>(counts.begin(), counts.end()), &M);
  if (rc) return rc;
  uint64_t n_recv = 0;
  std::vector<uint64_t> sb(G_), rb(G_);
  for (int r = 0; r < G_; r++) {
    n_recv += (uint64_t)M[(size_t)r * G_ + g_];
    sb[r] = counts[r] * rs;
    rb[r] = (uint64_t)M[(size_t)r * G_ + g_] * rs;
  }
  const uint8_t* recv = send;
  if (G_ > 1) {
    uint8_t* rv = cm_->exrecv.ensure(std::max<uint64_t>(1, n_recv) * rs);
    if (!rv) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
    std::string why;
    note(coll_rc(c_->all_to_all(send, sb.data(), rv, rb.data(), s_, &why), why));
    recv = rv;
  }
  sparkey_shard_exact_result rep;
  memset(&rep, 0, sizeof(rep));
  if (ok()) note(sparkey_shard_exact_build(pl_, n_recv ? recv : nullptr, n_recv, s_, &rep, err_, err_len_));
  std::vector<int64_t> rows;
  rc = gather_i64({rep.rc, rep.err_pos, rep.num_entries, rep.garbage_size}, &rows);
  if (rc) return rc;
  int64_t bad_pos = INT64_MAX, bad_rc = 0;
  int64_t n_entries = 0, garbage = 0;
  for (int r = 0; r < G_; r++) {
    const int64_t rrc = rows[(size_t)r * 4], pos = rows[(size_t)r * 4 + 1];
    if (rrc && (pos < bad_pos || (pos == bad_pos && rrc < bad_rc))) {
      bad_pos = pos;
      bad_rc = rrc;
    }
    n_entries += rows[(size_t)r * 4 + 2];
    garbage += rows[(size_t)r * 4 + 3];
  }
  if (bad_rc) return fail((int)bad_rc, std::string(code_text((int)bad_rc)) + " (log offset " + std::to_string(bad_pos) + ")");
  // the replayed slots to the ranks whose slices hold them (mostly a rank's own slice; the run before
  // the first empty slot of a slice was replayed by the previous range's owner)
  std::vector<std::pair<uint64_t, uint64_t>> slices(G_);
  for (int r = 0; r < G_; r++) sparkey_shard_slot_range(pl_, r, &slices[r].first, &slices[r].second);
  struct Piece {
    int q;
    uint64_t u, v;
  };
  auto pieces = [&](int r) {
    std::vector<Piece> got;
    auto it = ranges.find(r);
    if (it == ranges.end()) return got;
    const uint64_t a = it->second.first, b = it->second.second;
    std::vector<std::pair<uint64_t, uint64_t>> segs = {{a, std::min(b, cap)}};
    if (b > cap) segs.push_back({0, b - cap});
    for (int q = 0; q < G_; q++)
      for (auto& sg : segs) {
        const uint64_t u = std::max(sg.first, slices[q].first), v = std::min(sg.second, slices[q].second);
        if (u < v) got.push_back({q, u, v});
      }
    return got;
  };
  const std::vector<Piece> mine = pieces(g_);
  for (const Piece& p : mine)
    if (p.q == g_ && ok()) note(sparkey_shard_exact_extract(pl_, p.u, p.v, out + hdr_off + (p.u - slot_lo) * ss, s_, err_, err_len_));
  if (G_ > 1) {
    std::vector<uint64_t> to(G_, 0), frm(G_, 0), at(G_, 0);
    for (const Piece& p : mine)
      if (p.q != g_) to[p.q] += (p.v - p.u) * ss;
    uint64_t tot = 0;
    for (int q = 0; q < G_; q++) {
      at[q] = tot;
      tot += to[q];
    }
    uint8_t* send2 = cm_->send2.ensure(std::max<uint64_t>(1, tot));
    if (!send2) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
    for (const Piece& p : mine)
      if (p.q != g_) {
        if (ok()) note(sparkey_shard_exact_extract(pl_, p.u, p.v, send2 + at[p.q], s_, err_, err_len_));
        at[p.q] += (p.v - p.u) * ss;
      }
    uint64_t rtot = 0;
    for (int r = 0; r < G_; r++) {
      if (r == g_) continue;
      for (const Piece& p : pieces(r))
        if (p.q == g_) frm[r] += (p.v - p.u) * ss;
      rtot += frm[r];
    }
    uint8_t* recv2 = cm_->recv2.ensure(std::max<uint64_t>(1, rtot));
    if (!recv2) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
    std::string why;
    note(coll_rc(c_->all_to_all(send2, to.data(), recv2, frm.data(), s_, &why), why));
    uint64_t at2 = 0;
    for (int r = 0; r < G_ && ok(); r++) {
      if (r == g_) continue;
      for (const Piece& p : pieces(r))
        if (p.q == g_ && ok()) {
          const uint64_t nb = (p.v - p.u) * ss;
          note(gpu(hipMemcpyAsync(out + hdr_off + (p.u - slot_lo) * ss, recv2 + at2, nb, hipMemcpyDeviceToDevice, s_),
                   "D2D"));
          at2 += nb;
        }
    }
  }
  std::vector<int64_t> bnd;
  rc = range_stats(slot_lo, slot_hi, &bnd);
  if (rc) return rc;
  int64_t mx, col, tot;
  combine_stats(bnd, 8, 0, &mx, &col, &tot);
  if (g_ == 0) {
    uint8_t h[kIndexHeader];
    rc = sparkey_index_header(hdr_, &o, n_entries, garbage, mx, col, tot, h, err_, err_len_);
    if (!rc) rc = gpu(hipMemcpyAsync(out, h, kIndexHeader, hipMemcpyHostToDevice, s_), "H2D");
    if (!rc) rc = gpu(hipStreamSynchronize(s_), "sync");
    if (rc) return rc;
  }
  st->num_entries = n_entries;
  st->garbage_size = garbage;
  st->max_displacement = mx;
  st->hash_collisions = col;
  st->total_displacement = tot;
  st->placement_path = 2;
  st->sharded = 2;
  *done = true;
  return SPARKEY_OK;
}

// Logs the sharded steps do not cover: every rank gathers the whole log and builds it, then keeps its part.
int Rank::gathered(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo,
                   const sparkey_build_opts& o, uint8_t* out, uint64_t slot_lo, uint64_t out_len,
                   sparkey_build_stats* st) {
  uint64_t own_lo, own_hi;
  if (L_.small) {
    own_lo = 0;
    own_hi = g_ == 0 ? file_len : 0;
  } else {
    own_lo = g_ == 0 ? 0 : (uint64_t)L_.lo[g_];
    own_hi = g_ == G_ - 1 ? file_len : (uint64_t)L_.lo[g_ + 1];
  }
  const uint64_t n = own_hi > own_lo ? own_hi - own_lo : 0;
  uint64_t total = 0;
  int rc = gather_var(d_buf + (own_lo - buf_lo) * (n ? 1 : 0), n, cm_->glog, &total);
  if (rc) return rc;
  if (!ok()) return sticky_;  // (no collective follows: this rank fails alone)
  if (total != file_len) return fail(SPARKEY_E_GPU, "gathered log has the wrong length");
  const uint64_t full_len = kIndexHeader + geo_.cap * geo_.slot;
  uint8_t* full = cm_->full.ensure(full_len);
  if (!full) return fail(SPARKEY_E_GPU, "hipMalloc failed");
  rc = sparkey_plan_build_device(pl_, hdr, cm_->glog.p, file_len, full, full_len, &o, s_, st, err_, err_len_);
  if (rc) return rc;
  const uint64_t lo = g_ == 0 ? 0 : kIndexHeader + slot_lo * geo_.slot;
  if (out_len) rc = gpu(hipMemcpyAsync(out, full + lo, out_len, hipMemcpyDeviceToDevice, s_), "D2D");
  if (!rc) rc = gpu(hipStreamSynchronize(s_), "sync");
  st->sharded = 3;
  return rc;
}

// Compressed logs: each rank finds its part of the block chain from its own byte
// range (sk_cz_entry), follows it to the next rank's entry (sk_cz_count: induction from 84 as for the
// record chain) and decodes it into its slice of the virtual log (sk_cz_decode); the slices' starts
// become the ranks' entries and the NONE steps run over them.  *take = false (every rank alike): the
// gathered build, for logs these steps do not take (a record spanning two ranks' blocks, a link that
// misses, an irregular block -- the gathered build reports a corrupt log's error).  DELETEs and
// overwrites take the sharded exact path over the slices.
int Rank::compressed(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi,
                     const sparkey_build_opts& o, std::vector<int64_t>* cs, int64_t* vlen_out, bool* take) {
  *take = false;
  if (G_ == 1 || L_.small || !L_.cz_h || sk::knob_on(sk::Knob::ShardGatherCompressed))
    return SPARKEY_OK;
  auto together = [&](const std::vector<int64_t>& rows, int stride, int own) {
    std::vector<int64_t> codes(G_);
    for (int r = 0; r < G_; r++) codes[r] = rows[(size_t)r * stride + stride - 1];
    return fail_together(codes, own);
  };
  const int64_t lo = L_.lo[g_], hi = g_ + 1 < G_ ? L_.lo[g_ + 1] : L_.data_end;
  int64_t e = -1;
  int own = sk_cz_entry(pl_, hdr, file_len, d_buf, buf_lo, buf_hi, lo, hi, g_, s_, &e, err_, err_len_);
  std::vector<int64_t> E;
  int rc = gather_i64({e, own}, &E);
  if (!rc) rc = together(E, 2, own);
  if (rc) return rc;
  mark("cz_directory");
  std::vector<int64_t> ent(G_);
  for (int r = 0; r < G_; r++) ent[r] = E[2 * r];
  bool usable = ent[0] == kLogHeader;
  for (int r = 1; r < G_; r++) usable = usable && ent[r] >= L_.lo[r] && ent[r] >= ent[r - 1] && ent[r] <= L_.data_end;
  if (!usable) return SPARKEY_OK;
  int32_t ok = 0;
  uint64_t nb = 0, ul = 0;
  own = sk_cz_count(pl_, ent[g_], g_ + 1 < G_ ? ent[g_ + 1] : L_.data_end, s_, &ok, &nb, &ul, err_, err_len_);
  std::vector<int64_t> U;
  rc = gather_i64({ok, (int64_t)ul, own}, &U);
  if (!rc) rc = together(U, 3, own);
  if (rc) return rc;
  mark("cz_links");
  int64_t vbase = kLogHeader, vlen = kLogHeader;
  for (int r = 0; r < G_; r++) {
    if (!U[3 * r]) return SPARKEY_OK;
    if (r < g_) vbase += U[3 * r + 1];
    vlen += U[3 * r + 1];
  }
  int64_t carry = -1;
  own = sk_cz_decode(pl_, vbase, s_, &carry, err_, err_len_);
  rc = gather_i64({carry, own}, &E);
  if (!rc) rc = together(E, 2, own);
  if (rc) return rc;
  for (int r = 0; r < G_; r++)
    if (E[2 * r] != 0) return SPARKEY_OK;
  rc = agree(sk_cz_shard_begin(pl_, hdr, file_len, (uint64_t)vlen, &o, g_, G_, err_, err_len_));
  if (rc) return rc;
  cs->assign(G_, 0);
  int64_t v = kLogHeader;
  for (int r = 0; r < G_; r++) {
    (*cs)[r] = v;
    v += U[3 * r + 1];
  }
  uint8_t vh[kLogHeader];  // the virtual log's header (plan_build_snappy)
  memcpy(vh, hdr, kLogHeader);
  for (int i = 0; i < 8; i++) vh[32 + i] = (uint8_t)((uint64_t)vlen >> (8 * i));
  memset(vh + 64, 0, 4);
  vh[80] = 1;
  memset(vh + 81, 0, 3);
  F_ = make_layout(vh, G_);
  ce_ = ent;
  virt_ = true;
  *vlen_out = vlen;
  *take = true;
  mark("cz_decode");
  return SPARKEY_OK;
}

int Rank::run(const uint8_t* hdr, uint64_t file_len, const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi,
              const sparkey_build_opts& o, uint8_t* d_out, uint64_t out_cap, sparkey_build_stats* st, int rc0) {
  cm_->phase.clear();
  clock_ = now_ms();
  hdr_ = hdr;
  sticky_ = SPARKEY_OK;
  L_ = make_layout(hdr, G_);
  F_ = L_;
  virt_ = false;
  ce_.clear();
  geo_ = make_geo(L_, hdr, o);
  int64_t data_end = L_.data_end;
  memset(st, 0, sizeof(*st));
  st->capacity = (int64_t)geo_.cap;
  st->hash_size = geo_.hash_size;
  st->address_size = geo_.addr_size;
  st->num_puts = L_.num_puts;
  st->num_deletes = L_.num_deletes;
  uint64_t slot_lo = 0, slot_hi = 0;
  const uint64_t ss = (uint64_t)geo_.slot;
  const uint64_t hdr_off = g_ == 0 ? kIndexHeader : 0;
  uint64_t out_len = 0;
  if (!rc0) rc0 = sparkey_shard_begin(pl_, hdr, file_len, d_buf, buf_lo, buf_hi, &o, g_, G_, err_, err_len_);
  if (!rc0) {
    sparkey_shard_slot_range(pl_, g_, &slot_lo, &slot_hi);
    out_len = hdr_off + (slot_hi - slot_lo) * ss;
    if (out_cap < out_len) rc0 = fail(SPARKEY_E_BUFFER, "shard output buffer too small: need " + std::to_string(out_len));
  }
  const int RL = 8 + G_ + 256;  // the verification row
  uint8_t* row = rc0 ? nullptr : cm_->row.ensure((uint64_t)RL * 8);
  if (!rc0 && !row) rc0 = fail(SPARKEY_E_GPU, "hipMalloc failed");

  // ---- 1 entries: speculate, frame, verify by induction from c_0 = 84 ----
  auto uni_entry = [&](int r) {
    return std::min<int64_t>(data_end, kLogHeader + (L_.lo[r] - kLogHeader + L_.uni - 1) / L_.uni * L_.uni);
  };
  int64_t c_g = -1;
  if (!rc0) {
    if (g_ == 0) c_g = kLogHeader;
    else if (L_.small || L_.compression != 0) c_g = data_end;
    else if (L_.uni) c_g = uni_entry(g_);
    else rc0 = sparkey_shard_find_entry(pl_, (uint64_t)L_.lo[g_], (uint64_t)L_.window, s_, &c_g, err_, err_len_);
  }
  // the first checkpoint: every rank's entry and code (a rank that failed so far fails them all)
  std::vector<int64_t> cs(G_);
  if (G_ > 1) {
    std::vector<int64_t> ce;
    int rc = gather_i64({c_g, rc0}, &ce);
    if (rc) return rc;
    std::vector<int64_t> codes(G_);
    for (int r = 0; r < G_; r++) {
      cs[r] = ce[2 * r];
      codes[r] = ce[2 * r + 1];
    }
    rc = fail_together(codes, rc0);
    if (rc) return rc;
  } else {
    if (rc0) return rc0;
    cs[0] = c_g;
  }
  if (L_.compression != 0) {
    bool take = false;
    const int rc = compressed(hdr, file_len, d_buf, buf_lo, buf_hi, o, &cs, &data_end, &take);
    if (rc) return rc;
    if (!take) return gathered(hdr, file_len, d_buf, buf_lo, o, d_out, slot_lo, out_len, st);
  }
  mark("entries");
  entries_.assign(G_, 0);
  valid_.assign(G_, false);
  int64_t last_valid = -1;
  bool have_last = false;
  for (int r = 0; r < G_ && virt_; r++) {  // (the slices of the virtual log: every start is a record start)
    entries_[r] = cs[r];
    valid_[r] = true;
  }
  for (int r = 0; r < G_ && !virt_; r++) {
    const int64_t v = cs[r];
    bool ok = v >= 0 && (r == 0 || (L_.small && v == data_end) || (L_.lo[r] <= v && v <= data_end));
    if (ok && have_last && v < last_valid) ok = false;
    if (ok) {
      entries_[r] = v;
      valid_[r] = true;
    }
    // (sharded.py compares with the previous entry only when it is valid)
    have_last = valid_[r];
    last_valid = v;
  }
  std::vector<bool> todo(G_);
  for (int r = 0; r < G_; r++) todo[r] = valid_[r];
  std::vector<int64_t> framed;
  int rounds = 0;
  int rc = SPARKEY_OK;
  if (!todo[g_]) {  // (re-framed from the previous rank's exit in a later round)
    std::vector<int64_t> init(RL, 0);
    for (int i = 0; i < 7; i++) init[i] = -1;
    rc = gpu(hipMemcpyAsync(row, init.data(), (uint64_t)RL * 8, hipMemcpyHostToDevice, s_), "H2D");
    if (rc) return rc;
  }
  uint8_t* send = nullptr;
  uint64_t send_cap = 0;
  std::vector<int64_t> R((size_t)G_ * RL);
  const bool sync_frame = sk::knob_on(sk::Knob::ShardSyncFrame);  // (tests: every attempt retried)
  // a rank whose framing step fails posts a row with retry = -2 and its code (every rank then fails)
  auto post_failure = [&](int code) -> int {
    std::vector<int64_t> f(RL, 0);
    f[5] = code;
    f[6] = -1;
    f[7] = -2;
    const int e = gpu(hipMemcpyAsync(row, f.data(), (uint64_t)RL * 8, hipMemcpyHostToDevice, s_), "H2D");
    return e ? e : gpu(hipStreamSynchronize(s_), "sync");
  };
  int own = SPARKEY_OK;  // this rank's failed step, posted in its row
  for (;;) {
    rounds++;
    if (todo[g_] && !own) {
      const int64_t fend = fe(g_);
      if (std::find(framed.begin(), framed.end(), entries_[g_]) == framed.end()) {
        framed.push_back(entries_[g_]);
        uint64_t cap = 1ull << 62;  // (one rank: the entries stay in place, bounded by the plan's workspace)
        if (G_ > 1) {
          const int64_t c = sparkey_shard_frame_capacity(pl_, entries_[g_], fend);
          if (c < 0) own = fail(SPARKEY_E_ARG, "bad shard frame range");
          cap = (uint64_t)std::max<int64_t>(0, c);
        }
        if (sync_frame) cap = 0;
        send = nullptr;
        send_cap = cap;
        if (G_ > 1 && !own) {
          send = cm_->send.ensure(std::max<uint64_t>(1, cap) * kEntryBytes);
          if (!send) own = fail(SPARKEY_E_GPU, "hipMalloc failed");
        }
        if (!own) own = sparkey_shard_frame_bin_async(pl_, entries_[g_], fend, send, cap, (int64_t*)row, s_, err_, err_len_);
      } else {  // the speculative attempt did not hold: frame with every retry, then bin
        sparkey_shard_frame_result fr;
        memset(&fr, 0, sizeof(fr));
        own = sparkey_shard_frame(pl_, entries_[g_], fend, s_, &fr, err_, err_len_);
        const uint64_t n_mine = fr.rc ? 0 : (uint64_t)fr.num_records;
        send = nullptr;
        send_cap = 0;
        if (G_ > 1 && !own) {
          send = cm_->send.ensure(std::max<uint64_t>(1, n_mine) * kEntryBytes);
          if (!send) own = fail(SPARKEY_E_GPU, "hipMalloc failed");
          send_cap = cm_->send.cap / kEntryBytes;
        }
        const int64_t sc[8] = {entries_[g_], fend, fr.exit, fr.num_records, fr.num_deletes, fr.rc, fr.err_pos, 0};
        if (!own) own = sparkey_shard_bin_row(pl_, send, send_cap, n_mine, sc, (int64_t*)row, s_, err_, err_len_);
      }
    }
    if (own) {
      rc = post_failure(own);
      if (rc) return rc;
    }
    rc = all_gather(row, cm_->rows, (uint64_t)RL * 8);
    if (!rc) rc = to_host(R.data(), cm_->rows.p, (uint64_t)G_ * RL * 8);
    if (rc) return rc;
    {
      // a failed rank: retry -2 with its code (post_failure), or -1 when its row could not leave its
      // device (HostColl's all-ones row); valid rows carry retry 0 or 1
      std::vector<int64_t> codes(G_, 0);
      for (int r = 0; r < G_; r++)
        if (R[(size_t)r * RL + 7] < 0)
          codes[r] = R[(size_t)r * RL + 7] == -2 && R[(size_t)r * RL + 5] ? R[(size_t)r * RL + 5] : SPARKEY_E_GPU;
      rc = fail_together(codes, own);
      if (rc) return rc;
    }
    bool any = false;
    for (int r = 0; r < G_; r++) {
      todo[r] = R[(size_t)r * RL + 7] != 0;  // speculative attempts to redo, the entries unchanged
      any = any || todo[r];
    }
    if (any) continue;
    bool done = true;
    for (int r = 0; r < G_; r++) {
      const int64_t* x = &R[(size_t)r * RL];
      if (x[5]) return fail((int)x[5], std::string(code_text((int)x[5])) + " (log offset " + std::to_string(x[6]) + ")");
      if (r == G_ - 1) break;
      const int64_t nxt = std::min<int64_t>(x[2], data_end);
      if (R[(size_t)(r + 1) * RL] == nxt && valid_[r + 1] && entries_[r + 1] == nxt) continue;
      if (virt_) return gathered(hdr, file_len, d_buf, buf_lo, o, d_out, slot_lo, out_len, st);  // (not a slice end)
      entries_[r + 1] = nxt;  // rank r + 1 re-frames from the verified exit
      valid_[r + 1] = true;
      std::fill(todo.begin(), todo.end(), false);
      todo[r + 1] = true;
      done = false;
      break;
    }
    if (done) break;
  }
  int64_t n_total = 0, n_deletes = 0;
  for (int r = 0; r < G_; r++) {
    n_total += R[(size_t)r * RL + 3];
    n_deletes += R[(size_t)r * RL + 4];
  }
  st->num_records = n_total;
  mark("frame+verify");
  if (n_total - n_deletes >= (int64_t)geo_.cap)  // the PUT records may fill the table: one lane's replay
    return gathered(hdr, file_len, d_buf, buf_lo, o, d_out, slot_lo, out_len, st);

  // ---- 2 exchange: every PUT entry to the owner of its slot range ----
  std::vector<uint64_t> sb(G_), rb(G_);
  uint64_t n_recv = 0;
  for (int r = 0; r < G_; r++) {
    sb[r] = (uint64_t)R[(size_t)g_ * RL + 8 + r] * kEntryBytes;
    rb[r] = (uint64_t)R[(size_t)r * RL + 8 + g_] * kEntryBytes;
    n_recv += (uint64_t)R[(size_t)r * RL + 8 + g_];
  }
  // every buffer the exchange and the placement need, then one checkpoint: a rank that cannot
  // allocate them fails every rank here instead of leaving the others inside a collective
  const int FL = 4 + 4 * kSpillInline;
  uint64_t spill_cap = 4096;
  uint8_t* rv = nullptr;
  if (G_ > 1) {
    if (!send) send = cm_->send.ensure(16);
    rv = cm_->recv.ensure(std::max<uint64_t>(1, n_recv) * kEntryBytes);
  }
  uint8_t* spill = cm_->spill.ensure(spill_cap * kSpillBytes);
  uint8_t* flags = cm_->flags.ensure((uint64_t)FL * 8);
  uint8_t* fun = cm_->fun.ensure(16);
  uint8_t* fin = cm_->fin.ensure(12 * 8);
  const bool have = (G_ == 1 || (send && rv)) && spill && flags && fun && fin && cm_->funs.ensure(16ull * G_) &&
                    cm_->frows.ensure((uint64_t)FL * 8 * G_) && cm_->fins.ensure(12ull * 8 * G_);
  int cz_rc = SPARKEY_OK;  // compressed log: the entries' virtual offsets -> the compressed log's addresses
  if (have && virt_) {
    uint64_t n_send = 0;
    for (int r = 0; r < G_; r++) n_send += (uint64_t)R[(size_t)g_ * RL + 8 + r];
    cz_rc = sk_cz_to_real(pl_, send, n_send, kEntryBytes, s_, err_, err_len_);
  }
  rc = agree(have ? cz_rc : fail(SPARKEY_E_GPU, "hipMalloc failed"));
  if (rc) return rc;
  const uint8_t* recv = nullptr;
  // A collective that fails on this rank from here to the finish rows does not end its part: it skips
  // its device steps, posts neutral rows and its code, and joins every collective up to the finish-row
  // all_gather, where every rank fails together (its peers would otherwise wait in a collective it
  // never enters).  xrc: this rank's failure so far.
  int xrc = SPARKEY_OK;
  if (G_ > 1) {
    std::string why;
    xrc = coll_rc(c_->all_to_all(send, sb.data(), rv, rb.data(), s_, &why), why);
    recv = rv;
  }
  mark("all_to_all");

  // ---- 3 placement and stats on the device; the host sees one row per rank at the end ----
  // A rank whose step fails posts neutral rows (the identity carry function, no spilled slots) so
  // that the others' steps stay in bounds, and its code in its finish row: every rank then fails.
  std::vector<int64_t> F((size_t)G_ * 12);
  bool fixed = true;
  for (;;) {
    const int64_t* digits = (const int64_t*)cm_->rows.p + (8 + G_);  // &rows[0][8 + G]
    // (posting a neutral row can itself fail; the rank then still takes part in the collectives up to
    //  the finish rows, so that no peer waits in one it never enters, and returns that failure there)
    int post_rc = SPARKEY_OK;
    int lrc = xrc ? xrc
                  : sparkey_shard_summarize_dev(pl_, recv, n_recv, digits, RL, fixed ? 1 : 0, (int64_t*)fun, s_, err_, err_len_);
    if (lrc) post_rc = gpu(hipMemsetAsync(fun, 0, 16, s_), "memset");
    if (const int crc = all_gather(fun, cm_->funs, 16)) lrc = lrc ? lrc : crc;  // (joins the rest regardless)
    if (!lrc)
      lrc = sparkey_shard_place_dev(pl_, (const int64_t*)cm_->funs.p, d_out + hdr_off, spill, spill_cap, (int64_t*)flags,
                                    kSpillInline, s_, err_, err_len_);
    if (lrc && !post_rc) post_rc = gpu(hipMemsetAsync(flags, 0, (uint64_t)FL * 8, s_), "memset");
    if (const int crc = all_gather(flags, cm_->frows, (uint64_t)FL * 8)) lrc = lrc ? lrc : crc;
    if (!lrc) lrc = sparkey_shard_finish_dev(pl_, (const int64_t*)cm_->frows.p, FL, kSpillInline, (int64_t*)fin, s_, err_, err_len_);
    if (lrc) {
      int64_t f[12] = {0};
      f[3] = lrc;  // (a negative "aborted" flag: this rank failed)
      const int hrc = gpu(hipMemcpyAsync(fin, f, sizeof(f), hipMemcpyHostToDevice, s_), "H2D");
      if (!post_rc) post_rc = hrc;
    }
    rc = all_gather(fin, cm_->fins, 12 * 8);
    if (!rc) rc = post_rc;
    if (!rc) rc = to_host(F.data(), cm_->fins.p, (uint64_t)G_ * 12 * 8);
    if (rc) return rc;
    std::vector<int64_t> codes(G_, 0);
    for (int r = 0; r < G_; r++) codes[r] = F[(size_t)r * 12 + 3] < 0 ? F[(size_t)r * 12 + 3] : 0;
    rc = fail_together(codes, lrc);
    if (rc) return rc;
    bool aborted = false;
    for (int r = 0; r < G_; r++) aborted = aborted || F[(size_t)r * 12 + 3] != 0;
    if (aborted && fixed) {  // a bucket outgrew its fixed region on some rank: dense runs
      fixed = false;
      continue;
    }
    if (aborted) return fail(SPARKEY_E_GPU, "sharded placement aborted");
    if (g_ == 0) rc = sparkey_shard_header_dev(pl_, (const int64_t*)cm_->fins.p, 12, n_total, d_out, s_, err_, err_len_);
    if (rc) return rc;
    break;
  }
  mark("place");
  int64_t n_pairs_all = 0, max_spill = 0;
  bool noncanon = false;
  for (int r = 0; r < G_; r++) {

    max_spill = std::max(max_spill, F[(size_t)r * 12]);
    n_pairs_all += F[(size_t)r * 12 + 1];
    noncanon = noncanon || F[(size_t)r * 12 + 2] != 0;
  }
  // DELETE records, or equal-hash pairs this step cannot prove distinct: the exact path
  bool is_exact = n_deletes > 0 || noncanon;
  if (!is_exact && n_pairs_all > 0) {
    rc = pairs_share_a_key(F[(size_t)g_ * 12 + 1], &is_exact);
    if (rc) return rc;
  }
  bool host_header = is_exact;
  std::vector<int64_t> bnd((size_t)G_ * 8);
  for (int r = 0; r < G_; r++)
    for (int k = 0; k < 8; k++) bnd[(size_t)r * 8 + k] = F[(size_t)r * 12 + 4 + k];
  if (max_spill > kSpillInline) {  // more spilled slots than the rows carry: exchange them all
    host_header = true;
    const uint64_t n_spill = (uint64_t)F[(size_t)g_ * 12];
    // (a failure is noted and the rank joins the collectives up to the next checkpoint: gather_var's
    //  count gather, or range_stats' / the exact path's first gather)
    uint64_t n_send_spill = n_spill;
    if (n_spill > spill_cap) {
      spill_cap = n_spill;
      spill = cm_->spill.ensure(spill_cap * kSpillBytes);
      if (!spill) note(fail(SPARKEY_E_GPU, "hipMalloc failed"));
      if (ok()) note(sparkey_shard_place_dev(pl_, (const int64_t*)cm_->funs.p, d_out + hdr_off, spill, spill_cap,
                                             (int64_t*)flags, kSpillInline, s_, err_, err_len_));
    }
    if (!ok()) n_send_spill = 0;
    uint64_t total = 0;
    rc = gather_var(spill, n_send_spill * kSpillBytes, cm_->var_out, &total);
    if (rc) return rc;
    note(sparkey_shard_apply_spill(pl_, cm_->var_out.p, total / kSpillBytes, s_, err_, err_len_));
    if (!is_exact) rc = range_stats(slot_lo, slot_hi, &bnd);
    if (rc) return rc;
  }
  mark("spill");
  if (is_exact) {  // the ring splits at the slots the PUT placement left empty (now complete on every rank)
    bool done = false;
    rc = exact(d_out, hdr_off, R[(size_t)g_ * RL + 3], o, slot_lo, slot_hi, &done, st);
    if (rc) return rc;
    mark("exact");
    if (done) return SPARKEY_OK;
    return gathered(hdr, file_len, d_buf, buf_lo, o, d_out, slot_lo, out_len, st);
  }
  // ---- 4 stats ----
  int64_t mx, col, tot;
  combine_stats(bnd, 8, 0, &mx, &col, &tot);
  if (g_ == 0 && host_header) {
    uint8_t h[kIndexHeader];
    rc = sparkey_index_header(hdr, &o, n_total, 0, mx, col, tot, h, err_, err_len_);
    if (!rc) rc = gpu(hipMemcpyAsync(d_out, h, kIndexHeader, hipMemcpyHostToDevice, s_), "H2D");
    if (rc) return rc;
  }
  rc = gpu(hipStreamSynchronize(s_), "sync");
  if (rc) return rc;
  st->num_entries = n_total;
  st->garbage_size = 0;
  st->max_displacement = mx;
  st->hash_collisions = col;
  st->total_displacement = tot;
  st->placement_path = 0;
  st->sharded = 1;
  mark("stats");
  (void)rounds;
  return SPARKEY_OK;
}

}  // namespace

// One rank's sparkey_shard_build; rc0 != 0 (its log range could not be loaded, err holds why): the rank
// still meets the others at the first checkpoint so that they all return the error.
int shard_build_rank(sparkey_plan* plan, sparkey_shard_comm* comm, const uint8_t* log_header, uint64_t file_len,
                     const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi, const sparkey_build_opts* opts,
                     uint8_t* d_out, uint64_t out_cap, void* stream, sparkey_build_stats* stats_out, int rc0, char* err,
                     size_t err_len) {
  if (hipSetDevice(comm->device) != hipSuccess && !rc0) {
    set_err(err, err_len, "hipSetDevice failed");
    rc0 = SPARKEY_E_GPU;
  }
  hipStream_t s = (hipStream_t)stream;
  hipStream_t own = nullptr;
  if (!s) {
    if (hipStreamCreateWithFlags(&own, hipStreamNonBlocking) != hipSuccess) {
      set_err(err, err_len, "hipStreamCreate failed");
      own = nullptr;
      if (!rc0) rc0 = SPARKEY_E_GPU;
    }
    s = own;
  }
  sparkey_build_stats st;
  memset(&st, 0, sizeof(st));
  const double t0 = now_ms();
  Rank rank(plan, comm, s, err, err_len);
  int rc = rank.run(log_header, file_len, d_buf, buf_lo, buf_hi, *opts, d_out, out_cap, &st, rc0);
  if (rc) comm->coll->abort();  // (thread transport: release the other ranks)
  if (s) (void)hipStreamSynchronize(s);
  if (own) (void)hipStreamDestroy(own);
  st.device_ms = now_ms() - t0;
  if (stats_out) *stats_out = st;
  return rc;
}

// ---------------------------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------------------------
extern "C" {

int sparkey_shard_comm_unique_id(uint8_t* id128, char* err, size_t err_len) {
  std::string why;
  const RcclApi* api = rccl_api(&why);
  if (!api) {
    set_err(err, err_len, why);
    return SPARKEY_E_GPU;
  }
  ncclUniqueId id;
  if (api->GetUniqueId(&id) != ncclSuccess) {
    set_err(err, err_len, "ncclGetUniqueId failed");
    return SPARKEY_E_GPU;
  }
  memcpy(id128, &id, sizeof(id));
  return SPARKEY_OK;
}

int sparkey_shard_comm_create(sparkey_shard_comm** out, const uint8_t* id128, int32_t rank, int32_t world,
                              int32_t device, char* err, size_t err_len) {
  if (!out || !id128 || world < 1 || rank < 0 || rank >= world) {
    set_err(err, err_len, "bad communicator arguments");
    return SPARKEY_E_ARG;
  }
  std::string why;
  const RcclApi* api = rccl_api(&why);
  if (!api) {
    set_err(err, err_len, why);
    return SPARKEY_E_GPU;
  }
  if (hipSetDevice(device) != hipSuccess) {
    set_err(err, err_len, "hipSetDevice failed");
    return SPARKEY_E_GPU;
  }
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t r = api->CommInitRank(&c, world, id, rank);
  if (r != ncclSuccess) {
    set_err(err, err_len, std::string("ncclCommInitRank: ") + api->GetErrorString(r));
    return SPARKEY_E_GPU;
  }
  auto* cm = new sparkey_shard_comm();
  cm->coll.reset(new RcclColl(api, c, rank, world));
  cm->device = device;
  *out = cm;
  return SPARKEY_OK;
}

int sparkey_shard_comm_create_host(sparkey_shard_comm** out, const sparkey_shard_transport* t, int32_t rank,
                                   int32_t world, int32_t device, char* err, size_t err_len) {
  if (!out || !t || !t->all_gather || !t->all_to_all || world < 1 || rank < 0 || rank >= world) {
    set_err(err, err_len, "bad communicator arguments");
    return SPARKEY_E_ARG;
  }
  if (hipSetDevice(device) != hipSuccess) {
    set_err(err, err_len, "hipSetDevice failed");
    return SPARKEY_E_GPU;
  }
  auto* cm = new sparkey_shard_comm();
  cm->coll.reset(new HostColl(*t, rank, world));
  cm->device = device;
  *out = cm;
  return SPARKEY_OK;
}

void sparkey_shard_comm_destroy(sparkey_shard_comm* cm) {
  if (!cm) return;
  (void)hipSetDevice(cm->device);
  delete cm;
}

int sparkey_shard_geometry(const uint8_t* log_header, uint64_t file_len, const sparkey_build_opts* opts, int32_t rank,
                           int32_t world, uint64_t* buf_lo, uint64_t* buf_hi, uint64_t* out_off, uint64_t* out_len,
                           char* err, size_t err_len) {
  if (!log_header || !opts || world < 1 || rank < 0 || rank >= world) {
    set_err(err, err_len, "bad shard arguments");
    return SPARKEY_E_ARG;
  }
  const int64_t isz = sparkey_index_size(log_header, kLogHeader, opts);
  if (isz < 0) {
    set_err(err, err_len, sparkey_strerror((int)isz));
    return (int)isz;
  }
  const Layout L = make_layout(log_header, world);
  const Geo G = make_geo(L, log_header, *opts);
  buffer_range(L, file_len, rank, buf_lo, buf_hi);
  uint64_t s0, s1;
  shard_slot_split(G.cap, world, rank, &s0, &s1);
  *out_off = rank == 0 ? 0 : kIndexHeader + s0 * G.slot;
  *out_len = (rank == 0 ? kIndexHeader : 0) + (s1 - s0) * G.slot;
  return SPARKEY_OK;
}

int sparkey_shard_build(sparkey_plan* plan, sparkey_shard_comm* comm, const uint8_t* log_header, uint64_t file_len,
                        const uint8_t* d_buf, uint64_t buf_lo, uint64_t buf_hi, const sparkey_build_opts* opts,
                        uint8_t* d_out, uint64_t out_cap, void* stream, sparkey_build_stats* stats_out, char* err,
                        size_t err_len) {
  if (!plan || !comm || !log_header || !opts || !d_out) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  return shard_build_rank(plan, comm, log_header, file_len, d_buf, buf_lo, buf_hi, opts, d_out, out_cap, stream,
                          stats_out, SPARKEY_OK, err, err_len);
}

int32_t sparkey_shard_phase_count(const sparkey_shard_comm* comm) { return comm ? (int32_t)comm->phase.size() : 0; }
const char* sparkey_shard_phase_name(const sparkey_shard_comm* comm, int32_t i) {
  return comm && i >= 0 && i < (int32_t)comm->phase.size() ? comm->phase[i].first.c_str() : "";
}
double sparkey_shard_phase_ms(const sparkey_shard_comm* comm, int32_t i) {
  return comm && i >= 0 && i < (int32_t)comm->phase.size() ? comm->phase[i].second : 0.0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// N ranks as threads of this process (sparkey_build_index_mem / _file with opts.num_gpus > 1)
// ---------------------------------------------------------------------------------------------
namespace {

struct Group {  // communicators for one device list, kept across calls
  std::vector<int> devices;
  bool threads = false;
  std::vector<sparkey_shard_comm*> comms;
  std::mutex mu;  // one build at a time per group
  ~Group() {
    for (auto* c : comms) sparkey_shard_comm_destroy(c);
  }
};

// Groups are shared: a build holds its group for its whole length, so sparkey_release_cached_resources
// (which empties the map) never frees a group under a running build, and a failed group is dropped
// from the map and freed when its last build ends.
std::mutex g_groups_mu;
std::map<std::pair<std::vector<int>, bool>, std::shared_ptr<Group>> g_groups;
std::vector<std::vector<std::pair<std::string, double>>> g_multi_phases;  // per rank, the last build's

std::shared_ptr<Group> get_group(const std::vector<int>& devs, bool threads, std::string* why) {
  std::lock_guard<std::mutex> l(g_groups_mu);
  auto key = std::make_pair(devs, threads);
  auto it = g_groups.find(key);
  if (it != g_groups.end()) return it->second;
  auto gr = std::make_shared<Group>();
  gr->devices = devs;
  gr->threads = threads;
  const int n = (int)devs.size();
  if (threads) {
    auto sh = std::make_shared<ThreadShared>(n);
    for (int r = 0; r < n; r++) {
      auto* cm = new sparkey_shard_comm();
      cm->coll.reset(new ThreadColl(sh, r));
      cm->device = devs[r];
      gr->comms.push_back(cm);
    }
  } else {
    const RcclApi* api = rccl_api(why);
    if (!api) return nullptr;
    std::vector<ncclComm_t> cs(n);
    const ncclResult_t r = api->CommInitAll(cs.data(), n, devs.data());
    if (r != ncclSuccess) {
      *why = std::string("ncclCommInitAll: ") + api->GetErrorString(r);
      return nullptr;
    }
    for (int q = 0; q < n; q++) {
      auto* cm = new sparkey_shard_comm();
      cm->coll.reset(new RcclColl(api, cs[q], q, n));
      cm->device = devs[q];
      gr->comms.push_back(cm);
    }
  }
  g_groups[key] = gr;
  return gr;
}

}  // namespace

int shard_devices(const sparkey_build_opts& o, std::vector<int>* devs, bool* threads, char* err, size_t err_len) {
  const int n = o.num_gpus;
  const int64_t tr = sk::knob(sk::Knob::ShardTransport);  // (tests: 1 threads, 2 threads on opts.device)
  *threads = tr == 1 || tr == 2;
  const bool same = tr == 2;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
  devs->clear();
  for (int r = 0; r < n; r++) devs->push_back(same ? o.device : o.device + r);
  for (int d : *devs)
    if (d < 0 || d >= count) {
      set_err(err, err_len, "num_gpus = " + std::to_string(n) + " from device " + std::to_string(o.device) + " needs " +
                                "devices this process does not see (" + std::to_string(count) + " visible)");
      return SPARKEY_E_ARG;
    }
  return SPARKEY_OK;
}

int shard_run_threads(const sparkey_build_opts& o, const ShardRankFn& fn, char* err, size_t err_len) {
  std::vector<int> devs;
  bool threads = false;
  int rc = shard_devices(o, &devs, &threads, err, err_len);
  if (rc) return rc;
  std::string why;
  const std::shared_ptr<Group> gr = get_group(devs, threads, &why);
  if (!gr) {
    set_err(err, err_len, why);
    return SPARKEY_E_GPU;
  }
  std::lock_guard<std::mutex> l(gr->mu);
  const int n = (int)devs.size();
  const bool same = n > 1 && devs[0] == devs[1];  // every rank on one device (tests)
  std::vector<int> rcs(n, SPARKEY_OK);
  std::vector<std::string> msgs(n);
  std::vector<std::thread> ts;
  for (int r = 0; r < n; r++)
    ts.emplace_back([&, r] {
      char e[512] = {0};
      (void)hipSetDevice(devs[r]);
      rcs[r] = fn(r, n, devs[r], gr->comms[r], same, e, sizeof(e));
      msgs[r] = e;
      if (rcs[r]) gr->comms[r]->coll->abort();
    });
  for (auto& t : ts) t.join();
  {
    std::lock_guard<std::mutex> g2(g_groups_mu);
    g_multi_phases.resize(n);
    for (int r = 0; r < n; r++) g_multi_phases[r] = gr->comms[r]->phase;
  }
  rc = SPARKEY_OK;
  for (int r = 0; r < n && !rc; r++)  // the first rank's own error (not "another rank failed")
    if (rcs[r] && msgs[r].find("another rank") == std::string::npos) {
      set_err(err, err_len, msgs[r]);
      rc = rcs[r];
    }
  for (int r = 0; r < n && !rc; r++)
    if (rcs[r]) {
      set_err(err, err_len, msgs[r]);
      rc = rcs[r];
    }
  if (rc) {  // a failed group is not reused (a thread group's barrier is aborted; fresh communicators)
    std::lock_guard<std::mutex> g2(g_groups_mu);
    auto it = g_groups.find(std::make_pair(devs, threads));
    if (it != g_groups.end() && it->second == gr) g_groups.erase(it);
  }
  return rc;
}

extern "C" {
int32_t sparkey_multi_phase_count(int32_t rank) {
  std::lock_guard<std::mutex> l(g_groups_mu);
  return rank >= 0 && rank < (int32_t)g_multi_phases.size() ? (int32_t)g_multi_phases[rank].size() : 0;
}
const char* sparkey_multi_phase_name(int32_t rank, int32_t i) {
  thread_local std::string name;  // (a copy: a concurrent build may replace the phases)
  std::lock_guard<std::mutex> l(g_groups_mu);
  if (rank < 0 || rank >= (int32_t)g_multi_phases.size() || i < 0 || i >= (int32_t)g_multi_phases[rank].size()) return "";
  name = g_multi_phases[rank][i].first;
  return name.c_str();
}
double sparkey_multi_phase_ms(int32_t rank, int32_t i) {
  std::lock_guard<std::mutex> l(g_groups_mu);
  if (rank < 0 || rank >= (int32_t)g_multi_phases.size() || i < 0 || i >= (int32_t)g_multi_phases[rank].size()) return 0.0;
  return g_multi_phases[rank][i].second;
}
}  // extern "C"

void shard_release_groups() {
  std::map<std::pair<std::vector<int>, bool>, std::shared_ptr<Group>> old;
  {
    std::lock_guard<std::mutex> l(g_groups_mu);
    old.swap(g_groups);
  }
  // (each group is freed here, or by the build still holding it when that build ends)
}
