// file_build.cpp -- the drop-in entry points that start and end in host memory:
//   sparkey_build_index_file  log file in, .spi file out (what the JNI shim calls in place of
//                             IndexHash.createNew, IndexHash.java:131-167)
//   sparkey_build_index_mem   host bytes in, host bytes out
// Both run over the device-resident API (sparkey_plan_build_device) with a per-device context that
// is kept across calls: the plan's workspace, the device log and index buffers, a ring of pinned
// staging slots and a small reader/writer thread pool.  A log is read straight into the pinned
// slots by the pool while earlier slots are copied to the device, and the .spi comes back through
// the same slots while the previous slot is written out, so the file I/O overlaps PCIe both ways.
// The file is created only after the build succeeded, header then slots, then fsync when asked for
// (FileFlushingData.close, FileFlushingData.java:20-34); a failed write removes it.  Contexts are
// released by sparkey_release_cached_resources(), or never kept with SPARKEY_FILE_CACHE=0.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sparkey_gpu.h"
#include "knobs.hpp"
#include "shard_host.hpp"

using sk::Knob;
using sk::knob;

// Phases of the calling thread's last sparkey_build_index_file (sparkey_file_last_phases).
thread_local double t_file_phase[5] = {0, 0, 0, 0, 0};

// LogHeader.read's checks with the file's length (sparkey_gpu.cpp), message into err.
int sk_check_log_header(const uint8_t* b, uint64_t hdr_len, uint64_t file_len, char* err, size_t err_len);

namespace {

constexpr int kSlots = 4;                      // pinned staging ring
constexpr uint64_t kSlotBytes = 32ull << 20;   // bytes per slot (one H2D / D2H copy each)
constexpr uint64_t kPieceBytes = 4ull << 20;   // bytes per pool task inside a slot

void set_err(char* err, size_t err_len, const std::string& msg) {
  if (err && err_len > 0) snprintf(err, err_len, "%s", msg.c_str());
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Fixed threads; run(n, fn) calls fn(0..n-1) on the pool and the calling thread and returns when
// every call has returned.  Tasks are handed out under the lock, so an index always belongs to the
// job in progress.
class WorkerPool {
 public:
  explicit WorkerPool(int nthreads) {
    for (int i = 0; i < nthreads; i++) threads_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  void run(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      left_ = n;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [this] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  bool take(int* i, const std::function<void(int)>** f) {
    std::lock_guard<std::mutex> g(mu_);
    if (!fn_ || next_ >= n_) return false;
    *i = next_++;
    *f = fn_;
    return true;
  }
  void drain() {
    int i;
    const std::function<void(int)>* f;
    while (take(&i, &f)) {
      (*f)(i);
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || (fn_ != nullptr && next_ < n_); });
        if (stop_) return;
      }
      drain();
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, left_ = 0;
  bool stop_ = false;
};

struct FileCtx {
  int device = 0;
  bool cached = false;
  std::mutex mu;
  sparkey_plan* plan = nullptr;
  hipStream_t s = nullptr;
  uint8_t* d_log = nullptr;
  uint64_t c_log = 0;
  uint8_t* d_out = nullptr;
  uint64_t c_out = 0;
  uint8_t* slot[kSlots] = {};
  hipEvent_t ev[kSlots] = {};
  WorkerPool* pool = nullptr;

  ~FileCtx() {
    (void)hipSetDevice(device);
    if (s) (void)hipStreamSynchronize(s);
    delete pool;
    for (int i = 0; i < kSlots; i++) {
      if (slot[i]) (void)hipHostFree(slot[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
    if (d_log) (void)hipFree(d_log);
    if (d_out) (void)hipFree(d_out);
    if (plan) sparkey_plan_destroy(plan);
    if (s) (void)hipStreamDestroy(s);
  }

  int init(int dev, char* err, size_t err_len) {
    device = dev;
    int rc = sparkey_plan_create(&plan, dev, 0, 0, err, err_len);
    if (rc) return rc;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      set_err(err, err_len, "hipStreamCreate failed");
      return SPARKEY_E_GPU;
    }
    for (int i = 0; i < kSlots; i++) {
      if (hipHostMalloc((void**)&slot[i], kSlotBytes, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
        set_err(err, err_len, "pinned staging allocation failed");
        return SPARKEY_E_GPU;
      }
    }
    // the CPUs this process may run on (a container's share, not the machine's), at most 16
    cpu_set_t cs;
    unsigned hc = 0;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) hc = (unsigned)CPU_COUNT(&cs);
    if (!hc) hc = std::thread::hardware_concurrency();
    int nt = (int)std::min<unsigned>(16u, hc ? hc : 4u) - 1;  // the calling thread works too
    if (sk::knob_set(sk::Knob::FileThreads)) nt = (int)std::max<int64_t>(0, sk::knob(sk::Knob::FileThreads) - 1);
    pool = new WorkerPool(std::max(0, nt));
    return SPARKEY_OK;
  }

  int reserve(uint64_t log_bytes, uint64_t out_bytes, char* err, size_t err_len) {
    auto grow = [&](uint8_t** p, uint64_t& have, uint64_t want) -> bool {
      want = std::max<uint64_t>(want, 256);
      if (*p && have >= want) return true;
      if (*p) (void)hipFree(*p);
      *p = nullptr;
      have = 0;
      if (hipMalloc((void**)p, want) != hipSuccess) return false;
      have = want;
      return true;
    };
    if (!grow(&d_log, c_log, log_bytes) || !grow(&d_out, c_out, out_bytes)) {
      set_err(err, err_len, "hipMalloc of the log / index buffers failed");
      return SPARKEY_E_GPU;
    }
    return SPARKEY_OK;
  }
};

std::mutex g_mu;
std::map<int, FileCtx*> g_cache;

// A context for `device`, locked: the cached one when it is free, else a private one that the
// caller releases (so concurrent calls for different writers never share a context).
FileCtx* acquire_ctx(int device, char* err, size_t err_len, int* rc) {
  const char* env = getenv("SPARKEY_FILE_CACHE");
  const bool use_cache = !(env && env[0] == '0');
  *rc = SPARKEY_OK;
  if (use_cache) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_cache.find(device);
    if (it != g_cache.end() && it->second->mu.try_lock()) return it->second;
    if (it == g_cache.end()) {
      FileCtx* c = new FileCtx();
      *rc = c->init(device, err, err_len);
      if (*rc) {
        delete c;
        return nullptr;
      }
      c->cached = true;
      c->mu.lock();
      g_cache[device] = c;
      return c;
    }
  }
  FileCtx* c = new FileCtx();
  *rc = c->init(device, err, err_len);
  if (*rc) {
    delete c;
    return nullptr;
  }
  c->mu.lock();
  return c;
}

void release_ctx(FileCtx* c) {
  if (!c) return;
  if (c->cached) {
    c->mu.unlock();
  } else {
    c->mu.unlock();
    delete c;
  }
}

// Runs fn(slot, offset, bytes) for every kSlotBytes piece of [0, total) in order, with the slot of
// piece i free again (its previous copy done) before fn runs on it.  fn returns an error code.
template <class Fn>
int for_each_slot_piece(FileCtx* c, uint64_t total, Fn&& fn) {
  const uint64_t n = (total + kSlotBytes - 1) / kSlotBytes;
  for (uint64_t i = 0; i < n; i++) {
    const int k = (int)(i % kSlots);
    if (i >= (uint64_t)kSlots && hipEventSynchronize(c->ev[k]) != hipSuccess) return SPARKEY_E_GPU;
    const uint64_t off = i * kSlotBytes;
    const int rc = fn(k, off, std::min(kSlotBytes, total - off));
    if (rc) return rc;
  }
  return SPARKEY_OK;
}

// [off, off + len) of fd into buf by the pool, kPieceBytes per task.
// The first failure of a pool task: its errno, or kShortRead when the file ended early (it shrank
// after fstat).  errno is per thread, so the failing task records it for the caller's message.
constexpr int kShortRead = -1;

std::string io_error(int e) { return e == kShortRead ? std::string("the log file ended early (truncated)") : strerror(e); }

bool pool_pread(FileCtx* c, int fd, uint8_t* buf, uint64_t off, uint64_t len, int* err_no) {
  std::atomic<int> fail{0};
  const int ntask = (int)((len + kPieceBytes - 1) / kPieceBytes);
  c->pool->run(ntask, [&](int t) {
    uint64_t a = (uint64_t)t * kPieceBytes;
    const uint64_t b = std::min(len, a + kPieceBytes);
    while (a < b) {
      const ssize_t r = pread(fd, buf + a, (size_t)(b - a), (off_t)(off + a));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        int expect = 0;
        fail.compare_exchange_strong(expect, r == 0 ? kShortRead : errno);
        return;
      }
      a += (uint64_t)r;
    }
  });
  *err_no = fail.load();
  return *err_no == 0;
}

// Buffered writes to one file serialize on its inode lock: on the GPU box (overlayfs) one thread
// writes a new 208 MB file at 8.5 GB/s and 2-32 threads at 7.0-8.0 (tools/io_probe.c,
// DESIGN.md §5), so the index goes out from the calling thread unless the file_write_threads switch > 1.
int write_threads() { return (int)std::max<int64_t>(1, sk::knob(sk::Knob::FileWriteThreads)); }

bool pool_pwrite(FileCtx* c, int fd, const uint8_t* buf, uint64_t off, uint64_t len, int* err_no) {
  std::atomic<int> fail{0};
  const uint64_t piece = write_threads() > 1 ? kPieceBytes : std::max<uint64_t>(len, 1);
  const int ntask = (int)((len + piece - 1) / piece);
  auto task = [&](int t) {
    uint64_t a = (uint64_t)t * piece;
    const uint64_t b = std::min(len, a + piece);
    while (a < b) {
      const ssize_t w = pwrite(fd, buf + a, (size_t)(b - a), (off_t)(off + a));
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) {
        int expect = 0;
        fail.compare_exchange_strong(expect, w == 0 ? ENOSPC : errno);
        return;
      }
      a += (uint64_t)w;
    }
  };
  if (ntask == 1) task(0);
  else c->pool->run(ntask, task);
  *err_no = fail.load();
  return *err_no == 0;
}

// d_out[0, isz) -> fd at file offset file_off, through the staging ring: the copy of piece i + 1 runs
// while piece i is written.
int write_index(FileCtx* c, int fd, uint64_t isz, char* err, size_t err_len, uint64_t file_off = 0) {
  const uint64_t n = (isz + kSlotBytes - 1) / kSlotBytes;
  auto issue = [&](uint64_t i) -> bool {
    const int k = (int)(i % kSlots);
    const uint64_t off = i * kSlotBytes, len = std::min(kSlotBytes, isz - off);
    return hipMemcpyAsync(c->slot[k], c->d_out + off, len, hipMemcpyDeviceToHost, c->s) == hipSuccess &&
           hipEventRecord(c->ev[k], c->s) == hipSuccess;
  };
  for (uint64_t i = 0; i < std::min<uint64_t>(n, kSlots - 1); i++)
    if (!issue(i)) {
      set_err(err, err_len, "D2H copy failed");
      return SPARKEY_E_GPU;
    }
  for (uint64_t i = 0; i < n; i++) {
    const int k = (int)(i % kSlots);
    if (hipEventSynchronize(c->ev[k]) != hipSuccess) {
      set_err(err, err_len, "D2H copy failed");
      return SPARKEY_E_GPU;
    }
    if (i + kSlots - 1 < n && !issue(i + kSlots - 1)) {  // the slot written last round is free
      set_err(err, err_len, "D2H copy failed");
      return SPARKEY_E_GPU;
    }
    const uint64_t off = i * kSlotBytes, len = std::min(kSlotBytes, isz - off);
    int e = 0;
    if (!pool_pwrite(c, fd, c->slot[k], file_off + off, len, &e)) {
      set_err(err, err_len, std::string("write of the index file failed: ") + io_error(e));
      return SPARKEY_E_IO;
    }
  }
  return SPARKEY_OK;
}

// Log bytes [file_off, file_off + len) of fd -> c->d_log[0, len), through the staging ring (the pool
// reads piece i + 1 while piece i is copied).
int read_log_range(FileCtx* c, int fd, uint64_t file_off, uint64_t len, char* err, size_t err_len) {
  const int rc = for_each_slot_piece(c, len, [&](int k, uint64_t off, uint64_t n) -> int {
    int e = 0;
    if (!pool_pread(c, fd, c->slot[k], file_off + off, n, &e)) {
      set_err(err, err_len, std::string("read of the log file failed: ") + io_error(e));
      return SPARKEY_E_IO;
    }
    if (hipMemcpyAsync(c->d_log + off, c->slot[k], n, hipMemcpyHostToDevice, c->s) != hipSuccess ||
        hipEventRecord(c->ev[k], c->s) != hipSuccess) {
      set_err(err, err_len, "H2D copy failed");
      return SPARKEY_E_GPU;
    }
    return SPARKEY_OK;
  });
  if (rc) (void)hipStreamSynchronize(c->s);
  return rc;
}

struct CtxHold {  // acquire_ctx / release_ctx around one rank's work
  FileCtx* c = nullptr;
  ~CtxHold() { release_ctx(c); }
};

// One rank of a multi-GPU build (opts.num_gpus > 1): its log bytes in through `load`, the sharded build,
// its part of the .spi out through `store`.  Runs on the rank's own thread (shard_run_threads).  A rank
// whose context or load fails still enters the build with that code, so every rank returns it
// (shard_build_rank) instead of the others waiting for this one in a collective.
template <class Load, class Store>
int shard_rank(int rank, int world, int device, sparkey_shard_comm* comm, bool shared_device, const uint8_t* hdr,
               uint64_t log_len, const sparkey_build_opts* opts, sparkey_build_stats* stats_out, char* err,
               size_t err_len, Load&& load, Store&& store) {
  uint64_t blo = 0, bhi = 0, ooff = 0, olen = 0;
  int rc = sparkey_shard_geometry(hdr, log_len, opts, rank, world, &blo, &bhi, &ooff, &olen, err, err_len);
  if (rc) return rc;  // (the same on every rank: they all return here)
  CtxHold h;
  h.c = acquire_ctx(device, err, err_len, &rc);
  FileCtx* c = h.c;
  if (!rc && hipSetDevice(device) != hipSuccess) {
    set_err(err, err_len, "hipSetDevice failed");
    rc = SPARKEY_E_GPU;
  }
  if (!rc) rc = c->reserve(bhi - blo + 16, olen, err, err_len);
  if (!rc && knob(Knob::ShardFailRank) == rank) {  // (tests: one rank fails on its own)
    set_err(err, err_len, "rank " + std::to_string(rank) + ": injected load failure");
    rc = SPARKEY_E_IO;
  }
  if (!rc) rc = load(c, blo, bhi - blo);
  if (c) sk_plan_set_shared_device(c->plan, shared_device);
  sparkey_build_stats st;
  rc = shard_build_rank(c ? c->plan : nullptr, comm, hdr, log_len, c ? c->d_log : nullptr, blo, bhi, opts,
                        c ? c->d_out : nullptr, olen, c ? (void*)c->s : nullptr, &st, rc, err, err_len);
  if (c) sk_plan_set_shared_device(c->plan, false);
  if (!rc) rc = store(c, ooff, olen);
  if (!rc && rank == 0 && stats_out) *stats_out = st;
  return rc;
}

}  // namespace

extern "C" {

int sparkey_build_index_file(const char* log_path, const char* index_out_path, const sparkey_build_opts* opts,
                             int32_t fsync_out, sparkey_build_stats* stats_out, char* err, size_t err_len) {
  if (!log_path || !index_out_path || !opts) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  const bool dbg = sk::knob_on(sk::Knob::FileDebug);
  const double t0 = now_ms();
  const int fd = open(log_path, O_RDONLY);
  if (fd < 0) {
    set_err(err, err_len, std::string("cannot open log file ") + log_path + ": " + strerror(errno));
    return SPARKEY_E_IO;
  }
  struct Closer {
    int fd;
    ~Closer() { close(fd); }
  } closer{fd};
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    set_err(err, err_len, std::string("fstat failed: ") + strerror(errno));
    return SPARKEY_E_IO;
  }
  const uint64_t log_len = (uint64_t)sb.st_size;
  // LogHeader.read first (LogHeader.java:55-88): a file that is not a usable log fails before any
  // bulk read or device allocation
  uint8_t hdr[84];
  memset(hdr, 0, sizeof(hdr));
  const ssize_t hr = pread(fd, hdr, sizeof(hdr), 0);
  int rc = sk_check_log_header(hdr, hr > 0 ? (uint64_t)hr : 0, log_len, err, err_len);
  if (rc) return rc;
  const int64_t isz = sparkey_index_size(hdr, sizeof(hdr), opts);
  if (isz < 0) {
    set_err(err, err_len, sparkey_strerror((int)isz));
    return (int)isz;
  }
  if (opts->num_gpus > 1) {  // every rank reads its byte range and writes its part of the .spi itself
    const int ofd = open(index_out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (ofd < 0) {
      set_err(err, err_len, std::string("cannot create index file ") + index_out_path + ": " + strerror(errno));
      return SPARKEY_E_IO;
    }
    rc = ftruncate(ofd, (off_t)isz) == 0 ? SPARKEY_OK : SPARKEY_E_IO;
    if (rc) set_err(err, err_len, std::string("cannot size the index file: ") + strerror(errno));
    if (!rc)
      rc = shard_run_threads(*opts, [&](int rank, int world, int device, sparkey_shard_comm* comm, bool same, char* e,
                                        size_t el) {
        return shard_rank(
            rank, world, device, comm, same, hdr, log_len, opts, stats_out, e, el,
            [&](FileCtx* c, uint64_t lo, uint64_t n) { return read_log_range(c, fd, lo, n, e, el); },
            [&](FileCtx* c, uint64_t off, uint64_t n) { return write_index(c, ofd, n, e, el, off); });
      }, err, err_len);
    if (!rc && fsync_out && fsync(ofd) != 0) {
      set_err(err, err_len, std::string("fsync of the index file failed: ") + strerror(errno));
      rc = SPARKEY_E_IO;
    }
    if (close(ofd) != 0 && !rc) {
      set_err(err, err_len, std::string("close of the index file failed: ") + strerror(errno));
      rc = SPARKEY_E_IO;
    }
    if (rc) unlink(index_out_path);
    if (dbg) fprintf(stderr, "[file] %d GPUs: %.2f ms\n", opts->num_gpus, now_ms() - t0);
    return rc;
  }
  FileCtx* c = acquire_ctx(opts->device, err, err_len, &rc);
  if (!c) return rc;
  struct Releaser {
    FileCtx* c;
    ~Releaser() { release_ctx(c); }
  } releaser{c};
  if (hipSetDevice(c->device) != hipSuccess) {
    set_err(err, err_len, "hipSetDevice failed");
    return SPARKEY_E_GPU;
  }
  rc = c->reserve(log_len + 16, (uint64_t)isz, err, err_len);
  if (rc) return rc;
  const double t1 = now_ms();
  // log -> pinned slots (pool) -> device, piece by piece
  rc = read_log_range(c, fd, 0, log_len, err, err_len);
  if (rc) return rc;
  const double t2 = now_ms();
  rc = sparkey_plan_build_device(c->plan, hdr, c->d_log, log_len, c->d_out, (uint64_t)isz, opts, c->s, stats_out, err,
                                 err_len);
  if (rc) return rc;
  const double t3 = now_ms();
  // FileFlushingData.close: header then slots (+fsync)
  const int ofd = open(index_out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (ofd < 0) {
    set_err(err, err_len, std::string("cannot create index file ") + index_out_path + ": " + strerror(errno));
    return SPARKEY_E_IO;
  }
  rc = write_index(c, ofd, (uint64_t)isz, err, err_len);
  const double t4 = now_ms();
  if (!rc && fsync_out && fsync(ofd) != 0) {
    set_err(err, err_len, std::string("fsync of the index file failed: ") + strerror(errno));
    rc = SPARKEY_E_IO;
  }
  if (close(ofd) != 0 && !rc) {
    set_err(err, err_len, std::string("close of the index file failed: ") + strerror(errno));
    rc = SPARKEY_E_IO;
  }
  if (rc) {
    (void)hipStreamSynchronize(c->s);
    unlink(index_out_path);
    return rc;
  }
  const double t5 = now_ms();
  t_file_phase[0] = t1 - t0;
  t_file_phase[1] = t2 - t1;
  t_file_phase[2] = t3 - t2;
  t_file_phase[3] = t4 - t3;
  t_file_phase[4] = t5 - t4;
  if (dbg)
    fprintf(stderr, "[file] open+header %.2f ms, read+H2D %.2f ms, build %.2f ms, D2H+write %.2f ms, fsync+close %.2f ms\n",
            t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4);
  return SPARKEY_OK;
}

int sparkey_build_index_mem(const uint8_t* log, uint64_t log_len, uint8_t* index_out, uint64_t index_cap,
                            const sparkey_build_opts* opts, sparkey_build_stats* stats_out, char* err,
                            size_t err_len) {
  if (!log || !index_out || !opts) {
    set_err(err, err_len, "null argument");
    return SPARKEY_E_ARG;
  }
  int rc = sk_check_log_header(log, log_len, log_len, err, err_len);
  if (rc) return rc;
  const int64_t isz = sparkey_index_size(log, log_len, opts);
  if (isz < 0) {
    set_err(err, err_len, sparkey_strerror((int)isz));
    return (int)isz;
  }
  if ((uint64_t)isz > index_cap) {
    set_err(err, err_len, "index buffer too small: need " + std::to_string(isz));
    return SPARKEY_E_BUFFER;
  }
  if (opts->num_gpus > 1)
    return shard_run_threads(*opts, [&](int rank, int world, int device, sparkey_shard_comm* comm, bool same, char* e,
                                        size_t el) {
      return shard_rank(
          rank, world, device, comm, same, log, log_len, opts, stats_out, e, el,
          [&](FileCtx* c, uint64_t lo, uint64_t n) {
            if (hipMemcpyAsync(c->d_log, log + lo, n, hipMemcpyHostToDevice, c->s) != hipSuccess) {
              set_err(e, el, "H2D copy failed");
              return (int)SPARKEY_E_GPU;
            }
            return (int)SPARKEY_OK;
          },
          [&](FileCtx* c, uint64_t off, uint64_t n) {
            if (hipMemcpyAsync(index_out + off, c->d_out, n, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
                hipStreamSynchronize(c->s) != hipSuccess) {
              set_err(e, el, "D2H copy failed");
              return (int)SPARKEY_E_GPU;
            }
            return (int)SPARKEY_OK;
          });
    }, err, err_len);
  FileCtx* c = acquire_ctx(opts->device, err, err_len, &rc);
  if (!c) return rc;
  struct Releaser {
    FileCtx* c;
    ~Releaser() { release_ctx(c); }
  } releaser{c};
  if (hipSetDevice(c->device) != hipSuccess) {
    set_err(err, err_len, "hipSetDevice failed");
    return SPARKEY_E_GPU;
  }
  rc = c->reserve(log_len + 16, (uint64_t)isz, err, err_len);
  if (rc) return rc;
  rc = for_each_slot_piece(c, log_len, [&](int k, uint64_t off, uint64_t len) -> int {
    memcpy(c->slot[k], log + off, len);
    if (hipMemcpyAsync(c->d_log + off, c->slot[k], len, hipMemcpyHostToDevice, c->s) != hipSuccess ||
        hipEventRecord(c->ev[k], c->s) != hipSuccess) {
      set_err(err, err_len, "H2D copy failed");
      return SPARKEY_E_GPU;
    }
    return SPARKEY_OK;
  });
  if (rc) {
    (void)hipStreamSynchronize(c->s);
    return rc;
  }
  rc = sparkey_plan_build_device(c->plan, log, c->d_log, log_len, c->d_out, (uint64_t)isz, opts, c->s, stats_out, err,
                                 err_len);
  if (rc) return rc;
  if (hipMemcpyAsync(index_out, c->d_out, (size_t)isz, hipMemcpyDeviceToHost, c->s) != hipSuccess ||
      hipStreamSynchronize(c->s) != hipSuccess) {
    set_err(err, err_len, "D2H copy failed");
    return SPARKEY_E_GPU;
  }
  return SPARKEY_OK;
}

// The multi-GPU build over device-resident log ranges (include/sparkey_gpu.h): every rank reads its
// range in place and writes its part of the .spi in place.
int sparkey_build_index_sharded_device(const uint8_t* log_header, uint64_t file_len, const uint8_t* const* d_bufs,
                                       uint8_t* const* d_outs, const sparkey_build_opts* opts,
                                       sparkey_build_stats* stats_out, char* err, size_t err_len) {
  if (!log_header || !d_bufs || !d_outs || !opts || opts->num_gpus < 1) {
    set_err(err, err_len, "null argument or num_gpus < 1");
    return SPARKEY_E_ARG;
  }
  int rc = sk_check_log_header(log_header, 84, file_len, err, err_len);
  if (rc) return rc;
  sparkey_build_opts o = *opts;
  o.num_gpus = std::max(1, opts->num_gpus);
  return shard_run_threads(o, [&](int rank, int world, int device, sparkey_shard_comm* comm, bool same, char* e,
                                  size_t el) {
    uint64_t blo = 0, bhi = 0, ooff = 0, olen = 0;
    int r = sparkey_shard_geometry(log_header, file_len, &o, rank, world, &blo, &bhi, &ooff, &olen, e, el);
    if (r) return r;
    CtxHold h;
    h.c = acquire_ctx(device, e, el, &r);
    FileCtx* c = h.c;
    if (!r && hipSetDevice(device) != hipSuccess) {
      set_err(e, el, "hipSetDevice failed");
      r = SPARKEY_E_GPU;
    }
    if (!r && (!d_bufs[rank] || !d_outs[rank])) {
      set_err(e, el, "null device buffer for rank " + std::to_string(rank));
      r = SPARKEY_E_ARG;
    }
    if (c) sk_plan_set_shared_device(c->plan, same);
    sparkey_build_stats st;
    r = shard_build_rank(c ? c->plan : nullptr, comm, log_header, file_len, d_bufs[rank], blo, bhi, &o, d_outs[rank],
                         olen, c ? (void*)c->s : nullptr, &st, r, e, el);
    if (c) sk_plan_set_shared_device(c->plan, false);
    if (!r && rank == 0 && stats_out) *stats_out = st;
    return r;
  }, err, err_len);
}

int32_t sparkey_file_last_phases(double* ms_out, int32_t n) {
  const int32_t k = n < 5 ? n : 5;
  for (int32_t i = 0; i < k; i++) ms_out[i] = t_file_phase[i];
  return k;
}

void sparkey_release_cached_resources(void) {
  shard_release_groups();
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& kv : g_cache) {
    kv.second->mu.lock();  // waits for a call in flight
    kv.second->mu.unlock();
    delete kv.second;
  }
  g_cache.clear();
}

}  // extern "C"
