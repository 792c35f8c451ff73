// knobs.cpp -- storage and C-ABI of the test and diagnostic switches (knobs.hpp).
#include "knobs.hpp"

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>

#include "../../include/sparkey_gpu.h"

namespace sk {
namespace {

constexpr int kN = (int)Knob::kCount;

const char* const kNames[kN] = {
    "no_uniform",     "no_frame3",        "serial_framing",   "frame_cmin",     "frame_region",
    "frame_look",     "frame3_c",         "frame3_short",     "frame3_cover",   "frame3_stop",
    "frame_ticket",     "frame_spin_ticks", "frame_debug",    "part2_debug",
    "no_regions",     "no_buckets",       "region_cap",       "exact_serial",     "exact_debug",    "exact_reframe",
    "exact_full_table", "snappy_lds",     "snappy_dir_a",     "snappy_dir_debug", "snappy_chunk",
    "snappy_serial_dir", "zstd_lds",      "shard_sync_frame", "shard_transport", "shard_fail_rank", "file_threads",
    "file_write_threads", "file_debug", "reframe_spin_ticks",
    "shard_gather_compressed", "inject_foreign", "shard_coll_fail", "no_compact",
    "part2_two_level"};
static_assert(sizeof(kNames) / sizeof(kNames[0]) == kN, "one name per knob");

std::atomic<int64_t> g_val[kN];
std::once_flag g_once;

int find(const char* name, size_t len) {
  for (int i = 0; i < kN; i++)
    if (strlen(kNames[i]) == len && strncmp(kNames[i], name, len) == 0) return i;
  return -1;
}

// SPARKEY_DEBUG="name=value,name=value" (a bare name means 1), read once.
void init() {
  std::call_once(g_once, [] {
    for (auto& v : g_val) v.store(-1, std::memory_order_relaxed);
    const char* s = getenv("SPARKEY_DEBUG");
    while (s && *s) {
      const char* e = strchr(s, ',');
      const size_t n = e ? (size_t)(e - s) : strlen(s);
      const std::string item(s, n);
      const size_t eq = item.find('=');
      const int i = find(item.c_str(), eq == std::string::npos ? item.size() : eq);
      if (i >= 0) g_val[i].store(eq == std::string::npos ? 1 : atoll(item.c_str() + eq + 1), std::memory_order_relaxed);
      s = e ? e + 1 : nullptr;
    }
  });
}

}  // namespace

int64_t knob(Knob k) {
  init();
  return g_val[(int)k].load(std::memory_order_relaxed);
}

}  // namespace sk

extern "C" {

int sparkey_debug_set(const char* name, int64_t value) {
  if (!name) return SPARKEY_E_ARG;
  sk::init();
  const int i = sk::find(name, strlen(name));
  if (i < 0) return SPARKEY_E_ARG;
  sk::g_val[i].store(value < 0 ? -1 : value, std::memory_order_relaxed);
  return SPARKEY_OK;
}

int64_t sparkey_debug_get(const char* name) {
  if (!name) return SPARKEY_E_ARG;
  sk::init();
  const int i = sk::find(name, strlen(name));
  return i < 0 ? (int64_t)SPARKEY_E_ARG : sk::g_val[i].load(std::memory_order_relaxed);
}

}  // extern "C"
