// fastmod_check.cpp -- host check of the build kernels' "hash mod capacity" (device_common.hpp
// fast_mod / make_fastmod, the same __host__ __device__ code the kernels run) against the plain
// unsigned remainder IndexHash.getWantedSlot computes (Long.remainderUnsigned, IndexHash.java:667-669).
// Built and run by tests/test_fastmod.py.  Prints "ok <checks>" or the first mismatch.
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "device_common.hpp"

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  std::vector<uint64_t> caps = {1, 3, 5, 7, 1301, 13000001, 130000001, 1300000001, 0x7fffffffull, 0xffffffffull,
                                (1ull << 33) + 1, (1ull << 62) + 1, (1ull << 63) - 1};
  for (uint64_t c = 1; c < 4096; c += 2) caps.push_back(c);  // every odd capacity of small tables
  uint64_t seed = 12345, checks = 0;
  for (uint64_t cap : caps) {
    const sk::FastMod f = sk::make_fastmod(cap);
    std::vector<uint64_t> xs = {0, 1, cap - 1, cap, cap + 1, 2 * cap - 1, 2 * cap, ~0ull, ~0ull - 1, ~0ull - cap,
                                1ull << 63, (1ull << 63) - 1, (1ull << 32) - 1, 1ull << 32};
    // multiples of cap around the top of the range, where floor(2^64 / cap) is least exact
    const uint64_t top = ~0ull / cap;
    for (uint64_t i = 0; i < 4 && i <= top; i++)
      for (int d = -2; d <= 2; d++) xs.push_back((top - i) * cap + (uint64_t)(int64_t)d);
    const int nrand = cap < 4096 ? 2000 : 200000;
    for (int i = 0; i < nrand; i++) xs.push_back(splitmix(seed));
    if (cap < 4096)
      for (uint64_t x = 0; x < 20000; x++) xs.push_back(x);
    for (uint64_t x : xs) {
      const uint64_t got = sk::fast_mod(x, f), want = x % cap;
      checks++;
      if (got != want) {
        printf("mismatch cap=%llu x=%llu got=%llu want=%llu\n", (unsigned long long)cap, (unsigned long long)x,
               (unsigned long long)got, (unsigned long long)want);
        return 1;
      }
    }
  }
  printf("ok %llu\n", (unsigned long long)checks);
  return 0;
}
