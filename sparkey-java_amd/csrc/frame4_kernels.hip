// frame4_kernels.hip -- k_frame4: framing + MurmurHash3 of logs whose VLQs are all one byte (every key
// < 127 bytes, every value < 128 bytes: fr_fast), one log chunk per LANE.
//
// Where a record starts depends on every record before it (SparkeyLogIterator.java:86-138).  For
// these logs a record's length is a function of its first two bytes: next(p) = p + 2 + klen + vlen
// (UncompressedBlockOutput.java:67-87).  A wave stages 64 consecutive chunks of C = 2^fr_cshift bytes
// (plus the longest record) into LDS once; lane k owns chunk k, so every phase keeps the 64 lanes busy
// and a record costs a few instructions.  A chunk's exit is the first record start at or past its
// end; chunk k's entry is chunk k-1's exit.
//
//   1 speculate  the lane screens its chunk's first maxRecLen positions (SWAR, 8 a step) and walks the
//                plausible ones in position order until one walks out of the chunk on plausible
//                headers and lands on a plausible header: its starts in the chunk are the lane's spec
//                list, the landing its spec exit.  The true first start of the chunk is among the
//                candidates and always survives, so the first survivor lies at or before it (false
//                starts die within a record or two, or merge into the true chain).
//   2 converge   (waves after the first) every plausible start in chunk 0's window is walked, one per
//                lane, to the end of chunk m-1 (m C >= maxRecLen): when the survivors all land on one
//                start, that is chunk m-1's exit whatever the wave's entry -- the true first start is
//                one of them.  The chunks from m on are then verified at once (3) and the wave's exit
//                is published before the wave waits for its predecessor's.
//   3 verify     a lane walks the true chain from its entry until it meets its spec list (the rest of
//                the list and the spec exit are then the chain's) or leaves the chunk (the walk itself
//                is the chunk's records, its exit the chunk's).  All lanes verify at once against their
//                predecessor's current exit; a lane whose exit changed makes its successor verify again
//                (rare).  After the wait, chunks 0 .. m-1 are verified from the published entry.
//   4 hash       the wave's records in log order, 64 lanes a round: MurmurHash3 of every key out of LDS
//                (MurmurHash3.java:18-201), 16-byte (hash, address) entries in log order into the
//                wave's slab.
//
// A list longer than kF4Lcap, a verified chain outside the one-byte rules, or a chain that does not
// close flags Status.spec_fail, and the host redoes the framing with k_frame3 / k_frame / the serial
// walker (which alone reports the reference's errors).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "frame_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

namespace {

constexpr int kF4Lcap = 8;             // starts per chunk in a spec list and in a fix list
constexpr unsigned kF4Caps = 64u;      // Status.spec_fail: a list cap, or a chain that did not close
constexpr int32_t kUnk = -1;           // no exit known
constexpr int32_t kNever = -2;         // (a lane that has not verified)

// One record step from region offset p (one-byte VLQs within the header's maxima, the key inside the
// file): the next start, or -1.
__device__ __forceinline__ int32_t f4_step(const uint8_t* rgn, int32_t p, int32_t lim, int32_t mk, int32_t mv,
                                           bool nodel) {
  const int32_t b0 = rgn[p], b1 = rgn[p + 1];
  const int32_t klen = b0 ? b0 - 1 : b1;
  const int32_t vlen = b0 ? b1 : 0;
  const bool ok = ((b0 | b1) & 0x80) == 0 && (b0 || !nodel) && klen <= mk && vlen <= mv && p + 2 + klen <= lim;
  return ok ? p + 2 + klen + vlen : -1;
}

}  // namespace

// LDS of one k_frame4 wave: the staged region, then the spec lists and the fix lists (u16, entry n of
// lane k at n * 64 + k), which later hold the wave's record list.
uint32_t frame4_lds(const BuildParams& P) { return (uint32_t)P.f4_rgn + 2u * 64u * kF4Lcap * 2u; }

__device__ __forceinline__ void frame4_region(const BuildParams& P, const uint64_t wv, uint8_t* lds) {
  const int lane = threadIdx.x & 63;
  const int cs = P.fr_cshift;
  const int32_t C = 1 << cs;
  const int64_t R0 = (int64_t)((P.fr_k0 + wv * 64ull) << cs);
  const int64_t log_len = (int64_t)P.log_len;
  const int32_t RLEN = P.f4_rgn;
  uint8_t* rgn = lds;
  uint16_t* Lb = reinterpret_cast<uint16_t*>(lds + RLEN);  // spec lists
  uint16_t* Fb = Lb + 64 * kF4Lcap;                         // fix lists
  uint16_t* pos = Lb;                                        // (later) the wave's record list
  unsigned long long t_prev = P.dbg ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {  // diagnostic only: cycles per phase, per wave (no atomics)
    if (P.dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      P.dbg[wv * 16 + i] = t - t_prev;
      t_prev = t;
    }
  };
  // every return publishes the wave's exit first (successors wait on it); on a failure any value (the
  // host redoes the framing)
  bool published = false;
  auto fail = [&](unsigned bits) {
    if (lane == 0) {
      atomicOr(&P.st->spec_fail, bits);
      if (!published) granule_store(&P.exit_desc[wv], (unsigned long long)R0 | kReady);
    }
  };

  // ---- stage [R0, R0 + RLEN): every 1 KiB row in flight at once, straight into LDS ----
  {
    const int nvec = RLEN >> 4;
    if (R0 + 16ll * nvec <= log_len) {
      const uint4* src = reinterpret_cast<const uint4*>(P.log + R0);
      for (int v0 = 0; v0 < nvec; v0 += 64)
        if (v0 + lane < nvec)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + v0 + lane),
                                           (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16, 0,
                                           2);  // (non-temporal: the log is read once)
    } else {
      for (int v = lane; v < nvec; v += 64)
        *reinterpret_cast<uint4*>(rgn + 16u * v) = load16_guarded(P.log, R0 + 16ll * v, log_len);
    }
  }
  wave_sync();
  mark(0);

  const int32_t de = (int32_t)min((int64_t)0x7fffffff, P.data_end - R0);  // records start below this
  const int64_t lim64 = log_len - R0;
  const int32_t lim = lim64 > 0x7fffffff ? 0x7fffffff : (int32_t)lim64;
  const int32_t ruse = RLEN - 16;  // headers readable below this
  const int32_t mk = (int32_t)P.max_key_len, mv = (int32_t)P.max_value_len;
  const int32_t mrl = (int32_t)P.max_rec_len;
  const bool nodel = P.no_deletes != 0;
  const int32_t s = lane * C;  // this lane's chunk [s, e)
  const int32_t e = min(s + C, de);
  const bool pass = s >= de;   // past the frame's end: no record, the entry passes through
  auto step = [&](int32_t p) { return f4_step(rgn, p, lim, mk, mv, nodel); };
  auto Lat = [&](int n) -> int32_t { return Lb[n * 64 + lane]; };

  // ---- 1 speculate ----
  int32_t cnt = 0, sx = kUnk;  // spec list length, spec exit
  // a walk from c: its starts below e into the spec list; true when it leaves the chunk onto a
  // plausible header (or the frame's end)
  auto spec_walk = [&](int32_t c) -> bool {
    int32_t p = c, n = 0;
    while (p < e) {
      if (n < kF4Lcap) Lb[n * 64 + lane] = (uint16_t)p;
      n++;
      p = step(p);
      if (p < 0) return false;
    }
    if (p < de && p < ruse && step(p) < 0) return false;
    cnt = n;
    sx = p;
    return true;
  };
  if (!pass) {
    if (wv == 0 && lane == 0) {  // the frame's entry is known
      (void)spec_walk((int32_t)(P.fr_entry - R0));
    } else {
      const Screen8 scn = make_screen8(P);
      const uint64_t* r64 = reinterpret_cast<const uint64_t*>(rgn);
      const int32_t wend = min(min(s + mrl, de), ruse);
      bool found = false;
      for (int32_t w = s >> 3; !found && 8 * w < wend; w++) {
        const uint64_t x = r64[w];
        uint32_t bits = screen8(x, (x >> 8) | (r64[w + 1] << 56), scn);
        if (8 * w + 8 > wend) bits &= (1u << (wend - 8 * w)) - 1u;
        while (bits && !found) {
          const int32_t c = 8 * w + __builtin_ctz(bits);
          bits &= bits - 1;
          found = spec_walk(c);
        }
      }
    }
  }
  if (cnt > kF4Lcap) {  // (a spec list past the cap: the lane verifies without one)
    cnt = 0;
    sx = kUnk;
  }
  mark(1);

  // ---- 2 converge: chunk m-1's exit from every plausible start of chunk 0's window ----
  const int32_t m = P.f4_m;
  const int32_t Est = m * C;
  bool conv = false;
  int32_t cx = kUnk;
  if (wv > 0 && Est <= de && Est < ruse) {
    const int32_t wlim = min(mrl, de);
    int32_t mn = 0x7fffffff, mx = -1;
    for (int32_t c = lane; c < wlim; c += 64) {
      int32_t p = c;
      while (p >= 0 && p < Est) p = step(p);
      if (p >= 0) {
        mn = min(mn, p);
        mx = max(mx, p);
      }
    }
    const int32_t hi = wave_max_i32(mx), lo = -wave_max_i32(-mn);
    conv = hi >= 0 && hi == lo;
    cx = hi;
  }
  mark(2);

  // ---- 3 verify: the true chain from the entry meets the spec list, or is the chunk ----
  int32_t x = pass ? kUnk : sx;  // this lane's exit
  int32_t nf = 0, mi = 0;        // fix records, first spec record used
  bool bad = false;              // the walk from `seen` broke the one-byte rules
  int32_t seen = kNever;         // the entry this lane verified from
  auto verify = [&](int32_t px) {
    nf = 0;
    bad = false;
    if (pass) {
      mi = cnt;
      x = px;
      return;
    }
    int32_t t = px, j = 0;
    const int32_t n = min(cnt, kF4Lcap);
    while (t < e) {
      while (j < n && Lat(j) < t) j++;
      if (j < n && Lat(j) == t) {  // merged: the rest of the spec list is the chain's
        mi = j;
        x = sx;
        return;
      }
      if (nf < kF4Lcap) Fb[nf * 64 + lane] = (uint16_t)t;
      nf++;
      t = step(t);
      if (t < 0) {
        bad = true;
        x = kUnk;
        return;
      }
    }
    mi = cnt;
    x = t;
  };
  // rounds: every active lane whose predecessor's exit is known and not the entry it verified from
  auto ripple = [&](int32_t e0, bool act) {
    for (;;) {
      int32_t px = wave_prev_i32(x, kUnk);
      if (lane == 0) px = e0;
      const bool go = act && px != kUnk && px != seen;
      const int32_t before = x;
      if (go) {
        seen = px;
        verify(px);
      }
      if (!__any(go && x != before)) break;
    }
  };
  // closed: every lane verified from its predecessor's final exit
  auto closed = [&](int32_t e0, bool act) -> bool {
    int32_t px = wave_prev_i32(x, kUnk);
    if (lane == 0) px = e0;
    return !__any(act && (bad || x == kUnk || nf > kF4Lcap || seen != px));
  };
  int32_t early = kUnk;
  if (conv) {  // chunks m .. 63 from the converged exit, and the wave's exit published
    const bool act = lane >= m;
    if (lane == m - 1) x = cx;
    ripple(kUnk, act);
    if (closed(kUnk, act)) {
      early = __builtin_amdgcn_readlane(x, 63);
      if (lane == 0) granule_store(&P.exit_desc[wv], (unsigned long long)(R0 + early) | kReady);
      published = true;
    }
  }
  mark(3);
  int32_t e0 = 0;
  if (wv == 0) {
    e0 = (int32_t)(P.fr_entry - R0);
  } else {  // the previous wave's exit (lane 0 spins, bounded)
    unsigned long long extv = (unsigned long long)R0;
    if (lane == 0) {
      const unsigned long long t0 = wall_clock64();
      for (;;) {
        const unsigned long long v = granule_load(&P.exit_desc[wv - 1]);
        if (v & kReady) {
          extv = v & ~kReady;
          break;
        }
        if (wall_clock64() - t0 >= P.fr_spin_ticks) {  // bounded all the same: serial path
          atomicOr(&P.st->spec_fail, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    const int64_t ext = (int64_t)(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(extv >> 32))
                                   << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)extv));
    const int64_t d = ext - R0;
    if (d < 0 || d > (int64_t)64 * C + mrl) { fail(1u); return; }
    e0 = (int32_t)d;
  }
  mark(4);
  ripple(e0, true);
  if (!closed(e0, true)) { fail(kF4Caps); return; }
  const int32_t wexit = __builtin_amdgcn_readlane(x, 63);
  if (published && wexit != early) {  // the published exit was wrong (a corrupt log): the host redoes it
    if (lane == 0) atomicOr(&P.st->spec_fail, 1u);
    return;
  }
  if (!published && lane == 0) granule_store(&P.exit_desc[wv], (unsigned long long)(R0 + wexit) | kReady);
  published = true;
  if (lane == 0 && wv + 1 == (P.fr_nchunks + 63) / 64) P.st->exit = R0 + wexit;
  mark(5);

  // ---- counts; the wave's record list in log order over the lists (read into registers first) ----
  const uint32_t mine = pass ? 0u : (uint32_t)(nf + (cnt - mi));
  const uint32_t incl = wave_incl_sum_u32(mine);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (total > P.slab_cap || total > 2u * 64u * kF4Lcap) {
    if (lane == 0) {
      atomicMax(&P.st->max_wave_count, total);
      atomicOr(&P.st->overflow, 1u);
    }
    return;
  }
  {
    uint32_t fv[kF4Lcap], lv[kF4Lcap];
#pragma unroll
    for (int i = 0; i < kF4Lcap; i++) {
      fv[i] = Fb[i * 64 + lane];
      lv[i] = Lb[i * 64 + lane];
    }
    wave_sync();
    uint32_t o = incl - mine;
    if (!pass) {
#pragma unroll
      for (int i = 0; i < kF4Lcap; i++)
        if (i < nf) pos[o++] = (uint16_t)fv[i];
#pragma unroll
      for (int i = 0; i < kF4Lcap; i++)
        if (i >= mi && i < cnt) pos[o++] = (uint16_t)lv[i];
    }
  }
  if (lane == 0) P.wcount[wv] = total;
  wave_sync();
  mark(6);

  // ---- 4 hash ----
  const unsigned long long base = wv * (unsigned long long)P.slab_cap;
  unsigned long long ndel = 0;
  for (uint32_t r = (uint32_t)lane; r < total; r += 64) {
    const int32_t p = pos[r];
    const int32_t b0 = rgn[p], b1 = rgn[p + 1];
    const int32_t klen = b0 ? b0 - 1 : b1;
    const RgnKey ld{rgn, (uint32_t)(p + 2)};
    const uint64_t hash = P.hash_size == 8 ? murmur64_ld(ld, klen, (uint32_t)P.seed)
                                           : (uint64_t)murmur32_ld(ld, klen, (uint32_t)P.seed);
    uint64_t addr = (uint64_t)(R0 + p) << P.ebb;
    if (b0 == 0) {
      addr |= kDelBit;
      ndel++;
    }
    Entry en;
    en.hash = hash;
    en.addr = addr;
    P.ent[base + r] = en;
  }
  ndel = wave_sum_u64(ndel);
  if (ndel && lane == 0) add_deletes(P, wv, ndel);
  mark(7);
  if (P.dbg && lane == 0) {
    P.dbg[wv * 16 + 8] = (unsigned long long)total;
    P.dbg[wv * 16 + 10] = conv ? 0ull : 1ull;
  }
}

// One wave per workgroup, one 64-chunk region each (region i = workgroup i, or by ticket when builds
// share the device, as k_frame3).
__global__ __launch_bounds__(64, 4) void k_frame4(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint32_t tk = blockIdx.x;
  if (P.fr_ticket) {
    uint32_t t = 0;
    if (threadIdx.x == 0) t = atomicAdd(P.frame_ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  }
  const uint64_t nwaves = (P.fr_nchunks + 63) / 64;
  if (tk < nwaves) frame4_region(P, tk, lds);
}

// k_frame4's geometry on P (fr_fast logs): chunks of C = 2^cs bytes (64 .. 512; about one mean record
// unless the frame4_c switch sets it), 64 a wave, and m chunks to the converge target (m C >= maxRecLen).
// False when the lists cannot hold what the header's mean record implies.
bool frame4_geometry(BuildParams& P, double mean_record, int64_t want_c, int64_t entry, int64_t frame_end) {
  if (!P.fr_fast || P.max_rec_len > 256 || mean_record <= 0.0) return false;
  int64_t want = want_c > 0 ? want_c : (int64_t)(1.0 * mean_record);
  int cs = 6;
  while (cs < 9 && (1ll << cs) < want) cs++;
  const int64_t C = 1ll << cs;
  if ((double)C / mean_record > 0.5 * kF4Lcap) return false;
  P.fr_cshift = cs;
  P.fr_w = 64;
  P.fr_k0 = (uint64_t)entry >> cs;
  P.fr_nchunks = frame_end > entry ? (uint64_t)((frame_end + C - 1) / C) - P.fr_k0 : 0;
  P.f4_m = (int32_t)std::max<int64_t>(1, (P.max_rec_len + C - 1) / C);
  P.f4_rgn = (int32_t)((64 * C + P.max_rec_len + 32 + 15) & ~15ll);
  return frame4_lds(P) <= 64 * 1024;
}

void launch_frame4(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.fr_nchunks == 0) return;
  const uint64_t nwaves = (P.fr_nchunks + 63) / 64;
  hipLaunchKernelGGL(k_frame4, dim3((unsigned)nwaves), dim3(64), (size_t)frame4_lds(P), s, P);
  tm->mark("frame", s);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.wcount, P.woff, P.nslabs, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
}

}  // namespace sk
