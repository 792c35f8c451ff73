// frame3_kernels.hip -- k_frame3: framing + MurmurHash3 of logs whose records differ in size and
// whose VLQs are all one byte (every key < 127 bytes, every value < 128 bytes: fr_fast).
//
// The log is a chain of varint-framed records (SparkeyLogIterator.java:86-138): where a record
// starts depends on every record before it.  One wave owns W chunks of C = 2^fr_cshift bytes
// (C >= maxRecLen), staged once into LDS with LOOK bytes past the last one, like k_frame
// (fused_kernels.hip).  k_frame walks every candidate start of a chunk to the chunk end and then
// walks the verified chain a second time to list its records; here the walks are split so that
// all 64 lanes stay busy and every chain is walked once:
//
//   1 screen     plausible record starts in each chunk's first maxRecLen bytes (SWAR, 8 per step),
//                as in k_frame; the candidates of all chunks go to one position-sorted LDS list,
//                one 64-bit mask word per lane.
//   2 short walk every candidate K records on (K = 2..4), lanes taking candidates lane, lane + 64, ...:
//                a false start survives a step with the probability that two random bytes look like
//                a header (about 1 in 10 for 8-64 B keys: K = 2, 1 in 100 survives), and K grows
//                with that probability (the header's maxima).  A
//                surviving candidate marks the starts it reached inside its chunk: a candidate
//                reached from another one lies on that one's chain (its records are a suffix of the
//                other's), so only the unreached survivors -- the chain heads -- walk on.  The true
//                starts of a chunk form one chain: only the first is a head.
//   3 long walk  each head (about one per chunk: the true chain, rarely a false one) walks to its
//                chunk end + LOOK on its own lane, listing its record starts.  Its exit is the first
//                start at or past the chunk end.
//   4 resolve    chunk j's entry is chunk j-1's exit: a head whose list holds it gives the chunk's
//                records (that list from the entry on) and its exit (the true start of a chunk
//                always survives, as a head or on one's list: it is a plausible start of a valid
//                chain).  A chunk whose heads all reach one exit knows it without its entry, so the
//                wave's exit is usually published before the wave waits for its predecessor's; the
//                first entry is taken speculatively when chunk 0 has a single head (checked at the
//                end).
//   5 hash       the chosen lists back to back, every lane on every 64th record: MurmurHash3 of the
//                key out of LDS (MurmurHash3.java:18-201), 16-byte (hash, address) entries in log
//                order into the wave's slab.
//
// Anything outside what the lists can hold (too many candidates, survivors or records per chunk),
// a chunk whose entry no survivor starts at (the header understates its maxima, or the log is
// corrupt), or a wait that does not end, makes the host redo the framing with k_frame or the
// serial walker (Status.spec_fail).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "frame_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

namespace {

constexpr int kF3LcapMax = 128;  // record starts a survivor lists inside its chunk (P.f3_lcap, at most)
constexpr unsigned kF3Caps = 64u;  // Status.spec_fail: a list cap was exceeded (k_frame redoes it)
constexpr int kF3WavesPerSimd = 6;  // k_frame3's occupancy bound (its VGPR budget)

// Scratch after the staged region (bytes), sized on the host so that four waves of a workgroup and
// kF3WavesPerSimd workgroups fit a CU's LDS where the log allows (P.f3_cand_cap candidates, P.f3_surv_cap heads):
// candidate list; head starts / exits / counts / per-chunk choice (128 B) / a 16-byte sink that lanes
// with nothing to store write to (so no store needs an exec-mask branch); the heads' record lists,
// earlier the screen bitmap and then the short walk's reached-start bitmap (one bit per region byte).
__host__ __device__ __forceinline__ int f3_off_meta(int cand_cap) { return 2 * cand_cap; }
__host__ __device__ __forceinline__ int f3_off_sink(int cand_cap, int surv_cap) {
  return f3_off_meta(cand_cap) + surv_cap * 5 + 128;
}
__host__ __device__ __forceinline__ int f3_off_lists(int cand_cap, int surv_cap) {
  return (f3_off_sink(cand_cap, surv_cap) + 16 + 7) & ~7;
}

// One record step from region offset rp (screen rules, canonical one-byte VLQs): the next start,
// or -1 when the bytes at rp are no plausible header.  Branch-free: every rule is a difference whose
// sign says it failed, all ORed into one sign test (no chain of condition masks on the scalar unit).
// delmask = -1 when the header counts no DELETE (a 0x00 first byte is then no start).  Bytes >= 0x80
// (multi-byte VLQs) fail the maxima, which k_frame3's logs keep below 127 (fr_fast).
// kNoDel (the header counts no DELETE): a PUT's fields need no select (a zero first byte fails b0 - 1).
template <bool kNoDel>
__device__ __forceinline__ int32_t f3_step(const uint8_t* rgn, int32_t rp, int32_t lim, int32_t mk, int32_t mv) {
  const int32_t b0 = rgn[rp], b1 = rgn[rp + 1];
  if (kNoDel) {
    const int32_t kend = rp + 1 + b0;  // rp + 2 + (b0 - 1)
    const int32_t bad = (mk + 1 - b0) | (mv - b1) | (lim - kend) | (b0 - 1);
    return bad < 0 ? -1 : kend + b1;
  }
  const bool del = b0 == 0;
  const int32_t klen = del ? b1 : b0 - 1;
  const int32_t vlen = del ? 0 : b1;
  const int32_t kend = rp + 2 + klen;
  const int32_t bad = (mk - klen) | (mv - vlen) | (lim - kend);
  return bad < 0 ? -1 : kend + vlen;
}

// LDS hand-offs between the lanes of one wave: a wave's LDS accesses complete in issue order, so a
// compiler fence is all a later read of another lane's store needs (no s_waitcnt, no barrier).
__device__ __forceinline__ void lds_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace

// Stage region wv's bytes [R0, R0 + RLEN) into LDS: every 1 KiB row in flight at once, straight into
// LDS (the last row's lanes past the region masked off: the region is a 16-byte multiple, not whole
// rows).  Only issued here; the LDS-DMA completes under vmcnt (the wave_sync after it).
__device__ __forceinline__ void f3_stage(const BuildParams& P, const uint64_t wv, uint8_t* rgn, const int lane) {
  const int W = P.fr_w;
  const int cs = P.fr_cshift;
  const int64_t log_len = (int64_t)P.log_len;
  const uint64_t k0 = P.fr_k0 + wv * (uint64_t)W;
  const int nw = (int)min((uint64_t)W, P.fr_k0 + P.fr_nchunks - k0);
  const int64_t R0 = (int64_t)(k0 << cs);
  const int64_t RLEN = (int64_t)P.f3_rgn - ((int64_t)(W - nw) << cs);
  const int nvec = (int)((RLEN + 15) >> 4);
  if (R0 + 16ll * nvec <= log_len) {
    const uint4* src = reinterpret_cast<const uint4*>(P.log + R0);
    if (P.uni_nt) {  // non-temporal: the log is read once
      for (int v0 = 0; v0 < nvec; v0 += 64)
        if (v0 + lane < nvec)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + v0 + lane),
                                           (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16,
                                           0, 2);
    } else {
      for (int v0 = 0; v0 < nvec; v0 += 64)
        if (v0 + lane < nvec)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + v0 + lane),
                                           (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16,
                                           0, 0);
    }
  } else {
    for (int v = lane; v < nvec; v += 64)
      *reinterpret_cast<uint4*>(rgn + 16u * v) = load16_guarded(P.log, R0 + 16ll * v, log_len);
  }
}

// One region (wave index wv) of k_frame3; its exit is published before any return.
template <bool kNoDel>
__device__ __forceinline__ void frame3_region(const BuildParams& P, const uint64_t wv, uint8_t* lds) {
  const int lane = threadIdx.x & 63;
  const int cs = P.fr_cshift;
  const int W = P.fr_w;
  const int64_t LOOK = P.fr_look;
  const int64_t log_len = (int64_t)P.log_len;
  const uint64_t kf = P.fr_k0;
  const uint64_t k0 = kf + wv * (uint64_t)W;
  const int nw = (int)min((uint64_t)W, kf + P.fr_nchunks - k0);
  const int64_t R0 = (int64_t)(k0 << cs);
  // the staged bytes: the chunks, then at least max(LOOK, maxRecLen) + 16 more, so that every key a
  // listed record holds lies in LDS (records start inside the chunks)
  const int64_t RLEN = (int64_t)P.f3_rgn - ((int64_t)(W - nw) << cs);
  const int kF3CandCap = P.f3_cand_cap, kF3SurvCap = P.f3_surv_cap, kF3Lcap = P.f3_lcap;
  const int kF3Lstride = kF3Lcap + 1;  // (a head's list: kF3Lcap starts and a spare slot)
  const int kF3OffLists = f3_off_lists(kF3CandCap, kF3SurvCap);
  uint8_t* rgn = lds;
  uint8_t* scr = lds + P.f3_rgn;
  uint16_t* cand = reinterpret_cast<uint16_t*>(scr);             // candidates (bit 15: alive, with marks)
  uint16_t* s_start = reinterpret_cast<uint16_t*>(scr + f3_off_meta(kF3CandCap));
  uint16_t* s_exit = s_start + kF3SurvCap;                          // 0xffff: died in the long walk
  uint8_t* s_cnt = reinterpret_cast<uint8_t*>(s_exit + kF3SurvCap);
  int8_t* s_sel = reinterpret_cast<int8_t*>(s_cnt + kF3SurvCap);    // per chunk: first / last head
  uint16_t* sink = reinterpret_cast<uint16_t*>(scr + f3_off_sink(kF3CandCap, kF3SurvCap));
  uint16_t* lists = reinterpret_cast<uint16_t*>(scr + kF3OffLists);
  unsigned long long t_prev = P.dbg ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {  // diagnostic only: cycles per phase, per wave (no atomics)
    if (P.dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      P.dbg[wv * 16 + i] = t - t_prev;
      t_prev = t;
    }
  };
  // the previous wave's published exit (lane 0 spins, bounded), broadcast
  auto wait_prev = [&]() -> int64_t {
    unsigned long long extv = (unsigned long long)P.fr_entry;
    if (wv > 0 && lane == 0) {
      const unsigned long long t0 = wall_clock64();
      for (;;) {
        const unsigned long long v = granule_load(&P.exit_desc[wv - 1]);
        // (a bound of 0 gives up at once, even on a published exit: the tests of the host's redo)
        if ((v & kReady) && P.fr_spin_ticks) { extv = v & ~kReady; break; }
        if (wall_clock64() - t0 >= P.fr_spin_ticks) {  // bounded all the same: serial path
          atomicOr(&P.st->spec_fail, 2u);
          extv = (unsigned long long)R0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    return (int64_t)(((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(extv >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)extv));
  };
  // every return below publishes the wave's exit first (successors wait on it): on a failure, any
  // value (the host redoes the framing)
  auto fail = [&](unsigned bits) {
    if (lane == 0) {
      atomicOr(&P.st->spec_fail, bits);
      granule_store(&P.exit_desc[wv], (unsigned long long)R0 | kReady);
    }
  };
  // (frame3_stop: the exit published, the framing failed by wave 0 alone -- one atomic per wave on the
  //  status word would serialise and swamp what is measured)
  auto stop = [&]() {
    if (lane == 0) {
      if (wv == 0) atomicOr(&P.st->spec_fail, kF3Caps);
      granule_store(&P.exit_desc[wv], (unsigned long long)R0 | kReady);
    }
  };

  // ---- stage ----
  f3_stage(P, wv, rgn, lane);
  wave_sync();  // (the LDS-DMA counts in vmcnt)
  mark(0);
  if (P.f3_stop == 0) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)

  // region offsets (32-bit) of the wave's bounds
  const int32_t de = (int32_t)min((int64_t)0x7fffffff, P.data_end - R0);  // records start below this
  const int32_t ruse = (int32_t)(RLEN - 16);                              // headers readable below this
  const int64_t lim64 = log_len - R0;
  const int32_t lim = lim64 > 0x7fffffff ? 0x7fffffff : (int32_t)lim64;
  const int32_t mk = (int32_t)P.max_key_len, mv = (int32_t)P.max_value_len;
  const int32_t mrl = (int32_t)P.max_rec_len;
  const int32_t look = (int32_t)LOOK;
  const int32_t ent0 = (int32_t)(P.fr_entry - R0);  // (wave 0) the frame's entry
  const int32_t C = 1 << cs;
  auto chunk_end = [&](int32_t j) -> int32_t { return min((j + 1) * C, de); };

  // ---- 1 screen: one flag bit per byte of each chunk's candidate window ----
  const int nwl = (int)((min(C, mrl) + 63) >> 6);  // 64-position words per chunk
  unsigned long long* flags = reinterpret_cast<unsigned long long*>(scr + kF3OffLists);
  {
    const Screen8 scn = make_screen8(P);
    const uint64_t* r64 = reinterpret_cast<const uint64_t*>(rgn);
    uint8_t* fb = reinterpret_cast<uint8_t*>(flags);
    const int wpc = nwl * 8;
    const int nq = nw * wpc;
    for (int q = lane; q < nq; q += 64) {
      const int j = (int)(((uint32_t)q * P.fr_wpc_magic) >> 22);  // q / wpc (exact, checked on the host)
      const int rw = (j << (cs - 3)) + (q - j * wpc);
      const uint64_t x = r64[rw];
      fb[q] = (uint8_t)screen8(x, (x >> 8) | (r64[rw + 1] << 56), scn);
    }
  }
  lds_fence();
  mark(1);
  if (P.f3_stop == 1) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)

  // ---- candidates, position order: word q = chunk q / nwl, positions 64 (q % nwl) + bit.  Each lane
  //      writes one of its set bits per step; the wave's steps are its largest count ----
  int32_t T = 0;
  bool over = false;
  {
    const int nq = nw * nwl;
    for (int q0 = 0; q0 < nq; q0 += 64) {
      const int q = q0 + lane;
      unsigned long long m = 0;
      int32_t base = 0;
      if (q < nq) {
        const int j = q / nwl, wi = q - j * nwl;
        const int32_t s = j * C;
        const int32_t e = chunk_end(j);
        if (wv == 0 && j == 0) {  // the frame's entry chunk: its only start is the entry
          m = (wi == 0 && ent0 < e) ? 1ull : 0ull;
          base = ent0;
        } else {
          base = s + 64 * wi;
          const int32_t cend = min(e, s + mrl);
          if (base < cend) {
            m = flags[q];
            const int32_t valid = cend - base;
            if (valid < 64) m &= (1ull << valid) - 1ull;
          }
        }
      }
      const uint32_t c = (uint32_t)__builtin_popcountll(m);
      const uint32_t incl = wave_incl_sum_u32(c);
      const int32_t tot = __builtin_amdgcn_readlane((int)incl, 63);
      if (T + tot > kF3CandCap) {
        over = true;
        break;
      }
      uint32_t o = (uint32_t)T + incl - c;
      while (__ballot(m != 0)) {
        const bool has = m != 0;
        uint16_t* d = has ? cand + o : sink;
        *d = (uint16_t)(base + __builtin_ctzll(m));
        o += has ? 1u : 0u;
        m &= m - 1ull;
      }
      T += tot;
    }
  }
  if (over) {
    fail(kF3Caps);
    return;
  }
  lds_fence();
  mark(7);  // (the candidate list: reported after the other phases)

  // ---- 2 short walk: each candidate K records on (or to its stop); a survivor marks the starts it
  //      reached inside its chunk (bit 15 of its list entry: alive).  More heads than the lanes
  //      (rare: a stretch of bytes that look like headers) walk one step more.  A dead walk is
  //      p = -1; every lane runs the K steps (selects, no per-lane exits). ----
  uint32_t* reached = reinterpret_cast<uint32_t*>(scr + kF3OffLists);  // (the screen bitmap is dead)
  const bool cover = P.f3_cover != 0;  // (windows that hold several true starts: mark the reached ones)
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  int32_t S = 0;
  for (int K = P.f3_short;; K++) {
    if (cover) {
      for (int32_t i = lane; i < (ruse + 31) / 32 + 1; i += 64) reached[i] = 0u;
      lds_fence();
    }
    // without marks, a round's survivors are its heads: walk and compact in one pass
    S = 0;
    over = false;
    for (int32_t i0 = 0; i0 < T; i0 += 64) {
      const int32_t i = i0 + lane;
      const bool in = i < T;
      const int32_t st = in ? (int32_t)(cand[in ? i : 0] & 0x7fff) : 0;
      const int32_t e = chunk_end(st >> cs);
      const int32_t stop = min(min(e + look, de), ruse);
      int32_t p = in ? st : -1;
      for (int t = 0; t < K; t++) {
        const bool go = p >= 0 && p < stop;
        const int32_t q = f3_step<kNoDel>(rgn, go ? p : 0, lim, mk, mv);
        // (a start reached by a candidate that dies later dies too: marking it is harmless)
        if (cover && go && q >= 0 && q < e) atomicOr(&reached[q >> 5], 1u << (q & 31));
        p = go ? q : p;
      }
      const bool alive = in && p >= 0;
      if (cover) {
        uint16_t* d = in ? cand + i : sink;
        *d = (uint16_t)(st | (alive ? 0x8000 : 0));
        continue;
      }
      const unsigned long long bal = __ballot(alive);
      const int32_t n = (int32_t)__builtin_popcountll(bal);
      if (S + n > kF3SurvCap) {
        over = true;
        break;
      }
      uint16_t* d = alive ? s_start + S + (int32_t)__builtin_popcountll(bal & lt_mask) : sink;
      *d = (uint16_t)st;
      S += n;
    }
    if (cover) {
      lds_fence();
      // heads: alive and reached from no other survivor, compacted in position order
      for (int32_t i0 = 0; i0 < T; i0 += 64) {
        const int32_t i = i0 + lane;
        const int32_t v = i < T ? (int32_t)cand[i < T ? i : 0] : 0;
        const int32_t st = v & 0x7fff;
        const bool head = (v & 0x8000) && !((reached[st >> 5] >> (st & 31)) & 1u);
        const unsigned long long bal = __ballot(head);
        const int32_t n = (int32_t)__builtin_popcountll(bal);
        if (S + n > kF3SurvCap) {
          over = true;
          break;
        }
        uint16_t* d = head ? s_start + S + (int32_t)__builtin_popcountll(bal & lt_mask) : sink;
        *d = (uint16_t)st;
        S += n;
      }
    }
    if (!over) break;
    if (K >= 8) {
      fail(kF3Caps);
      return;
    }
    lds_fence();
  }
  lds_fence();
  mark(2);
  if (P.f3_stop == 2) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)

  // ---- 3 long walk: head `lane` to its exit (its first start at or past its chunk end), listing its
  //      starts in the chunk.  One wave-uniform loop while any head walks.  Every lane stores its p
  //      each step at its list's min(count, cap): a list has one spare slot past its cap, and a lane
  //      without a head stores to the sink, so no store needs a select or an exec-mask branch.  (Round
  //      5 walked on to the chunk end + LOOK, so that a false head dying there did not count; false
  //      heads are about 1 in 15 waves at C3's shape, and a chunk whose alive heads disagree is
  //      resolved from its entry all the same.) ----
  const bool hlane = lane < S;
  const int32_t hst = hlane ? (int32_t)s_start[hlane ? lane : 0] : 0;  // this lane's head
  int32_t hx = -1;                                                       // its exit (-1: died)
  int32_t hcnt = 0;                                                      // starts it lists
  {
    const int32_t e = chunk_end(hst >> cs);  // (<= de, and < ruse: every header below it is readable)
    uint16_t* my = hlane ? lists + lane * kF3Lstride : sink;
    int32_t p = hlane ? hst : -1;
    int32_t ex = -1;
    while (__ballot(p >= 0 && p < e)) {
      const bool go = p >= 0 && p < e;
      my[min(hcnt, kF3Lcap)] = (uint16_t)p;  // (a stopped lane's store lands past its count)
      hcnt += go ? 1 : 0;
      const int32_t q = f3_step<kNoDel>(rgn, max(p, 0), lim, mk, mv);
      ex = go && q >= e ? q : ex;
      p = go ? q : p;
    }
    hx = p >= 0 ? ex : -1;
    if (hlane) {
      s_exit[lane] = hx >= 0 ? (uint16_t)hx : (uint16_t)0xffff;
      s_cnt[lane] = (uint8_t)min(hcnt, 255);
    }
  }
  if (__ballot(hcnt > kF3Lcap)) {
    fail(kF3Caps);
    return;
  }
  lds_fence();
  mark(3);
  if (P.f3_stop == 3) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)

  // ---- 4 resolve, lane j = chunk j.  Heads are in position order: chunk j's are a contiguous run
  //      [c_first[j], c_last[j]].  A chunk whose alive heads all reach one exit is converged: its
  //      exit is known without its entry.  An entry is known from a converged predecessor, or from
  //      the predecessor's own entry (the head whose list holds it gives the exit); the frame's
  //      first entry is the previous wave's exit. ----
  uint8_t* c_first = reinterpret_cast<uint8_t*>(s_sel);
  uint8_t* c_last = c_first + 64;
  {
    if (lane < nw) c_first[lane] = 0xff;
    lds_fence();
    const int32_t hc = hlane ? (hst >> cs) : 127;
    const int32_t pc = wave_prev_i32(hc, -1), nc = wave_next_i32(hc, -1);
    uint8_t* df = hlane && (lane == 0 || pc != hc) ? c_first + hc : reinterpret_cast<uint8_t*>(sink);
    *df = (uint8_t)lane;
    uint8_t* dl = hlane && (lane == S - 1 || nc != hc) ? c_last + hc : reinterpret_cast<uint8_t*>(sink) + 1;
    *dl = (uint8_t)lane;
    lds_fence();
  }
  constexpr int32_t UNK = -2;
  int32_t hf = 0, hl = -1;  // this chunk's heads
  bool conv = false;
  int32_t cx = UNK;
  if (lane < nw) {
    const int32_t f = c_first[lane];
    if (f != 0xff) {
      hf = f;
      hl = c_last[lane];
    }
  }
  {
    // (the heads' exits by lane shuffles; a chunk's runs of heads are short: the loop runs to the
    //  longest, every lane on its own run with selects)
    const int32_t nh = hl - hf + 1;
    const int32_t nmax = __builtin_amdgcn_readlane(wave_incl_max_i32(nh), 63);
    bool any = false;
    conv = true;
    for (int32_t d = 0; d < nmax; d++) {
      const int32_t ex = __shfl(hx, min(hf + d, 63), 64);
      const bool use = d < nh && ex >= 0;
      conv = conv && (!use || !any || ex == cx);
      cx = use && !any ? ex : cx;
      any = any || use;
    }
    conv = conv && any;
  }
  // the head holding entry e of this chunk -> its exit (sel/at: head, index of e in its list); a
  // chunk entered at or past its end holds no record; -1: no head holds e
  auto find = [&](int32_t e, int32_t& sel, int32_t& at) -> int32_t {
    sel = -1;
    at = 0;
    if (e >= chunk_end(lane)) return e;
    for (int32_t g = hf; g <= hl; g++) {
      const int32_t st = s_start[g];
      if (st > e) break;
      if (s_exit[g] == 0xffff) continue;
      if (st == e) {
        sel = g;
        return s_exit[g];
      }
      const uint16_t* lg = lists + g * kF3Lstride;
      const int32_t n = min((int32_t)s_cnt[g], kF3Lcap);
      int32_t k = 1;
      while (k < n && (int32_t)lg[k] < e) k++;
      if (k < n && (int32_t)lg[k] == e) {
        sel = g;
        at = k;
        return s_exit[g];
      }
    }
    return -1;
  };
  // entries forward from whatever is known (converged chunks; chunk 0's entry e0 when given).  The
  // chunks resolved without e0 (pre = true) keep their result when e0 arrives or changes.
  int32_t ent = UNK, sel = -1, at = 0, myx = UNK;
  bool bad = false, pre = false;
  auto resolve = [&](int32_t e0) {
    if (!pre) {
      ent = lane == 0 ? e0 : UNK;
      myx = UNK;
      sel = -1;
      at = 0;
      bad = false;
    }
    for (;;) {
      if (lane < nw && myx == UNK && ent != UNK) {
        myx = find(ent, sel, at);
        if (myx < 0) bad = true;
      }
      const int32_t kx = myx >= 0 ? myx : (conv ? cx : UNK);
      const int32_t inx = wave_prev_i32(kx, UNK);
      const bool take = lane >= 1 && lane < nw && ent == UNK && inx != UNK;
      if (take) ent = inx;
      if (!__ballot(take || (lane < nw && myx == UNK && ent != UNK && !bad))) break;
    }
  };
  // early exit: the wave's exit known without the first entry
  resolve(UNK);
  pre = lane < nw && ent != UNK && !bad;
  int32_t early = -1;
  {
    const int32_t lastx = __builtin_amdgcn_readlane(myx >= 0 ? myx : (conv ? cx : UNK), nw - 1);
    if (wv > 0 && lastx >= 0) {
      early = lastx;
      if (lane == 0) granule_store(&P.exit_desc[wv], (unsigned long long)(R0 + early) | kReady);
    }
  }
  // the first entry: the previous wave's exit; with one alive head in chunk 0, speculatively its start
  int32_t spec_e0 = -1;
  {
    const int32_t h0f = __builtin_amdgcn_readfirstlane(hf), h0l = __builtin_amdgcn_readfirstlane(hl);
    const unsigned long long al = __ballot(hx >= 0 && lane >= h0f && lane <= h0l);
    if (wv > 0 && __builtin_popcountll(al) == 1) spec_e0 = __shfl(hst, (int)__builtin_ctzll(al), 64);
  }
  spec_e0 = __builtin_amdgcn_readfirstlane(spec_e0);
  bool spec = spec_e0 >= 0;
  int64_t ext = wv == 0 ? P.fr_entry : (spec ? R0 + spec_e0 : wait_prev());
  mark(4);
  if (P.f3_stop == 4) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)
  unsigned long long ndel = 0;
  uint32_t total = 0;
  unsigned long long base = 0;
  for (;;) {
    const int64_t e0 = ext - R0;
    resolve(e0 < 0 || e0 > 0x7fff ? UNK : (int32_t)e0);
    // every chunk resolved, and each exit the next chunk's entry
    const int32_t nxt = wave_next_i32(ent, UNK);
    const bool broken = lane < nw && (bad || myx < 0 || (lane + 1 < nw && nxt != myx));
    const int32_t wexit = __builtin_amdgcn_readlane(myx, nw - 1);
    if (__ballot(broken) || (early >= 0 && early != wexit)) {
      if (spec) {  // the guessed entry may be wrong: decide on the published one
        const int64_t real = wait_prev();
        spec = false;
        if (real != ext) {
          ext = real;
          continue;
        }
      }
      if (early < 0) fail(1u);
      else if (lane == 0) atomicOr(&P.st->spec_fail, 1u);
      return;
    }
    if (early < 0 && lane == 0) granule_store(&P.exit_desc[wv], (unsigned long long)(R0 + wexit) | kReady);
    if (lane == 0 && wv + 1 == (P.fr_nchunks + P.fr_w - 1) / P.fr_w) P.st->exit = R0 + wexit;
    // ---- counts: chunk `lane`'s records, their wave scan ----
    const int32_t scnt = __shfl(hcnt, max(sel, 0), 64);  // (every lane takes part in the shuffle)
    const uint32_t cnt = sel >= 0 ? (uint32_t)(scnt - at) : 0u;
    const uint32_t incl = wave_incl_sum_u32(cnt);
    total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (total > P.slab_cap) {
      if (spec) {
        const int64_t real = wait_prev();
        spec = false;
        if (real != ext) {
          ext = real;
          continue;
        }
      }
      if (lane == 0) {
        atomicMax(&P.st->max_wave_count, total);
        atomicOr(&P.st->overflow, 1u);
      }
      return;
    }
    if (lane == 0) P.wcount[wv] = total;
    // record r of the wave is entry r - base[j] of chunk j's chosen list (base: the scan of the
    // counts; the last chunk whose base is <= r, so empty chunks are passed over)
    const int32_t cbase = (int32_t)(incl - cnt);
    const int32_t csrc = sel >= 0 ? sel * kF3Lstride + at : 0;
    mark(5);
    if (P.f3_stop == 5) { stop(); return; }  // (SPARKEY_FRAME3_STOP: measurements)
    // Bucket regions: the entries leave as they are hashed, so a round redone after a wrong guess would
    // count twice.  With marks (f3_cover) the single head of chunk 0 can be a false start whose chain
    // joins the true one (the true start is then reached, not a head): the guess is checked first.
    // Without marks every survivor is a head and the true start always survives, so a single alive head
    // IS the true start of a log whose header holds: hash at once, and a mismatch (a header that lies)
    // fails the whole framing below, which the host redoes on k_frame.
    const bool spec_final = P.p1_bucket && spec && !cover;
    if (P.p1_bucket && spec && cover) {
      const int64_t real = wait_prev();
      spec = false;
      if (real != ext) {
        ext = real;
        continue;
      }
    }
    // ---- 5 hash: rounds of 64 records (a lane past the last record hashes the round's first one again
    //      and stores nothing) ----
    base = wv * (unsigned long long)P.slab_cap;
    ndel = 0;
    bool bovf = false;
    for (uint32_t r0 = 0; r0 < total; r0 += 64) {
      const uint32_t r = r0 + (uint32_t)lane;
      const bool act = r < total;
      int32_t src = 0;
      for (int j = 0; j < nw; j++) {  // (wave-uniform)
        const int32_t bj = __builtin_amdgcn_readlane(cbase, j);
        const int32_t sj = __builtin_amdgcn_readlane(csrc, j);
        if ((int32_t)r >= bj) src = sj + ((int32_t)r - bj);
      }
      const int32_t src0 = __builtin_amdgcn_readfirstlane(src);  // (lane 0's record: r0 < total)
      const uint32_t off = lists[act ? src : src0];
      // (listed records passed f3_step's rules on the walk that listed them: one-byte VLQs, PUT =
      //  klen + 1 then vlen, DELETE = 0 then klen; their keys lie in LDS, see RLEN)
      const uint32_t hb = rgn_u32(rgn, off);
      const int32_t b0 = (int32_t)(hb & 0xff), b1 = (int32_t)((hb >> 8) & 0xff);
      const bool put = b0 != 0;
      const int32_t klen = put ? b0 - 1 : b1;
      const RgnKey4 ld(rgn, off + 2u);
      const uint64_t hash = P.hash_size == 8 ? murmur64_ld(ld, klen, (uint32_t)P.seed)
                                             : (uint64_t)murmur32_ld(ld, klen, (uint32_t)P.seed);
      const int64_t p = R0 + (int64_t)off;
      uint64_t addr = (uint64_t)p << P.ebb;
      if (!put) {
        addr |= kDelBit;
        ndel += act ? 1 : 0;
      }
      Entry en;
      en.hash = hash;
      en.addr = addr;
      if (!P.p1_bucket) {
        if (act) P.ent[base + r] = en;
      } else {  // straight into the bucket's region (DELETEs stay out of the placement)
        const bool bput = act && put;
        const uint32_t b = bucket_of(P, hash);
        uint32_t a = 0;
        if (bput) a = atomicAdd(&P.bcount[b], 1u);
        if (bput) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          if (a < kPlaceLdsMax)
            __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(&en),
                                        reinterpret_cast<u32x4*>(&P.ent2[(uint64_t)b * kPlaceLdsMax + a]));
          else bovf = true;
        }
      }
    }
    if (bovf) atomicOr(&P.st->p2_overflow, 1u);
    if (spec) {  // check the guessed entry against the published exit; redo on a mismatch
      const int64_t real = wait_prev();
      spec = false;
      if (real != ext) {
        if (spec_final) {  // (the entries are out: the framing fails, see above)
          if (lane == 0) atomicOr(&P.st->spec_fail, 1u);
          return;
        }
        ext = real;
        continue;
      }
    }
    break;
  }
  ndel = wave_sum_u64(ndel);
  if (ndel && lane == 0) add_deletes(P, wv, ndel);
  mark(6);
  if (P.dbg && lane == 0) {
    P.dbg[wv * 16 + 8] = (unsigned long long)T;
    P.dbg[wv * 16 + 9] = (unsigned long long)S;
    P.dbg[wv * 16 + 10] = early >= 0 ? 0ull : 1ull;
  }
}

// One wave per workgroup, one region each: the waves share nothing, and each region's LDS is freed
// as soon as its wave ends (4-wave workgroups averaged 2.8 resident waves per SIMD of the 4 their
// LDS allowed, SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE).  Region i is workgroup i: a wave spins on its
// predecessor's exit, which the in-order dispatch has started before it (the spin is bounded all the
// same: the host redoes a framing whose wait ran out).  Builds that share the device take a ticket
// from one device-wide counter instead (fr_ticket): no wave then waits on one that is not resident.
// C3 10M on one box: one wave, no ticket 0.746 ms; 4 waves, ticket 0.856; 4 waves, no ticket 0.834;
// 8 waves 1.27.  Persistent waves that stage their next region while the current one
// finishes measured slower (round 5: 1.02-1.09 ms against 0.83).
template <bool kNoDel>
__global__ __launch_bounds__(64, kF3WavesPerSimd) void k_frame3(BuildParams P, uint32_t lds_per_wave) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint32_t tk = blockIdx.x;
  if (P.fr_ticket) {
    uint32_t t = 0;
    if (threadIdx.x == 0) t = atomicAdd(P.frame_ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  }
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  if (tk < nwaves) frame3_region<kNoDel>(P, tk, lds);
}

// LDS per wave: the staged region, then the scratch (candidates / record list, survivor data, lists
// or the screen bitmap).
uint32_t frame3_lds_per_wave(const BuildParams& P) {
  const size_t bitmap = (size_t)P.fr_w * (size_t)((std::min<int64_t>(1ll << P.fr_cshift, P.max_rec_len) + 63) / 64) * 8;
  const size_t reached = P.f3_cover ? (size_t)((((int64_t)P.fr_w << P.fr_cshift) + P.fr_look + 31) / 32 + 1) * 4 : 0;
  const size_t lists = (size_t)P.f3_surv_cap * (P.f3_lcap + 1) * 2;
  const size_t scratch =
      (size_t)f3_off_lists(P.f3_cand_cap, P.f3_surv_cap) + std::max<size_t>(std::max<size_t>(bitmap, reached), lists);
  return (uint32_t)(((size_t)P.f3_rgn + scratch + 15) & ~(size_t)15);
}

// The LDS layout of k_frame3 for this geometry (P.fr_w, fr_cshift, fr_look, f3_cover set): the region
// and the list caps.  The candidate cap is 2.2x the expected candidates of a wave (pass = the chance
// that a random byte pair passes the screen) plus 32, and at least 1.7x its expected records + 32;
// when that allows, it is trimmed so that as many workgroups as the VGPRs allow fit a CU.  False when the lists
// cannot hold what the header's mean record implies (k_frame frames such logs).
bool frame3_fits(BuildParams& P, double mean_record, double pass, double mean_short) {
  const double C = (double)(1ll << P.fr_cshift);
  if (!P.fr_fast || P.max_rec_len > 4096 || P.fr_cshift < 7) return false;
  if (mean_record <= 0.0 || C / mean_record > 0.6 * kF3LcapMax) return false;
  // a head's list: 16 starts while a chunk holds up to about 10 mean records, else 1 / 0.6 of its mean
  // records (long chunks: fewer, longer chains a wave)
  P.f3_lcap = C / mean_record <= 0.6 * 16 ? 16 : std::min(kF3LcapMax, ((int)std::ceil(C / mean_record / 0.6) + 7) & ~7);
  // and a chunk of the log's shorter records alone (the mean of its shorter kind, DELETEs or PUTs)
  if (mean_short > 0.0 && mean_short < mean_record)
    P.f3_lcap = std::max(P.f3_lcap, std::min(kF3LcapMax, ((int)std::ceil(C / mean_short) + 8 + 7) & ~7));
  const int64_t tail = std::max<int64_t>(P.fr_look, P.max_rec_len);  // (the keys of the last chunk's records)
  if (((int64_t)P.fr_w << P.fr_cshift) + tail + 16 >= 32768) return false;  // 15-bit region offsets
  P.f3_rgn = (int32_t)((((int64_t)P.fr_w << P.fr_cshift) + tail + 16 + 15) & ~15ll);
  const double recs = (double)P.fr_w * C / mean_record;
  const double false_cands = (double)P.fr_w * (double)std::min<int64_t>(1ll << P.fr_cshift, P.max_rec_len) * pass;
  if (recs > 0.6 * 512 || false_cands > 0.6 * 512) return false;
  const int need = std::min(512, (int)std::ceil(std::max(2.2 * (false_cands + P.fr_w) + 32.0, 1.7 * recs + 32.0)));
  // heads: about one per chunk plus a few false survivors; one long walk per lane
  P.f3_surv_cap = std::min(64, std::max(P.f3_lcap == 16 ? 32 : 16, (2 * P.fr_w + 8 + 7) & ~7));
  P.f3_cand_cap = 512;
  // the largest cap >= need (16-multiple) that keeps the most waves (up to kF3WavesPerSimd per SIMD) in
  // 160 KiB of LDS: workgroups of NW waves, + 16 B static each, in 512-byte allocation granules
  for (int wgs = 4 * kF3WavesPerSimd; wgs >= 1; wgs--)
    for (int cap = 512; cap >= need; cap -= 16) {
      P.f3_cand_cap = cap;
      const uint64_t wg = ((uint64_t)frame3_lds_per_wave(P) + 16 + 511) & ~511ull;
      if (wg * wgs <= 160 * 1024) return true;
    }
  P.f3_cand_cap = 512;  // (fewer waves per CU)
  return true;
}

void launch_frame3(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.fr_nchunks == 0) return;
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  const uint32_t per = frame3_lds_per_wave(P);
  hipLaunchKernelGGL(P.no_deletes ? k_frame3<true> : k_frame3<false>, dim3((unsigned)nwaves), dim3(64), (size_t)per, s, P,
                     per);
  tm->mark("frame", s);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.wcount, P.woff, P.nslabs, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
}

}  // namespace sk
