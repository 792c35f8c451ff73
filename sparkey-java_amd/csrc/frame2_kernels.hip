// frame2_kernels.hip -- k_frame2: framing + MurmurHash3 of logs whose records differ in size.
//
// The log is a chain of varint-framed records (SparkeyLogIterator.java:86-138): where a record
// starts depends on every record before it.  One wave owns a region of S segments of SEG bytes
// (SEG >= maxRecLen, so every segment but the frame's last holds a record start, and its first one
// lies within maxRecLen bytes of the segment start), staged once into LDS.
//
//   A  walkers    lane k (1 <= k < S) screens segment k's first maxRecLen bytes for plausible
//                 record starts (SWAR, 8 positions per step) and walks the chain of the first one
//                 that stays plausible up to the segment end, listing its record starts.  At the same
//                 time the lanes >= S take segment 0's candidate window one 8-byte word each and walk
//                 EVERY plausible candidate to segment 0's end.
//   B  segment 0  when all surviving candidates of segment 0 reach the same exit X, that exit holds
//                 for any entry the screen admits: the wave's chain is known without its entry.
//   C  chain      walker k's entry is walker k-1's exit (X for k = 1).  It is verified when it lies
//                 on walker k's listed chain (or is its exit); a walker whose speculative start missed
//                 is re-walked exactly from its entry.  The wave's exit (the last segment's) is then
//                 exact and is published at once for the next wave.
//   D  entry      segment 0 is walked exactly from the previous wave's published exit (a single
//                 surviving candidate is taken as that entry on speculation, checked at the end).
//                 Its exit must be X: otherwise the screen missed the true entry and the build reruns
//                 on the serial path (spec_fail).
//   E  hash       the verified record starts of all segments, every lane on every 64th record:
//                 MurmurHash3 of the key out of LDS (MurmurHash3.java:18-201), 16-byte
//                 (hash, address) entries in log order into the wave's slab.
//
// Compared with k_frame (fused_kernels.hip), only segment 0 of a wave walks every candidate; the
// other segments walk one chain each, so the speculative work is about one chain per segment.
// Waves are ordered by tickets (a wave waiting on its predecessor knows it is resident).
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

// One speculative step from region offset rp: the next record start, or -1 when the header there is
// not a plausible record (screen rules, key inside the log).
template <bool FAST>
__device__ __forceinline__ int32_t spec_step(const uint8_t* rgn, int64_t R0, int32_t rp, const BuildParams& P,
                                             int32_t lim, int32_t mk, int32_t mv) {
  if (FAST) {  // canonical one-byte VLQs only (keys < 127 bytes, values < 128 bytes)
    const uint64_t x = rgn_u64(rgn, (uint32_t)rp);
    const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
    const int32_t klen = b0 ? b0 - 1 : b1;
    const int32_t vlen = b0 ? b1 : 0;
    const bool ok = (x & 0x8080ull) == 0 && (b0 || !P.no_deletes) && klen <= mk && vlen <= mv && rp + 2 + klen <= lim;
    return ok ? rp + 2 + klen + vlen : -1;
  } else {
    const int64_t p = R0 + rp;
    const RecHdr h = decode_rgn(rgn, R0, p, (int64_t)P.log_len);
    if (!header_plausible(h, p, P.max_key_len, P.max_value_len, (int64_t)P.log_len) || (!h.put && P.no_deletes))
      return -1;
    return (int32_t)(record_end(h, p) - R0);
  }
}

}  // namespace

// One region (wave index wv) of k_frame2; its exit is published before any return.
template <bool FAST>
__device__ __forceinline__ void frame2_region(const BuildParams& P, const uint64_t wv, uint8_t* lds) {
  const int lane = threadIdx.x & 63;
  const int SS = P.fr_cshift;
  const int S = P.fr_w;
  const int LCAP = P.f2_lcap;
  const int64_t log_len = (int64_t)P.log_len;
  const int64_t fe = P.data_end;  // records are framed while they start below this
  const int64_t R0 = ((P.fr_entry >> SS) << SS) + (int64_t)wv * ((int64_t)S << SS);
  const int64_t RLEN = P.f2_rgn_bytes;  // staged bytes [R0, R0 + RLEN)
  uint8_t* rgn = lds;
  uint16_t* lists = reinterpret_cast<uint16_t*>(lds + RLEN);           // S x LCAP record starts (from R0)
  uint16_t* clist = lists + S * LCAP;                                   // the verified starts, compacted
  unsigned long long t_prev = P.dbg ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {  // diagnostic only: cycles per phase, per wave (no atomics)
    if (P.dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      P.dbg[wv * 16 + i] = t - t_prev;
      t_prev = t;
    }
  };

  // ---- stage [R0, R0 + RLEN): every 1 KiB row in flight at once, straight into LDS ----
  {
    const int nvec = (int)(RLEN >> 4);
    if (R0 + RLEN <= log_len) {
      const uint4* src = reinterpret_cast<const uint4*>(P.log + R0);
      for (int v0 = 0; v0 < nvec; v0 += 64)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + v0 + lane),
                                         (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16, 0,
                                         0);
      __builtin_amdgcn_s_waitcnt(0);
    } else {
      for (int v = lane; v < nvec; v += 64)
        *reinterpret_cast<uint4*>(rgn + 16u * v) = load16_guarded(P.log, R0 + 16ll * v, log_len);
    }
  }
  wave_sync();
  mark(0);

  const int64_t lim64 = log_len - R0;
  const int32_t lim = lim64 > 0x7fffffff ? 0x7fffffff : (int32_t)lim64;
  const int32_t mk = (int32_t)min(P.max_key_len, (int64_t)0x7fffffff), mv = (int32_t)min(P.max_value_len, (int64_t)0x7fffffff);
  const int32_t mrl = (int32_t)P.max_rec_len;
  const int64_t a0 = wv == 0 ? P.fr_entry : R0;                  // segment 0
  const int64_t b0 = min(R0 + (1ll << SS), fe);
  const bool walker = lane >= 1 && lane < S && R0 + ((int64_t)lane << SS) < fe;
  const int64_t a = R0 + ((int64_t)lane << SS);                  // (walkers) segment `lane`
  const int64_t b = min(R0 + ((int64_t)(lane + 1) << SS), fe);
  uint16_t* my = lists + (walker ? lane : 0) * LCAP;

  // ---- A: walkers (first chain that stays plausible) and segment 0's candidates (every one) ----
  const Screen8 scr = make_screen8(P);
  const int nwords0 = (mrl + 7) >> 3;                              // segment 0's candidate window in words
  const int ncl = 64 - S;                                          // candidate lanes
  int64_t xk = -1;                                                 // walker: exit of its chain
  int32_t m = 0;                                                   // walker: records listed
  bool found = false;
  unsigned long long nsurv = 0, exmin = ~0ull, cmin = ~0ull;
  long long exmax = -1;
  // One flat loop, one step per lane per iteration (no nested per-lane loops for the wave to run
  // through one after another): a lane either screens its next 8-byte word or takes its next
  // candidate, or advances its walk by one record.  Region offsets in 32 bits.
  const uint64_t* r64 = reinterpret_cast<const uint64_t*>(rgn);
  int32_t wpos = 0, wend = 0, rb = 0, pass = 0;
  if (walker) {
    wpos = (int32_t)(a - R0);
    wend = wpos + mrl;
    rb = (int32_t)(b - R0);
  } else if (lane >= S && wv > 0 && lane - S < nwords0) {
    wpos = (int32_t)(a0 - R0) + 8 * (lane - S);
    wend = min(wpos + 8, (int32_t)(a0 - R0) + mrl);
    rb = (int32_t)(b0 - R0);
  }
  bool done = wpos >= wend;
  uint32_t msk = 0;
  int32_t wbase = 0, rp = -1, cs = 0, cnt = 0;
  uint32_t iters = 0;
  for (;;) {
    iters++;
    if (!done && rp < 0) {
      if (msk == 0 && wpos >= wend && !walker) {  // a candidate lane's next word
        const int wi = (lane - S) + (++pass) * ncl;
        if (wi < nwords0) {
          wpos = (int32_t)(a0 - R0) + 8 * wi;
          wend = min(wpos + 8, (int32_t)(a0 - R0) + mrl);
        }
      }
      if (msk == 0) {
        if (wpos >= wend) {
          done = true;
        } else {  // screen one word (windows start 8-byte aligned)
          const uint64_t x = r64[wpos >> 3], x2 = r64[(wpos >> 3) + 1];
          msk = screen8(x, (x >> 8) | (x2 << 56), scr);
          if (wpos + 8 > wend) msk &= (1u << (uint32_t)(wend - wpos)) - 1u;
          wbase = wpos;
          wpos += 8;
        }
      }
      if (msk) {
        cs = wbase + __builtin_ctz(msk);
        msk &= msk - 1;
        rp = cs;
        cnt = 0;
      }
    }
    if (!__any(!done)) break;
    if (rp >= 0) {
      if (rp >= rb) {  // the chain from cs stayed plausible to the walk bound
        if (walker) {
          found = true;
          xk = R0 + rp;
          m = cnt;
          done = true;
        } else {
          nsurv++;
          exmin = min(exmin, (unsigned long long)(R0 + rp));
          exmax = max(exmax, (long long)(R0 + rp));
          cmin = min(cmin, (unsigned long long)(R0 + cs));
        }
        rp = -1;
      } else if (walker && cnt == LCAP) {  // more starts than a segment lists: not taken
        rp = -1;
      } else {
        if (walker) my[cnt] = (uint16_t)rp;
        cnt++;
        rp = spec_step<FAST>(rgn, R0, rp, P, lim, mk, mv);
      }
    }
  }
  mark(1);

  // ---- B: segment 0's exit, when its surviving candidates agree ----
  unsigned long long ns0 = wave_sum_u64(nsurv);
  unsigned long long xmin0 = exmin, cmin0 = cmin;
  long long xmax0 = exmax;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    xmin0 = min(xmin0, (unsigned long long)__shfl_xor(xmin0, o, 64));
    cmin0 = min(cmin0, (unsigned long long)__shfl_xor(cmin0, o, 64));
    xmax0 = max(xmax0, (long long)__shfl_xor(xmax0, o, 64));
  }
  // the previous wave's published exit (lane 0 spins, bounded), broadcast
  auto wait_prev = [&]() -> int64_t {
    unsigned long long extv = (unsigned long long)P.fr_entry;
    if (wv > 0 && lane == 0) {
      const unsigned long long t0 = wall_clock64();
      for (;;) {
        const unsigned long long v = granule_load(&P.exit_desc[wv - 1]);
        if (v & kReady) { extv = v & ~kReady; break; }
        if (wall_clock64() - t0 >= P.fr_spin_ticks) {  // bounded all the same: serial path
          atomicOr(&P.st->spec_fail, 2u);
          extv = (unsigned long long)a0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    return (int64_t)__shfl(extv, 0, 64);
  };
  auto at_glb = [&](int64_t q) -> uint32_t { return (uint32_t)P.log[q]; };
  auto hdr_at = [&](int64_t q) -> RecHdr {
    return q + 16 <= R0 + RLEN ? decode_rgn(rgn, R0, q, log_len) : decode_header(at_glb, q, log_len);
  };
  bool bad = false;
  // exact walk (the reference iterator's rules) of [from, end): lists the starts into `lst`, returns
  // the exit (the first start >= end), or sets the error on an invalid record
  auto exact_walk = [&](int64_t from, int64_t end, uint16_t* lst, int32_t& cnt) -> int64_t {
    int64_t q = from;
    cnt = 0;
    while (q < end) {
      const RecHdr h = hdr_at(q);
      if (!header_valid(h, q, P.max_key_len, log_len)) {
        set_error(P.st, q, h.rc ? h.rc : kErrCorruptRecord);
        bad = true;
        return end;
      }
      if (cnt < LCAP) lst[cnt] = (uint16_t)(q - R0);
      cnt++;
      q = record_end(h, q);
    }
    return q;
  };

  // segment 0: exact from the frame entry in wave 0; otherwise its exit X is known when the
  // candidates converged, else only from the entry
  int64_t X = 0, e0 = 0;
  bool seg0_done = false;
  int32_t m0 = 0;
  // (a segment 0 cut short by the frame end may hold no record start at all: its entry can be the
  // frame end itself, which no candidate screen sees -- it takes the entry)
  if (wv == 0 || b0 < R0 + (1ll << SS) || !(ns0 > 0 && (long long)xmin0 == xmax0)) {
    e0 = wv == 0 ? P.fr_entry : wait_prev();
    int64_t x0 = 0;
    if (lane == 0) x0 = exact_walk(e0, b0, lists, m0);
    X = __shfl(x0, 0, 64);
    m0 = __shfl(m0, 0, 64);
    seg0_done = true;
  } else {
    X = (int64_t)xmin0;
  }

  // ---- C: the walkers' entries along the wave, verified; misses re-walked exactly ----
  int32_t i0 = 0;  // (walkers) index of the verified entry in the list
  bool ok = false;
  auto verify = [&](int64_t e) {
    ok = false;
    if (!walker) return;
    if (found) {
      if (e == xk) { i0 = m; ok = true; return; }
      const int32_t er = (int32_t)(e - R0);
      const int32_t n = min(m, LCAP);
      for (int32_t i = 0; i < n; i++) {
        const int32_t v = (int32_t)my[i];
        if (v >= er) {
          if (v == er) { i0 = i; ok = true; }
          return;
        }
      }
    }
  };
  {
    int64_t xv = lane == 0 ? X : xk;
    int64_t e = __shfl_up(xv, 1, 64);
    verify(e);
    for (;;) {
      const unsigned long long fail = __ballot(walker && !ok);
      if (!fail) break;
      const int j = __builtin_ctzll(fail);
      if (lane == j) {
        xk = exact_walk(e, b, my, m);
        i0 = 0;
        found = true;
        ok = true;
      }
      xv = lane == 0 ? X : xk;
      const int64_t e2 = __shfl_up(xv, 1, 64);
      if (lane > j) {
        e = e2;
        verify(e);
      }
    }
  }
  // the wave's exit: the last active segment's
  const int last = (int)min((int64_t)S - 1, ((fe - 1 - R0) >> SS));
  const int64_t wexit = __shfl(lane == 0 ? X : xk, last, 64);
  if (lane == 0) {
    granule_store(&P.exit_desc[wv], (unsigned long long)wexit | kReady);
    if (wv + 1 == (P.fr_nchunks + P.fr_w - 1) / P.fr_w) P.st->exit = wexit;
  }
  mark(2);

  // ---- D + E: segment 0 from its entry, then every verified record hashed into the slab ----
  bool spec = !seg0_done && ns0 == 1;
  if (!seg0_done) e0 = spec ? (int64_t)cmin0 : wait_prev();
  unsigned long long ndel = 0;
  for (;;) {
    if (!seg0_done) {
      int64_t x0 = 0;
      if (lane == 0) x0 = exact_walk(e0, b0, lists, m0);
      x0 = __shfl(x0, 0, 64);
      m0 = __shfl(m0, 0, 64);
      seg0_done = true;
      if (x0 != X) {
        if (spec) {  // the guessed entry was not the entry
          spec = false;
          e0 = wait_prev();
          seg0_done = false;
          continue;
        }
        if (lane == 0) atomicOr(&P.st->spec_fail, 1u);  // the screen missed the real entry's chain
        return;
      }
    }
    // every list complete (segment 0's included): else the host redoes the build with k_frame
    const bool lovf = __any((walker && m > LCAP) || (lane == 0 && m0 > LCAP));
    if (lovf || __any(bad)) {
      if (lane == 0 && lovf) atomicOr(&P.st->spec_fail, 16u);
      return;
    }
    const uint32_t cnt = lane == 0 ? (uint32_t)m0 : (walker ? (uint32_t)(m - i0) : 0u);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    if (total > P.slab_cap) {
      if (spec) {  // the guessed entry may be wrong: decide on the published one
        const int64_t real = wait_prev();
        spec = false;
        if (real != e0) {
          e0 = real;
          seg0_done = false;
          continue;
        }
      }
      if (lane == 0) {
        atomicMax(&P.st->max_wave_count, total);
        atomicOr(&P.st->overflow, 1u);
      }
      return;
    }
    {  // each segment's verified starts to their place in the wave's list
      const uint32_t o = incl - cnt;
      const uint16_t* src = lane == 0 ? lists : my + i0;
      for (uint32_t i = 0; i < cnt; i++) clist[o + i] = src[i];
    }
    if (lane == 0) P.wcount[wv] = total;
    wave_sync();
    mark(3);
    const unsigned long long base = wv * (unsigned long long)P.slab_cap;
    ndel = 0;
    const uint32_t span = (uint32_t)S << SS;
    for (uint32_t r = (uint32_t)lane; r < total; r += 64) {
      const uint32_t off = clist[r];
      if (off >= span) {  // (cannot happen: every listed start lies in the wave's segments)
        atomicOr(&P.st->spec_fail, 32u);
        continue;
      }
      const int64_t p = R0 + (int64_t)off;
      const RecHdr h = hdr_at(p);
      const int64_t kp = p + h.hlen;
      uint64_t hash;
      if (kp + h.klen + 16 <= R0 + RLEN) {  // key in the region
        const RgnKey ld{rgn, (uint32_t)(kp - R0)};
        hash = P.hash_size == 8 ? murmur64_ld(ld, h.klen, (uint32_t)P.seed) : (uint64_t)murmur32_ld(ld, h.klen, (uint32_t)P.seed);
      } else if (kp + h.klen + 16 <= log_len) {
        const GlobalKey ld{P.log + kp};
        hash = P.hash_size == 8 ? murmur64_ld(ld, h.klen, (uint32_t)P.seed) : (uint64_t)murmur32_ld(ld, h.klen, (uint32_t)P.seed);
      } else {
        hash = key_hash(P.hash_size, P.log + kp, h.klen, (uint32_t)P.seed);
      }
      uint64_t addr = (uint64_t)p << P.ebb;
      if (!h.put) {
        addr |= kDelBit;
        ndel++;
      }
      Entry en;
      en.hash = hash;
      en.addr = addr;
      P.ent[base + r] = en;
    }
    if (spec) {  // check the guessed entry against the published exit; redo on a mismatch
      const int64_t real = wait_prev();
      spec = false;
      if (real != e0) {
        e0 = real;
        seg0_done = false;
        wave_sync();  // (the list is rewritten)
        continue;
      }
    }
    break;
  }
  ndel = wave_sum_u64(ndel);
  if (ndel && lane == 0) add_deletes(P, wv, ndel);
  mark(4);
  if (P.dbg && lane == 0) {
    P.dbg[wv * 16 + 9] = ns0;
    P.dbg[wv * 16 + 8] = iters;
  }
}

// One wave per workgroup, region = workgroup id, as k_frame (fused_kernels.hip); TICKET: the 4-wave
// ticket launch (SPARKEY_FRAME_TICKET).
template <bool FAST, int NW, bool TICKET>
__global__ __launch_bounds__(64 * NW, 5) void k_frame2(BuildParams P, uint32_t lds_per_wave) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint32_t tk = blockIdx.x;
  if (TICKET) {
    __shared__ unsigned int s_tk;
    if (threadIdx.x == 0) s_tk = atomicAdd(P.frame_ticket, 1u);
    __syncthreads();
    tk = s_tk;
  }
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  const uint32_t w = threadIdx.x >> 6;
  const uint64_t wv = (uint64_t)tk * NW + w;
  if (wv < nwaves) frame2_region<FAST>(P, wv, lds + w * lds_per_wave);
}

void launch_frame2(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.fr_nchunks == 0) return;
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  const size_t lds = (size_t)P.f2_rgn_bytes + 2 * (size_t)P.fr_w * P.f2_lcap * 2;
  const uint32_t per = (uint32_t)((lds + 15) & ~(size_t)15);
  if (getenv("SPARKEY_FRAME_TICKET")) {
    const dim3 grid((unsigned)((nwaves + kFrameWaves - 1) / kFrameWaves)), block(64 * kFrameWaves);
    if (P.fr_fast) hipLaunchKernelGGL((k_frame2<true, kFrameWaves, true>), grid, block, (size_t)per * kFrameWaves, s, P, per);
    else hipLaunchKernelGGL((k_frame2<false, kFrameWaves, true>), grid, block, (size_t)per * kFrameWaves, s, P, per);
  } else {
    const dim3 grid((unsigned)nwaves), block(64);
    if (P.fr_fast) hipLaunchKernelGGL((k_frame2<true, 1, false>), grid, block, (size_t)per, s, P, per);
    else hipLaunchKernelGGL((k_frame2<false, 1, false>), grid, block, (size_t)per, s, P, per);
  }
  tm->mark("frame", s);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.wcount, P.woff, P.nslabs, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
}

}  // namespace sk
