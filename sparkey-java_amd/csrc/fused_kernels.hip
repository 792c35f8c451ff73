// fused_kernels.hip -- the fast path of the .spi build on gfx950.
//
//   k_frame          ONE pass over the log: a wave owns 64 small chunks (lane = chunk):
//                    speculative framing -> wave exit published at once -> entry from the previous
//                    wave's exit -> MurmurHash3 of every key out of LDS -> (hash, address) entries
//                    in log order into the wave's slab.
//   k_frame_uniform  the same for logs whose header proves one record size (stride framing), also
//                    partition pass 1 into fixed per-digit regions.
//   k_part1_regions  partition pass 1 of the speculative framings' slabs into the digit regions
//                    (digit = the top 8 bits of the bucket id, bucket = wantedSlot >> 10).
//   k_part1_hist/    the two-pass partition (histogram, then LDS-staged scatter) for the serial walk's
//   k_part1_scatter  dense entries and for hash distributions that overflow a digit region.
//   k_part2st/s/d/   one workgroup per coarse digit: fine split into buckets (st/s: fixed bucket
//   k_part2          regions, slot counts and carry functions in the same pass; d: dense, staged).
//   k_place_reg      per bucket, entries in registers: counting sort by wanted slot, address order
//                    inside equal slots, canonical positions, every slot of the bucket written once.
//
// The only inter-workgroup hand-off in k_frame (a wave's exit -> the next wave's entry) uses 8-byte
// granules that carry their own state bits
// (MI355X_MICROARCH.md "Valid forms", R2: the data IS the flag) with relaxed agent-scope atomic
// loads/stores; every granule is zeroed before the launch and every spin is time-bounded.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"
#include "place_common.hpp"
#include "frame_common.hpp"
#include "knobs.hpp"

namespace sk {

// ================================================================================================
// k_frame: one wave owns W consecutive chunks of C = 2^fr_cshift bytes (lane j owns chunk k0 + j),
// staged contiguously in one XOR-swizzled LDS region together with fr_look + 16 bytes past the
// last chunk.  C >= maxRecLen, so every chunk but a short last one holds a record start, and its
// first one lies within maxRecLen bytes of the chunk start.
//   1 screen    every candidate start in [s, s + maxRecLen): 8 at a time from one u64, all lanes
//   2 walk      screened candidates in lock step, past the chunk end up to fr_look more bytes (the
//               next chunks' bytes are in the same region): a false start rarely stays plausible
//               that long.  exit = first record start >= chunk end on the chain.
//   3 entries   a chunk whose surviving chains share one exit knows it without its entry; the
//               wave's last exit is published at once, the first entry is the previous wave's
//               published exit, unresolved chunks are walked in order
//   4 counts    record counts and their wave scan: offsets inside the wave's slab of entries
//   5 hash      every lane walks its chunk from the verified entry and hashes each key from LDS
// ================================================================================================
// Balanced-walk candidate record: start (14 bits, region offset) | exit - chunk end (8) | steps to
// the exit (9) | survived (1).  The walk only runs with canonical one-byte VLQs (fr_fast), so a
// record is < 256 bytes and exit - chunk end always fits.  A survivor whose steps do not fit is
// recorded with steps = 511 and no survived bit: its chunk is then treated as unconverged and walked
// exactly in the entry phase (a dead candidate has steps 0).
constexpr uint32_t kCandOverflow = 511u;
__device__ __forceinline__ uint32_t pack_cand(int32_t start, int32_t dexit, int32_t steps) {
  if (steps >= (int32_t)kCandOverflow || dexit > 255) return (uint32_t)start | (kCandOverflow << 22);
  return (uint32_t)start | ((uint32_t)dexit << 14) | ((uint32_t)steps << 22) | 0x80000000u;
}
__device__ __forceinline__ uint32_t cand_start(uint32_t v) { return v & 0x3fffu; }
__device__ __forceinline__ uint32_t cand_dexit(uint32_t v) { return (v >> 14) & 0xffu; }
__device__ __forceinline__ int32_t cand_steps(uint32_t v) { return (int32_t)((v >> 22) & 0x1ffu); }

// One region (wave index wv) of k_frame; returns once its entries are in the slab (its exit was
// published before any return).
__device__ __forceinline__ void frame_region(const BuildParams& P, const uint64_t wv, uint8_t* lds) {
  const int lane = threadIdx.x & 63;
  const int cs = P.fr_cshift;
  const int64_t C = 1ll << cs;
  const int W = P.fr_w;
  const int64_t LOOK = P.fr_look;
  const int64_t log_len = (int64_t)P.log_len;
  const uint64_t kf = P.fr_k0;  // chunk of the framing entry
  const uint64_t k0 = kf + wv * (uint64_t)W;
  const int nw = (int)min((uint64_t)W, kf + P.fr_nchunks - k0);
  const int64_t R0 = (int64_t)(k0 << cs);
  const int64_t RLEN = ((int64_t)nw << cs) + LOOK + 16;  // staged bytes [R0, R0 + RLEN)
  const int64_t RUSE = R0 + RLEN - 16;                     // headers decodable in LDS below this
  uint8_t* rgn = lds;
  unsigned long long t_prev = P.dbg ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {  // diagnostic only: cycles per phase, per wave (no atomics)
    if (P.dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      P.dbg[wv * 16 + i] = t - t_prev;
      t_prev = t;
    }
  };

  // ---- stage: [R0, R0 + RLEN) once, coalesced, 16 bytes per lane per step ----
  {
    const int nvec = (int)((RLEN + 15) >> 4);
    if (R0 + 16ll * nvec <= log_len) {
      // every load of the region in flight at once, straight into LDS (global_load_lds_dwordx4:
      // 1 KiB per wave instruction at rgn + 1024 i; fr_rgn_bytes is a multiple of 1 KiB, lanes past
      // the end repeat the last vector)
      const uint4* src = reinterpret_cast<const uint4*>(P.log + R0);
      if (P.uni_nt) {  // non-temporal: the log is read once
        for (int v0 = 0; v0 < nvec; v0 += 64)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(src + min(v0 + lane, nvec - 1)),
              (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16, 0, 2);
      } else {
        for (int v0 = 0; v0 < nvec; v0 += 64)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(src + min(v0 + lane, nvec - 1)),
              (__attribute__((address_space(3))) void*)(rgn + 16u * (uint32_t)v0), 16, 0, 0);
      }
    } else {
      for (int v = lane; v < nvec; v += 64) {
        const uint4 val = load16_guarded(P.log, R0 + 16ll * v, log_len);
        *reinterpret_cast<uint4*>(rgn + 16u * v) = val;
      }
    }
  }
  wave_sync();
  mark(0);

  const bool act = lane < nw;
  const uint64_t k = k0 + lane;
  const int64_t wb = (int64_t)(k << cs);
  const int64_t s = (k == kf) ? P.fr_entry : wb;
  const int64_t e = act ? min(wb + C, P.data_end) : wb;
  const int64_t stop = min(min(e + LOOK, P.data_end), RUSE);  // speculative walks end here
  const bool passthrough = k > kf && s + P.max_rec_len - 1 >= e;
  const int64_t cand_end = !act || passthrough ? s : (k == kf ? s + 1 : min(e, s + P.max_rec_len));

  // ---- 1 screen: one flag bit per byte of the wave's chunks (is it a plausible record start?),
  //      lanes on consecutive 8-byte words, 8 positions per SWAR step; a chunk's mask words are
  //      then its slice of the bitmap.  Masks stay in registers when maxRecLen <= 128. ----
  const int nwl = (int)((min(C, P.max_rec_len) + 63) >> 6);
  unsigned long long* flags = reinterpret_cast<unsigned long long*>(lds + P.fr_rgn_bytes);
  {
    constexpr uint64_t H = 0x8080808080808080ull, L7 = 0x7f7f7f7f7f7f7f7full, ONES = 0x0101010101010101ull;
    // per byte: b <= T with b < 128 (T >= 127: every byte); thresholds replicated once, outside the loop
    const int64_t TK = P.max_key_len + 1 >= 128 ? 127 : P.max_key_len + 1;
    const bool allk = P.max_key_len + 1 >= 128, allv = P.max_value_len >= 127, alld = P.max_key_len >= 127;
    const uint64_t rk = ONES * (uint64_t)(min(TK, (int64_t)126) + 1);
    const uint64_t rv = ONES * (uint64_t)(min(P.max_value_len, (int64_t)126) + 1);
    const uint64_t rd = ONES * (uint64_t)(min(P.max_key_len, (int64_t)126) + 1);
    auto le_rep = [&](uint64_t x, uint64_t rep, bool all) -> uint64_t { return all ? H : ~(x | ((x | H) - rep)) & H; };
    const uint64_t* r64 = reinterpret_cast<const uint64_t*>(rgn);
    uint8_t* fb = reinterpret_cast<uint8_t*>(flags);
    // only each chunk's candidate window [chunk start, + nwl * 64) is screened: byte q of the
    // bitmap = word q % wpc of chunk q / wpc
    const int wpc = nwl * 8;
    const int nq = nw * wpc;
    for (int q = lane; q < nq; q += 64) {
      const int j = (int)(((uint32_t)q * P.fr_wpc_magic) >> 22);  // q / wpc (exact, checked on the host)
      const int rw = (j << (cs - 3)) + (q - j * wpc);
      const uint64_t x = r64[rw];
      const uint64_t y = (x >> 8) | (r64[rw + 1] << 56);
      const uint64_t z = ~(((x & L7) + L7) | x) & H;  // zero bytes
      const uint64_t put_first = le_rep(x, rk, allk) & ~z;
      // a log whose header counts no DELETE has none on its true chain: 0x00 starts no record
      const uint64_t r = (put_first & le_rep(y, rv, allv)) | (P.no_deletes ? 0ull : (z & le_rep(y, rd, alld)));
      // gather the 8 flags (bits 7, 15, ..., 63) into one byte: bit 8i -> bit 56 + i, no carries
      fb[q] = (uint8_t)((((r >> 7) & ONES) * 0x0102040810204080ull) >> 56);
    }
  }
  wave_sync();
  // mask word wi of this lane's chunk: bit i = candidate start s + 64 wi + i
  auto masked_word = [&](int wi) -> unsigned long long {
    if (k == kf) return (wi == 0 && cand_end > s) ? 1ull : 0ull;  // the entry chunk: its only start is the entry
    const int64_t cw = s + 64ll * wi;
    if (cw >= cand_end) return 0ull;
    unsigned long long word = flags[(uint32_t)lane * (uint32_t)nwl + (uint32_t)wi];
    const int64_t valid = cand_end - cw;
    if (valid < 64) word &= (1ull << valid) - 1ull;
    return word;
  };
  unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0;  // masks in registers when nwl <= 4
  if (nwl <= 4) {
    m0 = masked_word(0);
    m1 = nwl > 1 ? masked_word(1) : 0ull;
    m2 = nwl > 2 ? masked_word(2) : 0ull;
    m3 = nwl > 3 ? masked_word(3) : 0ull;
  }
  auto mask_word = [&](int wi) -> unsigned long long {
    if (nwl > 4) return masked_word(wi);
    return wi == 0 ? m0 : wi == 1 ? m1 : wi == 2 ? m2 : m3;
  };
  mark(1);

  // ---- 2 walk the screened candidates in lock step (one header per lane per step) ----
  unsigned long long nsurv = 0, min_exit = ~0ull, c_min = ~0ull;
  long long max_exit = -1;
  int32_t c_min_steps = 0;
  unsigned long long dbg_iters = 0;
  // Balanced walk (C = 128, masks in registers, canonical one-byte VLQs): the wave's candidates go
  // to one LDS list and lane L walks candidates L, L + 64, ..., so the walk takes about the mean
  // work per lane instead of the largest; each lane then folds its own chunk's results.
  // cand[i]: see pack_cand.
  bool balanced = false;
  bool unenc = false;  // a survivor of this chunk did not fit its candidate record
  uint32_t my_cpre = 0, my_ccnt = 0;
  if (P.fr_fast && nwl <= 4 && RLEN < 16384) {
    uint32_t* cand = reinterpret_cast<uint32_t*>(lds + P.fr_rgn_bytes);
    const bool has = act && cand_end > s;
    const uint32_t cnt_c = has ? (uint32_t)(__builtin_popcountll(m0) + __builtin_popcountll(m1) +
                                            __builtin_popcountll(m2) + __builtin_popcountll(m3))
                               : 0u;
    uint32_t incl = cnt_c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const uint32_t T = __shfl(incl, 63, 64);
    const uint32_t cpre = incl - cnt_c;
    my_cpre = cpre;
    my_ccnt = cnt_c;
    if (T <= (uint32_t)kCandCap) {
      balanced = true;
      wave_sync();  // every lane holds its masks: the list may overwrite the bitmap
      {  // enumerate: lane's candidates in ascending order at cand[cpre ..)
        unsigned long long a0 = has ? m0 : 0ull, a1 = has ? m1 : 0ull, a2 = has ? m2 : 0ull, a3 = has ? m3 : 0ull;
        uint32_t o = cpre;
        const uint32_t base = (uint32_t)(s - R0);
        while (__any((a0 | a1 | a2 | a3) != 0ull)) {
          if (a0) {
            cand[o++] = base + (uint32_t)__builtin_ctzll(a0);
            a0 &= a0 - 1;
          } else if (a1) {
            cand[o++] = base + 64u + (uint32_t)__builtin_ctzll(a1);
            a1 &= a1 - 1;
          } else if (a2) {
            cand[o++] = base + 128u + (uint32_t)__builtin_ctzll(a2);
            a2 &= a2 - 1;
          } else if (a3) {
            cand[o++] = base + 192u + (uint32_t)__builtin_ctzll(a3);
            a3 &= a3 - 1;
          }
        }
      }
      wave_sync();
      const int64_t lim64 = log_len - R0;
      const int32_t lim = lim64 > 0x7fffffff ? 0x7fffffff : (int32_t)lim64;
      const int32_t de = (int32_t)min((int64_t)0x7fffffff, P.data_end - R0);
      const int32_t ruse = (int32_t)(RUSE - R0);
      const int32_t mk = (int32_t)P.max_key_len, mv = (int32_t)P.max_value_len;
      const int32_t look = (int32_t)LOOK;
      uint32_t gi = (uint32_t)lane, cur = 0;
      int32_t rp = -1, rst = 0, rex = -1, st = 0, re = 0, rstop = 0;
      for (;;) {
        if (rp < 0 && gi < T) {
          cur = gi;
          gi += 64;
          rst = (int32_t)cand[cur];
          rp = rst;
          rex = -1;
          st = 0;
          re = min((((rst >> cs) + 1) << cs), de);
          rstop = min(min(re + look, de), ruse);
        }
        if (!__any(rp >= 0)) break;
        dbg_iters++;
        if (rp >= 0) {
          const uint64_t x = rgn_u64(rgn, (uint32_t)rp);
          const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
          const int32_t klen = b0 ? b0 - 1 : b1;
          const int32_t vlen = b0 ? b1 : 0;
          const bool ok = (x & 0x8080ull) == 0 && (b0 || !P.no_deletes) && klen <= mk && vlen <= mv &&
                          rp + 2 + klen <= lim;
          if (!ok) {
            rp = -1;  // dead: cand[cur] keeps its bare start
          } else {
            if (rex < 0) st++;
            rp += 2 + klen + vlen;
            if (rex < 0 && rp >= re) rex = rp;
            if (rp >= rstop) {
              cand[cur] = pack_cand(rst, rex - re, st);
              rp = -1;
            }
          }
        }
      }
      wave_sync();
      // fold the lane's own chunk
      for (uint32_t i = 0; i < cnt_c; i++) {
        const uint32_t v = cand[cpre + i];
        if (!(v & 0x80000000u) && cand_steps(v) == (int32_t)kCandOverflow) unenc = true;
        if (v & 0x80000000u) {
          const uint32_t st0 = cand_start(v);
          const unsigned long long pe = (unsigned long long)(e + cand_dexit(v));
          if (nsurv == 0) {
            c_min = (unsigned long long)(R0 + st0);
            c_min_steps = cand_steps(v);
          }
          nsurv++;
          min_exit = min(min_exit, pe);
          max_exit = max(max_exit, (long long)pe);
        }
      }
    }
  }
  if (!balanced) {
    int wi = 0;
    unsigned long long m = (act && cand_end > s) ? mask_word(0) : 0ull;
    bool done = !act || cand_end <= s;
    int32_t steps = 0;
    if (P.fr_fast) {
      // canonical one-byte VLQs only (keys < 127 bytes, values < 128 bytes): region offsets in
      // 32 bits, no generic decoder in the loop
      const int32_t re = (int32_t)(e - R0), rstop = (int32_t)(stop - R0);
      const int64_t lim64 = log_len - R0;
      const int32_t lim = lim64 > 0x7fffffff ? 0x7fffffff : (int32_t)lim64;
      const int32_t mk = (int32_t)P.max_key_len, mv = (int32_t)P.max_value_len;
      int32_t rp = -1, rst = 0, rex = 0;
      for (;;) {
        if (!done && rp < 0) {
          while (m == 0 && ++wi < nwl) m = mask_word(wi);
          if (m == 0) {
            done = true;
          } else {
            rst = (int32_t)(s - R0) + 64 * wi + __builtin_ctzll(m);
            m &= m - 1;
            rp = rst;
            rex = -1;
            steps = 0;
          }
        }
        if (__all(done)) break;
        dbg_iters++;
        if (!done) {
          const uint64_t x = rgn_u64(rgn, (uint32_t)rp);
          const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
          const int32_t klen = b0 ? b0 - 1 : b1;
          const int32_t vlen = b0 ? b1 : 0;
          const bool ok = (x & 0x8080ull) == 0 && (b0 || !P.no_deletes) && klen <= mk && vlen <= mv &&
                          rp + 2 + klen <= lim;
          if (!ok) {
            rp = -1;
          } else {
            if (rex < 0) steps++;
            rp += 2 + klen + vlen;
            if (rex < 0 && rp >= re) rex = rp;
            if (rp >= rstop) {  // survived the look-ahead: a candidate entry
              const unsigned long long pe = (unsigned long long)(R0 + rex);
              nsurv++;
              min_exit = min(min_exit, pe);
              max_exit = max(max_exit, (long long)pe);
              if ((unsigned long long)(R0 + rst) < c_min) { c_min = (unsigned long long)(R0 + rst); c_min_steps = steps; }
              rp = -1;
            }
          }
        }
      }
    } else {
      int64_t p = -1, cst = 0, pex = -1;
      for (;;) {
        if (!done && p < 0) {
          while (m == 0 && ++wi < nwl) m = mask_word(wi);
          if (m == 0) {
            done = true;
          } else {
            cst = s + 64ll * wi + __builtin_ctzll(m);
            m &= m - 1;
            p = cst;
            pex = -1;
            steps = 0;
          }
        }
        if (__all(done)) break;
        if (!done) {
          const RecHdr h = decode_rgn(rgn, R0, p, log_len);
          if (!header_plausible(h, p, P.max_key_len, P.max_value_len, log_len) || (!h.put && P.no_deletes)) {
            p = -1;
          } else {
            if (pex < 0) steps++;
            p = record_end(h, p);
            if (pex < 0 && p >= e) pex = p;
            if (p >= stop) {
              nsurv++;
              min_exit = min(min_exit, (unsigned long long)pex);
              max_exit = max(max_exit, (long long)pex);
              if ((unsigned long long)cst < c_min) { c_min = (unsigned long long)cst; c_min_steps = steps; }
              p = -1;
            }
          }
        }
      }
    }
  }
  const bool converged = act && !passthrough && !unenc && nsurv > 0 && (long long)min_exit == max_exit;
  mark(2);
  if (P.dbg) {
    const unsigned long long sv = wave_sum_u64(nsurv);
    const unsigned long long nc = wave_sum_u64(converged ? 0ull : (act ? 1ull : 0ull));
    if (lane == 0) { P.dbg[wv * 16 + 9] = sv; P.dbg[wv * 16 + 10] = nc; P.dbg[wv * 16 + 8] = dbg_iters; }
  }

  // balanced walk: the lane's own candidate that starts at p, if it survived -> its steps and exit
  // (cands_live: the list is overlaid by the record list once phase 5 ran)
  bool cands_live = true;
  auto find_surv = [&](int64_t p, int32_t& steps, int64_t& ex) -> bool {
    if (!balanced || !cands_live) return false;
    const uint32_t* cand = reinterpret_cast<const uint32_t*>(lds + P.fr_rgn_bytes);
    const uint32_t want = (uint32_t)(p - R0);
    for (uint32_t i = 0; i < my_ccnt; i++) {
      const uint32_t v = cand[my_cpre + i];
      if (cand_start(v) == want) {
        if (!(v & 0x80000000u)) return false;
        steps = cand_steps(v);
        ex = e + (int64_t)cand_dexit(v);
        return true;
      }
    }
    return false;
  };
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
          extv = (unsigned long long)s;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    return (int64_t)__shfl(extv, 0, 64);
  };
  auto at_glb = [&](int64_t a) -> uint32_t { return (uint32_t)P.log[a]; };
  auto hdr_at = [&](int64_t p) -> RecHdr {
    return p + 16 <= R0 + RLEN ? decode_rgn(rgn, R0, p, log_len) : decode_header(at_glb, p, log_len);
  };
  // ---- 3 entries ----
  const int64_t conv_exit = converged ? (int64_t)min_exit : -1;
  if (lane == nw - 1 && converged) granule_store(&P.exit_desc[wv], (unsigned long long)conv_exit | kReady);
  // The wave's first entry is the previous wave's published exit.  When every chunk converged and
  // the first one has a single survivor, that survivor is the entry of any consistent log: the wave
  // goes on with it and checks the published exit after hashing (phases 3-5 are redone on a
  // mismatch), so the hand-off latency hides behind the wave's own work.
  const unsigned long long c_min0 = __shfl(c_min, 0, 64);
  const unsigned long long nsurv0 = __shfl(nsurv, 0, 64);
  bool spec = wv > 0 && __all(!act || converged) && nsurv0 == 1;
  int64_t ext = spec ? (int64_t)c_min0 : wait_prev();
  mark(3);
  unsigned long long ndel = 0;
  for (;;) {
    int64_t my_exit = conv_exit;
    // chunks whose exit depends on their entry, in order (a serial walk each, rare)
    int32_t cnt = 0;
    bool bad = false;
    unsigned long long pending = __ballot(act && !converged);
    while (pending) {
      const int j = __builtin_ctzll(pending);
      pending &= pending - 1;
      const int64_t prev_exit = __shfl(my_exit, j > 0 ? j - 1 : 0, 64);
      if (lane == j) {
        int64_t p = j == 0 ? ext : prev_exit;
        int32_t fst = 0;
        int64_t fex = 0;
        if (p < e && find_surv(p, fst, fex)) {  // its chain was walked already
          cnt = fst;
          p = fex;
        }
        while (p < e) {
          const RecHdr h = hdr_at(p);
          if (!header_valid(h, p, P.max_key_len, log_len)) {
            set_error(P.st, p, header_error(h));
            bad = true;
            break;
          }
          cnt++;
          p = record_end(h, p);
        }
        my_exit = max(p, e);
      }
    }
    if (lane == nw - 1 && !converged) granule_store(&P.exit_desc[wv], (unsigned long long)my_exit | kReady);
    if (lane == nw - 1 && wv + 1 == (P.fr_nchunks + P.fr_w - 1) / P.fr_w) P.st->exit = my_exit;  // the framed chain's exit
    const int64_t up = __shfl_up(my_exit, 1, 64);
    const int64_t entry = lane == 0 ? ext : up;

    // ---- 4 counts ----
    bool need_walk = converged && !(nsurv == 1 && (unsigned long long)entry == c_min);
    if (converged && !need_walk) cnt = c_min_steps;
    if (need_walk) {  // the entry's own speculative walk, if it survived, is the verified one
      int32_t fst = 0;
      int64_t fex = 0;
      if (find_surv(entry, fst, fex) && fex == (int64_t)min_exit) {
        cnt = fst;
        need_walk = false;
      }
    }
    if (__any(need_walk)) {  // several survivors, or an entry the screen pruned: verified walk
      int64_t p = need_walk ? entry : e;
      for (;;) {
        const bool go = need_walk && !bad && p < e;
        if (!__any(go)) break;
        if (go) {
          const RecHdr h = hdr_at(p);
          if (!header_valid(h, p, P.max_key_len, log_len)) {
            set_error(P.st, p, header_error(h));
            bad = true;
          } else {
            cnt++;
            p = record_end(h, p);
          }
        }
      }
      if (need_walk && !bad && p != (int64_t)min_exit) atomicOr(&P.st->spec_fail, 1u);
    }
    if (!act || bad) cnt = 0;
    // wave-exclusive scan of the counts
    unsigned long long incl = (unsigned long long)cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const unsigned long long total = __shfl(incl, 63, 64);
    const unsigned long long local_off = incl - (unsigned long long)cnt;
    mark(4);
    // the wave's records go to its own slab; the radix partition compacts the slabs
    if (total > P.slab_cap) {
      if (spec) {  // the guessed entry may be wrong: decide on the published one
        const int64_t real = wait_prev();
        spec = false;
        if (real != ext) {
          ext = real;
          continue;
        }
      }
      if (lane == 0) {
        atomicMax(&P.st->max_wave_count, (unsigned int)min(total, 0xffffffffull));
        atomicOr(&P.st->overflow, 1u);
      }
      return;
    }
    if (lane == 0) P.wcount[wv] = (uint32_t)total;
    const unsigned long long base = wv * (unsigned long long)P.slab_cap;
    mark(5);

    // ---- 5 hash every record, entries in log order.  The lanes first list their chunks' record
    //      starts in LDS, then each lane hashes every 64th record of the wave (all lanes busy,
    //      consecutive entries written together); a wave holding more than kCandCap records hashes
    //      per chunk instead. ----
    ndel = 0;
    bool bovf = false;
    auto emit = [&](int64_t p, uint64_t dst) -> int64_t {
      const RecHdr h = hdr_at(p);
      const int64_t kp = p + h.hlen;
      uint64_t hash;
      if (kp + h.klen + 16 <= R0 + RLEN) {  // key in the region
        const RgnKey ld{rgn, (uint32_t)(kp - R0)};
        hash = P.hash_size == 8 ? murmur64_ld(ld, h.klen, (uint32_t)P.seed)
                                : (uint64_t)murmur32_ld(ld, h.klen, (uint32_t)P.seed);
      } else if (kp + h.klen + 32 <= log_len) {  // key runs past the region: unaligned global reads
        const GlobalKey ld{P.log + kp};
        hash = P.hash_size == 8 ? murmur64_ld(ld, h.klen, (uint32_t)P.seed)
                                : (uint64_t)murmur32_ld(ld, h.klen, (uint32_t)P.seed);
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
      if (!P.p1_bucket) {
        P.ent[dst] = en;
      } else if (h.put) {  // straight into the bucket's fixed region, as k_frame3 (DELETEs stay out)
        const uint32_t b = bucket_of(P, hash);
        const uint32_t a = atomicAdd(&P.bcount[b], 1u);
        if (a < kPlaceLdsMax) P.ent2[(uint64_t)b * kPlaceLdsMax + a] = en;
        else bovf = true;
      }
      return record_end(h, p);
    };
    if (total <= (unsigned long long)kCandCap) {  // wave-uniform
      uint32_t* list = reinterpret_cast<uint32_t*>(lds + P.fr_rgn_bytes);  // overlays the candidate list
      wave_sync();
      cands_live = false;
      {
        int64_t p = (act && cnt > 0) ? entry : e;
        uint32_t o = (uint32_t)local_off;
        for (;;) {
          const bool go = p < e;
          if (!__any(go)) break;
          if (go) {
            list[o++] = (uint32_t)(p - R0);
            p = record_end(hdr_at(p), p);
          }
        }
      }
      wave_sync();
      for (uint32_t i = (uint32_t)lane; i < (uint32_t)total; i += 64) emit(R0 + (int64_t)list[i], base + i);
    } else {
      int64_t p = (act && cnt > 0) ? entry : e;
      uint64_t dst = base + local_off;
      for (;;) {
        const bool go = p < e;
        if (!__any(go)) break;
        if (go) p = emit(p, dst++);
      }
    }
    if (bovf) atomicOr(&P.st->p2_overflow, 1u);
    if (spec) {  // check the guessed entry against the published exit; redo on a mismatch
      const int64_t real = wait_prev();
      spec = false;
      if (real != ext) {
        // (bucket regions: the entries are out, so a redone round would count twice.  The guess is a
        //  converged first chunk's single survivor, which the true entry of a log whose header holds
        //  always is: a mismatch is a header that lies, and the framing fails -- the host redoes it)
        if (P.p1_bucket) {
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
}

// One wave per workgroup, region = workgroup id (frame3_kernels.hip's measurements: in-order dispatch
// starts the predecessor first; the spin on its exit is bounded).  fr_ticket: regions by a device-wide
// ticket per workgroup, for builds that share the device.
__global__ __launch_bounds__(64, 5) void k_frame(BuildParams P, uint32_t lds_per_wave) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint32_t tk = blockIdx.x;
  if (P.fr_ticket) {
    uint32_t t = 0;
    if (threadIdx.x == 0) t = atomicAdd(P.frame_ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  }
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  (void)lds_per_wave;
  if (tk < nwaves) frame_region(P, tk, lds);
}


// ================================================================================================
// k_frame_uniform: logs whose header proves that every record has the same size R.  With no DELETE,
// putSize == numPuts * R (R = the largest PUT record the header allows) and dataEnd - 84 == putSize,
// every record is at most R bytes and together they fill putSize, so each is exactly R and record i
// starts at 84 + i * R.  One wave per 64 records stages their bytes into LDS with coalesced
// global_load_lds, and every lane checks its record's header against (maxKeyLen, maxValueLen) --
// anything else flags spec_fail and the build reruns the general framing -- then hashes its key.
// The entries are dense, in log order (the slab layout of the serial path).
// ================================================================================================
// s_waitcnt vmcnt(n) for n in 0..16 (gfx9 encoding: vmcnt in bits 3:0 and 15:14, expcnt and lgkmcnt
// left at their maxima)
__device__ __forceinline__ void wait_vmcnt_le(int n) {
#define SK_VM(v) __builtin_amdgcn_s_waitcnt(((v) & 0xF) | (((v) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
  switch (n) {
    case 1: SK_VM(1); break;
    case 2: SK_VM(2); break;
    case 3: SK_VM(3); break;
    case 4: SK_VM(4); break;
    case 5: SK_VM(5); break;
    case 6: SK_VM(6); break;
    case 7: SK_VM(7); break;
    case 8: SK_VM(8); break;
    case 9: SK_VM(9); break;
    case 10: SK_VM(10); break;
    case 11: SK_VM(11); break;
    case 12: SK_VM(12); break;
    case 13: SK_VM(13); break;
    case 14: SK_VM(14); break;
    case 15: SK_VM(15); break;
    case 16: SK_VM(16); break;
    default: __builtin_amdgcn_s_waitcnt(0); break;
  }
#undef SK_VM
}

// A workgroup barrier for LDS traffic only: LDS operations complete, global ones may stay in flight
// (__syncthreads waits for every outstanding load and store first)
__device__ __forceinline__ void lds_barrier() {
  // (a compiler barrier first: s_barrier is IntrNoMem, so without it earlier LDS stores could be
  //  scheduled past the barrier; it emits no instruction)
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt, expcnt at their maxima
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// W waves per workgroup; DB: each wave double-buffers its staging, the next round's LDS-DMA in flight
// while it hashes the current one (the only global loads of the rounds, so vmcnt counts just them).
template <int W, bool DB>
__global__ __launch_bounds__(64 * W) void k_frame_uniform(BuildParams P) {
  static_assert(W >= 4, "the write-out's digit steps take one thread per digit (256)");
  // A workgroup frames kSub partition tiles (kSub * kPartTile records), kRounds rounds of 64 records
  // per wave, each wave staging its own records by LDS-DMA.
  constexpr int kSub = 1;  // (2 or 4 -- longer runs per region -- measured slower: registers/scratch)
  constexpr int kTileRounds = kPartTile / 64 / W;
  constexpr int kRounds = kSub * kTileRounds;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];  // wave buffers | hist[kSub][256] rbase[256]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* buf0 = lds + (uint32_t)wave * P.uni_wbytes * (DB ? 2u : 1u);
  uint32_t* hist = reinterpret_cast<uint32_t*>(lds + P.uni_hist_off);  // per tile
  uint32_t* rbase = hist + kSub * 256;
  // to_regions: the entries go straight to their digit regions of ent3 (partition pass 1 done here);
  // else with p1_hist_ready each tile's digit counts are k_part1_hist's output
  const bool to_regions = P.p1_region != 0;
  const bool with_hist = to_regions || P.p1_hist_ready != 0;
  long long t_prev = P.dbg ? clock64() : 0;
  uint64_t dbg_tile = blockIdx.x;
  auto mark = [&](int i) {  // (frame_debug: thread 0's cycles per phase of the tile)
    if (P.dbg && threadIdx.x == 0) {
      const long long now = clock64();
      P.dbg[(uint64_t)dbg_tile * 16 + i] = (unsigned long long)(now - t_prev);
      t_prev = now;
    }
  };

  if (with_hist) {
    for (int t = threadIdx.x; t < kSub * 256; t += 64 * W) hist[t] = 0;
    __syncthreads();
  }
  const int64_t R = P.uni_rec;
  const int64_t log_len = (int64_t)P.log_len;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    P.st->n_records = P.uni_n;
    P.st->exit = P.fr_entry + (int64_t)P.uni_n * R;  // the framed chain's exit
  }
  const uint64_t nblk = (P.uni_n + kSub * kPartTile - 1) / (kSub * kPartTile);
  uint64_t hsh[kRounds];  // (the address follows from the round: record blk0 + (r * W + wave) * 64 + lane)
  uint32_t dr[kRounds];   // digit << 16 | rank within its tile's digit run, ~0 = none
  // Persistent workgroups (two a CU): tiles blockIdx.x, + gridDim.x, ...  A tile's entry stores drain
  // while the next tile's first rounds stream in (a workgroup that ended after its write-out held its
  // LDS until the stores completed).
  for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
  const uint64_t blk0 = blk * (kSub * kPartTile);
  dbg_tile = blk;
  // stage round r's records into b: LDS-DMA (returns the load instructions in flight), or guarded
  // loads near the end of the buffer (synchronous, returns 0)
  auto stage_round = [&](int r, uint8_t* b) -> int {
    const uint64_t i0 = blk0 + (uint64_t)(r * W + wave) * 64;
    if (i0 >= P.uni_n) return 0;  // (wave-uniform)
    const int64_t base = P.fr_entry + (int64_t)i0 * R;
    const int64_t a0 = base & ~15ll;
    const int nrec = (int)min((uint64_t)64, P.uni_n - i0);
    const int64_t want = base + (int64_t)nrec * R + 16 - a0;  // + 16: the 8-byte window reads past a key
    const int nvec = (int)((want + 15) >> 4);
    if (a0 + 16ll * nvec <= log_len) {
      const uint4* src = reinterpret_cast<const uint4*>(P.log + a0);
      if (P.uni_nt) {  // non-temporal: the log is read once
        for (int v0 = 0; v0 < nvec; v0 += 64)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(src + min(v0 + lane, nvec - 1)),
              (__attribute__((address_space(3))) void*)(b + 16u * (uint32_t)v0), 16, 0, 2);
      } else {
        for (int v0 = 0; v0 < nvec; v0 += 64)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(src + min(v0 + lane, nvec - 1)),
              (__attribute__((address_space(3))) void*)(b + 16u * (uint32_t)v0), 16, 0, 0);
      }
      return (nvec + 63) / 64;
    }
    for (int v = lane; v < nvec; v += 64) *reinterpret_cast<uint4*>(b + 16u * v) = load16_guarded(P.log, a0 + 16ll * v, log_len);
    return 0;
  };
  if (DB) stage_round(0, buf0);
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    dr[r] = ~0u;
    uint8_t* buf = DB ? buf0 + (r & 1) * P.uni_wbytes : buf0;
    const uint64_t i0 = blk0 + (uint64_t)(r * W + wave) * 64;
    if (DB) {
      // the next round's records in flight while this one is hashed; then wait for this one's (and
      // for anything issued before it: the previous tile's entry stores)
      const int nxt = r + 1 < kRounds ? stage_round(r + 1, buf0 + ((r + 1) & 1) * P.uni_wbytes) : 0;
      wait_vmcnt_le(nxt);
    } else {
      stage_round(r, buf);
      __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS-DMA has landed
    }
    if (i0 >= P.uni_n) continue;  // (wave-uniform)
    const int64_t base = P.fr_entry + (int64_t)i0 * R;
    const int64_t a0 = base & ~15ll;
    const int nrec = (int)min((uint64_t)64, P.uni_n - i0);
    __builtin_amdgcn_wave_barrier();
    if (lane < nrec) {
      const int64_t p = base + (int64_t)lane * R;
      const uint32_t off = (uint32_t)(p - a0);
      const uint64_t x = rgn_u64(buf, off);
      const int32_t klen = (int32_t)(x & 0xff) - 1, vlen = (int32_t)((x >> 8) & 0xff);
      if ((x & 0x8080ull) != 0 || klen != (int32_t)P.max_key_len || vlen != (int32_t)P.max_value_len) {
        atomicOr(&P.st->spec_fail, 4u);  // not the uniform log the header describes
      } else {
        // (klen is the header's maxKeyLen on every lane: the hash's loop and tail are scalar)
        const int32_t ukl = (int32_t)P.max_key_len;
        const RgnKey ld{buf, off + 2u};
        const uint64_t hash = P.hash_size == 8 ? murmur64_uni(ld, ukl, (uint32_t)P.seed)
                                               : (uint64_t)murmur32_uni(ld, ukl, (uint32_t)P.seed);
        hsh[r] = hash;
        if (!to_regions) {
          Entry en;
          en.hash = hash;
          en.addr = (uint64_t)p << P.ebb;
          P.ent[i0 + lane] = en;
        }
        if (with_hist) {
          const uint32_t d = digit_of(P, bucket_of(P, hash));
          const uint32_t rank = atomicAdd(&hist[(r / kTileRounds) * 256 + d], 1u);
          dr[r] = (d << 16) | rank;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // every lane is done with the buffer before the next round's DMA
  }
  if (!with_hist) continue;
  __syncthreads();
  mark(0);
  if (!to_regions) {  // k_part1_hist's output for these tiles
    for (int t = threadIdx.x; t < kSub * 256; t += 64 * W) {
      const uint64_t tile = blk * kSub + (t >> 8);
      if (tile < P.p1_tiles) P.p1_hist[(uint64_t)(t & 255) * P.p1_tiles + tile] = hist[t];
    }
    __syncthreads();  // (hist is cleared for the next tile)
    for (int t = threadIdx.x; t < kSub * 256; t += 64 * W) hist[t] = 0;
    __syncthreads();
    continue;
  }
  // One run per digit region for the workgroup's kSub tiles together (one atomic per non-empty
  // digit; runs kSub times longer than a tile's, so fewer partial lines at the run ends), then per
  // tile: its entries grouped by digit in LDS (the staging buffers are free now), each sub-run
  // written coalesced.
  Entry* stage = reinterpret_cast<Entry*>(lds);                      // kPartTile entries
  uint8_t* sdig = lds + kPartTile * sizeof(Entry);                    // digit of each staged entry
  uint32_t* lbase = reinterpret_cast<uint32_t*>(sdig + kPartTile);   // tile-local run starts
  __shared__ uint32_t wsum[4];
  static_assert(kSub == 1, "one tile a workgroup");
  // The digit runs' cursors: each returning atomic goes out first, and its round trip overlaps the
  // tile's scan and regroup (the write-out is the first to need rbase).
  uint32_t c = 0, incl = 0, b0 = 0;
  if (threadIdx.x < 256) {  // waves 0-3: the cursor, and the exclusive scan of the tile's 256 digit counts
    c = hist[threadIdx.x];
    hist[threadIdx.x] = 0;  // (for the next tile: its rounds count after the barriers below)
    b0 = c ? atomicAdd(&P.p1_fill[threadIdx.x], c) : 0u;
    incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
  }
  lds_barrier();
  if (threadIdx.x < 256) {
    uint32_t off = 0;
    for (int w = 0; w < wave; w++) off += wsum[w];
    lbase[threadIdx.x] = off + incl - c;
  }
  lds_barrier();
  mark(1);
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    if (dr[r] == ~0u) continue;
    const uint32_t d = dr[r] >> 16;
    const uint32_t i = lbase[d] + (dr[r] & 0xffffu);
    Entry en;
    en.hash = hsh[r];
    const uint64_t rec = blk0 + (uint64_t)(r * W + wave) * 64 + lane;
    // (compact: the record index, the write-out stores 12-byte CEntry)
    en.addr = (P.compact & kCompactIn) ? rec : (uint64_t)(P.fr_entry + (int64_t)rec * R) << P.ebb;
    stage[i] = en;
    sdig[i] = (uint8_t)d;
  }
  if (threadIdx.x < 256) {
    if ((uint64_t)b0 + c > P.p1_region) atomicOr(&P.st->spec_fail, kSpecRegionFull);
    rbase[threadIdx.x] = b0;
  }
  lds_barrier();
  mark(2);
  const uint32_t ntile = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  if (P.compact & kCompactIn) {
    for (uint32_t i = threadIdx.x; i < ntile; i += 64 * W) {
      const uint32_t d = sdig[i];
      const uint64_t pos = (uint64_t)rbase[d] + (i - lbase[d]);
      if (pos < P.p1_region) store_craw(reinterpret_cast<CEntry*>(P.ent3) + (uint64_t)d * P.p1_region + pos, stage[i]);
    }
  } else {
    for (uint32_t i = threadIdx.x; i < ntile; i += 64 * W) {
      const uint32_t d = sdig[i];
      const uint64_t pos = (uint64_t)rbase[d] + (i - lbase[d]);
      if (pos < P.p1_region) P.ent3[(uint64_t)d * P.p1_region + pos] = stage[i];
    }
  }
  if (P.dbg) {  // (the write-out to completion)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    mark(3);
  }
  lds_barrier();  // the stage's reads are done (its stores may still be in flight): the next tile's DMA
  }
}

// ================================================================================================
// Radix partition of the entries by bucket (bucket = wantedSlot >> kBucketShift).
// Pass 1: coarse digit = bucket / bpp (< 256; every digit holds bpp buckets, so the digits
// split the table evenly -- a sharded build gives each rank a run of digits) over tiles of slabs.
// ================================================================================================
// A partition tile is part_group (<= 64) consecutive slabs, <= kPartTile entries together.
// Wave 0 scans the slab counts with shuffles; slab_of maps a tile index to its slab, so every
// thread then loads its entries with independent reads.
template <int kMaxEntries>
struct SlabTileN {
  uint32_t pre[kMaxPartGroup + 1];  // entry prefix over the tile's slabs
  uint8_t slab_of[kMaxEntries];
};
using SlabTile = SlabTileN<kPartTile>;

template <int kMaxEntries>
__device__ __forceinline__ uint32_t load_tile(const BuildParams& P, SlabTileN<kMaxEntries>& T, uint64_t g0,
                                              uint32_t group) {
  const uint32_t ng = (uint32_t)min((uint64_t)group, P.nslabs > g0 ? P.nslabs - g0 : 0);
  const int tid = threadIdx.x;
  if (tid < 64) {
    const uint32_t c = (uint32_t)tid < ng ? P.wcount[g0 + tid] : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    T.pre[tid] = incl - c;
    if (tid == 63) T.pre[64] = incl;
  }
  __syncthreads();
  const int lane = tid & 63;
  for (uint32_t g = tid >> 6; g < ng; g += kPartBlock / 64) {
    const uint32_t lo = T.pre[g], n = T.pre[g + 1] - lo;
    for (uint32_t j = lane; j < n; j += 64) T.slab_of[lo + j] = (uint8_t)g;
  }
  __syncthreads();
  return T.pre[64];
}

template <int kMaxEntries>
__device__ __forceinline__ const Entry& tile_entry(const BuildParams& P, const SlabTileN<kMaxEntries>& T, uint64_t g0,
                                                   uint32_t i) {
  const uint32_t g = T.slab_of[i];
  return P.ent[(g0 + g) * (uint64_t)P.slab_cap + (i - T.pre[g])];
}

// k_part1_regions' tiles (up to 2 kPartTile entries): the slab of entry i found from the slab of
// entry 32 * (i / 32) (slabs hold ~60 entries: at most a step or two), 256 bytes where a byte per entry
// would take 8 KiB of the LDS that two workgroups per CU need.
struct SlabTileR {
  uint32_t pre[kMaxPartGroup + 1];
  uint8_t first[2 * kPartTile / 32];
};

// wave 0's part of load_tile_r: the tile's slab prefix and group map (a barrier must follow)
__device__ __forceinline__ void tile_r_hdr(const BuildParams& P, SlabTileR& T, uint64_t g0, uint32_t group) {
  const uint32_t ng = (uint32_t)min((uint64_t)group, P.nslabs > g0 ? P.nslabs - g0 : 0);
  const int tid = threadIdx.x;
  if (tid < 64) {
    const uint32_t c = (uint32_t)tid < ng ? P.wcount[g0 + tid] : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (tid >= o) incl += t;
    }
    T.pre[tid] = incl - c;
    if (tid == 63) T.pre[64] = incl;
    // slab g covers the 32-entry groups whose first entry it holds
    if ((uint32_t)tid < ng)
      for (uint32_t k = (incl - c + 31) / 32; k < (incl + 31) / 32 && k < 2 * kPartTile / 32; k++) T.first[k] = (uint8_t)tid;
  }
}

__device__ __forceinline__ const Entry& tile_entry_r(const BuildParams& P, const SlabTileR& T, uint64_t g0, uint32_t i) {
  uint32_t g = T.first[i >> 5];
  while (T.pre[g + 1] <= i) g++;
  return P.ent[(g0 + g) * (uint64_t)P.slab_cap + (i - T.pre[g])];
}

__global__ __launch_bounds__(kPartBlock) void k_part1_hist(BuildParams P) {
  __shared__ uint32_t hist[256];
  __shared__ SlabTile T;
  if (build_aborted(P)) return;
  const uint64_t g0 = (uint64_t)blockIdx.x * P.part_group;
  hist[threadIdx.x] = 0;
  const uint32_t n = load_tile(P, T, g0, P.part_group);
  // every load of the tile in flight at once, then the histogram
  Entry v[kPartItems];
#pragma unroll
  for (int i = 0; i < kPartItems; i++) {
    const uint32_t idx = (uint32_t)i * kPartBlock + threadIdx.x;
    if (idx < n) v[i] = tile_entry(P, T, g0, idx);
  }
#pragma unroll
  for (int i = 0; i < kPartItems; i++) {
    const uint32_t idx = (uint32_t)i * kPartBlock + threadIdx.x;
    if (idx >= n || (P.skip_del && (v[i].addr & kDelBit))) continue;  // exact path: DELETEs stay out
    atomicAdd(&hist[digit_of(P, bucket_of(P, v[i].hash))], 1u);
  }
  __syncthreads();
  P.p1_hist[(uint64_t)threadIdx.x * P.p1_tiles + blockIdx.x] = hist[threadIdx.x];  // digit-major
}

__global__ __launch_bounds__(kPartBlock) void k_part1_scatter(BuildParams P) {
  __shared__ Entry stage[kPartTile];
  __shared__ uint8_t sdig[kPartTile];  // digit of each staged entry
  __shared__ uint32_t lbase[256];
  __shared__ uint32_t cursor[256];
  __shared__ int64_t gdst[256];  // global offset of the digit's run minus its LDS start
  __shared__ uint64_t sh64[kPartBlock / 64 + 1];
  __shared__ SlabTile T;
  if (build_aborted(P)) return;  // the host grows the workspace and redoes the build
  const uint64_t g0 = (uint64_t)blockIdx.x * P.part_group;
  const int tid = threadIdx.x;
  const uint32_t h = P.p1_hist[(uint64_t)tid * P.p1_tiles + blockIdx.x];
  const uint64_t goff = P.p1_off[(uint64_t)tid * P.p1_tiles + blockIdx.x];
  const uint32_t lb = (uint32_t)block_excl_sum<kPartBlock>(h, sh64, &sh64[kPartBlock / 64]);
  lbase[tid] = lb;
  gdst[tid] = (int64_t)goff - (int64_t)lb;
  cursor[tid] = 0;
  const uint32_t n = load_tile(P, T, g0, P.part_group);
  Entry v[kPartItems];
#pragma unroll
  for (int i = 0; i < kPartItems; i++) {
    const uint32_t idx = (uint32_t)i * kPartBlock + tid;
    if (idx < n) v[i] = tile_entry(P, T, g0, idx);
  }
#pragma unroll
  for (int i = 0; i < kPartItems; i++) {
    const uint32_t idx = (uint32_t)i * kPartBlock + tid;
    if (idx < n && !(P.skip_del && (v[i].addr & kDelBit))) {
      const uint32_t d = digit_of(P, bucket_of(P, v[i].hash));
      const uint32_t pos = lbase[d] + atomicAdd(&cursor[d], 1u);
      stage[pos] = v[i];
      sdig[pos] = (uint8_t)d;
    }
  }
  __syncthreads();
  const uint32_t nkeep = (uint32_t)sh64[kPartBlock / 64];  // the tile's entries in the placement
  // coalesced write-out: LDS position i -> global offset of its digit run
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    const uint32_t i = (uint32_t)k * kPartBlock + tid;
    if (i < nkeep) P.ent3[gdst[sdig[i]] + (int64_t)i] = stage[i];
  }
}

// Pass 1 in one kernel, into fixed-capacity digit regions (P.p1_region, as k_frame_uniform writes
// them): the tile's digit counts in LDS, one atomic per non-empty digit on the region's fill cursor,
// the tile's entries grouped by digit in LDS and written as one run per digit.  No histogram pass over
// the entries and no global scan (k_part1_hist + k_part1_scatter read every entry twice).  A region
// that fills up flags kSpecRegionFull: the host redoes the build with the two-pass partition.
// Persistent workgroups (two a CU: the stage's LDS), each taking the rounds (kPartTile entries of a
// tile) of tiles blockIdx.x, + gridDim.x, ...: the next round's entries are loaded while this round's
// cursors are reserved, its runs grouped and written.  The barriers are LDS-only (lds_barrier): the
// loads and the cursor atomic stay in flight through them.
constexpr uint32_t kP1rGrid = 512;
__global__ __launch_bounds__(kPartBlock) void k_part1_regions(BuildParams P) {
  static_assert(kPartBlock == 256, "one thread per digit");
  __shared__ Entry stage[kPartTile];
  __shared__ uint8_t sdig[kPartTile];  // digit of each staged entry
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t lbase[256];
  __shared__ int64_t gdst[256];        // global index of the digit's run minus its LDS start
  __shared__ uint32_t wsum[kPartBlock / 64];
  __shared__ SlabTileR T[2];           // (p1r_group slabs: at most 2 kPartTile entries, host-checked)
  if (build_aborted(P)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t ntiles = P.p1r_tiles;
  uint64_t t = blockIdx.x;
  if (t >= ntiles) return;
  const uint32_t grp = P.p1r_group;
  tile_r_hdr(P, T[0], t * grp, grp);
  lds_barrier();
  int cb = 0;
  uint32_t ntile = T[0].pre[64], base = 0;
  Entry v[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    const uint32_t idx = (uint32_t)k * kPartBlock + tid;
    if (idx < ntile) v[k] = tile_entry_r(P, T[0], t * grp, idx);
  }
  for (;;) {
    const uint32_t n = min((uint32_t)kPartTile, ntile - base);
    uint64_t tn = t;
    uint32_t bn = base + kPartTile;
    int nb = cb;
    if (bn >= ntile) {
      tn = t + gridDim.x;
      bn = 0;
      nb = cb ^ 1;
    }
    const bool more = tn < ntiles;
    cnt[tid] = 0;
    if (more && nb != cb) tile_r_hdr(P, T[nb], tn * grp, grp);  // (T[nb]'s last reader was a load before this round's barriers)
    lds_barrier();  // (cnt clear, T[nb]; the previous round is done with stage, sdig, gdst, lbase, wsum)
    uint32_t dg[kPartItems];
#pragma unroll
    for (int k = 0; k < kPartItems; k++) {
      const uint32_t idx = (uint32_t)k * kPartBlock + tid;
      dg[k] = ~0u;
      if (idx < n && !(P.skip_del && (v[k].addr & kDelBit))) {  // exact path: DELETEs stay out
        const uint32_t d = digit_of(P, bucket_of(P, v[k].hash));
        dg[k] = d | (atomicAdd(&cnt[d], 1u) << 8);  // rank inside the round's digit run
      }
    }
    lds_barrier();
    // the digit's cursor first (its round trip overlaps the next round's loads and this one's scan)
    const uint32_t c = cnt[tid];
    const uint64_t b0 = c ? atomicAdd(&P.p1_fill[tid], c) : 0u;
    Entry nx[kPartItems];
    if (more) {
      const uint32_t nn = min((uint32_t)kPartTile, T[nb].pre[64] - bn);
#pragma unroll
      for (int k = 0; k < kPartItems; k++) {
        const uint32_t idx = (uint32_t)k * kPartBlock + tid;
        if (idx < nn) nx[k] = tile_entry_r(P, T[nb], tn * grp, bn + idx);
      }
    }
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o, 64);
      if (lane >= o) incl += x;
    }
    if (lane == 63) wsum[wave] = incl;
    lds_barrier();
    uint32_t off = 0;
    for (int w = 0; w < wave; w++) off += wsum[w];
    const uint32_t lb = off + incl - c;
    lbase[tid] = lb;
    if (b0 + c > P.p1_region) atomicOr(&P.st->spec_fail, kSpecRegionFull);
    gdst[tid] = (int64_t)((uint64_t)tid * P.p1_region + b0) - (int64_t)lb;
    lds_barrier();
#pragma unroll
    for (int k = 0; k < kPartItems; k++) {
      if (dg[k] == ~0u) continue;
      const uint32_t d = dg[k] & 255u, pos = lbase[d] + (dg[k] >> 8);
      stage[pos] = v[k];
      sdig[pos] = (uint8_t)d;
    }
    lds_barrier();
    const uint32_t nkeep = wsum[0] + wsum[1] + wsum[2] + wsum[3];
#pragma unroll
    for (int k = 0; k < kPartItems; k++) {
      const uint32_t i = (uint32_t)k * kPartBlock + tid;
      if (i < nkeep) {
        const uint32_t d = sdig[i];
        const uint64_t at = (uint64_t)(gdst[d] + (int64_t)i);
        if (at < (uint64_t)(d + 1) * P.p1_region) P.ent3[at] = stage[i];
      }
    }
    if (!more) break;
    t = tn;
    base = bn;
    cb = nb;
    ntile = T[nb].pre[64];
#pragma unroll
    for (int k = 0; k < kPartItems; k++) v[k] = nx[k];
  }
}

// Dense entries (serial framing path) seen as slabs of kPartTile.
__global__ void k_dense_slabs(BuildParams P) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= P.nslabs) return;
  const uint64_t N = P.st->n_records;
  const uint64_t lo = w * P.slab_cap;
  P.wcount[w] = (uint32_t)(N > lo ? min(N - lo, (uint64_t)P.slab_cap) : 0);
}

// Pass 2: one workgroup per coarse digit splits it into its bpp buckets.
__global__ __launch_bounds__(kPart2Block) void k_part2(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];  // hist[nbins] ++ cur[nbins]
  __shared__ uint64_t sh64[kPart2Block / 64 + 1];
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  // input: the digit's run of the pass-1 output, or (sharded receive) its run in every source rank's
  // block of the exchange buffer; output: ent2 from `lo` on
  uint64_t lo, hi;
  const uint64_t* seg = nullptr;  // nsrc (begin, end) runs of ent3
  uint32_t nseg = 1;
  if (P.p2_seg) {
    if (dpart < P.p2_d0 || dpart >= P.p2_d0 + P.p2_nd) return;
    const uint32_t k = dpart - P.p2_d0;
    lo = P.p2_out[k];
    hi = P.p2_out[k + 1];
    seg = P.p2_seg + 2ull * k * P.p2_nsrc;
    nseg = P.p2_nsrc;
  } else if (P.p1_region) {  // k_frame_uniform filled the digit's region of ent3
    lo = (uint64_t)dpart * P.p1_region;
    hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
  } else {
    lo = P.p1_off[(uint64_t)dpart * P.p1_tiles];
    hi = (dpart + 1 < 256) ? P.p1_off[(uint64_t)(dpart + 1) * P.p1_tiles] : P.p1_off_total[0];
  }
  const uint32_t nbins = P.bpp;
  const uint32_t b0 = dpart * nbins;
  uint32_t* hist = dyn;
  uint32_t* cur = dyn + nbins;
  const int tid = threadIdx.x;
  for (uint32_t b = tid; b < nbins; b += kPart2Block) hist[b] = 0;
  __syncthreads();
  bool bad = false;  // (kGuardForeign)
  // (kPart2Items loads per thread in flight: one workgroup per CU needs the memory-level parallelism)
  for (uint32_t q = 0; q < nseg; q++) {
    const uint64_t a = seg ? seg[2 * q] : lo, z = seg ? seg[2 * q + 1] : hi;
    for (uint64_t i0 = a; i0 < z; i0 += (uint64_t)kPart2Block * kPart2Items) {
      uint64_t h[kPart2Items];
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        if (i < z) h[k] = P.ent3[i].hash;
      }
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        if (i >= z) continue;
        const uint32_t b = bucket_of(P, h[k]) - b0;
        if (b < nbins) atomicAdd(&hist[b], 1u);
        else bad = true;
      }
    }
  }
  report_foreign(P, bad);
  __syncthreads();
  // exclusive scan of the bins (per consecutive bins per thread)
  const uint32_t per = (nbins + kPart2Block - 1) / kPart2Block;
  uint64_t local = 0;
  for (uint32_t q = 0; q < per; q++) {
    const uint32_t b = tid * per + q;
    if (b < nbins) local += hist[b];
  }
  uint64_t run = block_excl_sum<kPart2Block>(local, sh64, nullptr);
  for (uint32_t q = 0; q < per; q++) {
    const uint32_t b = tid * per + q;
    if (b < nbins) {
      const uint64_t bucket = (uint64_t)b0 + b;
      if (bucket < P.nbuckets) {
        P.boff[bucket] = lo + run;
        P.bcount[bucket] = hist[b];
      }
      cur[b] = (uint32_t)run;
      run += hist[b];
    }
  }
  __syncthreads();
  for (uint32_t q = 0; q < nseg; q++) {
    const uint64_t a = seg ? seg[2 * q] : lo, z = seg ? seg[2 * q + 1] : hi;
    for (uint64_t i0 = a; i0 < z; i0 += (uint64_t)kPart2Block * kPart2Items) {
      Entry v[kPart2Items];
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        if (i < z) v[k] = P.ent3[i];
      }
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        const uint32_t b = bucket_of(P, v[k].hash) - b0;
        if (i < z && b < nbins) P.ent2[lo + atomicAdd(&cur[b], 1u)] = v[k];  // (foreign: counted above)
      }
    }
  }
}

__device__ __forceinline__ MaxPlus shfl_up_mp(MaxPlus f, int o) {
  MaxPlus t;
  t.c = __shfl_up(f.c, o, 64);
  t.a = __shfl_up(f.a, o, 64);
  return t;
}

// fused_carry: the digit's bucket functions -> each bucket's exclusive prefix inside the digit (bpre)
// and the digit's composed function (dfun); the last block to finish composes the 256 digits around
// the ring: x0 = the composed function's constant (the carry into slot 0 when some slot stays
// empty), each digit's carry-in dcarry[d] = (digits before d)(x0), or `full` when no slot stays empty
// (k_carry's rules, evaluated per digit instead of per bucket).
// A digit's function travels as one 64-bit word, (epoch << 42) | c << 21 | (a + 2^20), stored with a
// relaxed agent-scope atomic; the last block reads each word until it carries this build's epoch.
// That needs no release fence (on gfx950 one writes the XCD's whole L2 back: 256 of them measured
// 0.11 ms).  With fixed bucket regions |a|, c <= 64 buckets x 1024 entries < 2^20; a digit past that
// overflowed its regions and the build is redone (the clamp only keeps the epoch bits intact).
constexpr int kDfunShift = 21;
__device__ __forceinline__ uint64_t pack_dfun(MaxPlus f, uint32_t epoch) {
  const int64_t lim = (1ll << 20) - 1;
  const uint64_t c = (uint64_t)min(max(f.c, (int64_t)0), lim), a = (uint64_t)(min(max(f.a, -lim), lim) + (1ll << 20));
  return ((uint64_t)epoch << (2 * kDfunShift)) | (c << kDfunShift) | a;
}

__device__ void part2_fused_carry(const BuildParams& P, const MaxPlus* s_fun, uint32_t nbins, uint64_t b0,
                                  uint32_t dpart) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const OpMaxPlus op;
  __shared__ bool s_last;
  uint64_t* dword = (uint64_t*)P.dfun;  // (256 packed words)
  __syncthreads();
  if (wave == 0) {
    MaxPlus f = (uint32_t)lane < nbins ? s_fun[lane] : MaxPlus{0, 0};
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const MaxPlus t = shfl_up_mp(f, o);
      if (lane >= o) f = op(t, f);
    }
    MaxPlus ex = shfl_up_mp(f, 1);
    if (lane == 0) ex = MaxPlus{0, 0};
    const uint64_t bucket = b0 + lane;
    if ((uint32_t)lane < nbins && bucket < P.nbuckets) P.bpre[bucket] = ex;
    if (lane == 63) __hip_atomic_store(&dword[dpart], pack_dfun(f, P.epoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&P.st->p2_ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last || wave != 0) return;
  static_assert(kPart2Block >= 64, "one wave composes the digits");
  MaxPlus g[4], agg{0, 0};
#pragma unroll
  for (int k = 0; k < 4; k++) {  // lane l: digits 4l .. 4l + 3 (every block stored its word before its ticket)
    uint64_t v;
    for (uint32_t spin = 0;; spin++) {  // (bounded: a word that never arrives is a bug, reported as such)
      v = __hip_atomic_load(&dword[4 * lane + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(v >> (2 * kDfunShift)) == P.epoch) break;
      if (spin > (1u << 24)) {
        atomicOr(&P.st->guard, 0x40u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    g[k].c = (int64_t)((v >> kDfunShift) & ((1ull << kDfunShift) - 1));
    g[k].a = (int64_t)(v & ((1ull << kDfunShift) - 1)) - (1ll << 20);
    agg = op(agg, g[k]);
  }
  MaxPlus incl = agg;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const MaxPlus t = shfl_up_mp(incl, o);
    if (lane >= o) incl = op(t, incl);
  }
  MaxPlus run = shfl_up_mp(incl, 1);
  if (lane == 0) run = MaxPlus{0, 0};
  MaxPlus tot;
  tot.c = __shfl(incl.c, 63, 64);
  tot.a = __shfl(incl.a, 63, 64);
  if (tot.a >= 0) {  // N >= capacity: no empty slot, the canonical layout does not apply
    if (lane == 0) atomicOr(&P.st->full, 1u);
    return;
  }
  const int64_t x0 = tot.c;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    P.dcarry[4 * lane + k] = max(run.c, x0 + run.a);
    run = op(run, g[k]);
  }
}

// k_part2d: k_part2 (dense bucket runs, tables of more than kP2SortedMaxBpp buckets per digit) with its
// scatter pass staged as in k_part2st: each round of kP2dPer entries a thread is grouped by bucket in
// LDS and leaves as one run per bucket, instead of one L2 request per 16-byte entry.  The round's
// bucket counts are double-buffered so that only the scan needs a barrier of its own.  Single GPU.
constexpr int kP2dPer = 6;

__global__ __launch_bounds__(kPart2Block) void k_part2d(BuildParams P) {
  // hist[nb] | cur[nb] | rc0[nb] | rc1[nb] | roff[nb] | gbase[nb] | stage[kPart2Block * kP2dPer]
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ uint64_t sh64[kPart2Block / 64 + 1];
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  uint64_t lo, hi;
  if (P.p1_region) {
    lo = (uint64_t)dpart * P.p1_region;
    hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
  } else {
    lo = P.p1_off[(uint64_t)dpart * P.p1_tiles];
    hi = (dpart + 1 < 256) ? P.p1_off[(uint64_t)(dpart + 1) * P.p1_tiles] : P.p1_off_total[0];
  }
  const uint32_t nbins = P.bpp;
  const uint32_t b0 = dpart * nbins;
  uint32_t* hist = dyn;
  uint32_t* cur = hist + nbins;
  uint32_t* rc[2] = {cur + nbins, cur + 2 * nbins};
  uint32_t* roff = cur + 3 * nbins;
  uint32_t* gbase = cur + 4 * nbins;
  Entry* stage = reinterpret_cast<Entry*>(dyn + ((6 * nbins + 3) & ~3u));
  constexpr uint32_t kRound = kPart2Block * kP2dPer;
  const int tid = threadIdx.x;
  for (uint32_t b = tid; b < 6 * nbins; b += kPart2Block) dyn[b] = 0;
  __syncthreads();
  bool bad = false;  // (kGuardForeign)
  // pass A: the bucket histogram (hashes only)
  for (uint64_t i0 = lo; i0 < hi; i0 += (uint64_t)kPart2Block * kPart2Items) {
    uint64_t h[kPart2Items];
#pragma unroll
    for (int k = 0; k < kPart2Items; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < hi) h[k] = P.ent3[i].hash;
    }
#pragma unroll
    for (int k = 0; k < kPart2Items; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i >= hi) continue;
      const uint32_t b = bucket_of(P, h[k]) - b0;
      if (b < nbins) atomicAdd(&hist[b], 1u);
      else bad = true;
    }
  }
  report_foreign(P, bad);
  __syncthreads();
  // bucket offsets: consecutive bins per thread
  const uint32_t per = (nbins + kPart2Block - 1) / kPart2Block;
  {
    uint64_t local = 0;
    for (uint32_t q = 0; q < per; q++) {
      const uint32_t b = tid * per + q;
      if (b < nbins) local += hist[b];
    }
    uint64_t run = block_excl_sum<kPart2Block>(local, sh64, nullptr);
    for (uint32_t q = 0; q < per; q++) {
      const uint32_t b = tid * per + q;
      if (b < nbins) {
        const uint64_t bucket = (uint64_t)b0 + b;
        if (bucket < P.nbuckets) {
          P.boff[bucket] = lo + run;
          P.bcount[bucket] = hist[b];
        }
        cur[b] = (uint32_t)run;
        run += hist[b];
      }
    }
  }
  __syncthreads();
  // pass B: rounds of kRound entries, grouped by bucket in the stage
  auto load_round = [&](Entry (&v)[kP2dPer], uint64_t i0) {
#pragma unroll
    for (int k = 0; k < kP2dPer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < hi) v[k] = P.ent3[i];
    }
  };
  Entry nx[kP2dPer];
  if (lo < hi) load_round(nx, lo);
  int par = 0;
  for (uint64_t i0 = lo; i0 < hi; i0 += kRound, par ^= 1) {
    Entry v[kP2dPer];
#pragma unroll
    for (int k = 0; k < kP2dPer; k++) v[k] = nx[k];
    if (i0 + kRound < hi) load_round(nx, i0 + kRound);
    uint32_t* rcnt = rc[par];
    uint32_t bk[kP2dPer], rk[kP2dPer];
#pragma unroll
    for (int k = 0; k < kP2dPer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      bk[k] = ~0u;
      const uint32_t b = bucket_of(P, v[k].hash) - b0;
      if (i >= hi || b >= nbins) continue;  // (foreign: reported by pass A)
      bk[k] = b;
      rk[k] = atomicAdd(&rcnt[b], 1u);
    }
    __syncthreads();
    {  // the round's run offsets; each bin's region cursor moves past the round; the other parity's
       // counts are cleared for the next round
      uint64_t local = 0;
      for (uint32_t q = 0; q < per; q++) {
        const uint32_t b = tid * per + q;
        if (b < nbins) local += rcnt[b];
      }
      uint64_t run = block_excl_sum<kPart2Block>(local, sh64, nullptr);
      for (uint32_t q = 0; q < per; q++) {
        const uint32_t b = tid * per + q;
        if (b < nbins) {
          roff[b] = (uint32_t)run;
          gbase[b] = cur[b];
          cur[b] += rcnt[b];
          run += rcnt[b];
          rc[par ^ 1][b] = 0;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kP2dPer; k++)
      if (bk[k] != ~0u) stage[roff[bk[k]] + rk[k]] = v[k];
    __syncthreads();
    const uint32_t nround = (uint32_t)min((uint64_t)kRound, hi - i0);
    for (uint32_t i = tid; i < nround; i += kPart2Block) {
      const Entry e = stage[i];
      const uint32_t b = bucket_of(P, e.hash) - b0;
      P.ent2[lo + gbase[b] + (i - roff[b])] = e;
    }
    __syncthreads();  // (the stage, roff and gbase are rewritten next round)
  }
}

// buckets of a sub-digit of the two-level pass 2 (k_part2_sub)
__host__ __device__ inline uint32_t sub_buckets(uint32_t bpp) { return (bpp + kSub - 1) / kSub; }

// k_part2f: k_part2d's staged scatter in ONE read of the digit's entries, into fixed bucket regions
// (bucket b's entries at ent2[b * kPlaceLdsMax ..), as k_part2st writes them) for tables of more than
// kP2SortedMaxBpp buckets per digit: no histogram pass, the bucket counts are the cursors at the end.
// A bucket past kPlaceLdsMax entries flags p2_overflow (the host redoes the build with k_part2d's dense
// runs; kPlaceLdsMax is 8 standard deviations over the mean bucket at the table's load).  The carry
// functions are k_summary's (no slot counts here: bpp x 1024 of them do not fit the LDS).  kPer entries
// a thread per round: 6 where the LDS holds them, fewer for the largest tables (C4's 4960 buckets a
// digit: 2, whose rounds are shorter than the bucket count -- runs of about one entry).  Single GPU.
// kC: 12-byte CEntry digit regions in and bucket regions out (BuildParams.compact).
// kSubIn: a workgroup per sub-digit of the two-level pass (k_part2_sub's regions in P.sub_ent: its
// bucket_sub buckets from the digit's sb-th on) instead of a workgroup per coarse digit.  A sub-digit's
// ~78 buckets leave room for their 8-bit slot counts beside a four-entry stage, so the pass also
// leaves each bucket's carry function, as k_part2st does (k_summary, which would read every entry
// again, does not run; a count past 255 flags p2_overflow and the host redoes the build dense).
template <int kPer, bool kC, bool kSubIn = false>
__global__ __launch_bounds__(kPart2Block) void k_part2f(BuildParams P) {
  // cur[nb] | rc0[nb] | rc1[nb] | roff[nb] | gbase[nb] | (kSubIn: h8[nb * 256]) | stage[kPart2Block * kPer]
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ uint64_t sh64[kPart2Block / 64 + 1];
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  uint64_t lo, hi;
  uint32_t nbins, b0;
  const Entry* src = P.ent3;
  if (kSubIn) {
    const uint32_t d = dpart / kSub, first = (dpart % kSub) * sub_buckets(P.bpp);
    nbins = first < P.bpp ? min(sub_buckets(P.bpp), P.bpp - first) : 0u;
    b0 = d * P.bpp + first;
    lo = (uint64_t)dpart * P.sub_region;
    hi = lo + min((uint64_t)P.sub_fill[dpart], P.sub_region);
    src = P.sub_ent;
  } else {
    lo = (uint64_t)dpart * P.p1_region;
    hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
    nbins = P.bpp;
    b0 = dpart * nbins;
  }
  uint32_t* cur = dyn;
  uint32_t* rc[2] = {cur + nbins, cur + 2 * nbins};
  uint32_t* roff = cur + 3 * nbins;
  uint32_t* gbase = cur + 4 * nbins;
  uint32_t* h = dyn + ((5 * nbins + 3) & ~3u);  // (kSubIn: 8-bit count per slot, four a word)
  const uint32_t hwords = kSubIn ? nbins * 256 : 0u;
  Entry* stage = reinterpret_cast<Entry*>(h + hwords);
  constexpr uint32_t kRound = kPart2Block * kPer;
  const int tid = threadIdx.x;
  for (uint32_t b = tid; b < ((5 * nbins + 3) & ~3u) + hwords; b += kPart2Block) dyn[b] = 0;
  __syncthreads();
  const uint32_t per = (nbins + kPart2Block - 1) / kPart2Block;
  bool ovf = false, bad = false;  // (bad: kGuardForeign)
  auto load_round = [&](Entry (&v)[kPer], uint64_t i0) {
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < hi) v[k] = kC ? load_craw(reinterpret_cast<const CEntry*>(src) + i) : src[i];
    }
  };
  Entry nx[kPer];
  if (lo < hi) load_round(nx, lo);
  int par = 0;
  for (uint64_t i0 = lo; i0 < hi; i0 += kRound, par ^= 1) {
    Entry v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) v[k] = nx[k];
    if (i0 + kRound < hi) load_round(nx, i0 + kRound);  // (in flight through this round)
    uint32_t* rcnt = rc[par];
    uint32_t bk[kPer], rk[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      bk[k] = ~0u;
      if (i >= hi) continue;
      const uint64_t slot = fast_mod(v[k].hash, P.mod);
      const uint32_t b = (uint32_t)(slot >> kBucketShift) - b0;
      bad |= b >= nbins;
      if (b >= nbins) continue;
      bk[k] = b;
      rk[k] = atomicAdd(&rcnt[b], 1u);
      if (kSubIn) {
        const uint32_t sl = (uint32_t)(slot & (kBucket - 1)), sh = (sl & 3u) * 8u;
        if (((atomicAdd(&h[(b << 8) + (sl >> 2)], 1u << sh) >> sh) & 0xffu) == 0xffu) ovf = true;  // (8-bit count full)
      }
    }
    __syncthreads();
    {  // the round's run offsets; each bucket's cursor moves past the round; the other parity's counts
       // are cleared for the next round
      uint64_t local = 0;
      for (uint32_t q = 0; q < per; q++) {
        const uint32_t b = tid * per + q;
        if (b < nbins) local += rcnt[b];
      }
      uint64_t run = block_excl_sum<kPart2Block>(local, sh64, nullptr);
      for (uint32_t q = 0; q < per; q++) {
        const uint32_t b = tid * per + q;
        if (b < nbins) {
          roff[b] = (uint32_t)run;
          gbase[b] = cur[b];
          cur[b] += rcnt[b];
          run += rcnt[b];
          rc[par ^ 1][b] = 0;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (bk[k] != ~0u) stage[roff[bk[k]] + rk[k]] = v[k];
    __syncthreads();
    const uint32_t nround = (uint32_t)min((uint64_t)kRound, hi - i0);
    for (uint32_t i = tid; i < nround; i += kPart2Block) {
      const Entry e = stage[i];
      const uint32_t b = bucket_of(P, e.hash) - b0;
      const uint32_t r = gbase[b] + (i - roff[b]);
      const uint64_t at = ((uint64_t)b0 + b - P.b_lo) * kPlaceLdsMax + r;
      if (r >= kPlaceLdsMax) ovf = true;
      else if (kC) store_craw(reinterpret_cast<CEntry*>(P.ent2) + at, e);
      else P.ent2[at] = e;
    }
    __syncthreads();  // (the stage, roff and gbase are rewritten next round)
  }
  if (ovf) atomicOr(&P.st->p2_overflow, 1u);
  report_foreign(P, bad);
  for (uint32_t b = tid; b < nbins; b += kPart2Block) {
    const uint64_t bucket = (uint64_t)b0 + b;
    if (bucket < P.nbuckets) {
      P.boff[bucket] = (bucket - P.b_lo) * (uint64_t)kPlaceLdsMax;
      P.bcount[bucket] = cur[b];
    }
  }
  if (!kSubIn) return;
  // per bucket (one wave each): the carry function from the slot counts (k_summary's, k_part2st's)
  const int lane = tid & 63, wave = tid >> 6;
  for (uint32_t b = wave; b < nbins; b += kPart2Block / 64) {
    const uint64_t bucket = (uint64_t)b0 + b;
    if (bucket >= P.nbuckets) continue;
    const uint32_t* hw = h + (b << 8) + lane * 4;  // this lane's 16 slots: 16 * lane ...
    uint32_t cnts[16];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t w = hw[k];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        cnts[4 * k + q] = (w >> (8 * q)) & 0xffu;
        tot += cnts[4 * k + q];
      }
    }
    const uint32_t incl = wave_incl_sum_u32(tot);
    uint32_t run = incl - tot;
    long long mx = -(1ll << 40);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (cnts[k]) mx = max(mx, (long long)(16 * lane + k) - (long long)run);
      run += cnts[k];
    }
    mx = wave_max_i64(mx);
    if (lane == 0) {
      const int64_t n = (int64_t)cur[b];
      const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - (bucket << kBucketShift));
      const int64_t mlast = mx < 0 ? 0 : mx;
      MaxPlus f;
      f.a = n - bsize;
      f.c = n ? max((int64_t)0, n + mlast - bsize) : 0;
      P.bfun[bucket] = f;
    }
  }
}

// k_part2f for tables whose rounds would hold about one entry per bucket (more than 3072 buckets a
// digit: C4's 4960): no stage, each entry stored at its bucket cursor's place (an LDS atomic), eight
// loads a thread in flight.  The stores scatter as the staged kernel's would at that size.
// kCI / kCO: 12-byte CEntry digit regions in / bucket regions out (BuildParams.compact's bits).
template <bool kCI, bool kCO>
__global__ __launch_bounds__(kPart2Block) void k_part2f_direct(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];  // per bucket of the digit
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  const uint64_t lo = (uint64_t)dpart * P.p1_region;
  const uint64_t hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
  const uint32_t nbins = P.bpp;
  const uint32_t b0 = dpart * nbins;
  const int tid = threadIdx.x;
  for (uint32_t b = tid; b < nbins; b += kPart2Block) cur[b] = 0;
  __syncthreads();
  constexpr int kIn = 8;
  bool ovf = false, bad = false;  // (bad: kGuardForeign)
  for (uint64_t i0 = lo; i0 < hi; i0 += (uint64_t)kPart2Block * kIn) {
    Entry v[kIn];
#pragma unroll
    for (int k = 0; k < kIn; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < hi) {
        const CEntry* c = reinterpret_cast<const CEntry*>(P.ent3) + i;
        v[k] = !kCI ? P.ent3[i] : kCO ? load_craw(c) : load_centry(P, c);
      }
    }
#pragma unroll
    for (int k = 0; k < kIn; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i >= hi) continue;
      const uint32_t b = bucket_of(P, v[k].hash) - b0;
      bad |= b >= nbins;
      if (b >= nbins) continue;
      const uint32_t r = atomicAdd(&cur[b], 1u);
      const uint64_t at = ((uint64_t)b0 + b - P.b_lo) * kPlaceLdsMax + r;
      if (r >= kPlaceLdsMax) ovf = true;
      else if (kCO) store_craw(reinterpret_cast<CEntry*>(P.ent2) + at, v[k]);
      else P.ent2[at] = v[k];
    }
  }
  if (ovf) atomicOr(&P.st->p2_overflow, 1u);
  report_foreign(P, bad);
  __syncthreads();
  for (uint32_t b = tid; b < nbins; b += kPart2Block) {
    const uint64_t bucket = (uint64_t)b0 + b;
    if (bucket < P.nbuckets) {
      P.boff[bucket] = (bucket - P.b_lo) * (uint64_t)kPlaceLdsMax;
      P.bcount[bucket] = cur[b];
    }
  }
}

// Two-level pass 2, for tables of thousands of buckets a digit (C4's 4960).  k_part2f_direct stores
// every entry at its bucket's cursor across the bucket regions of 256 digits at once: the stores land
// as partial lines, 3.15x their bytes written (26.5 GB for 8.4 GB of entries at 700M records,
// profiles/r06/meas/c4_700000000_write.txt).  Here k_part2_sub first splits each digit region into
// kSub regions of consecutive buckets (sub-digits) -- per tile of kPartTile entries, grouped in LDS and
// written as one run per sub-digit -- and k_part2f<.., kSubIn> then stages one sub-digit per
// workgroup into its bucket regions (runs of about a hundred entries a bucket and round).  A sub-digit region that fills up flags
// kSpecRegionFull (the host redoes the build with the two-pass partition).

// One tile of kPartTile entries a workgroup (persistent workgroups that load the next tile during this
// one's grouping measured 9.3 against 5.1 ms at C4: 235 VGPRs, two waves a SIMD,
// profiles/r06/c4/part2_sub_persistent_ab.txt).
template <bool kC>  // 12-byte CEntry regions in and out (BuildParams.compact)
__global__ __launch_bounds__(kPartBlock) void k_part2_sub(BuildParams P, uint32_t tiles_per_digit) {
  __shared__ Entry stage[kPartTile];
  __shared__ uint8_t ssub[kPartTile];  // sub-digit of each staged entry
  __shared__ uint32_t cnt[kSub], lbase[kSub + 1];
  __shared__ int64_t gdst[kSub];       // global index of the sub-digit's run minus its LDS start
  if (build_aborted(P)) return;
  const uint32_t d = blockIdx.x / tiles_per_digit, t = blockIdx.x % tiles_per_digit;
  const uint64_t fill = min((uint64_t)P.p1_fill[d], P.p1_region);
  const uint64_t lo = (uint64_t)t * kPartTile;
  if (lo >= fill) return;
  const uint32_t n = (uint32_t)min((uint64_t)kPartTile, fill - lo);
  const uint64_t base = (uint64_t)d * P.p1_region + lo;
  const uint32_t b0 = d * P.bpp, bps = sub_buckets(P.bpp);
  const int tid = threadIdx.x;
  if (tid < (int)kSub) cnt[tid] = 0;
  __syncthreads();
  Entry v[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    const uint32_t idx = (uint32_t)k * kPartBlock + tid;
    if (idx < n) v[k] = kC ? load_craw(reinterpret_cast<const CEntry*>(P.ent3) + base + idx) : P.ent3[base + idx];
  }
  uint32_t sg[kPartItems];
  bool bad = false;  // (kGuardForeign)
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    const uint32_t idx = (uint32_t)k * kPartBlock + tid;
    sg[k] = ~0u;
    if (idx >= n) continue;
    const uint32_t b = bucket_of(P, v[k].hash) - b0;
    bad |= b >= P.bpp;
    if (b >= P.bpp) continue;
    const uint32_t sb = b / bps;
    sg[k] = sb | (atomicAdd(&cnt[sb], 1u) << 8);  // rank inside the tile's sub-digit run
  }
  __syncthreads();
  if (tid < (int)kSub) {  // (wave 0: reserve each run, scan the counts)
    const uint32_t c = cnt[tid];
    const uint64_t g = c ? atomicAdd(&P.sub_fill[d * kSub + tid], c) : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o, 64);
      if (tid >= o) incl += x;
    }
    lbase[tid] = incl - c;
    if (tid == (int)kSub - 1) lbase[kSub] = incl;
    if (g + c > P.sub_region) atomicOr(&P.st->spec_fail, kSpecRegionFull);
    gdst[tid] = (int64_t)((uint64_t)(d * kSub + tid) * P.sub_region + g) - (int64_t)(incl - c);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    if (sg[k] == ~0u) continue;
    const uint32_t sb = sg[k] & 255u, pos = lbase[sb] + (sg[k] >> 8);
    stage[pos] = v[k];
    ssub[pos] = (uint8_t)sb;
  }
  __syncthreads();
  const uint32_t nkeep = lbase[kSub];
#pragma unroll
  for (int k = 0; k < kPartItems; k++) {
    const uint32_t i = (uint32_t)k * kPartBlock + tid;
    if (i >= nkeep) continue;
    const uint32_t sb = ssub[i];
    const uint64_t at = (uint64_t)(gdst[sb] + (int64_t)i);
    if (at >= (uint64_t)(d * kSub + sb + 1) * P.sub_region) continue;  // (flagged above)
    if (kC) store_craw(reinterpret_cast<CEntry*>(P.sub_ent) + at, stage[i]);
    else P.sub_ent[at] = stage[i];
  }
  report_foreign(P, bad);
}

// Sharded receive into fixed bucket regions, for tables of more than kP2SortedMaxBpp buckets a digit.
// Workgroup (x, k) takes slice x of coarse digit k's entries (its runs from every source rank,
// seg: nsrc (begin, end) runs of ent3, read back to back): it counts the slice per bucket in LDS,
// reserves each bucket's share of the bucket's fixed region with one returning global atomic on the
// bucket's count (zeroed by the host), and reads the slice again to store each entry at its place.
// The entries land in any order -- k_place_reg orders a bucket by (wanted slot, address) itself.
// Every CU is busy whatever the rank's share of the digits (k_part2 gives a digit one workgroup: 32
// workgroups a rank at N = 8); one atomic per entry instead of per (slice, bucket) measured 4.2 ms
// against k_part2's 1.9 at 125M entries.  A bucket past kPlaceLdsMax entries flags p2_overflow (the
// host redoes the step with dense runs).
__global__ __launch_bounds__(kPart2Block) void k_part2_recv(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cnt[];  // per bucket of the digit
  if (build_aborted(P)) return;
  constexpr int kIn = kPart2Items;
  const int tid = threadIdx.x;
  const uint32_t k = blockIdx.y, X = gridDim.x, x = blockIdx.x;
  const uint32_t nbins = P.bpp;
  const uint64_t b0 = (uint64_t)(P.p2_d0 + k) * nbins;
  const uint64_t* seg = P.p2_seg + 2ull * k * P.p2_nsrc;
  uint64_t tot = 0;
  for (uint32_t q = 0; q < P.p2_nsrc; q++) tot += seg[2 * q + 1] - seg[2 * q];
  const uint64_t vlo = tot * x / X, vhi = tot * (x + 1) / X;  // the slice, in the runs' concatenation
  for (uint32_t b = tid; b < nbins; b += kPart2Block) cnt[b] = 0;
  __syncthreads();
  // f(i, e) over the slice's entries, kIn loads a thread in flight
  auto each = [&](auto&& f) {
    uint64_t v0 = 0;
    for (uint32_t q = 0; q < P.p2_nsrc; q++) {
      const uint64_t a = seg[2 * q], n = seg[2 * q + 1] - a;
      const uint64_t lo = max(vlo, v0), hi = min(vhi, v0 + n);
      v0 += n;
      if (lo >= hi) continue;
      const uint64_t pa = a + (lo - (v0 - n)), pz = pa + (hi - lo);
      for (uint64_t i0 = pa; i0 < pz; i0 += (uint64_t)kPart2Block * kIn) {
        Entry v[kIn];
#pragma unroll
        for (int u = 0; u < kIn; u++) {
          const uint64_t i = i0 + (uint64_t)u * kPart2Block + tid;
          if (i < pz) v[u] = P.ent3[i];
        }
#pragma unroll
        for (int u = 0; u < kIn; u++)
          if (i0 + (uint64_t)u * kPart2Block + tid < pz) f(v[u]);
      }
    }
  };
  bool bad = false;  // (kGuardForeign)
  each([&](const Entry& e) {
    const uint32_t b = (uint32_t)(bucket_of(P, e.hash) - b0);
    if (b < nbins) atomicAdd(&cnt[b], 1u);
    else bad = true;
  });
  report_foreign(P, bad);
  __syncthreads();
  for (uint32_t b = tid; b < nbins; b += kPart2Block) {
    const uint32_t c = cnt[b];
    cnt[b] = c ? atomicAdd(&P.bcount[b0 + b], c) : 0u;
  }
  __syncthreads();
  bool ovf = false;
  each([&](const Entry& e) {
    const uint32_t b = (uint32_t)(bucket_of(P, e.hash) - b0);
    if (b >= nbins) return;  // (reported by the count pass)
    const uint32_t r = atomicAdd(&cnt[b], 1u);
    if (r < kPlaceLdsMax) P.ent2[(b0 + b - P.b_lo) * kPlaceLdsMax + r] = e;
    else ovf = true;
  });
  if (ovf) atomicOr(&P.st->p2_overflow, 1u);
  const uint64_t nblk = (uint64_t)gridDim.x * gridDim.y;
  for (uint64_t b = P.b_lo + ((uint64_t)k * gridDim.x + x) * kPart2Block + tid; b < P.b_hi; b += nblk * kPart2Block)
    P.boff[b] = (b - P.b_lo) * (uint64_t)kPlaceLdsMax;
}

bool part2_recv_fits(uint32_t bpp) { return (size_t)bpp * sizeof(uint32_t) <= 64 * 1024; }

void launch_part2_recv(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.p2_nd == 0) return;
  // about two workgroups a CU over the rank's digits
  const unsigned x = (unsigned)std::max<uint32_t>(1u, (512u + P.p2_nd - 1) / P.p2_nd);
  hipLaunchKernelGGL(k_part2_recv, dim3(x, P.p2_nd), dim3(kPart2Block), (size_t)P.bpp * sizeof(uint32_t), s, P);
  tm->mark("partition", s);
}

// Pass 2 for a table of up to kP2SortedMaxBpp buckets per digit (single GPU): the digit's entries
// are also counted per (bucket, wanted slot) in LDS (16-bit counts), so that the same pass leaves
// each bucket's max-plus carry function -- k_summary's output: F(x) = max(x + n - bsize,
// n + mlast - bsize), mlast = max over occupied s of s - base[s] -- without k_summary's read of the
// entries.  The entries themselves go out grouped by bucket as in k_part2 (each bucket's run written
// in order: ordering them by wanted slot here scattered the writes and measured 2x slower).  A digit
// with a bucket of more than 65535 entries (the counts could overflow) asks for the k_summary pass.
__global__ __launch_bounds__(kPart2Block) void k_part2s(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];  // h[bpp * 512] | btot[bpp] | boffl[bpp]
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  // input: the digit's run of the pass-1 output, or (sharded receive) its run in every source
  // rank's block of the exchange buffer; dense output (not p2_fixed) from `lo` on
  uint64_t lo, hi;
  const uint64_t* seg = nullptr;  // nseg (begin, end) runs of ent3
  uint32_t nseg = 1;
  if (P.p2_seg) {
    if (dpart < P.p2_d0 || dpart >= P.p2_d0 + P.p2_nd) return;
    const uint32_t k = dpart - P.p2_d0;
    lo = P.p2_out[k];
    hi = P.p2_out[k + 1];
    seg = P.p2_seg + 2ull * k * P.p2_nsrc;
    nseg = P.p2_nsrc;
  } else if (P.p1_region) {
    lo = (uint64_t)dpart * P.p1_region;
    hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
  } else {
    lo = P.p1_off[(uint64_t)dpart * P.p1_tiles];
    hi = (dpart + 1 < 256) ? P.p1_off[(uint64_t)(dpart + 1) * P.p1_tiles] : P.p1_off_total[0];
  }
  const uint32_t nbins = P.bpp;
  const uint64_t b0 = (uint64_t)dpart * nbins;
  __shared__ MaxPlus s_fun[kP2SortedMaxBpp];  // (fused_carry) the digit's bucket functions
  uint32_t* h = dyn;
  uint32_t* btot = dyn + nbins * 512;
  uint32_t* boffl = btot + nbins;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // p2_fixed: bucket b's entries go to its region ent2[b * kPlaceLdsMax ..) in this same pass (the
  // region cursor is the bucket count), so the digit is read once; a bucket that outgrows its region
  // (more entries than k_place_reg stages anyway) makes the host redo the build with dense runs
  const bool fixed = P.p2_fixed != 0;
  long long t_prev2 = P.part_dbg ? clock64() : 0;
  auto mark2 = [&](int i) {  // (SPARKEY_PART2_DEBUG: thread 0's cycles per phase)
    if (P.part_dbg && tid == 0) {
      const long long now = clock64();
      P.part_dbg[8 * (uint64_t)dpart + i] = now - t_prev2;
      t_prev2 = now;
    }
  };
  for (uint32_t i = tid; i < nbins * 512 + 2 * nbins; i += kPart2Block) dyn[i] = 0;
  if (tid < (int)kP2SortedMaxBpp) s_fun[tid] = MaxPlus{0, 0};
  __syncthreads();
  mark2(0);
  bool ovf = false, bad = false;  // (bad: kGuardForeign)
  // (software-pipelined: the next round's entries are in flight while this round's are counted and
  // stored -- one workgroup per CU, so nothing else hides the load latency; measured 5 rounds of
  // ~31K cycles each at C2 without it, SPARKEY_PART2_DEBUG)
  auto load_round = [&](Entry (&v)[kPart2Items], uint64_t i0, uint64_t rz) {
#pragma unroll
    for (int k = 0; k < kPart2Items; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < rz) {
        if (fixed) v[k] = P.ent3[i];
        else v[k].hash = P.ent3[i].hash;
      }
    }
  };
  for (uint32_t q = 0; q < nseg; q++) {
    const uint64_t ra = seg ? seg[2 * q] : lo, rz = seg ? seg[2 * q + 1] : hi;
    Entry nx[kPart2Items];
    if (ra < rz) load_round(nx, ra, rz);
    for (uint64_t i0 = ra; i0 < rz; i0 += (uint64_t)kPart2Block * kPart2Items) {
      Entry v[kPart2Items];
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) v[k] = nx[k];
      if (i0 + (uint64_t)kPart2Block * kPart2Items < rz) load_round(nx, i0 + (uint64_t)kPart2Block * kPart2Items, rz);
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        if (i >= rz) continue;
        const uint64_t slot = fast_mod(v[k].hash, P.mod);
        const uint32_t b = (uint32_t)((slot >> kBucketShift) - b0), sl = (uint32_t)(slot & (kBucket - 1));
        bad |= b >= nbins;
        if (b >= nbins) continue;
        atomicAdd(&h[(b << 9) + (sl >> 1)], 1u << ((sl & 1) * 16));
        const uint32_t r = atomicAdd(&btot[b], 1u);
        if (fixed) {  // (regions from the range's first bucket: a sharded rank holds its range only)
          if (r < kPlaceLdsMax) P.ent2[(b0 + b - P.b_lo) * (uint64_t)kPlaceLdsMax + r] = v[k];
          else ovf = true;
        }
      }
    }
  }
  if (ovf) atomicOr(&P.st->p2_overflow, 1u);
  report_foreign(P, bad);
  mark2(1);
  __syncthreads();
  mark2(2);
  bool big = false;
  for (uint32_t b = tid; b < nbins; b += kPart2Block) big |= btot[b] > 65535u;
  const bool summarise = !__syncthreads_or(big);
  if (!summarise && tid == 0) atomicOr(&P.st->need_summary, 1u);  // (rare)
  // bucket offsets within the digit (one wave; nbins <= 64)
  if (wave == 0) {
    const uint32_t c = (uint32_t)lane < nbins ? btot[lane] : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if ((uint32_t)lane < nbins) {
      boffl[lane] = incl - c;  // then the bucket's cursor
      const uint64_t bucket = b0 + lane;
      if (bucket < P.nbuckets) {
        P.boff[bucket] = fixed ? (bucket - P.b_lo) * (uint64_t)kPlaceLdsMax : lo + incl - c;
        P.bcount[bucket] = c;
      }
    }
  }
  // per bucket (one wave each): the carry function from the slot counts
  for (uint32_t b = wave; summarise && b < nbins; b += kPart2Block / 64) {
    const uint64_t bucket = b0 + b;
    if (bucket >= P.nbuckets) continue;
    const uint32_t* hw = h + (b << 9) + lane * 8;  // this lane's 16 slots: 16 * lane ...
    uint32_t cnts[16];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t w = hw[k];
      cnts[2 * k] = w & 0xffffu;
      cnts[2 * k + 1] = w >> 16;
      tot += cnts[2 * k] + cnts[2 * k + 1];
    }
    uint32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    uint32_t run = incl - tot;
    long long mx = -(1ll << 40);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (cnts[k]) mx = max(mx, (long long)(16 * lane + k) - (long long)run);
      run += cnts[k];
    }
    mx = wave_max_i64(mx);
    if (lane == 0) {
      const int64_t n = (int64_t)btot[b];
      const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - (bucket << kBucketShift));
      const int64_t mlast = mx < 0 ? 0 : mx;
      MaxPlus f;
      f.a = n - bsize;
      f.c = n ? max((int64_t)0, n + mlast - bsize) : 0;
      P.bfun[bucket] = f;
      s_fun[b] = f;
    }
  }
  mark2(3);
  if (P.fused_carry) {
    part2_fused_carry(P, s_fun, nbins, b0, dpart);
    mark2(4);
    return;
  }
  if (fixed) return;
  __syncthreads();
  for (uint32_t q = 0; q < nseg; q++) {
    const uint64_t ra = seg ? seg[2 * q] : lo, rz = seg ? seg[2 * q + 1] : hi;
    for (uint64_t i0 = ra; i0 < rz; i0 += (uint64_t)kPart2Block * kPart2Items) {
      Entry v[kPart2Items];
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        if (i < rz) v[k] = P.ent3[i];
      }
#pragma unroll
      for (int k = 0; k < kPart2Items; k++) {
        const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
        const uint32_t b = (uint32_t)(bucket_of(P, v[k].hash) - b0);
        if (i < rz && b < nbins) P.ent2[lo + atomicAdd(&boffl[b], 1u)] = v[k];  // (foreign: reported above)
      }
    }
  }
}

// k_part2st: k_part2s's fixed-region pass with its stores staged.  k_part2s stores every entry on
// its own (one L2 request per 16 bytes: 100K of its 160K cycles per digit at C2,
// profiles/r03/k_part2s_phases_c2.log).  Here each round of kP2Stage entries is grouped by bucket in
// LDS and leaves as one run per bucket.  The slot counts are 8-bit (4 per word), which frees the LDS
// for the stage; a count that would pass 255 flags p2_overflow, and the host redoes the build with
// dense runs (k_part2s's two-pass path).  Single GPU, fixed regions only.
// kCI / kCO: 12-byte CEntry digit regions in / bucket regions out (BuildParams.compact's bits; with
// both the entries keep the record index in their addr word from the load to the store)
template <int kP2StagePer, bool kCI, bool kCO>
__global__ __launch_bounds__(kPart2Block) void k_part2st(BuildParams P) {
  constexpr int kP2Stage = kPart2Block * kP2StagePer;
  // h8[bpp * 256] | btot[bpp] | rcnt[bpp] | roff[bpp] | gbase[bpp] | stage[kP2Stage]
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  if (build_aborted(P)) return;
  const uint32_t dpart = blockIdx.x;
  const uint64_t lo = (uint64_t)dpart * P.p1_region;
  const uint64_t hi = lo + min((uint64_t)P.p1_fill[dpart], P.p1_region);
  const uint32_t nbins = P.bpp;
  const uint64_t b0 = (uint64_t)dpart * nbins;
  __shared__ MaxPlus s_fun[kP2SortedMaxBpp];
  uint32_t* h = dyn;
  uint32_t* btot = dyn + nbins * 256;
  uint32_t* rcnt = btot + nbins;
  uint32_t* roff = rcnt + nbins;
  uint32_t* gbase = roff + nbins;
  Entry* stage = reinterpret_cast<Entry*>(dyn + ((nbins * 260 + 3) & ~3u));
  uint8_t* sbk = reinterpret_cast<uint8_t*>(stage + kP2Stage);  // each staged entry's bucket (no second fast_mod)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long t_prev2 = P.part_dbg ? clock64() : 0;
  auto mark2 = [&](int i) {  // (SPARKEY_PART2_DEBUG: thread 0's cycles per phase)
    if (P.part_dbg && tid == 0) {
      const long long now = clock64();
      P.part_dbg[8 * (uint64_t)dpart + i] = now - t_prev2;
      t_prev2 = now;
    }
  };
  for (uint32_t i = tid; i < nbins * 260; i += kPart2Block) dyn[i] = 0;
  if (tid < (int)kP2SortedMaxBpp) s_fun[tid] = MaxPlus{0, 0};
  __syncthreads();
  mark2(0);
  bool ovf = false, bad = false;  // (bad: kGuardForeign)
  auto load_round = [&](Entry (&v)[kP2StagePer], uint64_t i0) {
#pragma unroll
    for (int k = 0; k < kP2StagePer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      if (i < hi) {
        const CEntry* c = reinterpret_cast<const CEntry*>(P.ent3) + i;
        v[k] = !kCI ? P.ent3[i] : kCO ? load_craw(c) : load_centry(P, c);
      }
    }
  };
  Entry nx[kP2StagePer];
  if (lo < hi) load_round(nx, lo);
  for (uint64_t i0 = lo; i0 < hi; i0 += kP2Stage) {
    Entry v[kP2StagePer];
#pragma unroll
    for (int k = 0; k < kP2StagePer; k++) v[k] = nx[k];
    if (i0 + kP2Stage < hi) load_round(nx, i0 + kP2Stage);  // (in flight through this round)
    uint32_t bk[kP2StagePer], rk[kP2StagePer];
#pragma unroll
    for (int k = 0; k < kP2StagePer; k++) {
      const uint64_t i = i0 + (uint64_t)k * kPart2Block + tid;
      bk[k] = ~0u;
      if (i >= hi) continue;
      const uint64_t slot = fast_mod(v[k].hash, P.mod);
      const uint32_t b = (uint32_t)((slot >> kBucketShift) - b0), sl = (uint32_t)(slot & (kBucket - 1));
      bad |= b >= nbins;  // (bk stays ~0u: no LDS index, no store)
      if (b >= nbins) continue;
      const uint32_t sh = (sl & 3u) * 8u;
      if (((atomicAdd(&h[(b << 8) + (sl >> 2)], 1u << sh) >> sh) & 0xffu) == 0xffu) ovf = true;  // (8-bit count full)
      bk[k] = b;
      rk[k] = atomicAdd(&rcnt[b], 1u);
    }
    __syncthreads();
    if (wave == 0) {  // the round's run offsets, and each bucket's region cursor before the round
      const uint32_t c = (uint32_t)lane < nbins ? rcnt[lane] : 0u;
      uint32_t incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if ((uint32_t)lane < nbins) {
        roff[lane] = incl - c;
        gbase[lane] = btot[lane];
        btot[lane] += c;
        rcnt[lane] = 0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kP2StagePer; k++) {
      if (bk[k] == ~0u) continue;
      stage[roff[bk[k]] + rk[k]] = v[k];
      sbk[roff[bk[k]] + rk[k]] = (uint8_t)bk[k];
    }
    __syncthreads();
    // the runs: consecutive lanes on consecutive entries of a bucket's region
    const uint32_t nround = (uint32_t)min((uint64_t)kP2Stage, hi - i0);
    for (uint32_t i = tid; i < nround; i += kPart2Block) {
      const Entry e = stage[i];
      const uint32_t b = sbk[i];
      const uint32_t r = gbase[b] + (i - roff[b]);
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const uint64_t at = (b0 + b - P.b_lo) * (uint64_t)kPlaceLdsMax + r;
      if (r >= kPlaceLdsMax) ovf = true;
      else if (kCO) store_craw(reinterpret_cast<CEntry*>(P.ent2) + at, e);  // (a non-temporal 3-dword store measured slower)
      else __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(&e), reinterpret_cast<u32x4*>(&P.ent2[at]));
    }
    __syncthreads();  // (the stage and the offsets are rewritten next round)
  }
  if (ovf) atomicOr(&P.st->p2_overflow, 1u);
  report_foreign(P, bad);
  mark2(1);
  mark2(2);
  // bucket offsets (fixed regions) and counts
  if (wave == 0 && (uint32_t)lane < nbins) {
    const uint64_t bucket = b0 + lane;
    if (bucket < P.nbuckets) {
      P.boff[bucket] = (bucket - P.b_lo) * (uint64_t)kPlaceLdsMax;
      P.bcount[bucket] = btot[lane];
    }
  }
  // per bucket (one wave each): the carry function from the slot counts
  for (uint32_t b = wave; b < nbins; b += kPart2Block / 64) {
    const uint64_t bucket = b0 + b;
    if (bucket >= P.nbuckets) continue;
    const uint32_t* hw = h + (b << 8) + lane * 4;  // this lane's 16 slots: 16 * lane ...
    uint32_t cnts[16];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t w = hw[k];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        cnts[4 * k + q] = (w >> (8 * q)) & 0xffu;
        tot += cnts[4 * k + q];
      }
    }
    uint32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    uint32_t run = incl - tot;
    long long mx = -(1ll << 40);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (cnts[k]) mx = max(mx, (long long)(16 * lane + k) - (long long)run);
      run += cnts[k];
    }
    mx = wave_max_i64(mx);
    if (lane == 0) {
      const int64_t n = (int64_t)btot[b];
      const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - (bucket << kBucketShift));
      const int64_t mlast = mx < 0 ? 0 : mx;
      MaxPlus f;
      f.a = n - bsize;
      f.c = n ? max((int64_t)0, n + mlast - bsize) : 0;
      P.bfun[bucket] = f;
      s_fun[b] = f;
    }
  }
  mark2(3);
  part2_fused_carry(P, s_fun, nbins, b0, dpart);
  mark2(4);
}

// ================================================================================================
// Placement: one bucket per workgroup (buckets above kPlaceLdsMax entries are left to the
// global-memory k_place, flagged in P.st->big_buckets).
// ================================================================================================
__device__ __forceinline__ bool is_put_pair(const Entry& x, const Entry& y) {  // a duplicate-key candidate
  return x.hash == y.hash && !(x.addr & kDelBit) && !(y.addr & kDelBit);
}

// ================================================================================================
// k_place_reg: the canonical placement of one bucket, its entries kept in registers.  Per bucket: the 16-bit count of each wanted slot (its atomic is the entry's place
// in its group), one scan for base[s] (entries wanted before s) and M[s] (the prefix max of
// s - base[s] over occupied s), the entries copied to base[w] + cursor so that each group of equal
// wanted slots lies together, then every entry's rank in its group by address (IndexHash.java:647-650,
// SortHelper's (wantedSlot, address) order) and its position j + max(carry, M[w]).  The block writes
// its slots [x, hi) in order (coalesced: scattered 16-byte stores cost one L2 request each, which
// measured 2.4x slower), entries out of LDS through a slot -> entry map.  27 KiB of LDS (the round-2
// kernel that staged the bucket in LDS took 36 KiB and 0.170 against 0.154 ms on C2), 4 waves per
// block, 5 blocks per CU; the fixed regions' entry loads go out before the head.
// ================================================================================================
constexpr int kPlaceRegBlock = 256;
constexpr int kPlaceRegPer = kPlaceLdsMax / kPlaceRegBlock;

// One bucket of k_place_reg: bucket b_lo + bi; pre[] holds its fixed-region entries when kFixed.
template <bool kFixed>
__device__ __forceinline__ void place_reg_bucket(const BuildParams& P, uint64_t bi, const Entry (&pre)[kPlaceRegPer]) {
  constexpr int NW = kPlaceRegBlock / 64;
  static_assert(kBucket == 4 * kPlaceRegBlock, "four wanted slots per thread in the scan");
  // (each array has one more element: the place of the lanes past the bucket's count, so that the
  //  unrolled loops below run without a branch per entry -- the kernel is SALU-bound)
  __shared__ uint32_t cnt[kBucket / 2 + 1];      // 16-bit entry count per wanted slot
  __shared__ uint32_t meta[kBucket + 1];         // base[s] | (M[s] + 32768) << 16
  __shared__ Entry buf[kPlaceLdsMax + 1];        // each group's members together (any order inside)
  __shared__ int16_t slot_of[2 * kBucket + 2];   // slot x + t -> its entry's buf index, -1: empty
  __shared__ uint32_t wsum[NW];
  __shared__ int32_t wmax[NW];
  __shared__ uint64_t sh64[NW + 1];
  __shared__ unsigned long long pair_base;
  __shared__ unsigned long long r_sum[NW], r_col[NW];
  __shared__ long long r_max[NW];
  __shared__ int32_t s_pend;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  Entry mine[kPlaceRegPer];
  constexpr bool fixed = kFixed;
  if (fixed) {
#pragma unroll
    for (int k = 0; k < kPlaceRegPer; k++) mine[k] = pre[k];
  }
  const Status* st = P.st;
  const unsigned ovf = st->overflow | st->p2_overflow | (P.abort_on_fail ? st->spec_fail : 0u), full = st->full;
  const unsigned long long nrec = st->n_records, ndel = st->n_deletes, npairs0 = st->n_pairs;
  const bool failed = P.abort_on_fail && st->err != ~0ull;
  const uint64_t b = P.b_lo + bi;
  const uint32_t n = P.bcount[b];
  const uint64_t eoff = P.boff[b];
  int64_t x;
  if (P.fused_carry) {
    const MaxPlus pre = P.bpre[b];
    x = max(pre.c, P.dcarry[b / P.bpp] + pre.a);
  } else {
    x = P.carry[b];
  }
  if (ovf != 0 || failed || nrec > P.max_records) return;  // build_aborted
  if (P.fused_carry && tid == 0) P.carry[b] = x;  // (for the global-memory placement's readers)
  const uint64_t start = b << kBucketShift;
  const int64_t bsize = (int64_t)min((uint64_t)kBucket, P.cap - start);
  if (n > kPlaceLdsMax) {  // (never with fixed regions: p2_overflow above)
    if (tid == 0) atomicOr(&P.st->big_buckets, 1u);
    return;
  }
  if (!fixed) {
#pragma unroll
    for (int k = 0; k < kPlaceRegPer; k++) {
      const uint32_t i = tid + k * kPlaceRegBlock;
      if (i < n) mine[k] = P.ent2[eoff + i];
    }
  }
  // (the loads are in flight while the counts are cleared)
  for (int t = tid; t < kBucket / 2; t += kPlaceRegBlock) cnt[t] = 0;
  for (int t = tid; t < kBucket; t += kPlaceRegBlock) reinterpret_cast<uint32_t*>(slot_of)[t] = 0xffffffffu;
  if (tid == 0) s_pend = 0;
  __syncthreads();
  uint32_t want[kPlaceRegPer], cur[kPlaceRegPer];
  bool bad = false;  // (kGuardForeign: an entry of another bucket in this bucket's region)
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    const uint32_t i = tid + k * kPlaceRegBlock;
    const uint64_t w = fast_mod(mine[k].hash, P.mod) - start;
    bad |= i < n && w >= (uint64_t)kBucket;
    want[k] = i < n && w < (uint64_t)kBucket ? (uint32_t)w : (uint32_t)kBucket;  // (kBucket: past n, or foreign)
    const uint32_t sh = (want[k] & 1u) * 16u;
    cur[k] = (atomicAdd(&cnt[want[k] >> 1], 1u << sh) >> sh) & 0xffffu;
  }
  report_foreign(P, bad);
  __syncthreads();
  // scan of slots 4 tid .. 4 tid + 3: base (exclusive count) and M (prefix max of s - base[s] over
  // occupied s), one barrier: a wave's max of (s - its local base) needs only the waves' sums after it
  {
    const uint32_t w0 = cnt[2 * tid], w1 = cnt[2 * tid + 1];
    const uint32_t c[4] = {w0 & 0xffffu, w0 >> 16, w1 & 0xffffu, w1 >> 16};
    const uint32_t tot = c[0] + c[1] + c[2] + c[3];
    const uint32_t incl = wave_incl_sum_u32(tot);  // (DPP: no LDS crossbar round trips)
    constexpr int32_t kNone = -(1 << 20);
    uint32_t lb[4];
    int32_t v = kNone;  // max over this thread's occupied slots of s - (wave-local base)
    {
      uint32_t run = incl - tot;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        lb[i] = run;
        if (c[i]) v = max(v, (int32_t)(4 * tid + i) - (int32_t)run);
        run += c[i];
      }
    }
    const int32_t mi = wave_incl_max_i32(v);  // inclusive wave prefix max
    if (lane == 63) {
      wsum[wv] = incl;
      wmax[wv] = mi;
    }
    __syncthreads();
    uint32_t off = 0;
    int32_t pre = kNone;
#pragma unroll
    for (int u = 0; u < NW; u++) {
      if (u < wv) {
        pre = max(pre, wmax[u] == kNone ? kNone : wmax[u] - (int32_t)off);
        off += wsum[u];
      }
    }
    const int32_t ex = wave_prev_i32(mi, kNone);  // exclusive wave prefix max (wave-local), then block-level
    int32_t m = max(pre, ex == kNone ? kNone : ex - (int32_t)off);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t base = off + lb[i];
      if (c[i]) m = max(m, (int32_t)(4 * tid + i) - (int32_t)base);
      const int32_t mc = max(m, -32768);
      meta[4 * tid + i] = base | ((uint32_t)(mc + 32768) << 16);
    }
  }
  __syncthreads();
  uint32_t bw[kPlaceRegPer], g[kPlaceRegPer];
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    const bool valid = want[k] < (uint32_t)kBucket;
    bw[k] = valid ? meta[want[k]] & 0xffffu : (uint32_t)kPlaceLdsMax;
    g[k] = valid ? (cnt[want[k] >> 1] >> ((want[k] & 1u) * 16u)) & 0xffffu : 0u;
    buf[bw[k] + (valid ? cur[k] : 0u)] = mine[k];
  }
  __syncthreads();
  // Equal wanted slots in address order: each member counts the members with smaller addresses.
  const bool want_pairs = ndel == 0 && npairs0 <= P.pair_cap;
  uint32_t npair = 0;
  uint32_t rank[kPlaceRegPer];
  // One loop per wave over its lanes' largest group (a wave-uniform trip count), selects instead of
  // branches: per-lane loops' exec-mask bookkeeping made this kernel SALU-bound
  uint32_t gl = 0;
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    rank[k] = 0;
    gl = max(gl, g[k] >= 2 ? g[k] : 0u);
    if (g[k] > kGroupMax && cur[k] == 0) atomicOr(&P.st->dup_overflow, 1u);
  }
  const uint32_t gw = (uint32_t)wave_max_i32((int32_t)gl);
  uint32_t eqh = 0;  // another member with this entry's hash (duplicate keys: rare)
  for (uint32_t u = 0; u < gw; u++) {
#pragma unroll
    for (int k = 0; k < kPlaceRegPer; k++) {
      const bool act = u < g[k];  // (a lone entry meets only itself)
      const Entry e = buf[bw[k] + (act ? u : 0u)];
      const uint64_t ai = mine[k].addr & ~kDelBit;
      const uint64_t aj = e.addr & ~kDelBit;
      rank[k] += act && aj < ai ? 1u : 0u;
      eqh |= (uint32_t)act & (uint32_t)(aj != ai) & (uint32_t)(e.hash == mine[k].hash);  // (no branches)
    }
  }
  // Equal-hash PUT pairs (duplicate-key candidates, for the pair list): counted and written only by
  // blocks that met an equal hash at all
  if (__syncthreads_or(eqh != 0 && want_pairs)) {  // (block-uniform)
#pragma unroll
    for (int k = 0; k < kPlaceRegPer; k++) {
      if (g[k] < 2 || g[k] > kGroupMax || (mine[k].addr & kDelBit)) continue;
      const uint64_t ai = mine[k].addr & ~kDelBit;
      for (uint32_t u = 0; u < g[k]; u++) {
        const Entry e = buf[bw[k] + u];
        npair += (e.addr & ~kDelBit) > ai && is_put_pair(mine[k], e) ? 1u : 0u;
      }
    }
    uint64_t pair_total = 0;
    const uint64_t pair_off = block_excl_sum<kPlaceRegBlock>(npair, sh64, &pair_total);
    if (tid == 0) pair_base = atomicAdd(&P.st->n_pairs, (unsigned long long)pair_total);
    __syncthreads();
    unsigned long long slotn = pair_base + pair_off;
#pragma unroll
    for (int k = 0; k < kPlaceRegPer; k++) {
      if (!npair || g[k] < 2 || g[k] > kGroupMax || (mine[k].addr & kDelBit)) continue;
      const Entry* grp = buf + bw[k];
      const uint64_t ai = mine[k].addr & ~kDelBit;
      for (uint32_t u = 0; u < g[k]; u++) {
        const Entry e = grp[u];
        if ((e.addr & ~kDelBit) <= ai || !is_put_pair(mine[k], e)) continue;
        if (slotn < P.pair_cap) {
          P.pairs[2 * slotn] = mine[k].addr;
          P.pairs[2 * slotn + 1] = e.addr;
        }
        slotn++;
      }
    }
  }
  if (full) return;
  // positions, the entries' slots, the occupancy bitmap and the displacements
  const bool nt16 = P.slot_size == 16 && !P.sharded && P.uni_nt;
  const uint64_t lim = P.sharded ? P.slot_hi : ~0ull;
  unsigned long long sum_d = 0, col = 0;
  long long max_d = 0;
  int32_t pend = 0;
  int64_t pos[kPlaceRegPer];
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    const bool valid = want[k] < (uint32_t)kBucket;
    const int32_t M = (int32_t)(meta[want[k]] >> 16) - 32768;
    const int64_t p = (int64_t)(bw[k] + rank[k]) + max(x, (int64_t)M);
    pos[k] = valid ? p : -1;
    slot_of[valid ? p - x : (int64_t)(2 * kBucket + 1)] = (int16_t)(bw[k] + cur[k]);  // (where the entry sits in buf)
    const int64_t d = valid ? p - (int64_t)want[k] : 0;
    sum_d += (unsigned long long)d;  // getDisplacement (IndexHash.java:671-678)
    max_d = max(max_d, (long long)d);
    pend = max(pend, valid ? (int32_t)(p + 1) : 0);
  }
  pend = wave_max_i32(pend);
  if (lane == 0 && pend > 0) atomicMax(&s_pend, pend);
  __syncthreads();
  // the pair (slot - 1, slot) inside the block's range: equal hashes share a wanted slot, so they are
  // members of one group ranked next to each other -- the member in slot p - 1 of a member ranked
  // after another (calculateMaxDisplacement, IndexHash.java:195-245)
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    const int64_t p = pos[k];
    const bool act = p >= 0 && rank[k] > 0;
    const Entry e = buf[act ? slot_of[p - 1 - x] : 0];
    col += act && e.hash == mine[k].hash && wrap_slot(start + (uint64_t)p, P.cap) != 0 && start + (uint64_t)p < lim;
  }
  const int64_t hi = max(bsize, (int64_t)s_pend);
  // the block's slots [x, hi) in order, consecutive lanes on consecutive slots: its entries out of
  // buf, zeros where none landed (the run spilled past the bucket has no gap)
  if (hi <= bsize) {  // (block-uniform, the usual case: no run spilled past the bucket, so every slot
    // is in a sharded rank's range too) no wrap, no per-slot branches: 32-bit offsets, selects,
    // non-temporal stores of the slot's words (16-, 12- and 8-byte slots: write_slot's layouts)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const uint32_t ss = P.slot_size;
    const bool h8 = P.hash_size == 8;
    uint8_t* dst = P.out + kIndexHeaderSize + start * (uint64_t)ss;
    for (int32_t t = (int32_t)x + tid; t < (int32_t)hi; t += kPlaceRegBlock) {
      const int32_t v = slot_of[t - (int32_t)x];
      const Entry en = buf[v >= 0 ? v : 0];
      const uint64_t hh = v >= 0 ? en.hash : 0ull, aa = v >= 0 ? en.addr & ~kDelBit : 0ull;
      uint8_t* q = dst + (uint32_t)t * ss;
      if (ss == 16) {
        u32x4 w;
        w.x = (uint32_t)hh;
        w.y = (uint32_t)(hh >> 32);
        w.z = (uint32_t)aa;
        w.w = (uint32_t)(aa >> 32);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(q));
      } else if (ss == 8) {
        u32x2 w;
        w.x = (uint32_t)hh;
        w.y = (uint32_t)aa;
        __builtin_nontemporal_store(w, reinterpret_cast<u32x2*>(q));
      } else {  // 12: 8 + 4 or 4 + 8 (4-byte aligned: three dword stores)
        uint32_t* d = reinterpret_cast<uint32_t*>(q);
        __builtin_nontemporal_store((uint32_t)hh, d);
        __builtin_nontemporal_store(h8 ? (uint32_t)(hh >> 32) : (uint32_t)aa, d + 1);
        __builtin_nontemporal_store(h8 ? (uint32_t)aa : (uint32_t)(aa >> 32), d + 2);
      }
    }
  } else {
    for (int64_t t = x + tid; t < hi; t += kPlaceRegBlock) {
      const int32_t v = slot_of[t - x];
      const uint64_t slot = t < bsize ? start + (uint64_t)t : wrap_slot(start + (uint64_t)t, P.cap);
      uint64_t hh = 0, aa = 0;
      if (v >= 0) {
        const Entry en = buf[v];
        hh = en.hash;
        aa = en.addr & ~kDelBit;
      }
      if (nt16) {  // the table is written once: non-temporal stores
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 w;
        w.x = (uint32_t)hh;
        w.y = (uint32_t)(hh >> 32);
        w.z = (uint32_t)aa;
        w.w = (uint32_t)(aa >> 32);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(P.out + kIndexHeaderSize + slot * 16ull));
      } else if (v >= 0) {
        put_slot(P, slot, hh, aa);
      } else {
        write_slot(P, slot, 0, 0);
      }
    }
  }
  if (!P.fold_stats) return;
  // an entry of hash 0 before an empty slot of the range (an empty slot reads as hash 0)
#pragma unroll
  for (int k = 0; k < kPlaceRegPer; k++) {
    const int64_t p = pos[k];
    if (p < 0 || mine[k].hash != 0 || p + 1 >= hi) continue;
    if (slot_of[p + 1 - x] < 0 && wrap_slot(start + (uint64_t)p + 1, P.cap) != 0 &&
        start + (uint64_t)p + 1 < lim)
      col++;
  }
  if (x < (1ll << 20)) {  // (block-uniform) every displacement < 2^21: 32-bit DPP reductions
    sum_d = wave_sum_u32((uint32_t)sum_d);
    max_d = wave_max_i32((int32_t)max_d);
  } else {
    sum_d = wave_sum_u64(sum_d);
    max_d = wave_max_i64(max_d);
  }
  col = wave_sum_u32((uint32_t)col);
  if (lane == 0) {
    r_sum[wv] = sum_d;
    r_col[wv] = col;
    r_max[wv] = max_d;
  }
  __syncthreads();
  if (tid == 0) {
    StatPart sp{0, 0, 0};
    for (int w = 0; w < NW; w++) {
      sp.sum_disp += r_sum[w];
      sp.collisions += r_col[w];
      sp.max_disp = max(sp.max_disp, r_max[w]);
    }
    P.parts[b] = sp;
    P.bstat_start[b] = hi > x ? wrap_slot(start + (uint64_t)x, P.cap) : ~0ull;
  }
}


// k_place_reg: one block per bucket.  With fixed regions (kFixed: a template parameter, so that no
// branch joins the loads and the wave runs on to the head's scalar loads with them in flight) the first
// three quarters of the region are loaded with the bucket's count (a bucket at load 0.77 holds about
// 790 entries), the last quarter only up to the count (it read 23% more bytes than the entries).
// kC: the fixed regions hold 12-byte CEntry (BuildParams.compact), expanded to Entry on the load.
template <bool kFixed, bool kC = false>
__global__ __launch_bounds__(kPlaceRegBlock) void k_place_reg(BuildParams P) {
  Entry pre[kPlaceRegPer];
  if (kFixed) {
    const uint64_t e0 = (uint64_t)blockIdx.x * kPlaceLdsMax;
    const uint32_t n = P.bcount[P.b_lo + blockIdx.x];
    constexpr uint32_t kLast = (kPlaceRegPer - 1) * kPlaceRegBlock;
    // (no branch: lanes past the count reload their first entry's line, which the cache holds)
    const uint64_t last = e0 + threadIdx.x + (threadIdx.x + kLast < n ? kLast : 0u);
    if (kC) {
      const CEntry* c2 = reinterpret_cast<const CEntry*>(P.ent2);
#pragma unroll
      for (int k = 0; k < kPlaceRegPer - 1; k++) pre[k] = load_centry(P, c2 + e0 + threadIdx.x + k * kPlaceRegBlock);
      pre[kPlaceRegPer - 1] = load_centry(P, c2 + last);
    } else {
#pragma unroll
      for (int k = 0; k < kPlaceRegPer - 1; k++) pre[k] = P.ent2[e0 + threadIdx.x + k * kPlaceRegBlock];
      pre[kPlaceRegPer - 1] = P.ent2[last];
    }
  }
  place_reg_bucket<kFixed>(P, blockIdx.x, pre);
}

// (inject_foreign switch: tests of kGuardForeign) The first entry of digit 0's region (ent3, before
// pass 2: where 1) or of the range's first bucket region (ent2, before the placement: where 2) becomes
// an entry of the table's last bucket -- a region whose contents disagree with its count, as a bug or
// a half-written region would leave it.  Its hash is below the capacity, so it wants slot hash.
__global__ void k_inject_foreign(BuildParams P, int where) {
  if (threadIdx.x || blockIdx.x || P.nbuckets < 2 || build_aborted(P)) return;
  const uint64_t h = (P.nbuckets - 1) << kBucketShift;
  if (where == 1 && P.p1_region && P.p1_fill[0] > 0) P.ent3[0].hash = h;
  if (where == 2 && P.p2_fixed && P.bcount[P.b_lo] > 0) P.ent2[0].hash = h;
}

// ================================================================================================
// launchers
// ================================================================================================
void launch_frame_fused(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.fr_nchunks == 0) return;
  const uint64_t nwaves = (P.fr_nchunks + P.fr_w - 1) / P.fr_w;
  // the screen's bitmap (one bit per candidate-window byte), later overlaid by the balanced walk's
  // candidate list and then by the record list
  const size_t lds = (size_t)P.fr_rgn_bytes + std::max<size_t>((size_t)P.fr_w * P.fr_mask_words * 8 + 8, kCandCap * 4);
  const uint32_t per = (uint32_t)((lds + 15) & ~(size_t)15);
  hipLaunchKernelGGL(k_frame, dim3((unsigned)nwaves), dim3(64), (size_t)per, s, P, per);
  tm->mark("frame", s);  // the stage is k_frame alone (its rocprof row); the slab scan counts as partition
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.wcount, P.woff, P.nslabs, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
}

void launch_frame_uniform(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.uni_n == 0) return;
  BuildParams Q = P;
  // 4 waves per workgroup, double-buffered: two workgroups per CU, each wave's next DMA in flight while
  // it hashes (single-buffered 16- and 8-wave workgroups, one per CU, measured slower)
  constexpr int W = 4;
  Q.uni_wbytes = (uint32_t)((64 * P.uni_rec + 32 + 1023) & ~1023ll);
  Q.uni_nt = 1u;  // (the log is read once: non-temporal staging measured 10% faster)
  const uint64_t nblk = (P.uni_n + kPartTile - 1) / kPartTile;  // a partition tile a workgroup
  // the wave buffers, then the tile regrouped by digit in the same space (entries, digits, run
  // starts), and hist + rbase after either (tiles of 2048 records measured slower: profiles/r05/c2/)
  const size_t body = std::max<size_t>((size_t)W * Q.uni_wbytes * 2, (size_t)kPartTile * (sizeof(Entry) + 1) + 1024);
  Q.uni_hist_off = (uint32_t)body;
  // persistent: two workgroups a CU (the LDS), each over every 512th tile
  hipLaunchKernelGGL((k_frame_uniform<W, true>), dim3((unsigned)std::min<uint64_t>(nblk, 512)), dim3(64 * W), body + 2048, s, Q);
  tm->mark("frame", s);
}

void launch_dense_slabs(const BuildParams& P, hipStream_t s) {
  hipLaunchKernelGGL(k_dense_slabs, dim3((unsigned)((P.nslabs + 255) / 256)), dim3(256), 0, s, P);
}

void launch_partition1(const BuildParams& P, hipStream_t s) {
  if (!P.p1_hist_ready) hipLaunchKernelGGL(k_part1_hist, dim3((unsigned)P.p1_tiles), dim3(kPartBlock), 0, s, P);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.p1_hist, P.p1_off, (uint64_t)P.p1_tiles * 256, P.p1_off_total,
                                            OpAdd(), P.scan_scratch_u64, s);
  hipLaunchKernelGGL(k_part1_scatter, dim3((unsigned)P.p1_tiles), dim3(kPartBlock), 0, s, P);
}

void launch_partition_quiet(const BuildParams& P, hipStream_t s) {
  launch_partition1(P, s);
  hipLaunchKernelGGL(k_part2, dim3(256), dim3(kPart2Block), (size_t)(2u * P.bpp) * sizeof(uint32_t), s, P);
}

void launch_partition2(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.p2_sorted)
    hipLaunchKernelGGL(k_part2s, dim3(256), dim3(kPart2Block), (size_t)(514u * P.bpp) * sizeof(uint32_t), s, P);
  else
    hipLaunchKernelGGL(k_part2, dim3(256), dim3(kPart2Block), (size_t)(2u * P.bpp) * sizeof(uint32_t), s, P);
  tm->mark("partition", s);
}

// k_part2d's dynamic LDS (six words a bucket, the stage)
static size_t part2d_lds(uint32_t bpp) {
  return (size_t)((6 * bpp + 3) & ~3u) * 4 + (size_t)kPart2Block * kP2dPer * sizeof(Entry);
}

static size_t part2f_lds(uint32_t bpp, int per) {
  return (size_t)((5 * bpp + 3) & ~3u) * 4 + (size_t)kPart2Block * per * sizeof(Entry);
}
bool part2f_fits(uint32_t bpp) { return bpp > kPart2Block * 3 ? bpp * 4 <= 158 * 1024 : part2f_lds(bpp, 2) <= 158 * 1024; }

// k_part2st's dynamic LDS (the 8-bit counts, the bucket words, the stage of `per` entries a thread)
static size_t part2st_lds(uint32_t bpp, int per) {
  return (size_t)((bpp * 260 + 3) & ~3u) * 4 + (size_t)kPart2Block * per * (sizeof(Entry) + 1);
}

// k_part2st's entries a thread per round for this build: the largest stage that fits (fewer rounds,
// fewer barriers), or 0 when pass 2 is not the staged kernel
int part2st_per(const BuildParams& P) {
  constexpr size_t kLdsMax = 158 * 1024;
  if (!(P.p2_sorted && P.p2_fixed && P.fused_carry && P.p1_region && !P.p2_seg)) return 0;
  for (int per = 6; per >= 4; per--)
    if (part2st_lds(P.bpp, per) <= kLdsMax) return per;
  return 0;
}

// pass 2 is k_part2f_direct (more buckets a digit than a staged round would group: C4's tables) or
// k_part2f: fixed bucket regions straight from the digit regions, with k_summary's carries
bool part2_direct(const BuildParams& P) {
  return part2st_per(P) == 0 && !P.p2_sorted && P.p2_fixed && P.p1_region && !P.p2_seg &&
         (P.bpp > kPart2Block * 3 || part2f_lds(P.bpp, 2) <= 158 * 1024);
}

void launch_partition(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.p1_bucket) return;  // (the framing wrote the bucket regions)
  if (!P.p1_region) launch_partition1(P, s);
  else if (P.p1_kernel) hipLaunchKernelGGL(k_part1_regions, dim3(std::min<unsigned>(P.p1r_tiles, kP1rGrid)), dim3(kPartBlock), 0, s, P);
  constexpr size_t kLdsMax = 158 * 1024;
  const int per = part2st_per(P);  // (the staged kernel: the largest stage that fits; compact only with it)
  if (per == 6)
    hipLaunchKernelGGL((P.compact ? k_part2st<6, true, true> : k_part2st<6, false, false>),
                       dim3(256), dim3(kPart2Block),
                       part2st_lds(P.bpp, 6), s, P);
  else if (per == 5)
    hipLaunchKernelGGL((P.compact ? k_part2st<5, true, true> : k_part2st<5, false, false>),
                       dim3(256), dim3(kPart2Block),
                       part2st_lds(P.bpp, 5), s, P);
  else if (per == 4)
    hipLaunchKernelGGL((P.compact ? k_part2st<4, true, true> : k_part2st<4, false, false>),
                       dim3(256), dim3(kPart2Block),
                       part2st_lds(P.bpp, 4), s, P);
  else if (P.p2_sorted)
    hipLaunchKernelGGL(k_part2s, dim3(256), dim3(kPart2Block), (size_t)(514u * P.bpp) * sizeof(uint32_t), s, P);
  else if (part2_direct(P) && P.sub_region) {  // (two levels: sub-digit regions, then the buckets)
    const uint32_t tpd = (uint32_t)((P.p1_region + kPartTile - 1) / kPartTile);
    hipLaunchKernelGGL((P.compact ? k_part2_sub<true> : k_part2_sub<false>), dim3(256u * tpd), dim3(kPartBlock), 0, s,
                       P, tpd);
    hipLaunchKernelGGL((P.compact ? k_part2f<4, true, true> : k_part2f<4, false, true>), dim3(256u * kSub),
                       dim3(kPart2Block), part2f_lds(sub_buckets(P.bpp), 4) + (size_t)sub_buckets(P.bpp) * 1024, s, P);
  } else if (part2_direct(P))
    hipLaunchKernelGGL((P.compact ? k_part2f_direct<true, true> : k_part2f_direct<false, false>),
                       dim3(256), dim3(kPart2Block),
                       (size_t)P.bpp * sizeof(uint32_t), s, P);
  else if (P.p2_fixed && P.p1_region && !P.p2_seg && part2f_lds(P.bpp, 6) <= kLdsMax)
    hipLaunchKernelGGL((P.compact ? k_part2f<6, true> : k_part2f<6, false>), dim3(256), dim3(kPart2Block),
                       part2f_lds(P.bpp, 6), s, P);
  else if (P.p2_fixed && P.p1_region && !P.p2_seg && part2f_lds(P.bpp, 4) <= kLdsMax)
    hipLaunchKernelGGL((P.compact ? k_part2f<4, true> : k_part2f<4, false>), dim3(256), dim3(kPart2Block),
                       part2f_lds(P.bpp, 4), s, P);
  else if (P.p2_fixed && P.p1_region && !P.p2_seg && part2f_lds(P.bpp, 2) <= kLdsMax)
    hipLaunchKernelGGL((P.compact ? k_part2f<2, true> : k_part2f<2, false>), dim3(256), dim3(kPart2Block),
                       part2f_lds(P.bpp, 2), s, P);
  else if (!P.p2_seg && part2d_lds(P.bpp) <= kLdsMax)
    hipLaunchKernelGGL(k_part2d, dim3(256), dim3(kPart2Block), part2d_lds(P.bpp), s, P);
  else
    hipLaunchKernelGGL(k_part2, dim3(256), dim3(kPart2Block), (size_t)(2u * P.bpp) * sizeof(uint32_t), s, P);
  tm->mark("partition", s);
}

void launch_inject_foreign(const BuildParams& P, hipStream_t s, int where) {
  hipLaunchKernelGGL(k_inject_foreign, dim3(1), dim3(64), 0, s, P, where);
}

void launch_place_buckets(const BuildParams& P, hipStream_t s) {
  if (P.b_hi > P.b_lo)
    hipLaunchKernelGGL(((P.compact & kCompactOut) ? k_place_reg<true, true> : P.p2_fixed ? k_place_reg<true> : k_place_reg<false>),
                       dim3((unsigned)(P.b_hi - P.b_lo)), dim3(kPlaceRegBlock), 0, s, P);
  // buckets above kPlaceLdsMax entries (normally none; never with fixed bucket regions, whose
  // overflow redoes the build with dense runs)
  if (!P.p2_fixed) launch_place_global(P, s, 0, 1);
}


void launch_place_fast(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (!P.fused_carry) launch_summary_carry(P, s, tm);
  launch_place_buckets(P, s);
  tm->mark("place", s);
  if (!P.fused_carry) launch_verify(P, s, tm);  // (fused_carry: k_stats_folded verifies the pairs)
}

}  // namespace sk
