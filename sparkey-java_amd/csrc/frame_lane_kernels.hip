// frame_lane_kernels.hip -- k_frame_lane: framing + MurmurHash3 with ONE LANE PER REGION of the log.
//
// The log is a chain of varint-framed records (SparkeyLogIterator.java:86-138): where record i + 1
// starts depends on every record before it.  The wave-per-region framings (k_frame, k_frame3) spend
// their lanes on that dependence: most of a wave's instructions screen, walk and resolve candidate
// starts, and only one of its phases hashes.  Here a lane owns a whole region of R bytes and walks
// its records itself, one dependent header load per record, hashing each key as it goes; the 64 lanes
// of a wave (and every wave of the grid) walk 64 different regions at once, so the dependent loads of
// thousands of lanes are in flight together and the HBM stream, not the chain, sets the pace.
//
//   entry   region r > 0 starts at s = base + r * R.  Its entry is the first record start >= s.  The
//           lane screens [s, s + maxRecLen) 16 positions at a time (SWAR, the header maxima) and walks
//           each plausible position kLaneTrial records on; the first that survives is its entry.
//   walk    from the entry while records start below the region end: decode the header (one-byte
//           VLQs from registers, else the reference's VLQ rules from memory), load the key's 16-byte
//           chunks, prefetch the next header, MurmurHash3 the key (MurmurHash3.java:18-201) from
//           registers, write the (hash, address) entry into the region's slab.  The walk applies the
//           reference iterator's rules (SparkeyLogIterator.java:117-136); its exit is the first record
//           start at or past the region end.
//   fix     region r's records are right when its walk started at region r - 1's exit (by induction
//           from the frame's verified entry).  k_frame_lane_flags + k_frame_lane_act re-walk, from
//           r - 1's exit, every region whose start disagrees (the screened candidate was a false start,
//           or the walk failed); kLanePasses such passes settle what the speculation leaves in practice,
//           and a final check pass flags any disagreement left: the host then redoes the framing with
//           k_frame3 / k_frame / the serial walker.  A walk error on the verified chain leaves its
//           region without an exit, so it reaches the serial walker too, which reports it.
//
// Per region r (P.qpos / P.exitp / P.tail / P.wcount, one word each): the position its walk started
// from, its exit (-1: the walk failed), its DELETE count and its record count; entries in slab r of
// P.ent (slab_cap each).  Regions are the framing's "chunks" with fr_w = 1 (fr_cshift = log2 R).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "frame_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

namespace {

constexpr int kLanePasses = 4;    // fix passes (one settles what C3-like logs leave; pathological ones need more)
constexpr int kLaneMaxChunks = 10;  // 16-byte chunks of a record's header + key (+ 8 bytes): maxKeyLen <= 126

__device__ __forceinline__ uint4 chunk_at(const BuildParams& P, int64_t a) {  // the 16 bytes at a (16-aligned)
  return load16_guarded(P.log, a, (int64_t)P.log_len);
}

// Plausible record start at byte o of c0 ++ c1 (the screen's rules: one-byte VLQs, the header's
// maxima, no DELETE when the header counts none); returns the record's length, or 0.
__device__ __forceinline__ int32_t plausible_len(const BuildParams& P, uint64_t x) {
  const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
  if ((b0 | b1) & 0x80) return 0;
  if (b0 == 0) {
    if (P.no_deletes || b1 > P.max_key_len) return 0;
    return 2 + b1;
  }
  if (b0 - 1 > P.max_key_len || b1 > P.max_value_len) return 0;
  return 1 + b0 + b1;
}

// Walks the records from p while they start below rend: for each, emit(position, hash, put) (false:
// stop there).  Returns the first record start >= rend, the position emit stopped at, or -1 at a
// record the reference's iterator rejects (SparkeyLogIterator.java:117-136) or one outside the
// header's maxima (below).
template <int N, class Emit>
__device__ int64_t walk_records(const BuildParams& P, int64_t p, int64_t rend, Emit&& emit) {
  const int64_t log_len = (int64_t)P.log_len;
  uint4 c[N];
  if (p < rend) {
    const int64_t a = p & ~15ll;
    c[0] = chunk_at(P, a);
    c[1] = chunk_at(P, a + 16);
  }
#pragma unroll 1
  while (p < rend) {
    const int o = (int)(p & 15);
    const uint64_t x = bytes8(c[0], c[1], o);
    // The header's maxima make every VLQ of the log one byte (frame_lane_supported): a longer one, a
    // value over maxValueLen or a DELETE in a log that counts none cannot be on the true chain of a
    // log the header describes, so the walk stops there as on a record the iterator rejects.  (On a
    // false chain such a record would send the walk anywhere; on the verified chain the region keeps
    // no exit and the host's serial walker decides, by the reference's rules.)
    if (x & 0x8080ull) return -1;
    const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
    const int32_t hlen = 2;
    const bool put = b0 != 0;
    const int32_t klen = put ? b0 - 1 : b1;
    const int32_t vlen = put ? b1 : 0;
    if (klen > P.max_key_len || vlen > P.max_value_len || (!put && P.no_deletes) || p + hlen + klen > log_len ||
        o + hlen + klen + 8 > 16 * N)
      return -1;
    const int64_t pn = p + hlen + klen + vlen;
    // the key's remaining chunks, then the next header's two (prefetch: its latency under the hash)
    const int64_t a = p & ~15ll;
    const int nch = (o + hlen + klen + 8 + 15) >> 4;  // chunks holding the header, the key, 8 slack bytes
#pragma unroll
    for (int k = 2; k < N; k++)
      if (k < nch) c[k] = chunk_at(P, a + 16 * k);
    uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0;
    if (pn < rend) {
      const int64_t an = pn & ~15ll;
      n0 = chunk_at(P, an);
      n1 = chunk_at(P, an + 16);
    }
    const int ko = o + hlen;
    const uint64_t hash = P.hash_size == 8 ? lane_murmur64(c, ko, klen, (uint32_t)P.seed)
                                           : (uint64_t)lane_murmur32(c, ko, klen, (uint32_t)P.seed);
    if (!emit(p, hash, put)) return p;
    p = pn;
    c[0] = n0;
    c[1] = n1;
  }
  return p;
}

__device__ __forceinline__ uint64_t entry_addr(const BuildParams& P, int64_t p, bool put) {
  return ((uint64_t)p << P.ebb) | (put ? 0ull : kDelBit);
}
__device__ __forceinline__ int64_t entry_pos(const BuildParams& P, uint64_t addr) {
  return (int64_t)((addr & ~kDelBit) >> P.ebb);
}

// Walks region r from `entry` (see the file comment): its slab and per-region words.
template <int N>
__device__ void walk_region(const BuildParams& P, uint64_t r, int64_t entry, int64_t rend) {
  const uint64_t slab0 = r * (uint64_t)P.slab_cap;
  uint32_t n = 0, nd = 0;
  const int64_t ex = walk_records<N>(P, entry, rend, [&](int64_t p, uint64_t hash, bool put) {
    if (n < P.slab_cap) {
      Entry en;
      en.hash = hash;
      en.addr = entry_addr(P, p, put);
      P.ent[slab0 + n] = en;
    }
    nd += put ? 0u : 1u;
    n++;
    return true;
  });
  if (n > P.slab_cap) atomicMax(&P.st->max_wave_count, n);  // the host grows the slabs and redoes the build
  P.qpos[r] = entry;
  P.exitp[r] = ex;
  P.tail[r] = nd;
  P.wcount[r] = n;
}

constexpr int kPatchMax = 16;  // records a fix may put in front of the original walk's suffix

// Region r again from x, the verified previous exit.  A screened entry that was a false start almost
// always joins the true chain within a record or two, so the original walk's records are right from
// the first position both walks reach: the new records before it replace the original's before it (the
// suffix is moved in the slab) and the exit stands.  A walk that meets no original position within
// kPatchMax records, or an original walk without an exit, is redone whole.
template <int N>
__device__ void fix_region(const BuildParams& P, uint64_t r, int64_t x, int64_t rend) {
  const uint64_t slab0 = r * (uint64_t)P.slab_cap;
  const int64_t old_exit = P.exitp[r];
  const uint32_t n0 = P.wcount[r];
  if (old_exit < 0 || P.qpos[r] < 0 || n0 > P.slab_cap) {
    walk_region<N>(P, r, x, rend);
    return;
  }
  Entry nb[kPatchMax];
  int k = 0;
  uint32_t i = 0, nd_old = 0, nd_new = 0;
  bool merged = false, full = false;
  int64_t ipos = n0 ? entry_pos(P, P.ent[slab0].addr) : INT64_MAX;
  const int64_t ex = walk_records<N>(P, x, rend, [&](int64_t p, uint64_t hash, bool put) {
    while (i < n0 && ipos < p) {  // the original's records before p: replaced
      nd_old += (P.ent[slab0 + i].addr & kDelBit) ? 1u : 0u;
      i++;
      ipos = i < n0 ? entry_pos(P, P.ent[slab0 + i].addr) : INT64_MAX;
    }
    if (ipos == p) {  // both walks reach p: the original is right from here on
      merged = true;
      return false;
    }
    if (k == kPatchMax) {
      full = true;
      return false;
    }
    nb[k].hash = hash;
    nb[k].addr = entry_addr(P, p, put);
    nd_new += put ? 0u : 1u;
    k++;
    return true;
  });
  if (full || ex < 0) {  // no meeting point close by (or a bad record): the whole region again
    walk_region<N>(P, r, x, rend);
    return;
  }
  uint32_t n;
  if (merged && i == 0 && r > 0) {
    // The walk from x reached the region's first record: nb is the run between the previous region's
    // exit and this region's entry.  It follows the previous region's records in the log, so it goes
    // at the end of that region's slab (this region's slab is right as it is).
    const uint64_t pslab = (r - 1) * (uint64_t)P.slab_cap;
    const uint32_t pn = P.wcount[r - 1];
    if (pn + (uint32_t)k > P.slab_cap) {
      atomicMax(&P.st->max_wave_count, pn + (uint32_t)k);
      P.wcount[r - 1] = pn + (uint32_t)k;
      return;
    }
    for (int t = 0; t < kPatchMax; t++)
      if (t < k) P.ent[pslab + pn + t] = nb[t];
    P.wcount[r - 1] = pn + (uint32_t)k;
    P.tail[r - 1] += nd_new;
    P.exitp[r - 1] = P.qpos[r];
    return;
  }
  if (merged) {  // new prefix nb[0, k) + original [i, n0)
    n = (uint32_t)k + (n0 - i);
    if (n > P.slab_cap) {
      atomicMax(&P.st->max_wave_count, n);
      P.wcount[r] = n;
      return;
    }
    if ((uint32_t)k > i) {
      for (uint32_t t = n0; t-- > i;) P.ent[slab0 + t + (k - i)] = P.ent[slab0 + t];
    } else if ((uint32_t)k < i) {
      for (uint32_t t = i; t < n0; t++) P.ent[slab0 + t - (i - k)] = P.ent[slab0 + t];
    }
    P.tail[r] = P.tail[r] - nd_old + nd_new;
  } else {  // the walk reached the region end within kPatchMax records: nb is the region
    n = (uint32_t)k;
    P.exitp[r] = ex;
    P.tail[r] = nd_new;
  }
  for (int t = 0; t < kPatchMax; t++)
    if (t < k) P.ent[slab0 + t] = nb[t];
  P.qpos[r] = x;
  P.wcount[r] = n;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// k_frame_lane: the ring.  Lane L of a wave walks region r = 64 w + L, but the wave loads the log
// for all 64 lanes together: slice k of a lane's stream is bytes [b + kZ, b + (k + 1)Z) of its
// region (b = region start rounded down to 16), and one slice of every lane is 64 Z bytes fetched by
// 64 Z / 1024 LDS-DMA instructions in which Z / 16 consecutive lanes fetch the Z bytes of one region
// -- whole lines, 1 KiB per instruction, as coalesced as a contiguous copy.  The ring holds kRingNS
// slices per lane (512 bytes: slot-major, lane-minor, Z bytes each); the wave refills the slots the
// slowest lane has left, and each lane walks as far as the landed bytes allow.
// ------------------------------------------------------------------------------------------------
constexpr int kRingWin = 512;     // bytes of a lane's stream the ring holds
constexpr int kLaneTail = 768;    // bytes a lane streams past its region end (the walk on to the next entry)
constexpr int kConvMax = 12;      // record starts of the first surviving chain kept for the join test

template <int Z>
struct Ring {
  static constexpr int NS = kRingWin / Z;  // slots
  static constexpr int SLOT = 64 * Z;      // bytes of one slot (a slice of every lane)
  const uint8_t* lds;
  uint32_t lane_off;  // lane * Z
  __device__ __forceinline__ uint64_t al8(int32_t a) const {  // a: stream offset, multiple of 8
    const uint32_t u = (uint32_t)a;
    return *reinterpret_cast<const uint64_t*>(lds + ((u / Z) % NS) * SLOT + lane_off + (u % Z));
  }
  __device__ __forceinline__ uint64_t u64(int32_t a) const {  // the 8 bytes at stream offset a
    const int32_t a0 = a & ~7;
    const uint64_t lo = al8(a0), hi = al8(a0 + 8);
    const int sh = (a & 7) * 8;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
};

template <int Z>
struct RingKey {  // a key at stream offset base (murmur*_ld's loader)
  const Ring<Z>& R;
  int32_t base;
  __device__ __forceinline__ uint64_t u64(int o) const { return R.u64(base + o); }
};

// The entry of a region: a record start m at or after its start, on the log's true chain whatever
// the record before the region is.  Candidates are the plausible starts in [so, so + span) (the screen
// of §2.1; the true first start is one of them).  A = the first candidate whose chain stays plausible
// through the ring's first 512 bytes (or to the frame end); every later candidate must die or join
// A's chain (land on one of its starts) inside that window.  The true first start is A or a joiner,
// so the true chain runs through m = the last join point (A when none joins).  Returns -1 when that
// cannot be decided inside the window (the fix pass walks the region from the previous exit).
template <int Z>
__device__ int32_t ring_entry(const BuildParams& P, const Ring<Z>& R, int32_t so, int32_t span, int32_t deo) {
  constexpr int32_t hlim = kRingWin - 16;  // headers readable below this (16 bytes from the 8-aligned offset)
  int32_t ca[kConvMax];
  int nca = 0;
  int32_t A = -1, mj = -1, alast = -1;
  bool undecided = false;
  const Screen8 scn = make_screen8(P);
  const int32_t cend = min(so + span, deo);
#pragma unroll 1
  for (int32_t a = so & ~15; a < cend; a += 16) {
    const uint64_t x0 = R.al8(a), x1 = R.al8(a + 8), x2 = R.al8(a + 16);
    uint32_t m = screen8(x0, (x0 >> 8) | (x1 << 56), scn) | (screen8(x1, (x1 >> 8) | (x2 << 56), scn) << 8);
    if (a < so) m &= ~0u << (int)(so - a);
    if (cend - a < 16) m &= (1u << (int)(cend - a)) - 1u;
#pragma unroll 1
    while (m) {
      const int32_t c = a + (int32_t)__builtin_ctz(m);
      m &= m - 1;
      if (A < 0) {  // the chain of c through the window
        int32_t p = c;
        int n = 0;
        bool alive = true;
#pragma unroll 1
        while (p < deo && p < hlim && n < kConvMax) {  // (tiny records: the list's first kConvMax starts)
          const int32_t L = plausible_len(P, R.u64(p));
          if (!L) {
            alive = false;
            break;
          }
#pragma unroll
          for (int k = 0; k < kConvMax; k++)
            if (k == n) ca[k] = p;
          n++;
          alast = p;
          p += L;
        }
        if (alive) {
          A = c;
          nca = n;
        }
      } else {  // c dies, or joins A's chain, or stays undecided
        int32_t p = c;
#pragma unroll 1
        for (;;) {
          bool on = false;
#pragma unroll
          for (int k = 0; k < kConvMax; k++) on |= k < nca && ca[k] == p;
          if (on) {
            mj = max(mj, p);
            break;
          }
          if (p >= deo || p >= hlim || (nca == kConvMax && p > alast)) {  // undecided: A, speculatively
            undecided = true;
            break;
          }
          const int32_t L = plausible_len(P, R.u64(p));
          if (!L) break;
          p += L;
        }
      }
    }
  }
  // (undecided: the boundary check after the walk decides, and the fix pass repairs a wrong guess)
  (void)undecided;
  return A < 0 ? -1 : max(A, mj);
}

// Regions of the frame: region k (k from fr_k0) covers [k << fr_cshift, (k + 1) << fr_cshift) of the
// log, clipped to [fr_entry, frame end).  One wave per 64 regions.
template <int Z>
__global__ __launch_bounds__(64) void k_frame_lane(BuildParams P) {
  using RingT = Ring<Z>;
  constexpr int NS = RingT::NS;
  constexpr int LPR = Z / 16;     // lanes fetching one row (region) of a slice
  constexpr int RPI = 64 / LPR;   // rows per DMA instruction
  constexpr int NI = 64 / RPI;    // DMA instructions per slice
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x;
  const uint64_t nreg = P.fr_nchunks;
  const uint64_t r0 = (uint64_t)blockIdx.x * 64;
  const uint64_t r = r0 + lane;
  const bool active = r < nreg;
  const int64_t log_len = (int64_t)P.log_len, frame_end = P.data_end;
  const int cs = P.fr_cshift;
  auto reg_start = [&](uint64_t q) -> int64_t { return q == 0 ? P.fr_entry : (int64_t)((P.fr_k0 + q) << cs); };
  auto reg_end = [&](uint64_t q) -> int64_t { return min((int64_t)((P.fr_k0 + q + 1) << cs), frame_end); };
  // the wave's base (its first region's 16-aligned start): every row base below is 32-bit from it
  const int64_t Wb = reg_start(r0) & ~15ll;
  // this lane's region [s, e), its stream base b (16-aligned) and streamed bytes [b, se)
  const int64_t s = active ? reg_start(r) : Wb, e = active ? reg_end(r) : Wb;
  const int64_t b = s & ~15ll;
  const int64_t se = active ? min(e + kLaneTail, log_len) : b;
  // per DMA instruction i: the row this lane fetches for (LPR lanes a row), its base and stream length
  int32_t rowb[NI], rowl[NI];
#pragma unroll
  for (int i = 0; i < NI; i++) {
    const uint64_t q = r0 + (uint64_t)(RPI * i + lane / LPR);
    rowb[i] = 0;
    rowl[i] = 0;
    if (q < nreg) {
      const int64_t qb = reg_start(q) & ~15ll;
      rowb[i] = (int32_t)(qb - Wb);
      rowl[i] = (int32_t)(min(reg_end(q) + kLaneTail, log_len) - qb);
    }
  }
  unsigned long long streaming = __ballot(active);  // rows whose lanes still walk
  // Slice k of every row into its slot: NI instructions, always all of them (the wait below counts
  // them), lanes of finished or absent rows fetching the log's first line into their unused cells.
  auto issue = [&](int k) {
    uint8_t* slot = lds + (uint32_t)(k % NS) * RingT::SLOT;
    const int32_t off = k * Z + (lane % LPR) * 16;
#pragma unroll
    for (int i = 0; i < NI; i++) {
      const int row = RPI * i + lane / LPR;
      const bool need = off < rowl[i] && ((streaming >> row) & 1ull);
      const int64_t a = Wb + rowb[i] + off;
      const bool tail = need && a + 16 > log_len;  // (the log's last bytes: a guarded copy instead)
      if (!tail)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(P.log + (need ? a : 0)),
                                         (__attribute__((address_space(3))) void*)(slot + i * 1024), 16, 0, 2);
      if (tail) *reinterpret_cast<uint4*>(slot + i * 1024 + lane * 16) = load16_guarded(P.log, a, log_len);
    }
  };
  // prologue: the ring's NS slices (the entry phase reads all of them)
#pragma unroll 1
  for (int k = 0; k < NS; k++) issue(k);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const RingT R{lds, (uint32_t)lane * Z};
  const int32_t so = (int32_t)(s - b), eo = (int32_t)(e - b);
  const int32_t deo = (int32_t)min((int64_t)0x3fffffff, frame_end - b);
  const int32_t slim = (int32_t)(se - b);  // streamed bytes of this lane
  const int32_t lo_max = (int32_t)min((int64_t)0x3fffffff, log_len - b);
  int32_t m = -1;
  if (active) m = r == 0 ? so : ring_entry<Z>(P, R, so, (int32_t)min((int64_t)P.max_rec_len, e - s), deo);
  // the next region's entry (lane + 1; the wave's last lane leaves that boundary to the fix pass):
  // the lane walks on past its region end to it, so that the boundary agrees without a fix
  const int32_t mn = __shfl(m, (lane + 1) & 63, 64);
  int32_t tgt = -1;  // (stream offset)
  if (active && lane < 63 && r + 1 < nreg && mn >= 0) tgt = (int32_t)((reg_start(r + 1) & ~15ll) + mn - b);
  const uint64_t slab0 = r * (uint64_t)P.slab_cap;
  uint32_t n = 0, nd = 0;
  int32_t pos = m, ex = -1;
  bool done = !active || m < 0, failed = false;
  int kb = 0, kl = NS, kland = NS;  // ring: slices [kb, kb + NS); issued below kl, landed below kland
#pragma unroll 1
  for (;;) {
    const int32_t hv = kland * Z;  // landed stream bytes
    const bool all_in = hv >= slim;
    // every lane walks the records whose bytes have landed (a lane whose next key has not: blocked
    // until the next slice)
    bool blocked = false;
#pragma unroll 1
    for (;;) {
      bool go = false;
      if (!done && !blocked) {
        if (pos >= eo && pos >= tgt) {  // past the region end, at (or past) the next region's entry
          done = true;
          ex = pos;
        } else if ((pos & ~7) + 16 > slim) {  // the stream ends (a walk to the next entry longer than the tail)
          done = true;
          ex = pos >= eo ? pos : -1;
        } else if ((pos & ~7) + 16 <= hv) {
          go = true;
        } else {
          blocked = true;
        }
      }
      if (!__any(go)) break;
      if (go) {
        const uint64_t x = R.u64(pos);
        const int32_t b0 = (int32_t)(x & 0xff), b1 = (int32_t)((x >> 8) & 0xff);
        const bool put = b0 != 0;
        const int32_t klen = put ? b0 - 1 : b1;
        const int32_t vlen = put ? b1 : 0;
        const int32_t kend = pos + 2 + klen;
        // The header's maxima make every VLQ of the log one byte (frame_lane_supported): anything else
        // ends the walk, as a record the iterator rejects would (SparkeyLogIterator.java:117-136); the
        // fix pass and then the serial walker decide on such a region.
        if ((x & 0x8080ull) || klen > P.max_key_len || vlen > P.max_value_len || (!put && P.no_deletes) ||
            kend > lo_max) {
          done = true;
          failed = true;
        } else if (kend + 16 > slim && slim < lo_max) {  // the key runs past the stream (a long walk on)
          done = true;
          ex = pos >= eo ? pos : -1;
        } else if (all_in || ((kend + 16) & ~7) + 8 <= hv) {
          const RingKey<Z> ld{R, pos + 2};
          const uint64_t hash = P.hash_size == 8 ? murmur64_ld(ld, klen, (uint32_t)P.seed)
                                                 : (uint64_t)murmur32_ld(ld, klen, (uint32_t)P.seed);
          if (n < P.slab_cap) {
            Entry en;
            en.hash = hash;
            en.addr = ((uint64_t)(b + pos) << P.ebb) | (put ? 0ull : kDelBit);
            P.ent[slab0 + n] = en;
          }
          n++;
          nd += put ? 0u : 1u;
          pos = kend + vlen;
        } else {
          blocked = true;  // (the key's bytes have not all landed: the lane waits for the next slice)
        }
      }
    }
    streaming = __ballot(!done);
    if (!streaming) break;
    // slots below the slowest lane's slice are free: refill them, then wait for the next slice
    int32_t kmin = done ? 0x7fffffff : pos / Z;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) kmin = min(kmin, __shfl_xor(kmin, o, 64));
    kb = max(kb, (int)kmin);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the ring's reads are done before its slots refill
#pragma unroll 1
    while (kl < kb + NS) issue(kl++);
    if (kland < kl) {
      wait_vmcnt_upto((kl - kland - 1) * NI);  // loads complete in order: the later slices stay in flight
      kland++;
    } else {  // (unreachable: the slowest lane's next record always lies in a full ring)
      if (!done) failed = true;
      break;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!active) return;
  if (n > P.slab_cap) atomicMax(&P.st->max_wave_count, n);  // the host grows the slabs and redoes the build
  P.qpos[r] = m < 0 ? -2 : b + m;
  P.exitp[r] = (m < 0 || failed || ex < 0) ? -1 : b + ex;
  P.tail[r] = m < 0 ? 0 : nd;
  P.wcount[r] = m < 0 ? 0 : n;
}

// The fix (see the file comment), in passes of two launches so that no region is read while it is
// rewritten.  k_frame_lane_flags: P.conv[r] = 1 when region r's walk started at region r - 1's exit (region
// 0: at the frame's entry) and ended with an exit.  check = 1 (the last pass): any region left without
// the flag sets spec_fail (the host reruns the framing another way); the DELETE counts are summed and
// the frame's exit recorded.
__global__ __launch_bounds__(256) void k_frame_lane_flags(BuildParams P, int check) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nreg = P.fr_nchunks;
  bool good = true;
  uint32_t nd = 0;
  if (r < nreg) {
    good = P.exitp[r] >= 0 && (r == 0 || (P.exitp[r - 1] >= 0 && P.exitp[r - 1] == P.qpos[r]));
    P.conv[r] = good ? 1 : 0;
    nd = P.tail[r];
    if (check && r + 1 == nreg) P.st->exit = P.exitp[r];
  }
  if (!check) return;
  const bool any_bad = __any(!good);
  const unsigned long long ndw = wave_sum_u64((unsigned long long)nd);
  if ((threadIdx.x & 63) == 0) {
    if (any_bad) atomicOr(&P.st->spec_fail, 1u);
    if (ndw) add_deletes(P, blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), ndw);
  }
}

// k_frame_lane_act: a run of regions without the flag (region r - 1 before it has the flag, so no thread
// of this pass rewrites it) is fixed by one thread, region by region, from region r - 1's exit: every
// region of the run belongs to that thread only.
template <int N>
__global__ __launch_bounds__(256) void k_frame_lane_act(BuildParams P) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nreg = P.fr_nchunks;
  if (r == 0 || r >= nreg || P.conv[r] || !P.conv[r - 1] || P.exitp[r - 1] < 0) return;
#pragma unroll 1
  for (uint64_t q = r; q < nreg; q++) {
    const int64_t rend = min((int64_t)((P.fr_k0 + q + 1) << P.fr_cshift), P.data_end);
    const int64_t old_exit = P.exitp[q];
    fix_region<N>(P, q, P.exitp[q - 1], rend);
    if (P.exitp[q] < 0 || q + 1 >= nreg) break;
    // on into the next region when it is part of this run, or when this fix moved the exit it agreed
    // with and the region after it is no other run's head (whose thread reads the next region's exit)
    if (P.conv[q + 1] && !(P.exitp[q] != old_exit && (q + 2 >= nreg || P.conv[q + 2]))) break;
  }
}

// Chunks (16 bytes) a record's header + key + 8 slack bytes can span at the header maxima.
static int lane_chunks(const BuildParams& P) {
  const int64_t need = 15 + 2 + P.max_key_len + 8;
  return (int)((need + 15) / 16);
}

// One-byte VLQs (the ring walk decodes 2-byte headers), records within a region, and an entry screen
// (maxRecLen positions plus the 16-byte reads past them) inside the ring's first 512 bytes.
bool frame_lane_supported(const BuildParams& P) {
  return P.fr_fast && lane_chunks(P) <= kLaneMaxChunks && P.max_rec_len <= (1ll << P.fr_cshift) &&
         P.max_rec_len + 15 + 32 <= kRingWin - 16;
}

// SPARKEY_LANE_DEBUG: regions without the flag before each fix pass (stderr; synchronizes)
static void lane_debug(const BuildParams& P, hipStream_t s, int pass) {
  std::vector<uint8_t> conv(P.fr_nchunks);
  std::vector<int64_t> qp(P.fr_nchunks), ex(P.fr_nchunks);
  if (hipMemcpyAsync(conv.data(), P.conv, conv.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(qp.data(), P.qpos, qp.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(ex.data(), P.exitp, ex.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return;
  uint64_t bad = 0, runs = 0, nofound = 0, failed = 0, first = ~0ull;
  for (uint64_t r = 0; r < conv.size(); r++) {
    if (!conv[r]) {
      bad++;
      if (r > 0 && conv[r - 1]) runs++;
      if (first == ~0ull) first = r;
    }
    nofound += qp[r] == -2;
    failed += ex[r] < 0;
  }
  fprintf(stderr, "[lane] pass %d: %llu of %llu regions unflagged, %llu run heads, %llu without entry, %llu without exit, first %lld\n",
          pass, (unsigned long long)bad, (unsigned long long)conv.size(), (unsigned long long)runs,
          (unsigned long long)nofound, (unsigned long long)failed, first == ~0ull ? -1ll : (long long)first);
  if (first != ~0ull && first > 0)
    fprintf(stderr, "[lane]   region %lld: qpos %lld exit %lld; previous exit %lld\n", (long long)first,
            (long long)qp[first], (long long)ex[first], (long long)ex[first - 1]);
}

template <int N>
static void launch_lane_n(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  const unsigned g = (unsigned)((P.fr_nchunks + 255) / 256);
  const bool dbg = getenv("SPARKEY_LANE_DEBUG") != nullptr;
  // the ring kernel: one wave per 64 regions, 512 bytes of LDS per lane; slices of 128 bytes (or 64:
  // SPARKEY_LANE_Z=64, a measurement)
  const unsigned gw = (unsigned)((P.fr_nchunks + 63) / 64);
  static const int z = [] {
    const char* v = getenv("SPARKEY_LANE_Z");
    return v && atoi(v) == 64 ? 64 : 128;
  }();
  if (z == 64) hipLaunchKernelGGL(k_frame_lane<64>, dim3(gw), dim3(64), 64 * kRingWin, s, P);
  else hipLaunchKernelGGL(k_frame_lane<128>, dim3(gw), dim3(64), 64 * kRingWin, s, P);
  for (int pass = 0; pass < kLanePasses; pass++) {
    hipLaunchKernelGGL(k_frame_lane_flags, dim3(g), dim3(256), 0, s, P, 0);
    if (dbg) lane_debug(P, s, pass);
    hipLaunchKernelGGL(k_frame_lane_act<N>, dim3(g), dim3(256), 0, s, P);
  }
  if (dbg) {
    hipLaunchKernelGGL(k_frame_lane_flags, dim3(g), dim3(256), 0, s, P, 0);
    lane_debug(P, s, kLanePasses);
  }
  hipLaunchKernelGGL(k_frame_lane_flags, dim3(g), dim3(256), 0, s, P, 1);
  tm->mark("frame", s);
}

void launch_frame_lane(const BuildParams& P, hipStream_t s, StageTimer* tm) {
  if (P.fr_nchunks == 0) return;
  // the chunk array holds a record's header and key: its size is static (registers)
  const int n = lane_chunks(P);
  if (n <= 4) launch_lane_n<4>(P, s, tm);
  else if (n <= 6) launch_lane_n<6>(P, s, tm);
  else launch_lane_n<kLaneMaxChunks>(P, s, tm);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.wcount, P.woff, P.nslabs, (uint64_t*)&P.st->n_records, OpAdd(),
                                            P.scan_scratch_u64, s);
}

}  // namespace sk
