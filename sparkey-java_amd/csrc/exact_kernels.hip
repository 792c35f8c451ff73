// exact_kernels.hip -- IndexHash.put / delete replayed exactly (IndexHash.java:454-665) for logs the
// canonical layout does not cover: DELETE records and duplicate keys (overwrites).
//
//   k_sequential      one lane over the whole table: tables whose PUT records leave no empty slot
//   k_seg_dcount      distinct keys per wanted slot, from the canonical placement of every PUT record
//   scan, k_seg_dmarks the occupied slots of the distinct keys' placement, and their runs (segments)
//   k_seg_first/runs  each segment's placed PUT records (contiguous in that placement) and its length
//   k_seg_assign      every DELETE -> the slot segment holding its wanted slot
//   k_seg_puts/scatter records grouped by segment (the table is then cleared for the replay)
//   k_seg_classify    segments listed by size class
//   k_seg_lanes       one lane per small segment: records numbered in replay order, key classes, the
//                     segment's slots in LDS
//   k_seg_replay_wave one wave per larger segment: records, their header fields, short keys and the
//                     segment's slots staged in LDS, bitonic sort, put / delete evaluated 64 slots
//                     per step, slots written back
//
// Why segments are independent.  occ(S), the set of slots a linear-probing table of the multiset S of
// wanted slots occupies, depends neither on insertion order, nor on the Robin-Hood tie rule, nor on
// in-place replacement or backward-shift deletion (every entry sits at w + d with slots w .. w + d
// all occupied), and it grows with S.  Every table state IndexHash passes through holds each of the
// log's distinct PUT keys at most once: a put of a key the table holds meets it before it can steal
// a slot (IndexHash.java:606-653: the key's wanted-slot group comes first, and the tie rule never
// steals inside it, since the new address is the group's largest -- log order, or SortHelper's
// (wantedSlot, address) order).  So a slot that the canonical placement of the DISTINCT PUT keys
// leaves empty is empty in every state: no put probe, delete probe or backward shift ever crosses it.
// The runs of occupied slots of that placement -- segments -- therefore evolve independently.  (Round
// 5 placed every PUT record, repeats included: a sparser placement with repeats left out has far
// shorter runs -- churn's 9M PUT records hold 5.4M keys.)  Each segment replays its own records in the
// reference's order (log order for IN_MEMORY; SortHelper's (wantedSlot, address) for SORTING,
// SortHelper.java:153-171) with the reference's put / delete on its own slots; a DELETE whose wanted
// slot is empty there is a no-op in every state.  The result is the reference's table byte for byte.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "build_kernels.hpp"
#include "device_common.hpp"
#include "kernel_utils.hpp"
#include "scan.hpp"

namespace sk {

constexpr uint64_t kNoSeg = ~0ull;
// segment size classes (records per segment): 1 small -> one thread, slots in HBM; 2 mid, 3 large,
// 4 huge -> one wave, records and slots in LDS (keys of up to 32 / 16 / 0 bytes staged too); past
// kHugeSegMax records lane 0 replays against HBM
constexpr uint32_t kSmallSegOps = 24;
constexpr uint32_t kMidSegMax = 128;
constexpr uint32_t kLargeSegMax = 384;
constexpr uint32_t kHugeSegMax = 1024;
constexpr unsigned kMidGrid = 4096;
constexpr unsigned kLargeGrid = 2048;
constexpr unsigned kHugeGrid = 512;
constexpr unsigned kLaneGrid = 4096;  // k_seg_lanes: 64 small segments a wave at a time, from a work queue
constexpr int kSegClasses = 4;   // small (k_seg_lanes), mid, large, huge (k_seg_replay_wave)
constexpr int kSmallLists = 6;   // the small class's lists, by record count
constexpr int kSegLists = kSmallLists + kSegClasses - 1;
constexpr int kClsBlock = 256;            // k_seg_classify: 4 slots per thread
constexpr int kClsItems = 4;
constexpr uint64_t kClsSlots = (uint64_t)kClsBlock * kClsItems;

// Every global access of the exact path is bounds-checked: a violation (a bug, never a property of
// the input) sets a bit of st->guard, skips the access, and the host fails the build loudly.
__device__ __forceinline__ void guard_trip(const BuildParams& P, unsigned bit) { atomicOr(&P.st->guard, bit); }

// 16 log bytes from position p >= 0, as four little-endian words: five aligned dword loads, issued
// together, each 4 bytes out one v_alignbit (a byte loop is one dependent round trip per byte).  A
// dword is read only when it starts inside the log (the buffer is 16-byte aligned, so the rest of
// that dword is allocated); bytes at or past log_len are left to the caller's bounds.
struct Bytes16 {
  uint32_t w[4];
  __device__ __forceinline__ uint32_t byte(uint32_t k) const {  // k < 16 (shifts and a select: a dynamic
    const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);  // index into w would go to scratch)
    const uint64_t hi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    return (uint32_t)((k < 8 ? lo >> (8u * k) : hi >> (8u * (k - 8u))) & 0xffu);
  }
};
__device__ __forceinline__ Bytes16 log16(const BuildParams& P, int64_t p) {
  const int64_t b = p & ~3ll;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(P.log + b);
  uint32_t x[5];
#pragma unroll
  for (int i = 0; i < 5; i++) x[i] = b + 4 * i < (int64_t)P.log_len ? d[i] : 0u;
  const uint32_t sh = (uint32_t)(p & 3) * 8u;
  Bytes16 r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.w[i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], sh);
  return r;
}

__device__ __forceinline__ bool keys_equal(const BuildParams& P, int64_t k1, int64_t k2, int32_t len) {
  if (len < 0 || k1 < 0 || k2 < 0 || k1 + len > (int64_t)P.log_len || k2 + len > (int64_t)P.log_len) {
    guard_trip(P, 1u);
    return false;
  }
  for (int32_t j = 0; j < len; j += 16) {  // 16 bytes of each key a step
    const Bytes16 x = log16(P, k1 + j), y = log16(P, k2 + j);
    const int32_t r = len - j;
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int32_t nb = min(max(r - 4 * i, 0), 4);  // bytes of word i inside the key
      const uint32_t m = nb >= 4 ? ~0u : (1u << (8 * nb)) - 1u;
      diff |= (x.w[i] ^ y.w[i]) & m;
    }
    if (diff) return false;
  }
  return true;
}
// The record header at address (decode_header's rules, on 16 bytes loaded at once: a header is at
// most 10 bytes).
__device__ __forceinline__ RecHdr log_header(const BuildParams& P, uint64_t address) {
  const int64_t p = (int64_t)(address >> P.ebb);
  const Bytes16 b = log16(P, p);
  auto at = [&](int64_t a) -> uint32_t { return b.byte((uint32_t)(a - p)); };
  return decode_header(at, p, (int64_t)P.log_len);
}

// ------------------------------------------------------------------------------------------------
// Table views the replay runs against.  get/set carry, per slot, the occupant's (hash, address), its
// wanted slot and an opaque record id; rec() gives a record's header fields, same_key() compares two
// records' keys (IndexHash.java:606-636).
//   HbmTable: the .spi slots in HBM, headers and keys read from the log.
//   LdsTable: one segment's slots staged in LDS (index = slot - s0 on the ring; the slot after the
//             segment is staged too and stays empty); records are the segment's staged records,
//             their headers decoded once, keys of up to KEYB bytes staged too.
// ------------------------------------------------------------------------------------------------
struct HbmTable {
  const BuildParams* P;
  __device__ __forceinline__ void get(uint64_t slot, uint64_t& h, uint64_t& a, uint64_t& w, uint32_t& o) const {
    read_slot(*P, slot, h, a);
    w = a ? fast_mod(h, P->mod) : 0;
    o = 0;
  }
  __device__ __forceinline__ void set(uint64_t slot, uint64_t h, uint64_t a, uint64_t, uint32_t) const {
    write_slot(*P, slot, h, a);
  }
  __device__ __forceinline__ RecHdr rec(uint32_t, uint64_t address) const { return log_header(*P, address); }
  __device__ __forceinline__ bool same_key(uint32_t, const RecHdr& x, uint64_t ax, uint32_t, const RecHdr& y,
                                           uint64_t ay) const {
    return keys_equal(*P, (int64_t)(ax >> P->ebb) + x.hlen, (int64_t)(ay >> P->ebb) + y.hlen, x.klen);
  }
};

template <uint32_t KEYB>
struct LdsTable {
  const BuildParams* P;
  uint64_t* h;
  uint64_t* a;
  uint32_t* w;   // wanted slot - s0 (ring)
  uint16_t* o;   // record id of the occupant
  const RecHdr* hdr;
  const uint64_t* keys;  // KEYB bytes per record, zero padded (klen <= KEYB)
  uint64_t s0;
  uint64_t cap;
  __device__ __forceinline__ uint32_t at(uint64_t slot) const {
    return (uint32_t)(slot >= s0 ? slot - s0 : slot + cap - s0);
  }
  __device__ __forceinline__ void get(uint64_t slot, uint64_t& hh, uint64_t& aa, uint64_t& ww, uint32_t& oo) const {
    const uint32_t i = at(slot);
    hh = h[i];
    aa = a[i];
    const uint64_t wr = s0 + w[i];
    ww = wr >= cap ? wr - cap : wr;
    oo = o[i];
  }
  __device__ __forceinline__ void set(uint64_t slot, uint64_t hh, uint64_t aa, uint64_t ww, uint32_t oo) const {
    const uint32_t i = at(slot);
    h[i] = hh;
    a[i] = aa;
    w[i] = at(ww);
    o[i] = (uint16_t)oo;
  }
  __device__ __forceinline__ RecHdr rec(uint32_t id, uint64_t) const { return hdr[id]; }
  __device__ __forceinline__ bool same_key(uint32_t ix, const RecHdr& x, uint64_t ax, uint32_t iy, const RecHdr& y,
                                           uint64_t ay) const {
    if (KEYB > 0 && x.klen <= (int32_t)KEYB) {
      for (uint32_t q = 0; q < KEYB / 8; q++)
        if (keys[ix * (KEYB / 8) + q] != keys[iy * (KEYB / 8) + q]) return false;
      return true;
    }
    return keys_equal(*P, (int64_t)(ax >> P->ebb) + x.hlen, (int64_t)(ay >> P->ebb) + y.hlen, x.klen);
  }
};

template <class Tab>
struct Replay {
  const BuildParams* P;
  Tab tab;
  int64_t num_entries;  // entries this replay added (the whole table, or one segment)
  int64_t garbage;
};

__device__ __forceinline__ int64_t disp_at(const BuildParams& P, uint64_t slot, uint64_t wanted) {
  const int64_t d = (int64_t)slot - (int64_t)wanted;
  return d >= 0 ? d : d + (int64_t)P.cap;
}
__device__ __forceinline__ int32_t vlq_size_i32(int64_t v) {
  if (v < (1 << 7)) return 1;
  if (v < (1 << 14)) return 2;
  if (v < (1 << 21)) return 3;
  if (v < (1 << 28)) return 4;
  return 5;
}
__device__ __forceinline__ int64_t garbage_of(int32_t k2, int32_t v2) {  // IndexHeader.java:221-228
  return (int32_t)((uint32_t)k2 + (uint32_t)v2 + (uint32_t)vlq_size_i32((int64_t)k2 + 1) + (uint32_t)vlq_size_i32(v2));
}

// IndexHash.put (IndexHash.java:562-665) of record `id`; returns 0 or an error code
template <class Tab>
__device__ int replay_put(Replay<Tab>& r, uint64_t hash, uint64_t address, uint32_t id) {
  const BuildParams& P = *r.P;
  const int64_t cap = (int64_t)P.cap;
  if (r.num_entries >= cap) return kErrNoFreeSlots;
  uint64_t wanted = fast_mod(hash, P.mod);
  uint64_t slot = wanted;
  int64_t displacement = 0, tries = cap;
  bool might = true;
  bool have_mine = false;
  RecHdr mine;
  const uint32_t my_id = id;
  const uint64_t my_addr = address;
  while (--tries >= 0) {
    uint64_t hash2, address2, wanted2;
    uint32_t id2;
    r.tab.get(slot, hash2, address2, wanted2, id2);
    if (address2 == 0) {
      r.tab.set(slot, hash, address, wanted, id);
      r.num_entries++;
      return 0;
    }
    if (might && hash == hash2) {  // same hash: same key?  (IndexHash.java:606-636)
      if (!have_mine) {
        mine = r.tab.rec(my_id, my_addr);
        if (mine.rc) return header_error(mine);
        if (!mine.put) return kErrCorruptData;
        have_mine = true;
      }
      const RecHdr other = r.tab.rec(id2, address2);
      if (other.rc) return header_error(other);
      if (!other.put) return kErrCorruptData;  // "Invalid data - reference to delete entry"
      if (mine.klen == other.klen && r.tab.same_key(my_id, mine, my_addr, id2, other, address2)) {
        r.tab.set(slot, hash, address, wanted, id);  // replace in place
        r.garbage += garbage_of(other.klen, other.vlen);
        return 0;
      }
    }
    const int64_t d2 = disp_at(P, slot, wanted2);
    if (displacement > d2 || (displacement == d2 && (int64_t)address < (int64_t)address2)) {
      r.tab.set(slot, hash, address, wanted, id);  // steal the slot, carry the evicted entry on
      address = address2;
      displacement = d2;
      hash = hash2;
      wanted = wanted2;
      id = id2;
      might = false;
    }
    displacement++;
    slot = slot + 1 == (uint64_t)cap ? 0 : slot + 1;
  }
  return kErrNoFreeSlots;
}

// IndexHash.delete (IndexHash.java:454-548) of record `id`: find the key, backward-shift the run
template <class Tab>
__device__ int replay_delete(Replay<Tab>& r, uint64_t hash, uint64_t address, uint32_t id) {
  const BuildParams& P = *r.P;
  const int64_t cap = (int64_t)P.cap;
  uint64_t slot = fast_mod(hash, P.mod);
  int64_t displacement = 0;
  bool have_mine = false;
  RecHdr mine;
  for (int64_t guard = 0; guard <= cap; guard++) {
    uint64_t hash2, address2, wanted2;
    uint32_t id2;
    r.tab.get(slot, hash2, address2, wanted2, id2);
    if (address2 == 0) return 0;
    if (hash == hash2) {
      if (!have_mine) {
        mine = r.tab.rec(id, address);
        if (mine.rc) return header_error(mine);
        if (mine.put) return kErrCorruptData;
        have_mine = true;
      }
      const RecHdr other = r.tab.rec(id2, address2);
      if (other.rc) return header_error(other);
      if (!other.put) return kErrCorruptData;
      if (mine.klen == other.klen && r.tab.same_key(id, mine, address, id2, other, address2)) {
        for (int64_t g2 = 0; g2 < cap; g2++) {  // backward shift, IndexHash.java:503-524
          const uint64_t next = slot + 1 == (uint64_t)cap ? 0 : slot + 1;
          uint64_t hash3, pos3, wanted3;
          uint32_t id3;
          r.tab.get(next, hash3, pos3, wanted3, id3);
          if (pos3 == 0) break;
          if (wanted3 == next) break;
          r.tab.set(slot, hash3, pos3, wanted3, id3);
          slot = next;
        }
        r.tab.set(slot, 0, 0, slot, 0);
        r.garbage += garbage_of(other.klen, other.vlen);
        r.num_entries--;
        return 0;
      }
    }
    const int64_t d2 = disp_at(P, slot, wanted2);
    if (displacement > d2) return 0;
    displacement++;
    slot = slot + 1 == (uint64_t)cap ? 0 : slot + 1;
  }
  return 0;
}

template <class Tab>
__device__ __forceinline__ bool replay_one(Replay<Tab>& r, const Entry& en, uint32_t id) {
  const uint64_t addr = en.addr & ~kDelBit;
  const int rc = (en.addr & kDelBit) ? replay_delete(r, en.hash, addr, id) : replay_put(r, en.hash, addr, id);
  if (rc) set_error(r.P->st, (int64_t)(addr >> r.P->ebb), rc);
  return rc == 0;
}

// numEntries / garbageSize of a segment replay: summed over the wave, one atomic per wave (every lane
// of the wave calls this)
__device__ __forceinline__ void commit_counts(const BuildParams& P, int64_t entries, int64_t garbage) {
  const unsigned long long e = wave_sum_u64((unsigned long long)entries);
  const unsigned long long g = wave_sum_u64((unsigned long long)garbage);
  if ((threadIdx.x & 63) == 0) {
    if (e) atomicAdd((unsigned long long*)&P.st->num_entries, e);
    if (g) atomicAdd((unsigned long long*)&P.st->garbage, g);
  }
}

// ================================================================================================
// k_sequential: the whole log on one lane.  IN_MEMORY: entries in log order (the slabs).
// SORTING: (wantedSlot, address) order per bucket (ent3, from k_place sort_only).
// ================================================================================================
__global__ void k_sequential(BuildParams P, int sorted_order) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Replay<HbmTable> r{&P, HbmTable{&P}, 0, 0};
  const uint64_t N = min((uint64_t)P.st->n_records, P.max_records);
  uint64_t w = 0, j = 0;
  for (uint64_t i = 0; i < N; i++) {
    Entry en;
    if (sorted_order) {
      en = P.ent3[i];
    } else {
      while (j >= P.wcount[w]) { w++; j = 0; }
      en = P.ent[w * P.slab_cap + j];
      j++;
    }
    if (!replay_one(r, en, 0)) break;
  }
  P.st->num_entries = r.num_entries;
  P.st->garbage = r.garbage;
}

// ================================================================================================
// Segments
// ================================================================================================
__device__ __forceinline__ uint64_t prev_slot(const BuildParams& P, uint64_t t) { return t == 0 ? P.cap - 1 : t - 1; }
__device__ __forceinline__ uint64_t next_slot(const BuildParams& P, uint64_t t) { return t + 1 == P.cap ? 0 : t + 1; }
// The wanted slot of the record the canonical placement left in slot t (kNoSeg: t is empty).
__device__ __forceinline__ uint64_t placed_wanted(const BuildParams& P, uint64_t t, uint64_t& h, uint64_t& a) {
  read_slot(P, t, h, a);
  return a ? fast_mod(h, P.mod) : kNoSeg;
}

// A record's first 32 bytes (header and, for keys of up to 22-30 bytes, the whole key), loaded at once,
// and its header decoded from them.
struct Rec32 {
  Bytes16 lo, hi;
  RecHdr h;
};
__device__ __forceinline__ Rec32 log32(const BuildParams& P, uint64_t address) {
  const int64_t p = (int64_t)(address >> P.ebb);
  const Bytes16 lo = log16(P, p), hi = log16(P, p + 16);
  auto at = [&](int64_t x) -> uint32_t { return lo.byte((uint32_t)(x - p)); };  // (a header: <= 10 bytes)
  return Rec32{lo, hi, decode_header(at, p, (int64_t)P.log_len)};
}

// Do the records at addresses a and a2 hold the same key?  (IndexHash.java:606-636)  From the loaded
// 32 bytes when both headers have one length and the key ends inside them, else from the log.
__device__ __forceinline__ bool same_key_at(const BuildParams& P, uint64_t a, const Rec32& ra, uint64_t a2, const Rec32& rb) {
  const RecHdr &ha = ra.h, &hb = rb.h;
  if (ha.rc || hb.rc || ha.klen != hb.klen) return false;
  if (ha.hlen == hb.hlen && ha.hlen + ha.klen <= 32 && ha.klen >= 0 &&
      (int64_t)(max(a, a2) >> P.ebb) + ha.hlen + ha.klen <= (int64_t)P.log_len) {  // (else keys_equal's guard)
    const int32_t k0 = ha.hlen, k1 = ha.hlen + ha.klen;  // key bytes [k0, k1) of both windows
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int32_t lo = min(max(k0 - 4 * i, 0), 4), hi = min(max(k1 - 4 * i, 0), 4);
      const uint32_t m = (uint32_t)(((1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull));
      const uint32_t x = i < 4 ? ra.lo.w[i & 3] : ra.hi.w[i & 3], y = i < 4 ? rb.lo.w[i & 3] : rb.hi.w[i & 3];
      diff |= (x ^ y) & m;
    }
    return diff == 0;
  }
  return keys_equal(P, (int64_t)(a >> P.ebb) + ha.hlen, (int64_t)(a2 >> P.ebb) + hb.hlen, ha.klen);
}

// The first member of slot g0's group, from g0 up to (not including) slot `end`, with hash h and the
// key of the record at address a (its bytes ra): its slot, or kNoSeg.
__device__ __forceinline__ uint64_t first_with_key(const BuildParams& P, uint64_t g0, uint64_t end, uint64_t h, uint64_t a,
                                   const Rec32& ra) {
  for (uint64_t j = g0, g = 0; j != end && g < P.cap; j = next_slot(P, j), g++) {
    uint64_t h2, a2;
    read_slot(P, j, h2, a2);
    if (h2 == h && same_key_at(P, a, ra, a2, log32(P, a2))) return j;
  }
  return kNoSeg;
}

// c[w] (P.seg_len, zeroed) = the distinct keys among the placed PUT records that want slot w, and each
// placed record's key class: seg_krep[t] = slots back to the group's first record with its key (0:
// itself, the key's first).  The canonical placement orders each run by wanted slot, so a wanted
// slot's records (its group) sit in consecutive slots, and equal keys share a hash and so a group.
// Each wave sums its lanes' first-of-key flags per group; a group that continues past the wave adds
// atomically.
__global__ __launch_bounds__(256) void k_seg_dcount(BuildParams P) {
  const int lane = threadIdx.x & 63;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t h = 0, a = 0;
  const uint64_t w = t < P.cap ? placed_wanted(P, t, h, a) : kNoSeg;
  bool first_of_key = w != kNoSeg;
  if (first_of_key) {
    // the group's first member with this hash (the whole group back: a repeated key's records are
    // usually its only members with that hash)
    constexpr int kStep = 4;  // slots read together, backwards
    uint64_t e = kNoSeg, ae = 0;
    bool more = true;
    for (uint64_t g = 0, j = t; more && g < P.cap; g += kStep) {
      uint64_t hb[kStep], ab[kStep], jb[kStep];
#pragma unroll
      for (int q = 0; q < kStep; q++) {
        const uint64_t back = (uint64_t)(q + 1) % P.cap;
        jb[q] = j >= back ? j - back : j + P.cap - back;
        read_slot(P, jb[q], hb[q], ab[q]);
      }
#pragma unroll
      for (int q = 0; q < kStep; q++) {
        if (!more) continue;
        if (!ab[q] || fast_mod(hb[q], P.mod) != w || g + (uint64_t)q + 1 >= P.cap) {
          more = false;
          continue;
        }
        if (hb[q] == h) {
          e = jb[q];
          ae = ab[q];
        }
      }
      j = jb[kStep - 1];
    }
    uint32_t back = 0;
    if (e != kNoSeg) {  // (both records' bytes in one round trip: the first member with this hash
                        //  usually holds the key -- a second key of that hash is a collision)
      const Rec32 ra = log32(P, a), re = log32(P, ae);
      const uint64_t r = same_key_at(P, a, ra, ae, re) ? e : first_with_key(P, next_slot(P, e), t, h, a, ra);
      if (r != kNoSeg) back = (uint32_t)(t >= r ? t - r : t + P.cap - r);
    }
    P.seg_krep[t] = back;
    first_of_key = back == 0;
  }
  // this wave's lanes of the group: consecutive, from the head lane (hidx) to the group's last lane
  const uint32_t wl = (uint32_t)w, wh = (uint32_t)(w >> 32);
  const uint64_t wp = ((uint64_t)(uint32_t)wave_prev_i32((int32_t)wh, -1) << 32) | (uint32_t)wave_prev_i32((int32_t)wl, -1);
  const uint64_t wn = ((uint64_t)(uint32_t)wave_next_i32((int32_t)wh, -1) << 32) | (uint32_t)wave_next_i32((int32_t)wl, -1);
  const bool head = lane == 0 || wp != w;
  const bool last = lane == 63 || wn != w;
  const uint32_t incl = wave_incl_sum_u32(first_of_key ? 1u : 0u);
  const int32_t hidx = wave_incl_max_i32(head ? lane : -1);
  const uint32_t before = (uint32_t)__shfl((int)incl, max(hidx - 1, 0), 64);
  if (w == kNoSeg || !last) return;
  const uint32_t cnt = incl - (hidx > 0 ? before : 0u);
  // the group may go on before the wave's first slot or after this one (around the ring too)
  uint64_t h2, a2;
  bool open = hidx == 0 && placed_wanted(P, prev_slot(P, t - (uint64_t)lane), h2, a2) == w;
  if (!open && (lane == 63 || t + 1 == P.cap)) open = placed_wanted(P, next_slot(P, t), h2, a2) == w;
  if (!open) P.seg_len[w] = cnt;
  else if (cnt) atomicAdd(&P.seg_len[w], cnt);
}

// The carry out of a slot of the distinct keys' placement: max(0, carry in + c - 1).
struct DistinctCount {
  uint32_t c;
  __device__ __forceinline__ explicit operator MaxPlus() const { return MaxPlus{0, (int64_t)c - 1}; }
};

// mark[s] = s + 1 for a slot the distinct keys' placement leaves empty, 0 for an occupied one: carry
// in + c[s] >= 1.  F[s] composes the carry functions of the slots before s from slot 0 (F[cap]: all of
// them); the carry into slot 0 is F[cap](0), the carry out of the last slot when slot 0 starts from 0
// -- exact, because the placement of every PUT record has an empty slot (else k_sequential), empty
// in the sparser placement too, where both carries are 0 and agree from there on.  Its exclusive
// max-scan gives every slot the first slot of its run (<= 0: the run wraps, it starts after the
// table's last empty slot).
__global__ __launch_bounds__(256) void k_seg_dmarks(BuildParams P) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= P.cap) return;
  const MaxPlus tot = P.seg_fun[P.cap];
  const int64_t c0 = max(tot.c, tot.a);
  const MaxPlus f = P.seg_fun[s];
  const int64_t cin = max(f.c, c0 + f.a);
  P.seg_mark[s] = cin + (int64_t)P.seg_len[s] >= 1 ? 0 : (int64_t)(s + 1);
}

// kSegSlabs slabs a 64-thread workgroup: each thread follows that many records' dependent random
// reads at once (one slab a workgroup left one chain a thread: 0.51 + 0.59 ms for churn's 10M).
constexpr uint32_t kSegSlabs = 4;

// The first slot of the run holding occupied slot t (a run with no empty slot before it wraps: it
// starts after the table's last empty slot).
__device__ __forceinline__ uint64_t run_start(const BuildParams& P, uint64_t t, int64_t last) {
  const int64_t m = P.seg_start[t];
  return m > 0 ? (uint64_t)m : (uint64_t)last % P.cap;
}

// The segment of the placed record in slot t (kNoSeg: t is empty); its wanted slot lies in the
// distinct keys' placement (its key's first record wants it too).
__device__ __forceinline__ uint64_t placed_segment(const BuildParams& P, uint64_t t, uint64_t& h, uint64_t& a,
                                                   int64_t last) {
  const uint64_t w = placed_wanted(P, t, h, a);
  if (w == kNoSeg) return kNoSeg;
  if (P.seg_mark[w] != 0) {
    guard_trip(P, 256u);
    return kNoSeg;
  }
  return run_start(P, w, last);
}

// A segment's PUT records are the placed records whose wanted slots lie in its run: consecutive in
// the placement, which orders each of its runs by wanted slot.  The first of them records its slot.
__global__ __launch_bounds__(256) void k_seg_first(BuildParams P) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P.cap) return;
  const int64_t last = P.seg_mark[P.cap];
  uint64_t h, a;
  const uint64_t d = placed_segment(P, t, h, a, last);
  if (d == kNoSeg) return;
  if (placed_segment(P, prev_slot(P, t), h, a, last) != d) P.seg_first[d] = t;
}

// Per segment: its PUT record count (added by its last placed record: k_seg_assign adds the DELETEs to
// the same counter, concurrently) into seg_cnt, and its length (written by the empty slot that ends
// it) into seg_len.
__global__ __launch_bounds__(256) void k_seg_runs(BuildParams P) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P.cap) return;
  const int64_t last = P.seg_mark[P.cap];
  uint64_t h, a;
  const uint64_t d = placed_segment(P, t, h, a, last);
  if (d != kNoSeg && placed_segment(P, next_slot(P, t), h, a, last) != d) {
    const uint64_t f = P.seg_first[d];
    atomicAdd(&P.seg_cnt[d], (uint32_t)((t >= f ? t - f : t + P.cap - f) + 1));
  }
  if (P.seg_mark[t] != 0 && P.seg_mark[prev_slot(P, t)] == 0) {
    const uint64_t st = run_start(P, prev_slot(P, t), last);
    P.seg_len[st] = (uint32_t)(t >= st ? t - st : t + P.cap - st);
  }
}

// A DELETE's key class: the rank in its segment d of the first placed PUT record with its key, or kNoSeg
// when no PUT record holds its key (the DELETE then removes nothing in any state).  The placement's
// slots from the wanted slot w on hold records of earlier wanted slots, then w's group.
__device__ uint64_t delete_class(const BuildParams& P, uint64_t w, uint64_t h, uint64_t a, uint64_t d) {
  const Rec32 ra = log32(P, a);  // (its header and key: loaded while the slots are probed)
  constexpr int kStep = 4;             // slots read together (the probe passes about as many at 0.77 load)
  uint64_t t = w;
  for (uint64_t g = 0; g < P.cap; g += kStep) {
    uint64_t hb[kStep], ab[kStep], tb[kStep];
#pragma unroll
    for (int j = 0; j < kStep; j++) {
      tb[j] = wrap_slot(t + (uint64_t)j, P.cap);
      read_slot(P, tb[j], hb[j], ab[j]);
    }
#pragma unroll
    for (int j = 0; j < kStep; j++) {
      if (!ab[j]) return kNoSeg;
      const uint64_t w2 = fast_mod(hb[j], P.mod), u = tb[j];
      const uint64_t dt = u >= w2 ? u - w2 : u + P.cap - w2;  // (displacements at u)
      const uint64_t dw = u >= w ? u - w : u + P.cap - w;
      if (dt < dw) return kNoSeg;  // past where w's group would be: no record wants w
      if (dt == dw && hb[j] == h && same_key_at(P, a, ra, ab[j], log32(P, ab[j]))) {  // w's group: the first with the key
        const uint64_t f = P.seg_first[d];
        return u >= f ? u - f : u + P.cap - f;
      }
    }
    t = wrap_slot(t + kStep, P.cap);
  }
  return kNoSeg;
}

// The segment and key class of DELETE entry idx (delete_class), counted at the segment's start.
__device__ __forceinline__ void delete_segment(const BuildParams& P, uint64_t idx, int64_t last) {
  const Entry en = P.ent[idx];
  const uint64_t w = fast_mod(en.hash, P.mod);
  uint64_t seg = run_start(P, w, last);
  const uint64_t cls = delete_class(P, w, en.hash, en.addr & ~kDelBit, seg);
  if (cls == kNoSeg) {
    seg = kNoSeg;  // (no PUT record holds its key: a no-op in every state too)
  } else if (cls >= (1ull << 24) || seg >= (1ull << 40)) {
    guard_trip(P, 512u);
    seg = kNoSeg;
  } else {
    atomicAdd(&P.seg_cnt[seg], 1u);
    seg |= cls << 40;
  }
  P.eseg[idx] = seg;
}

// DELETE records (the PUT records come from the table, k_seg_puts): each whose wanted slot lies in a
// segment is queued in LDS and the wave works them 64 at a time, one a lane (its probe of the placement
// is a chain of dependent reads: a lane per record, not one per slab entry, keeps the lanes busy); a
// DELETE whose wanted slot is empty there is a no-op in every state.  kSegSlabs slabs a 64-thread
// workgroup.
__global__ __launch_bounds__(64) void k_seg_assign(BuildParams P) {
  __shared__ uint64_t q[64 * (kSegSlabs + 1)];
  const int64_t last = P.seg_mark[P.cap];
  const int lane = threadIdx.x;
  uint32_t n[kSegSlabs], nmax = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSegSlabs; k++) {
    const uint64_t w = (uint64_t)blockIdx.x * kSegSlabs + k;
    n[k] = w < P.nslabs ? P.wcount[w] : 0u;
    nmax = max(nmax, n[k]);
  }
  uint32_t qn = 0;  // (wave-uniform)
  for (uint32_t j0 = 0; j0 < nmax; j0 += 64) {
    const uint32_t j = j0 + (uint32_t)lane;
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      const uint64_t idx = ((uint64_t)blockIdx.x * kSegSlabs + k) * P.slab_cap + j;
      bool listed = false;
      if (j < n[k]) {
        const Entry en = P.ent[idx];
        if (en.addr & kDelBit) {
          listed = P.seg_mark[fast_mod(en.hash, P.mod)] == 0;
          if (!listed) P.eseg[idx] = kNoSeg;
        }
      }
      const unsigned long long bal = __ballot(listed);
      if (listed) q[qn + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull))] = idx;
      qn += (uint32_t)__builtin_popcountll(bal);
    }
    __syncthreads();
    for (; qn >= 64; qn -= 64) delete_segment(P, q[qn - 64 + (uint32_t)lane], last);  // (one a lane)
    __syncthreads();
  }
  if ((uint32_t)lane < qn) delete_segment(P, q[lane], last);
}

// The PUT records grouped by segment straight from the table: placed record t is record t - first of
// its segment's list (slot order; the replay sorts a segment itself).  Reads and writes in slot order.
__global__ __launch_bounds__(256) void k_seg_puts(BuildParams P) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P.cap) return;
  uint64_t h, a;
  const uint64_t d = placed_segment(P, t, h, a, P.seg_mark[P.cap]);
  if (d == kNoSeg) return;
  const uint64_t f = P.seg_first[d];
  const uint64_t r = t >= f ? t - f : t + P.cap - f;
  const uint64_t dst = P.seg_off[d] + r;
  const uint32_t back = P.seg_krep[t];
  if (dst >= P.max_records || dst >= P.seg_off[d + 1] || back > r) {
    guard_trip(P, 32u);
    return;
  }
  P.ent3[dst] = Entry{h, a};
  P.ecls[dst] = (uint32_t)(r - back);  // (the rank of its key's first record)
}

// The DELETE records after their segment's PUT records: seg_cnt still holds run length + DELETEs, and
// each DELETE takes the place its decrement names (the top ones, above the run's PUT records).
__global__ __launch_bounds__(64) void k_seg_scatter(BuildParams P) {
  uint32_t n[kSegSlabs], nmax = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSegSlabs; k++) {
    const uint64_t w = (uint64_t)blockIdx.x * kSegSlabs + k;
    n[k] = w < P.nslabs ? P.wcount[w] : 0u;
    nmax = max(nmax, n[k]);
  }
  for (uint32_t j = threadIdx.x; j < nmax; j += 64) {
    uint64_t idx[kSegSlabs], seg[kSegSlabs];
    uint32_t r[kSegSlabs];
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      idx[k] = ((uint64_t)blockIdx.x * kSegSlabs + k) * P.slab_cap + j;
      seg[k] = kNoSeg;
      if (j < n[k] && (P.ent[idx[k]].addr & kDelBit)) seg[k] = P.eseg[idx[k]];
    }
    uint32_t cls[kSegSlabs];
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      cls[k] = seg[k] != kNoSeg ? (uint32_t)(seg[k] >> 40) : 0u;  // (delete_class, packed by k_seg_assign)
      if (seg[k] != kNoSeg) seg[k] &= (1ull << 40) - 1;
      if (seg[k] != kNoSeg && seg[k] >= P.cap) {
        guard_trip(P, 32u);
        seg[k] = kNoSeg;
      }
      r[k] = seg[k] != kNoSeg ? atomicSub(&P.seg_cnt[seg[k]], 1u) - 1u : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      if (seg[k] == kNoSeg) continue;
      const uint64_t dst = P.seg_off[seg[k]] + r[k];
      if (dst >= P.max_records) {
        guard_trip(P, 32u);
        continue;
      }
      P.ent3[dst] = P.ent[idx[k]];
      P.ecls[dst] = cls[k];
    }
  }
}

// Segment lists by size class (the arrays are free once the records are grouped): small segments in
// seg_mark, mid ones from the front of eseg, big ones from its back.  Stream compaction without
// global atomics: per-workgroup class counts, one scan, then every workgroup writes its runs.
// List of segment s: small ones by record count (1, 2, 3-4, 5-8, 9-16, 17-24: lists 0-5, one list in
// that order, so that a wave's 64 lanes replay segments of about one size), then mid, large, huge (6-8).
__device__ __forceinline__ int seg_class(const BuildParams& P, uint64_t s) {
  if (s >= P.cap) return -1;
  const uint64_t n = P.seg_off[s + 1] - P.seg_off[s];
  if (n == 0) return -1;
  if (n <= kSmallSegOps) return n <= 1 ? 0 : n <= 2 ? 1 : n <= 4 ? 2 : n <= 8 ? 3 : n <= 16 ? 4 : 5;
  return n <= kMidSegMax ? 6 : n <= kLargeSegMax ? 7 : 8;
}
__device__ __forceinline__ int list_class(int l) { return l < kSmallLists ? 0 : l - kSmallLists + 1; }
// list of size class c: small in seg_mark, mid at the front of eseg, large at its back, huge in
// seg_start (all free once the records are grouped)
__device__ __forceinline__ uint64_t seg_list_cap(const BuildParams& P, int c) {
  return c == 0 ? P.cap + 1 : c == 3 ? P.cap : P.nslabs * (uint64_t)P.slab_cap;
}
__device__ __forceinline__ uint64_t* seg_list_slot(const BuildParams& P, int c, uint64_t i) {
  switch (c) {
    case 0: return reinterpret_cast<uint64_t*>(P.seg_mark) + i;
    case 1: return P.eseg + i;
    case 2: return P.eseg + (P.nslabs * (uint64_t)P.slab_cap - 1 - i);
    default: return reinterpret_cast<uint64_t*>(P.seg_start) + i;
  }
}

__global__ __launch_bounds__(kClsBlock) void k_seg_classify(BuildParams P, int write) {
  __shared__ uint32_t wsum[kSegLists][kClsBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t s0 = (uint64_t)blockIdx.x * kClsSlots + (uint64_t)tid * kClsItems;
  int cls[kClsItems];
  uint32_t c[kSegLists];
#pragma unroll
  for (int k = 0; k < kSegLists; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < kClsItems; i++) {
    cls[i] = seg_class(P, s0 + i);
#pragma unroll
    for (int k = 0; k < kSegLists; k++) c[k] += cls[i] == k ? 1u : 0u;
  }
  const uint32_t nblk = gridDim.x;
  if (!write) {  // per-workgroup counts, list-major
    for (int k = 0; k < kSegLists; k++) {
      uint32_t v = c[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) wsum[k][wv] = v;
    }
    __syncthreads();
    if (tid < kSegLists) {
      uint32_t t = 0;
      for (int w = 0; w < kClsBlock / 64; w++) t += wsum[tid][w];
      P.seg_cls_cnt[(uint64_t)tid * nblk + blockIdx.x] = t;
    }
    return;
  }
  // exclusive rank of this thread's segments inside the workgroup, per list
  uint32_t ex[kSegLists];
  for (int k = 0; k < kSegLists; k++) {
    uint32_t incl = c[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[k][wv] = incl;
    ex[k] = incl - c[k];
  }
  __syncthreads();
  for (int k = 0; k < kSegLists; k++)
    for (int w = 0; w < wv; w++) ex[k] += wsum[k][w];
  // a list's place in its class list: the small lists one after another, the others alone
  const uint64_t* off = P.seg_cls_off;
  uint64_t pos[kSegLists];
  for (int k = 0; k < kSegLists; k++)
    pos[k] = off[(uint64_t)k * nblk + blockIdx.x] - off[(uint64_t)(k < kSmallLists ? 0 : k) * nblk] + ex[k];
#pragma unroll
  for (int i = 0; i < kClsItems; i++) {
    if (cls[i] < 0) continue;
    uint64_t at = 0;
#pragma unroll
    for (int k = 0; k < kSegLists; k++)
      if (cls[i] == k) at = pos[k]++;
    const int cl = list_class(cls[i]);
    if (at < seg_list_cap(P, cl)) *seg_list_slot(P, cl, at) = s0 + i;
    else guard_trip(P, 64u);
  }
  if (blockIdx.x == 0 && tid < kSegClasses) {
    const int l0 = tid == 0 ? 0 : tid + kSmallLists - 1, l1 = tid == 0 ? kSmallLists : l0 + 1;
    P.st->n_segs[tid] = off[(uint64_t)l1 * nblk] - off[(uint64_t)l0 * nblk];
  }
}

// replay order: IN_MEMORY = address (log order); SORTING = (wantedSlot, address), the table's wanted
// slot (a window's run may wrap the table's end)
__device__ __forceinline__ bool seg_before(const BuildParams& P, const Entry& a, const Entry& b, int sorted_order) {
  if (sorted_order) {
    const uint64_t wa = window_to_table(fast_mod(a.hash, P.mod), P.mod);
    const uint64_t wb = window_to_table(fast_mod(b.hash, P.mod), P.mod);
    if (wa != wb) return wa < wb;
  }
  return (a.addr & ~kDelBit) < (b.addr & ~kDelBit);
}

// A segment replayed by one thread against the .spi slots in HBM; adds its counts to `acc`.
__device__ void replay_segment_hbm(const BuildParams& P, uint64_t s, Entry* L, uint64_t n, int sorted_order,
                                   int64_t acc[2]) {
  for (uint64_t i = 1; i < n; i++) {  // insertion sort: small segments, and the lane-0 fallback of
    const Entry v = L[i];              // huge ones (thousands of writes of one key)
    uint64_t j = i;
    while (j > 0 && seg_before(P, v, L[j - 1], sorted_order)) {
      L[j] = L[j - 1];
      j--;
    }
    L[j] = v;
  }
  (void)s;  // (the table was cleared after the grouping: the segment's slots start empty)
  Replay<HbmTable> r{&P, HbmTable{&P}, 0, 0};
  for (uint64_t i = 0; i < n; i++)
    if (!replay_one(r, L[i], 0)) break;
  acc[0] += r.num_entries;
  acc[1] += r.garbage;
}

// ------------------------------------------------------------------------------------------------
// k_seg_lanes: the small segments (<= kSmallSegOps records), one lane each, replayed in LDS.  Every
// record carries its key's class (ecls: the rank in its segment of the first placed PUT record with
// that key), so where IndexHash compares hashes and then both keys (IndexHash.java:606-636) a lane
// compares two bytes, and the log is read only for the garbage sizes of removed records.  Records are
// renumbered in replay order (IN_MEMORY: address; SORTING: the table's wanted slot, then address), which
// inside one wanted slot's group is address order: the tie rule (address < address2) compares the
// numbers.  Slots hold record numbers (0xff: empty); local slot index = slot - segment start, and a
// record's local wanted slot is its displacement origin (the segment's run never wraps in local terms).
// LDS arrays are [element][lane]: a lane's accesses to element i of its own arrays hit consecutive
// words across the wave, free of bank conflicts.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kLaneRecs = kSmallSegOps;
constexpr uint32_t kLaneDel = 0x80;         // class byte: a DELETE record
constexpr uint32_t kLaneFree = 0xffffffffu;  // an empty slot
constexpr uint32_t kLaneBatch = 8;          // global loads a lane issues together
// KeyT: 32-bit replay keys where every address fits (IN_MEMORY order over a log below 4 GB): 17 KB of
// LDS a wave instead of 23 KB, so 9 waves a CU instead of 6 hide the lanes' dependent loads.
template <typename KeyT>
struct LaneLds {
  KeyT key[kLaneRecs][64];           // replay-order keys; then the removed records' numbers (bytes)
  uint32_t slot[kLaneRecs + 1][64];  // local slot -> its record: number | wanted << 8 | class << 16
  uint16_t attr[kLaneRecs][64];      // list index, then record number -> local wanted slot | class << 8
  uint8_t perm[kLaneRecs][64];       // record number -> list index
};

template <typename KeyT>
__global__ __launch_bounds__(64) void k_seg_lanes(BuildParams P, int sorted_order) {
  static_assert(sizeof(KeyT) * kLaneRecs >= 2 * kLaneRecs, "the key array holds the u16 and byte lists after it");
  __shared__ LaneLds<KeyT> L;
  const int lane = threadIdx.x;
  const unsigned long long nseg = P.st->n_segs[0];
  int64_t entries = 0, garbage = 0;
  uint8_t* rem = reinterpret_cast<uint8_t*>(&L.key[0][0]);  // (removed numbers: rem[q * 64 + lane])
  unsigned long long* dbg = P.dbg ? P.dbg + (kMidGrid + kLargeGrid + kHugeGrid + blockIdx.x) * 8 : nullptr;
  unsigned long long t_prev = 0;
  auto mark = [&](int i) {  // diagnostic only (SPARKEY_EXACT_DEBUG=1): cycles per phase, per wave
    if (dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (i >= 0) dbg[i] += t - t_prev;
      t_prev = t;
    }
  };
  for (;;) {
    uint32_t kq = 0;
    if (lane == 0) kq = atomicAdd(&P.st->seg_next[0], 64u);
    const unsigned long long k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)kq);
    if (k0 >= nseg) break;
    mark(-1);
    const unsigned long long k = k0 + (uint64_t)lane;
    uint64_t s0 = 0, lo = 0;
    uint32_t n = 0, len = 0;
    if (k < nseg) {
      s0 = *seg_list_slot(P, 0, k);
      if (s0 < P.cap && P.seg_off[s0 + 1] <= P.max_records && P.seg_off[s0 + 1] - P.seg_off[s0] <= kLaneRecs) {
        lo = P.seg_off[s0];
        n = (uint32_t)(P.seg_off[s0 + 1] - lo);
        len = min(n, P.seg_len[s0]);
      } else {
        guard_trip(P, 4u);
      }
    }
    // replay-order keys (IN_MEMORY: address; SORTING: the table's wanted slot -- the segment's local
    // order, except that slots past the table's end come first -- then address), local wanted slots
    // and key classes (list indices of first records)
    const uint64_t t0 = window_to_table(s0, P.mod);
    for (uint32_t i0 = 0; i0 < n; i0 += kLaneBatch) {  // (a batch's loads in flight together)
      Entry eb[kLaneBatch];
      uint32_t cb[kLaneBatch];
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++) {
        eb[j] = i0 + j < n ? P.ent3[lo + i0 + j] : Entry{0, 0};
        cb[j] = i0 + j < n ? P.ecls[lo + i0 + j] : 0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++) {
        if (i0 + j >= n) continue;
        const uint64_t wl = fast_mod(eb[j].hash, P.mod);
        const uint64_t l = wl >= s0 ? wl - s0 : wl + P.cap - s0;
        const uint64_t addr = eb[j].addr & ~kDelBit;
        if (l >= len || (addr >> 58)) guard_trip(P, 1024u);
        uint64_t key = addr;
        if (sorted_order) key |= (l + (window_to_table(wl, P.mod) < t0 ? 0ull : 32ull)) << 58;
        if (sizeof(KeyT) < 8 && (key >> 32)) guard_trip(P, 1024u);  // (the host picks 32 bits only below 4 GB)
        L.key[i0 + j][lane] = (KeyT)key;
        L.attr[i0 + j][lane] = (uint16_t)(min(l, (uint64_t)kLaneRecs) |
                                          ((min(cb[j], kLaneRecs - 1) | ((eb[j].addr & kDelBit) ? kLaneDel : 0u)) << 8));
      }
    }
    mark(0);
    // record number = rank of the key (addresses are distinct, so are the keys); perm keeps the list
    // index and slot[i] (free until the replay) the number of list index i
    for (uint32_t i = 0; i < n; i++) {
      const KeyT ki = L.key[i][lane];
      uint32_t r = 0;
#pragma unroll
      for (uint32_t j = 0; j < kLaneRecs; j++) r += j < n && L.key[j][lane] < ki ? 1u : 0u;
      L.perm[r][lane] = (uint8_t)i;
      L.slot[i][lane] = r;
    }
    // attributes by number (through the key array, free now), the classes (first records' list
    // indices) as numbers too
    uint16_t* tmp = reinterpret_cast<uint16_t*>(&L.key[0][0]);
    for (uint32_t r = 0; r < n; r++) tmp[r * 64 + lane] = L.attr[L.perm[r][lane]][lane];
    for (uint32_t r = 0; r < n; r++) {
      const uint32_t v = tmp[r * 64 + lane];
      const uint32_t c = v >> 8;
      const uint32_t cn = L.slot[c & 0x7f][lane];
      L.attr[r][lane] = (uint16_t)((v & 0xff) | ((cn | (c & kLaneDel)) << 8));
    }
    for (uint32_t i = 0; i <= len; i++) L.slot[i][lane] = kLaneFree;
    mark(1);
    // the replay: IndexHash.put / delete (IndexHash.java:454-665) on the lane's slots, each probe step
    // one LDS word (the occupant's number, wanted slot and class)
    uint32_t nrem = 0;
    for (uint32_t r = 0; r < n; r++) {
      const uint32_t at = L.attr[r][lane];
      uint32_t s = at & 0xff;
      if (!((at >> 8) & kLaneDel)) {
        uint32_t C = r | (at << 8);  // the carried entry, packed as a slot word
        bool might = true;
        for (uint32_t g = 0; g <= len; g++, s++) {
          if (s > len) {
            guard_trip(P, 2048u);
            break;
          }
          const uint32_t o = L.slot[s][lane];
          if (o == kLaneFree) {
            L.slot[s][lane] = C;
            entries++;
            break;
          }
          if (might && ((o >> 16) & 0x7f) == ((C >> 16) & 0x7f)) {  // same key: replaced in place
            L.slot[s][lane] = C;
            rem[nrem++ * 64 + lane] = (uint8_t)o;
            break;
          }
          const uint32_t d = s - ((C >> 8) & 0xff), d2 = s - ((o >> 8) & 0xff);
          if (d > d2 || (d == d2 && (C & 0xff) < (o & 0xff))) {  // steal the slot, carry its occupant on
            L.slot[s][lane] = C;
            C = o;
            might = false;
          }
        }
      } else {
        const uint32_t myc = (at >> 8) & 0x7f;
        const uint32_t w0 = s;
        for (uint32_t g = 0; g <= len; g++, s++) {
          if (s > len) {
            guard_trip(P, 2048u);
            break;
          }
          const uint32_t o = L.slot[s][lane];
          if (o == kLaneFree) break;
          if (((o >> 16) & 0x7f) == myc) {  // found: backward shift (IndexHash.java:503-524)
            rem[nrem++ * 64 + lane] = (uint8_t)o;
            entries--;
            for (uint32_t g2 = 0; g2 < len && s < len; g2++) {
              const uint32_t o3 = L.slot[s + 1][lane];
              if (o3 == kLaneFree || ((o3 >> 8) & 0xff) == s + 1) break;
              L.slot[s][lane] = o3;
              s++;
            }
            L.slot[s][lane] = kLaneFree;
            break;
          }
          if (s - w0 > s - ((o >> 8) & 0xff)) break;  // displacement > the other's: not there
        }
      }
    }
    mark(2);
    // garbage of the removed records (IndexHeader.java:221-228), their headers read together
    for (uint32_t q0 = 0; q0 < nrem; q0 += kLaneBatch) {
      uint64_t ab8[kLaneBatch];
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++)
        ab8[j] = q0 + j < nrem ? P.ent3[lo + L.perm[rem[(q0 + j) * 64 + lane]][lane]].addr & ~kDelBit : 0ull;
      RecHdr hb[kLaneBatch];
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++)
        if (q0 + j < nrem) hb[j] = log_header(P, ab8[j]);
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++) {
        if (q0 + j >= nrem) continue;
        if (hb[j].rc) set_error(P.st, (int64_t)(ab8[j] >> P.ebb), header_error(hb[j]));
        else garbage += garbage_of(hb[j].klen, hb[j].vlen);
      }
    }
    // the segment's slots to the table (cleared before the replay)
    for (uint32_t i0 = 0; i0 < len; i0 += kLaneBatch) {
      Entry eb[kLaneBatch];
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++) {
        const uint32_t o = i0 + j < len ? L.slot[i0 + j][lane] : kLaneFree;
        eb[j] = o != kLaneFree ? P.ent3[lo + L.perm[o & 0xff][lane]] : Entry{0, 0};
      }
#pragma unroll
      for (uint32_t j = 0; j < kLaneBatch; j++) {
        if (i0 + j >= len || !eb[j].addr) continue;
        uint64_t t = s0 + i0 + j;
        if (t >= P.cap) t -= P.cap;
        write_slot(P, t, eb[j].hash, eb[j].addr & ~kDelBit);
      }
    }
    mark(3);
    if (dbg) {
      const unsigned long long nw = wave_sum_u64(n);
      if (lane == 0) {
        dbg[4] += 1;
        dbg[5] += nw;
      }
    }
  }
  commit_counts(P, entries, garbage);
}

// ------------------------------------------------------------------------------------------------
// k_seg_replay_wave: one wave per listed segment (grid-stride).  The segment's records go to LDS with
// their header fields (and keys of up to KEYB bytes), its slots too (local index = slot - s0 on the
// ring; local wanted slots, so a displacement is index - wanted), a bitonic sort orders the records,
// and the wave replays put / delete with 64 slots per step:
//   put, probe phase   the carried entry C is fixed until its first event, so every lane evaluates
//                      one slot: empty, error, same key (might), steal (d > d2 || d == d2 && a < a2);
//                      the first event in slot order is the one the sequential loop meets
//   put, shift phase   after a steal the carried entry is the previous slot's original occupant as
//                      long as every slot steals, so lane k checks "o[q-1] beats o[q] at q"; the
//                      slots before the first failure shift by one at once, an empty slot ends the
//                      put, a failure hands the carried entry back to the probe phase
//   delete             probe for the key (empty / displacement > other end it), then backward-shift
//                      the run behind it up to the first empty slot or entry at its wanted slot
// Exactly IndexHash.put / delete (IndexHash.java:454-665), in O(run / 64) steps per record.
// Segments of more than CAP records replay on lane 0 against HBM.
// ------------------------------------------------------------------------------------------------
struct SlotV {  // a slot's content as the wave sees it (local wanted slot, record id)
  uint64_t h, a;
  uint32_t w, id;
};

constexpr uint32_t pow2_ceil(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

template <uint32_t CAP, uint32_t KEYB>
struct SegLds {
  static constexpr uint32_t kOrd = pow2_ceil(CAP);  // the bitonic sort runs over the next power of two
  Entry ops[CAP];
  RecHdr hdr[CAP];
  uint64_t keys[KEYB ? CAP * (KEYB / 8) : 1];
  uint64_t th[CAP + 1];
  uint64_t ta[CAP + 1];
  uint16_t tw[CAP + 1];
  uint16_t to[CAP + 1];
  uint16_t ord[kOrd];
  uint32_t len;
  uint32_t nrec;
  __device__ __forceinline__ SlotV get(uint32_t i) const { return SlotV{th[i], ta[i], tw[i], to[i]}; }
  // header fields of record `id` (ids come from the replay's own slots; clamped all the same)
  __device__ __forceinline__ const RecHdr& rec(const BuildParams& P, uint32_t id) const {
    if (id >= nrec) {
      guard_trip(P, 128u);
      id = 0;
    }
    return hdr[id];
  }
  __device__ __forceinline__ void set(uint32_t i, const SlotV& v) {
    th[i] = v.h;
    ta[i] = v.a;
    tw[i] = (uint16_t)v.w;
    to[i] = (uint16_t)v.id;
  }
  __device__ __forceinline__ void clear(uint32_t i) {
    th[i] = 0;
    ta[i] = 0;
    tw[i] = 0;
    to[i] = 0;
  }
  __device__ __forceinline__ bool same_key(const BuildParams& P, uint32_t ix, uint32_t iy) const {
    if (ix >= nrec || iy >= nrec) {
      guard_trip(P, 16u);
      return false;
    }
    const RecHdr& x = hdr[ix];
    if (KEYB > 0 && x.klen <= (int32_t)KEYB) {
      for (uint32_t q = 0; q < KEYB / 8; q++)
        if (keys[ix * (KEYB / 8) + q] != keys[iy * (KEYB / 8) + q]) return false;
      return true;
    }
    const RecHdr& y = hdr[iy];
    return keys_equal(P, (int64_t)((ops[ix].addr & ~kDelBit) >> P.ebb) + x.hlen,
                      (int64_t)((ops[iy].addr & ~kDelBit) >> P.ebb) + y.hlen, x.klen);
  }
};

// broadcasts from a wave-uniform lane: v_readlane (no LDS round trip)
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)v, src); }
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int src) {
  return (uint64_t)lane_u32((uint32_t)v, src) | ((uint64_t)lane_u32((uint32_t)(v >> 32), src) << 32);
}
__device__ __forceinline__ SlotV lane_slot(const SlotV& v, int src) {
  return SlotV{lane_u64(v.h, src), lane_u64(v.a, src), lane_u32(v.w, src), lane_u32(v.id, src)};
}
__device__ __forceinline__ SlotV lane_slot_up(const SlotV& v) {
  return SlotV{(uint64_t)__shfl_up((unsigned long long)v.h, 1, 64), (uint64_t)__shfl_up((unsigned long long)v.a, 1, 64),
               (uint32_t)__shfl_up((int)v.w, 1, 64), (uint32_t)__shfl_up((int)v.id, 1, 64)};
}
__device__ __forceinline__ int first_lane(unsigned long long m) { return m ? __builtin_ctzll(m) : 64; }
// LDS written by some lanes is read by others in the next step: order the wave's LDS accesses (the
// compiler may otherwise move a lane's later loads above its own earlier stores to other addresses)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// put of record `id` (wave-uniform arguments); returns 0 or an error code
template <uint32_t CAP, uint32_t KEYB>
__device__ int wave_put(const BuildParams& P, SegLds<CAP, KEYB>& L, const Entry& en, uint32_t id, uint32_t wl,
                        int64_t& entries, int64_t& garbage) {
  const int lane = threadIdx.x & 63;
  const uint32_t len = L.len;
  SlotV C{en.hash, en.addr & ~kDelBit, wl, id};
  bool might = true;
  uint32_t s = wl;  // next slot the carried entry C looks at
  for (;;) {
    // ---- probe: C fixed, first slot >= s with an event ----
    int kind = 0;  // 1 empty, 2 error, 3 same key, 4 steal
    uint32_t at = 0;
    SlotV occ;
    int err = 0;
    for (;;) {
      const uint32_t i = s + (uint32_t)lane;
      int ev = 0, e_rc = 0;
      SlotV o{0, 0, 0, 0};
      if (i <= len) {
        o = L.get(i);
        if (o.a == 0) {
          ev = 1;
        } else {
          if (might && o.h == C.h) {
            const RecHdr& mine = L.rec(P, C.id);
            const RecHdr& other = L.rec(P, o.id);
            if (mine.rc) e_rc = header_error(mine);
            else if (!mine.put) e_rc = kErrCorruptData;
            else if (other.rc) e_rc = header_error(other);
            else if (!other.put) e_rc = kErrCorruptData;
            if (e_rc) ev = 2;
            else if (mine.klen == other.klen && L.same_key(P, C.id, o.id)) ev = 3;
          }
          if (!ev) {
            const int64_t d = (int64_t)i - (int64_t)C.w, d2 = (int64_t)i - (int64_t)o.w;
            if (d > d2 || (d == d2 && (int64_t)C.a < (int64_t)o.a)) ev = 4;
          }
        }
      }
      const int k = first_lane(__ballot(ev != 0));
      if (k < 64) {
        kind = (int)lane_u32((uint32_t)ev, k);
        err = (int)lane_u32((uint32_t)e_rc, k);
        occ = lane_slot(o, k);
        at = s + (uint32_t)k;
        break;
      }
      s += 64;
      if (s > len) return kErrNoFreeSlots;  // unreachable: slot len is empty
    }
    if (kind == 2) return err;
    if (kind == 1) {
      if (lane == 0) L.set(at, C);
      wave_lds_sync();
      entries++;
      return 0;
    }
    if (kind == 3) {  // replace in place (IndexHash.java:630-636)
      if (lane == 0) L.set(at, C);
      wave_lds_sync();
      garbage += garbage_of(L.rec(P, occ.id).klen, L.rec(P, occ.id).vlen);
      return 0;
    }
    // ---- steal at `at`: C takes the slot, its occupant is carried on; shift while every slot steals ----
    if (lane == 0) L.set(at, C);
    wave_lds_sync();
    C = occ;
    might = false;
    uint32_t q0 = at + 1;
    for (;;) {
      const uint32_t q = q0 + (uint32_t)lane;
      SlotV o{0, 0, 0, 0};
      if (q <= len) o = L.get(q);
      SlotV prev = lane_slot_up(o);  // the original occupant of q - 1 (lane 0: the carried entry)
      if (lane == 0) prev = C;
      bool ev = false;
      if (q <= len) {
        if (o.a == 0) {
          ev = true;
        } else {
          const int64_t d = (int64_t)q - (int64_t)prev.w, d2 = (int64_t)q - (int64_t)o.w;
          ev = !(d > d2 || (d == d2 && (int64_t)prev.a < (int64_t)o.a));
        }
      }
      const int k = first_lane(__ballot(ev));
      if (lane < k && q <= len) L.set(q, prev);  // the chain's steals: everything moves up one slot
      wave_lds_sync();
      if (k == 64) {
        C = lane_slot(o, 63);
        q0 += 64;
        if (q0 > len) return kErrNoFreeSlots;  // unreachable
        continue;
      }
      const SlotV pk = lane_slot(prev, k);
      const bool empty = lane_u64(o.a, k) == 0;
      if (empty) {
        if (lane == k) L.set(q, prev);
        wave_lds_sync();
        entries++;
        return 0;
      }
      C = pk;  // does not steal at q0 + k: probe on from the next slot
      s = q0 + (uint32_t)k + 1;
      break;
    }
  }
}

// delete of record `id`; returns 0 or an error code
template <uint32_t CAP, uint32_t KEYB>
__device__ int wave_delete(const BuildParams& P, SegLds<CAP, KEYB>& L, const Entry& en, uint32_t id, uint32_t wl,
                           int64_t& entries, int64_t& garbage) {
  const int lane = threadIdx.x & 63;
  const uint32_t len = L.len;
  const uint64_t h = en.hash;
  uint32_t s = wl;
  int kind = 0;  // 1 not there, 2 error, 3 found
  uint32_t at = 0;
  SlotV occ;
  int err = 0;
  for (;;) {
    const uint32_t i = s + (uint32_t)lane;
    int ev = 0, e_rc = 0;
    SlotV o{0, 0, 0, 0};
    if (i <= len) {
      o = L.get(i);
      if (o.a == 0) {
        ev = 1;
      } else {
        if (o.h == h) {
          const RecHdr& mine = L.rec(P, id);
          const RecHdr& other = L.rec(P, o.id);
          if (mine.rc) e_rc = header_error(mine);
          else if (mine.put) e_rc = kErrCorruptData;
          else if (other.rc) e_rc = header_error(other);
          else if (!other.put) e_rc = kErrCorruptData;
          if (e_rc) ev = 2;
          else if (mine.klen == other.klen && L.same_key(P, id, o.id)) ev = 3;
        }
        if (!ev && (int64_t)i - (int64_t)wl > (int64_t)i - (int64_t)o.w) ev = 1;
      }
    }
    const int k = first_lane(__ballot(ev != 0));
    if (k < 64) {
      kind = (int)lane_u32((uint32_t)ev, k);
      err = (int)lane_u32((uint32_t)e_rc, k);
      occ = lane_slot(o, k);
      at = s + (uint32_t)k;
      break;
    }
    s += 64;
    if (s > len) return 0;
  }
  if (kind == 1) return 0;
  if (kind == 2) return err;
  // backward shift (IndexHash.java:503-524): entries after `at` move down one slot until an empty
  // slot or an entry at its wanted slot; the last moved-from slot is cleared
  uint32_t q0 = at + 1;
  for (;;) {
    const uint32_t q = q0 + (uint32_t)lane;
    SlotV o{0, 0, 0, 0};
    bool stop = true;
    if (q <= len) {
      o = L.get(q);
      stop = o.a == 0 || o.w == q;
    }
    const int k = first_lane(__ballot(stop));
    if (lane < k) L.set(q - 1, o);
    wave_lds_sync();
    if (k < 64) {
      if (lane == k) L.clear(q - 1);
      wave_lds_sync();
      break;
    }
    q0 += 64;
  }
  garbage += garbage_of(L.rec(P, occ.id).klen, L.rec(P, occ.id).vlen);
  entries--;
  return 0;
}

template <uint32_t CAP, uint32_t KEYB, int CLS>
__global__ __launch_bounds__(64) void k_seg_replay_wave(BuildParams P, int sorted_order) {
  __shared__ SegLds<CAP, KEYB> L;
  const int lane = threadIdx.x;
  const unsigned long long nseg = P.st->n_segs[CLS];
  int64_t acc[2] = {0, 0};  // this wave's numEntries / garbageSize (lane 0)
  unsigned long long* dbg =
      P.dbg ? P.dbg + ((CLS == 1 ? 0 : CLS == 2 ? kMidGrid : kMidGrid + kLargeGrid) + blockIdx.x) * 8 : nullptr;
  unsigned long long t_prev = 0;
  auto mark = [&](int i) {  // diagnostic only (SPARKEY_EXACT_DEBUG=1): cycles per phase, per wave
    if (dbg && lane == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (i >= 0) dbg[i] += t - t_prev;
      t_prev = t;
    }
  };
  // segments from a work queue: a wave that drew short ones draws again (a static stride left the
  // waves whose segments ran long to finish the class alone, and the grid is larger than what fits)
  for (;;) {
    uint32_t kq = 0;
    if (lane == 0) kq = atomicAdd(&P.st->seg_next[CLS], 1u);
    const unsigned long long k = (uint32_t)__builtin_amdgcn_readfirstlane((int)kq);
    if (k >= nseg) break;
    mark(-1);
    const uint64_t s0 = *seg_list_slot(P, CLS, k);
    if (s0 >= P.cap || P.seg_off[s0 + 1] > P.max_records) {
      if (lane == 0) guard_trip(P, 8u);
      continue;
    }
    const uint64_t lo = P.seg_off[s0];
    const uint64_t n64 = P.seg_off[s0 + 1] - lo;
    if (n64 > CAP) {
      if (lane == 0) replay_segment_hbm(P, s0, P.ent3 + lo, n64, sorted_order, acc);
      __syncthreads();
      continue;
    }
    const uint32_t n = (uint32_t)n64;
    if (lane == 0) {
      L.len = min(n, P.seg_len[s0]);  // (the run of the distinct keys' placement: at most n slots)
      L.nrec = n;
    }
    __syncthreads();
    // stage the records (header fields, short keys)
    for (uint32_t i = lane; i < n; i += 64) {
      const Entry en = P.ent3[lo + i];
      L.ops[i] = en;
      const RecHdr h = log_header(P, en.addr & ~kDelBit);
      L.hdr[i] = h;
      if (KEYB > 0) {
        uint64_t kw[KEYB ? KEYB / 8 : 1];
#pragma unroll
        for (uint32_t q = 0; q < KEYB / 8; q++) kw[q] = 0;
        if (h.rc == 0 && h.klen >= 0 && h.klen <= (int32_t)KEYB) {
          const int64_t kp = (int64_t)((en.addr & ~kDelBit) >> P.ebb) + h.hlen;
          if (kp + h.klen <= (int64_t)P.log_len) {
            static_assert(KEYB <= 16, "keys staged from one 16-byte load");
            const Bytes16 kb = log16(P, kp);
#pragma unroll
            for (uint32_t q = 0; q < KEYB / 8; q++) {
              const int32_t nb = min(max(h.klen - 8 * (int32_t)q, 0), 8);  // key bytes of word q
              const uint64_t v = (uint64_t)kb.w[2 * q] | ((uint64_t)kb.w[2 * q + 1] << 32);
              kw[q] = nb >= 8 ? v : v & ((1ull << (8 * nb)) - 1ull);
            }
          } else {
            guard_trip(P, 2u);
          }
        }
#pragma unroll
        for (uint32_t q = 0; q < KEYB / 8; q++) L.keys[i * (KEYB / 8) + q] = kw[q];
      }
    }
    uint32_t n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (uint32_t i = lane; i < n2; i += 64) L.ord[i] = i < n ? (uint16_t)i : (uint16_t)0xffff;
    for (uint32_t i = lane; i <= n; i += 64) L.clear(i);
    __syncthreads();
    mark(0);
    // bitonic sort of the record indices (0xffff pads sort last)
    for (uint32_t kk = 2; kk <= n2; kk <<= 1) {
      for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
        for (uint32_t i = lane; i < n2; i += 64) {
          const uint32_t ixj = i ^ j;
          if (ixj > i) {
            const uint16_t a = L.ord[i], b = L.ord[ixj];
            const bool b_first = a == 0xffff ? b != 0xffff
                                             : (b != 0xffff && seg_before(P, L.ops[b], L.ops[a], sorted_order));
            if (b_first == ((i & kk) == 0)) {
              L.ord[i] = b;
              L.ord[ixj] = a;
            }
          }
        }
        __syncthreads();
      }
    }
    mark(1);
    int64_t entries = 0, garbage = 0;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t id = L.ord[i];
      const Entry en = L.ops[id];
      const uint64_t wg = fast_mod(en.hash, P.mod);
      const uint32_t wl = (uint32_t)(wg >= s0 ? wg - s0 : wg + P.cap - s0);
      const int rc = (en.addr & kDelBit) ? wave_delete(P, L, en, id, wl, entries, garbage)
                                         : wave_put(P, L, en, id, wl, entries, garbage);
      __syncthreads();
      if (rc) {
        if (lane == 0) set_error(P.st, (int64_t)((en.addr & ~kDelBit) >> P.ebb), rc);
        break;
      }
    }
    mark(2);
    if (lane == 0) {
      acc[0] += entries;
      acc[1] += garbage;
    }
    if (dbg && lane == 0) {
      dbg[4] += 1;
      dbg[5] += n;
    }
    const uint32_t len = min(L.len, n);
    for (uint32_t i = lane; i < len; i += 64) {
      uint64_t slot = s0 + i;
      if (slot >= P.cap) slot -= P.cap;
      write_slot(P, slot, L.th[i], L.ta[i]);
    }
    __syncthreads();
    mark(3);
  }
  commit_counts(P, acc[0], acc[1]);
}

// ================================================================================================
// launchers
// ================================================================================================
void launch_sequential(const BuildParams& P, hipStream_t s, int sorted_order) {
  hipLaunchKernelGGL(k_sequential, dim3(1), dim3(64), 0, s, P, sorted_order);
}

// seg_cnt zeroed and num_entries / garbage / segment counters reset by the caller; ent3 receives the
// grouped records
// check_each (SPARKEY_EXACT_DEBUG=2, diagnostics): synchronize after every launch and report it
void launch_segments(const BuildParams& P, hipStream_t s, int sorted_order, StageTimer* tm, bool check_each,
                     const SideStreams* side) {
  auto step = [&](const char* what) {
    if (!check_each) return;
    const hipError_t e = hipStreamSynchronize(s);
    fprintf(stderr, "[exact] %s: %s\n", what, hipGetErrorString(e));
    fflush(stderr);
  };
  const unsigned slot_grid = (unsigned)((P.cap + 255) / 256);
  // the distinct keys' placement: its occupied slots, their runs (the segments), each segment's PUT
  // records in the placement of every PUT record and its length (seg_len zeroed by the caller)
  hipLaunchKernelGGL(k_seg_dcount, dim3(slot_grid), dim3(256), 0, s, P);
  step("distinct counts");
  scan_exclusive<DistinctCount, MaxPlus, OpMaxPlus>(reinterpret_cast<const DistinctCount*>(P.seg_len), P.seg_fun,
                                                    P.cap, P.seg_fun + P.cap, OpMaxPlus(), P.seg_fun + P.cap + 1, s);
  step("carry scan");
  hipLaunchKernelGGL(k_seg_dmarks, dim3(slot_grid), dim3(256), 0, s, P);
  step("marks");
  scan_exclusive<int64_t, int64_t, OpMaxI64>(P.seg_mark, P.seg_start, P.cap, P.seg_mark + P.cap, OpMaxI64(),
                                             reinterpret_cast<int64_t*>(P.scan_scratch_u64), s);
  step("start scan");
  hipLaunchKernelGGL(k_seg_first, dim3(slot_grid), dim3(256), 0, s, P);
  // k_seg_runs on a side stream beside k_seg_assign: both latency-bound, and they share only seg_cnt,
  // which both add to
  const bool fork = side && !check_each;
  if (fork) {
    (void)hipEventRecord(side->fork, s);
    (void)hipStreamWaitEvent(side->s[0], side->fork, 0);
  }
  hipLaunchKernelGGL(k_seg_runs, dim3(slot_grid), dim3(256), 0, fork ? side->s[0] : s, P);
  step("runs");
  const unsigned seg_grid = (unsigned)((P.nslabs + kSegSlabs - 1) / kSegSlabs);
  if (P.nslabs) hipLaunchKernelGGL(k_seg_assign, dim3(seg_grid), dim3(64), 0, s, P);
  step("assign");
  if (fork) {
    (void)hipEventRecord(side->join[0], side->s[0]);
    (void)hipStreamWaitEvent(s, side->join[0], 0);
  }
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.seg_cnt, P.seg_off, P.cap, P.seg_off + P.cap, OpAdd(),
                                            P.scan_scratch_u64, s);
  step("count scan");
  // the PUT and DELETE records to their places (disjoint: the DELETEs take the top of each segment's
  // list), the DELETEs on a side stream, and the size classes' counts (they read seg_off only) on
  // another; joined before the class lists are written (into arrays k_seg_puts / k_seg_scatter read)
  const unsigned cls_grid = (unsigned)((P.cap + kClsSlots - 1) / kClsSlots);
  hipStream_t sd = fork ? side->s[0] : s, sc = fork ? side->s[1] : s;
  if (fork) {
    (void)hipEventRecord(side->fork, s);
    (void)hipStreamWaitEvent(sd, side->fork, 0);
    (void)hipStreamWaitEvent(sc, side->fork, 0);
  }
  hipLaunchKernelGGL(k_seg_classify, dim3(cls_grid), dim3(kClsBlock), 0, sc, P, 0);
  step("classify counts");
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.seg_cls_cnt, P.seg_cls_off, (uint64_t)kSegLists * cls_grid,
                                            P.seg_cls_off + (uint64_t)kSegLists * cls_grid, OpAdd(), P.scan_scratch_u64, sc);
  step("classify scan");
  if (P.nslabs) hipLaunchKernelGGL(k_seg_scatter, dim3(seg_grid), dim3(64), 0, sd, P);
  hipLaunchKernelGGL(k_seg_puts, dim3(slot_grid), dim3(256), 0, s, P);
  step("scatter");
  // the records are grouped: the replays start from an empty table (slots outside every segment stay
  // empty; the placement of every PUT record filled some of them)
  (void)hipMemsetAsync(P.out + kIndexHeaderSize, 0, (size_t)P.cap * (size_t)P.slot_size, s);
  if (fork) {
    for (int i = 0; i < 2; i++) {
      (void)hipEventRecord(side->join[i], side->s[i]);
      (void)hipStreamWaitEvent(s, side->join[i], 0);
    }
  }
  hipLaunchKernelGGL(k_seg_classify, dim3(cls_grid), dim3(kClsBlock), 0, s, P, 1);
  step("classify lists");
  if (check_each) {
    Status h;
    if (hipMemcpy(&h, P.st, sizeof(Status), hipMemcpyDeviceToHost) == hipSuccess)
      fprintf(stderr, "[exact] segments per class: %llu %llu %llu %llu, guard %u\n", h.n_segs[0], h.n_segs[1],
              h.n_segs[2], h.n_segs[3], h.guard);
  }
  // the size classes replay disjoint slots: huge, large and mid on the side streams, concurrent with
  // small on the build stream (longest tails first), joined back before the stats
  (void)hipMemsetAsync(P.st->seg_next, 0, sizeof(P.st->seg_next), s);  // (the classes' work queues)
  hipStream_t sh = fork ? side->s[0] : s, sl = fork ? side->s[1] : s, sm = fork ? side->s[2] : s;
  if (fork) {
    (void)hipEventRecord(side->fork, s);
    for (int i = 0; i < 3; i++) (void)hipStreamWaitEvent(side->s[i], side->fork, 0);
  }
  hipLaunchKernelGGL((k_seg_replay_wave<kHugeSegMax, 0, 3>), dim3(kHugeGrid), dim3(64), 0, sh, P, sorted_order);
  step("huge");
  hipLaunchKernelGGL((k_seg_replay_wave<kLargeSegMax, 16, 2>), dim3(kLargeGrid), dim3(64), 0, sl, P, sorted_order);
  step("large");
  hipLaunchKernelGGL((k_seg_replay_wave<kMidSegMax, 16, 1>), dim3(kMidGrid), dim3(64), 0, sm, P, sorted_order);
  step("mid");
  if (!sorted_order && (((uint64_t)P.log_len + 1) << P.ebb) <= (1ull << 32))
    hipLaunchKernelGGL(k_seg_lanes<uint32_t>, dim3(kLaneGrid), dim3(64), 0, s, P, sorted_order);
  else
    hipLaunchKernelGGL(k_seg_lanes<uint64_t>, dim3(kLaneGrid), dim3(64), 0, s, P, sorted_order);
  step("small");
  if (fork) {
    for (int i = 0; i < 3; i++) {
      (void)hipEventRecord(side->join[i], side->s[i]);
      (void)hipStreamWaitEvent(s, side->join[i], 0);
    }
  }
  tm->mark("exact", s);
}

}  // namespace sk
