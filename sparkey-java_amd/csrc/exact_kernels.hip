// exact_kernels.hip -- IndexHash.put / delete replayed exactly (IndexHash.java:454-665) for logs the
// canonical layout does not cover: DELETE records and duplicate keys (overwrites).
//
//   k_sequential      one lane over the whole table: tables whose PUT records leave no empty slot
//   k_seg_marks/scan  the first slot of every run of occupied slots of the canonical PUT placement
//   k_seg_assign      every record -> the slot segment holding its wanted slot
//   k_seg_scatter     records grouped by segment
//   k_seg_classify    segments listed by size class
//   k_seg_small       one thread per small segment: sort, clear, replay on the .spi slots in HBM
//   k_seg_replay_wave one wave per larger segment: records, their header fields, short keys and the
//                     segment's slots staged in LDS, bitonic sort, put / delete evaluated 64 slots
//                     per step, slots written back
//
// Why segments are independent.  occ(S), the set of slots a linear-probing table of the multiset S of
// wanted slots occupies, depends neither on insertion order, nor on the Robin-Hood tie rule, nor on
// in-place replacement or backward-shift deletion (every entry sits at w + d with slots w .. w + d
// all occupied), and it grows with S.  Every table state IndexHash passes through holds a subset of
// the log's PUT keys, so a slot the canonical placement of ALL PUT records (duplicates included,
// DELETEs left out) leaves empty is empty in every state: no put probe, delete probe or backward
// shift ever crosses it.  The runs of occupied slots of that placement -- segments -- therefore
// evolve independently.  Each one replays its own records in the reference's order (log order for
// IN_MEMORY; SortHelper's (wantedSlot, address) for SORTING, SortHelper.java:153-171) with the
// reference's put / delete on its own slots; a DELETE whose wanted slot is empty there is a no-op in
// every state.  The result is the reference's table byte for byte.
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
constexpr int kSegClasses = 4;
constexpr int kClsBlock = 256;            // k_seg_classify: 4 slots per thread
constexpr int kClsItems = 4;
constexpr uint64_t kClsSlots = (uint64_t)kClsBlock * kClsItems;

// Every global access of the exact path is bounds-checked: a violation (a bug, never a property of
// the input) sets a bit of st->guard, skips the access, and the host fails the build loudly.
__device__ __forceinline__ void guard_trip(const BuildParams& P, unsigned bit) { atomicOr(&P.st->guard, bit); }

__device__ __forceinline__ bool keys_equal(const BuildParams& P, int64_t k1, int64_t k2, int32_t len) {
  if (len < 0 || k1 < 0 || k2 < 0 || k1 + len > (int64_t)P.log_len || k2 + len > (int64_t)P.log_len) {
    guard_trip(P, 1u);
    return false;
  }
  for (int32_t j = 0; j < len; j++)
    if (P.log[k1 + j] != P.log[k2 + j]) return false;
  return true;
}
__device__ __forceinline__ RecHdr log_header(const BuildParams& P, uint64_t address) {
  auto at = [&](int64_t a) -> uint32_t { return P.log[a]; };
  return decode_header(at, (int64_t)(address >> P.ebb), (int64_t)P.log_len);
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
__device__ __forceinline__ bool slot_occupied(const BuildParams& P, uint64_t slot) {
  uint64_t h, a;
  read_slot(P, slot, h, a);
  return a != 0;
}

// mark[i] = i + 1 for an empty slot, 0 for an occupied one; its exclusive max-scan gives every slot
// the first slot of its run (<= 0: the run wraps, it starts after the table's last empty slot)
__global__ __launch_bounds__(256) void k_seg_marks(BuildParams P) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.cap) P.seg_mark[i] = slot_occupied(P, i) ? 0 : (int64_t)(i + 1);
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

// The PUT records of a segment are exactly the entries the canonical placement left in its run (every
// PUT record, duplicates included, was placed; occ(S) does not depend on the order), so a run's PUT
// count is its length: the empty slot that ends a run writes it at the run's start, with no atomics.
__global__ __launch_bounds__(256) void k_seg_runs(BuildParams P) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.cap || P.seg_mark[e] == 0) return;  // (occupied)
  const uint64_t p = e == 0 ? P.cap - 1 : e - 1;
  if (P.seg_mark[p] == 0) {
    const uint64_t st = run_start(P, p, P.seg_mark[P.cap]);
    P.seg_cnt[st] = (uint32_t)(e >= st ? e - st : e + P.cap - st);
  }
}

// DELETE records (the PUT records come from the table, k_seg_puts): each finds the first slot of the
// segment holding its wanted slot and counts itself there.  A slot is occupied when its mark is 0.
// kSegSlabs slabs a 64-thread workgroup (several chains a thread in flight).
__global__ __launch_bounds__(64) void k_seg_assign(BuildParams P) {
  const int64_t last = P.seg_mark[P.cap];  // (last empty slot) + 1
  uint32_t n[kSegSlabs], nmax = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSegSlabs; k++) {
    const uint64_t w = (uint64_t)blockIdx.x * kSegSlabs + k;
    n[k] = w < P.nslabs ? P.wcount[w] : 0u;
    nmax = max(nmax, n[k]);
  }
  for (uint32_t j = threadIdx.x; j < nmax; j += 64) {
    uint64_t idx[kSegSlabs], sl[kSegSlabs];
    bool del[kSegSlabs];
    int64_t mk[kSegSlabs];
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      idx[k] = ((uint64_t)blockIdx.x * kSegSlabs + k) * P.slab_cap + j;
      Entry en{0, 0};
      if (j < n[k]) en = P.ent[idx[k]];
      del[k] = j < n[k] && (en.addr & kDelBit);
      sl[k] = del[k] ? fast_mod(en.hash, P.mod) : 0;
    }
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) mk[k] = del[k] ? P.seg_mark[sl[k]] : 1;
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
      if (!del[k]) continue;
      uint64_t seg = kNoSeg;
      if (mk[k] == 0) {  // (a DELETE whose wanted slot is empty is a no-op in every state)
        seg = run_start(P, sl[k], last);
        atomicAdd(&P.seg_cnt[seg], 1u);
      }
      P.eseg[idx[k]] = seg;
    }
  }
}

// The PUT records grouped by segment straight from the table: occupied slot t is record t - start of
// its segment's list (slot order; the replay sorts a segment itself).  Reads and writes in slot order.
__global__ __launch_bounds__(256) void k_seg_puts(BuildParams P) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P.cap || P.seg_mark[t] != 0) return;
  const uint64_t st = run_start(P, t, P.seg_mark[P.cap]);
  const uint64_t dst = P.seg_off[st] + (t >= st ? t - st : t + P.cap - st);
  if (dst >= P.max_records) {
    guard_trip(P, 32u);
    return;
  }
  uint64_t h, a;
  read_slot(P, t, h, a);
  P.ent3[dst] = Entry{h, a};
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
#pragma unroll
    for (uint32_t k = 0; k < kSegSlabs; k++) {
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
    }
  }
}

// Segment lists by size class (the arrays are free once the records are grouped): small segments in
// seg_mark, mid ones from the front of eseg, big ones from its back.  Stream compaction without
// global atomics: per-workgroup class counts, one scan, then every workgroup writes its runs.
__device__ __forceinline__ int seg_class(const BuildParams& P, uint64_t s) {
  if (s >= P.cap) return -1;
  const uint64_t n = P.seg_off[s + 1] - P.seg_off[s];
  if (n == 0) return -1;
  return n <= kSmallSegOps ? 0 : n <= kMidSegMax ? 1 : n <= kLargeSegMax ? 2 : 3;
}
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
  __shared__ uint32_t wsum[kSegClasses][kClsBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t s0 = (uint64_t)blockIdx.x * kClsSlots + (uint64_t)tid * kClsItems;
  int cls[kClsItems];
  uint32_t c[kSegClasses] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < kClsItems; i++) {
    cls[i] = seg_class(P, s0 + i);
    if (cls[i] >= 0) c[cls[i]]++;
  }
  const uint32_t nblk = gridDim.x;
  if (!write) {  // per-workgroup counts, class-major
    for (int k = 0; k < kSegClasses; k++) {
      uint32_t v = c[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) wsum[k][wv] = v;
    }
    __syncthreads();
    if (tid < kSegClasses) {
      uint32_t t = 0;
      for (int w = 0; w < kClsBlock / 64; w++) t += wsum[tid][w];
      P.seg_cls_cnt[(uint64_t)tid * nblk + blockIdx.x] = t;
    }
    return;
  }
  // exclusive rank of this thread's segments inside the workgroup, per class
  uint32_t ex[kSegClasses];
  for (int k = 0; k < kSegClasses; k++) {
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
  for (int k = 0; k < kSegClasses; k++)
    for (int w = 0; w < wv; w++) ex[k] += wsum[k][w];
  const uint64_t* off = P.seg_cls_off;
  uint64_t pos[kSegClasses];
  for (int k = 0; k < kSegClasses; k++) pos[k] = off[(uint64_t)k * nblk + blockIdx.x] - off[(uint64_t)k * nblk] + ex[k];
#pragma unroll
  for (int i = 0; i < kClsItems; i++) {
    if (cls[i] < 0) continue;
    const uint64_t at = pos[cls[i]]++;
    if (at < seg_list_cap(P, cls[i])) *seg_list_slot(P, cls[i], at) = s0 + i;
    else guard_trip(P, 64u);
  }
  if (blockIdx.x == 0 && tid < kSegClasses) P.st->n_segs[tid] = off[(uint64_t)(tid + 1) * nblk] - off[(uint64_t)tid * nblk];
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
  uint64_t t = s;
  for (uint64_t g = 0; g < P.cap && slot_occupied(P, t); g++) {  // clear the canonical placement
    write_slot(P, t, 0, 0);
    t = t + 1 == P.cap ? 0 : t + 1;
  }
  Replay<HbmTable> r{&P, HbmTable{&P}, 0, 0};
  for (uint64_t i = 0; i < n; i++)
    if (!replay_one(r, L[i], 0)) break;
  acc[0] += r.num_entries;
  acc[1] += r.garbage;
}

__global__ __launch_bounds__(256) void k_seg_small(BuildParams P, int sorted_order) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t acc[2] = {0, 0};
  if (i < P.st->n_segs[0]) {
    const uint64_t s = *seg_list_slot(P, 0, i);
    if (s < P.cap && P.seg_off[s + 1] <= P.max_records) {
      const uint64_t lo = P.seg_off[s];
      replay_segment_hbm(P, s, P.ent3 + lo, P.seg_off[s + 1] - lo, sorted_order, acc);
    } else {
      guard_trip(P, 4u);
    }
  }
  commit_counts(P, acc[0], acc[1]);
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
      L.len = n;
      L.nrec = n;
    }
    __syncthreads();
    // stage the records (header fields, short keys); the segment's length = its first empty slot,
    // at most n slots in
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
            for (int32_t b = 0; b < h.klen; b++) kw[b >> 3] |= (uint64_t)P.log[kp + b] << (8 * (b & 7));
          } else {
            guard_trip(P, 2u);
          }
        }
#pragma unroll
        for (uint32_t q = 0; q < KEYB / 8; q++) L.keys[i * (KEYB / 8) + q] = kw[q];
      }
      uint64_t slot = s0 + i;
      if (slot >= P.cap) slot -= P.cap;
      if (!slot_occupied(P, slot)) atomicMin(&L.len, i);
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
  hipLaunchKernelGGL(k_seg_marks, dim3(slot_grid), dim3(256), 0, s, P);
  step("marks");
  scan_exclusive<int64_t, int64_t, OpMaxI64>(P.seg_mark, P.seg_start, P.cap, P.seg_mark + P.cap, OpMaxI64(),
                                             reinterpret_cast<int64_t*>(P.scan_scratch_u64), s);
  step("start scan");
  hipLaunchKernelGGL(k_seg_runs, dim3(slot_grid), dim3(256), 0, s, P);
  step("runs");
  const unsigned seg_grid = (unsigned)((P.nslabs + kSegSlabs - 1) / kSegSlabs);
  if (P.nslabs) hipLaunchKernelGGL(k_seg_assign, dim3(seg_grid), dim3(64), 0, s, P);
  step("assign");
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.seg_cnt, P.seg_off, P.cap, P.seg_off + P.cap, OpAdd(),
                                            P.scan_scratch_u64, s);
  step("count scan");
  hipLaunchKernelGGL(k_seg_puts, dim3(slot_grid), dim3(256), 0, s, P);
  if (P.nslabs) hipLaunchKernelGGL(k_seg_scatter, dim3(seg_grid), dim3(64), 0, s, P);
  step("scatter");
  const unsigned cls_grid = (unsigned)((P.cap + kClsSlots - 1) / kClsSlots);
  hipLaunchKernelGGL(k_seg_classify, dim3(cls_grid), dim3(kClsBlock), 0, s, P, 0);
  step("classify counts");
  scan_exclusive<uint32_t, uint64_t, OpAdd>(P.seg_cls_cnt, P.seg_cls_off, (uint64_t)kSegClasses * cls_grid,
                                            P.seg_cls_off + (uint64_t)kSegClasses * cls_grid, OpAdd(), P.scan_scratch_u64, s);
  step("classify scan");
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
  const bool fork = side && !check_each;
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
  hipLaunchKernelGGL(k_seg_small, dim3(slot_grid), dim3(256), 0, s, P, sorted_order);
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
