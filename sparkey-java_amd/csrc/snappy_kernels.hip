// snappy_kernels.hip -- SNAPPY log front end on the device (snappy.hpp).
//
//   k_snappy_dir      block directory: the chain of VLQ(compressedSize) block headers from offset 84 to
//                     dataEnd (CompressedReader.fetchBlock, CompressedReader.java:66-74), one lane
//   k_snappy_lds      one wave per block: the Snappy stream read through an LDS window, decoded
//                     element by element into LDS (every lane copies a slice of each literal /
//                     match), streamed out to the virtual log
//   k_snappy_walk     one lane per block: the block's records
//   k_snappy_global   the same, lane-serial in global memory, for blocks too large for LDS
//   k_snappy_rewrite  one lane per slot: virtual offset -> (blockPosition << ebb) | entryIndex
#include "device_common.hpp"
#include "snappy.hpp"
#include "knobs.hpp"

namespace sk {

namespace {

__device__ __forceinline__ int64_t align16(int64_t x) { return (x + 15) & ~15LL; }

// len bytes: one byte per lane per round for short copies (one LDS round trip for the usual
// <= 256-byte element), 16 consecutive bytes per lane per round for long ones.  32-bit indices:
// blocks are < 2^31 bytes (compressionBlockSize is a Java int).
// kVol: src is output in global memory written by this wave (volatile loads, past the vector L1).
template <bool kVol = false>
__device__ __forceinline__ uint8_t ld_byte(const uint8_t* p) {
  if (kVol) return *(const volatile uint8_t*)p;
  return *p;
}

template <bool kVol = false>
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint32_t len, uint32_t lane,
                                           uint32_t nlanes) {
  if (len <= 4 * nlanes) {
    for (uint32_t k = lane; k < len; k += nlanes) dst[k] = ld_byte<kVol>(src + k);
    return;
  }
  for (uint32_t k = lane * 16; k < len; k += nlanes * 16) {
    if (k + 16 <= len) {
      uint8_t t[16];
#pragma unroll
      for (int i = 0; i < 16; i++) t[i] = ld_byte<kVol>(src + k + i);
#pragma unroll
      for (int i = 0; i < 16; i++) dst[k + i] = t[i];
    } else {
      for (uint32_t i = k; i < len; i++) dst[i] = ld_byte<kVol>(src + i);
    }
  }
}

// Where snappy_decode reads the stream.  FlatIn: the whole stream in one buffer.
struct FlatIn {
  const uint8_t* in;
  __device__ __forceinline__ void ensure(uint32_t, uint32_t) {}
  __device__ __forceinline__ uint32_t byte(uint32_t q) const { return in[q]; }
  __device__ __forceinline__ const uint8_t* src(uint32_t q, uint32_t) const { return in + q; }
};

// RingIn: a kSnappyWindow-byte LDS window over the stream, refilled by the whole wave with aligned
// 16-byte loads when the parse nears its end; literals that reach past it are copied from global
// memory directly.  Keeps the LDS per block to the decoded block + the window (two waves per CU at
// 64 KiB blocks instead of one with the whole stream staged).
constexpr uint32_t kSnappyWindow = 8192;
struct RingIn {
  const uint8_t* g;       // the stream in global memory
  int64_t readable;       // bytes readable from g (to the end of the log buffer)
  uint32_t n;             // stream bytes
  uint8_t* win;           // kSnappyWindow + 16 bytes of LDS
  int64_t a;              // stream offset of win[0] (16-byte aligned in global memory; may be < 0)
  int64_t wend;           // stream offset past the window's valid bytes
  uint32_t lane;
  __device__ __forceinline__ void refill(uint32_t p) {
    a = (int64_t)p - (int64_t)(((uintptr_t)(g + p)) & 15);
#pragma unroll 4
    for (uint32_t w = lane; w < kSnappyWindow / 16; w += 64) {
      const int64_t q = a + 16 * (int64_t)w;
      if (q + 16 <= readable) {
        *(uint4*)(win + 16 * w) = *(const uint4*)(g + q);
      } else {
        for (int i = 0; i < 16 && q + i < readable; i++) win[16 * w + i] = g[q + i];
      }
    }
    wend = min<int64_t>(a + kSnappyWindow, (int64_t)n);
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ void ensure(uint32_t p, uint32_t need) {
    if ((int64_t)p + need > wend && wend < (int64_t)n) refill(p);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t q) const { return win[(int64_t)q - a]; }
  __device__ __forceinline__ const uint8_t* src(uint32_t q, uint32_t len) const {
    return (int64_t)q + len <= wend ? win + ((int64_t)q - a) : g + q;
  }
};

// Snappy raw format: varint uncompressed length, then literal (tag 00), copy-1 (01), copy-2 (10) and
// copy-4 (11) elements.  Lanes [lane, nlanes) share each element's copy; every lane parses the same
// tags (uniform control flow).  A match copies out[o + k] = out[o - off + k % off]: only bytes before
// o are read, so overlapping matches need no ordering between the lanes.  Returns kWalkBadStream on a
// malformed stream.
// kGlobal: `out` is global memory (k_snappy_gw): a match reads what the wave stored, so its source
// must be complete first -- the wave waits for its stores when the source reaches past `safe`, the
// output offset below which every store is known complete.
template <bool kSync, class In, bool kGlobal = false>
__device__ __forceinline__ uint32_t snappy_decode(In& in, uint32_t n, uint32_t p, uint8_t* out, uint32_t ulen,
                                                  uint32_t lane, uint32_t nlanes) {
  uint32_t o = 0;
  uint32_t safe = 0;
  while (p < n) {
    // the tag and the four bytes after it in one round trip
    in.ensure(p, 5);
    // uniform across the wave: held in scalar registers, so the element's control flow is scalar
    const uint32_t t = __builtin_amdgcn_readfirstlane(in.byte(p));
    const uint32_t e0 = __builtin_amdgcn_readfirstlane(p + 1 < n ? in.byte(p + 1) : 0u);
    const uint32_t e1 = __builtin_amdgcn_readfirstlane(p + 2 < n ? in.byte(p + 2) : 0u);
    const uint32_t e2 = __builtin_amdgcn_readfirstlane(p + 3 < n ? in.byte(p + 3) : 0u);
    const uint32_t e3 = __builtin_amdgcn_readfirstlane(p + 4 < n ? in.byte(p + 4) : 0u);
    p++;
    uint32_t len, off = 0;
    if ((t & 3u) == 0) {
      len = (t >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = len - 60;
        if (p + nb > n) return kWalkBadStream;
        const uint32_t w = e0 | (e1 << 8) | (e2 << 16) | (e3 << 24);
        const uint64_t lm1 = nb == 4 ? (uint64_t)w : (uint64_t)(w & ((1u << (8 * nb)) - 1u));
        if (lm1 + 1 > (uint64_t)(n - p - nb)) return kWalkBadStream;
        len = (uint32_t)lm1 + 1;
        p += nb;
      }
      if (len > n - p || len > ulen - o) return kWalkBadStream;
      copy_bytes(out + o, in.src(p, len), len, lane, nlanes);
      p += len;
    } else {
      if ((t & 3u) == 1) {
        if (p + 1 > n) return kWalkBadStream;
        len = ((t >> 2) & 7u) + 4;
        off = ((t >> 5) << 8) | e0;
        p += 1;
      } else if ((t & 3u) == 2) {
        if (p + 2 > n) return kWalkBadStream;
        len = (t >> 2) + 1;
        off = e0 | (e1 << 8);
        p += 2;
      } else {
        if (p + 4 > n) return kWalkBadStream;
        len = (t >> 2) + 1;
        off = e0 | (e1 << 8) | (e2 << 16) | (e3 << 24);
        p += 4;
      }
      if (off == 0 || off > o || len > ulen - o) return kWalkBadStream;
      if (kGlobal && o - off + min(off, len) > safe) {
        __builtin_amdgcn_s_waitcnt(0);
        safe = o;
      }
      if (off >= len) copy_bytes<kGlobal>(out + o, out + o - off, len, lane, nlanes);
      else
        for (uint32_t k = lane; k < len; k += nlanes) out[o + k] = ld_byte<kGlobal>(out + o - off + k % off);
    }
    o += len;
    if (kSync) __builtin_amdgcn_wave_barrier();  // one-wave workgroup: LDS ops run in order
  }
  return o == ulen ? 0u : kWalkBadStream;
}

// The block's records, assuming it starts at a record (SparkeyLogIterator.java:86-138): their offsets
// go to rec_off, and the last record's bytes past the block end to overflow.  The first four header
// bytes are read together; one-byte VLQs (the common case) decode from them without another trip.
__device__ __forceinline__ void walk_block(const SnappyParams& S, uint64_t b, const uint8_t* buf, int64_t ulen) {
  auto at = [&](int64_t i) -> uint32_t { return buf[i]; };
  uint32_t j = 0, flags = 0;
  int64_t u = 0;
  uint32_t* offs = S.rec_off + b * S.mepb;
  while (u < ulen) {
    if (j < S.mepb) offs[j] = (uint32_t)u;
    else flags |= kWalkTooMany;
    j++;
    const uint32_t b0 = buf[u], b1 = u + 1 < ulen ? buf[u + 1] : 0x80u;
    if (b0 < 0x80u && b1 < 0x80u) {  // VLQ(first) VLQ(second), one byte each
      u += 2 + (b0 == 0 ? b1 : (b0 - 1) + b1);
      continue;
    }
    const RecHdr h = decode_header(at, u, ulen);
    if (h.rc == kEndOfLog) {  // (not a record: the host accepts this only in the last block)
      flags |= kWalkEofFirst;
      j--;
      u = ulen;
      break;
    }
    if (h.rc || h.klen < 0 || h.vlen < 0) {
      flags |= kWalkBadHeader;
      break;
    }
    u = record_end(h, u);
  }
  SnappyWalk w;
  w.count = j;
  w.flags = flags;
  w.overflow = u - ulen;
  S.walk[b] = w;
}

// The 16 bytes from p as two little-endian words, from one pair of aligned 16-byte loads (one memory
// round trip per hop of the block chain); byte loads near the end of the buffer.
struct Window {
  uint64_t lo, hi;
  __device__ __forceinline__ uint32_t at(int j) const {
    return (uint32_t)((j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8))) & 0xffu);
  }
};

__device__ __forceinline__ Window load_window(const uint8_t* log, int64_t p, int64_t len) {
  Window w;
  const int64_t a = p & ~15LL;
  if (a + 32 <= len) {
    const uint4 v0 = *(const uint4*)(log + a);
    const uint4 v1 = *(const uint4*)(log + a + 16);
    const uint64_t q0 = v0.x | ((uint64_t)v0.y << 32), q1 = v0.z | ((uint64_t)v0.w << 32);
    const uint64_t q2 = v1.x | ((uint64_t)v1.y << 32), q3 = v1.z | ((uint64_t)v1.w << 32);
    const int o = (int)(p - a);
    const uint64_t s0 = o >= 8 ? q1 : q0, s1 = o >= 8 ? q2 : q1, s2 = o >= 8 ? q3 : q2;
    const int sh = 8 * (o & 7);
    w.lo = sh ? (s0 >> sh) | (s1 << (64 - sh)) : s0;
    w.hi = sh ? (s1 >> sh) | (s2 << (64 - sh)) : s1;
  } else {
    w.lo = w.hi = 0;
    for (int j = 0; j < 16 && p + j < len; j++) {
      if (j < 8) w.lo |= (uint64_t)log[p + j] << (8 * j);
      else w.hi |= (uint64_t)log[p + j] << (8 * (j - 8));
    }
  }
  return w;
}

// Util.readUnsignedVLQInt over the window from byte j; bytes at >= avail are EOF.
__device__ __forceinline__ int32_t dir_vlq(const Window& w, int& j, int avail, int32_t& err) {
  uint32_t v = 0;
  for (int i = 0; i < 5; i++) {
    if (j >= avail) { err = 1; return 0; }
    const uint32_t b = w.at(j++);
    if (b < 0x80u) return (int32_t)(v | (b << (7 * i)));
    v |= (b & 0x7fu) << (7 * i);
  }
  err = 1;
  return 0;
}

}  // namespace

__global__ void __launch_bounds__(64) k_snappy_dir(SnappyParams S) {
  if (threadIdx.x != 0) return;
  const SnappyDirResult d0 = *S.dir;
  int64_t p = d0.p ? d0.p : 84;
  uint64_t nb = d0.nblk, total = d0.total;
  int32_t err = 0;
  while (p < S.data_end && nb < S.dir_limit) {
    const Window w = load_window(S.log, p, S.log_len);
    int j = 0;
    const int32_t clen = dir_vlq(w, j, (int)min<int64_t>(16, S.data_end - p), err);   // Util.readUnsignedVLQInt
    const int64_t q = p + j;
    if (err || clen < 0 || q + clen > S.data_end) { err = 1; break; }
    const int32_t ulen = dir_vlq(w, j, (int)min<int64_t>(16, q + clen - p), err);     // the Snappy preamble
    if (err || ulen < 0) { err = 1; break; }
    // the reader's buffers: maxBlockSize decompressed, Snappy.maxCompressedLength(maxBlockSize) compressed
    // (CompressedReader.java:40-49)
    if ((int64_t)ulen > S.max_block || (int64_t)clen > 32 + S.max_block + S.max_block / 6) { err = 2; break; }
    if (S.vcap >= 0 && (int64_t)(total + (uint64_t)ulen) > S.vcap) { err = 3; break; }
    {
      SnappyBlock B;
      B.file_pos = p;
      B.data = q;
      B.voff = 84 + (int64_t)total;
      B.clen = (uint32_t)clen;
      B.ulen = (uint32_t)ulen;
      S.blocks[nb] = B;
    }
    nb++;
    total += (uint64_t)ulen;
    p = q + clen;
  }
  SnappyDirResult d;
  d.nblk = nb;
  d.total = total;
  d.p = p;
  d.err = err;
  d.done = err == 0 && p >= S.data_end;
  *S.dir = d;
}

__global__ void __launch_bounds__(64) k_snappy_lds(SnappyParams S) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint64_t b = S.blk_base + blockIdx.x;
  const SnappyBlock B = S.blocks[b];
  const uint32_t lane = threadIdx.x;
  // outb: the decoded block at the alignment of its place in the virtual log (16-byte stores out);
  // then the stream window
  uint8_t* outb = lds;
  const int64_t oa = B.voff & ~15LL;
  uint8_t* out = outb + (B.voff - oa);
  RingIn in;
  in.g = S.log + B.data;
  in.readable = S.log_len - B.data;
  in.n = B.clen;
  in.win = lds + align16(S.max_block) + 16;
  in.lane = lane;
  in.refill(0);
  uint32_t p = 0;
  while (in.byte(p) & 0x80u) p++;                              // preamble (<= 5 bytes, validated by k_snappy_dir)
  p++;
  const uint32_t flags = snappy_decode<true>(in, B.clen, p, out, B.ulen, lane, 64u);
  __syncthreads();
  {
    const int64_t lo = B.voff - oa, hi = lo + B.ulen;  // the block's bytes in outb coordinates
    const int64_t nw = (hi + 15) / 16;
    for (int64_t w = lane; w < nw; w += 64) {
      if (16 * w >= lo && 16 * w + 16 <= hi) {
        *(uint4*)(S.vlog + oa + 16 * w) = *(const uint4*)(outb + 16 * w);
      } else {
        for (int64_t i = max<int64_t>(16 * w, lo); i < min<int64_t>(16 * w + 16, hi); i++) S.vlog[oa + i] = outb[i];
      }
    }
  }
  if (lane == 0) {  // the records are walked by k_snappy_walk, many blocks per wave
    SnappyWalk w;
    w.count = 0;
    w.flags = flags;
    w.overflow = 0;
    S.walk[b] = w;
  }
}

// k_snappy_gw: one wave per block, decoding straight into the virtual log.  In LDS only a window over
// the stream (refilled with aligned 16-byte loads as the parse nears its end) and a ring of the last
// kSnappyRing output bytes, from which matches copy (a longer-range match waits for the wave's stores
// and reads global memory): 12 KiB per wave instead of the whole decoded block, so many blocks decode
// at once.  Every LDS access indexes the __shared__ arrays themselves (never a pointer that may point
// to global memory as well), so the loads are ds_* and do not wait for the wave's global stores.
constexpr uint32_t kSnappyRing = 4096;
constexpr uint32_t kGwWindow = 4096;  // k_snappy_gw's stream window (8 KiB of LDS per wave with the ring)
template <int kExp>
__global__ void __launch_bounds__(64) k_snappy_gw(SnappyParams S) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kGwWindow + 16];
  __shared__ __attribute__((aligned(16))) uint8_t ring[kSnappyRing];
  constexpr uint32_t RM = kSnappyRing - 1;
  const uint64_t b = S.blk_base + blockIdx.x;
  const SnappyBlock B = S.blocks[b];
  const uint32_t lane = threadIdx.x;
  const uint8_t* g = S.log + B.data;
  const int64_t readable = S.log_len - B.data;
  const uint32_t n = B.clen, ulen = B.ulen;
  uint8_t* out = S.vlog + B.voff;
  int32_t wa = 0, wend = 0;  // the window holds stream bytes [wa, wend) (a Snappy block is < 2^31 bytes)
  auto refill = [&](uint32_t p) {
    wa = (int32_t)p - (int32_t)(((uintptr_t)(g + p)) & 15);
#pragma unroll 4
    for (uint32_t w = lane; w < kGwWindow / 16; w += 64) {
      const int64_t q = (int64_t)wa + 16 * (int64_t)w;
      if (q + 16 <= readable) {
        *(uint4*)(win + 16 * w) = *(const uint4*)(g + q);
      } else {
        for (int i = 0; i < 16 && q + i < readable; i++) win[16 * w + i] = g[q + i];
      }
    }
    wend = min(wa + (int32_t)kGwWindow, (int32_t)n);
    __builtin_amdgcn_wave_barrier();
  };
  auto byte = [&](uint32_t q) -> uint32_t { return win[(int32_t)q - wa]; };
  refill(0);
  uint32_t p = 0;
  while (byte(p) & 0x80u) p++;  // preamble (<= 5 bytes, validated by the directory)
  p++;
  uint32_t o = 0, flags = 0;
  while (p < n) {
    if ((int32_t)p + 5 > wend && wend < (int32_t)n) refill(p);
    // the tag and the four bytes after it: one aligned 8-byte LDS read (the window has 16 bytes of
    // slack; bytes at or past the stream end are not used: every use is bounds-checked against n)
    uint64_t v;
    {
      const uint32_t r = (uint32_t)((int32_t)p - wa);
      const uint32_t a4 = r & ~3u, sh = (r & 3u) * 8u;
      const uint32_t d0 = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(win + a4));
      const uint32_t d1 = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(win + a4 + 4));
      const uint32_t d2 = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(win + a4 + 8));
      const uint64_t lo = ((uint64_t)d1 << 32 | d0) >> sh;
      const uint32_t hi = sh ? (d2 << (32 - sh)) : 0u;
      v = lo | ((uint64_t)hi << 32);
    }
    // the element from its tag with selects: the bytes after the tag are a literal's length (tag
    // length field >= 60: 1-4 bytes) or a copy's offset (1, 2 or 4 bytes)
    const uint32_t t = (uint32_t)v & 0xffu, w = (uint32_t)(v >> 8);
    const uint32_t kind = t & 3u, hi6 = t >> 2;
    const uint32_t nb = kind == 0 ? (hi6 >= 60 ? hi6 - 59 : 0u) : (kind == 3 ? 4u : kind);
    const uint32_t m = nb >= 4 ? 0xffffffffu : (1u << (8 * nb)) - 1u;
    p++;
    if (p + nb > n) { flags = kWalkBadStream; break; }
    p += nb;
    uint32_t len, off = 0;
    if (kind == 0) {
      const uint64_t len64 = hi6 >= 60 ? (uint64_t)(w & m) + 1 : (uint64_t)hi6 + 1;
      if (len64 > (uint64_t)(n - p) || len64 > (uint64_t)(ulen - o)) { flags = kWalkBadStream; break; }
      len = (uint32_t)len64;
      if ((int32_t)(p + len) <= wend && len <= 128) {  // the usual literal: two lane steps, no loop
        const uint32_t r = (uint32_t)((int32_t)p - wa), k1 = lane + 64u;
        const uint8_t v0 = win[r + min(lane, len - 1u)];
        const uint8_t v1 = win[r + min(k1, len - 1u)];
        if (lane < len) {
          if (kExp != 1) out[o + lane] = v0;
          ring[(o + lane) & RM] = v0;
        }
        if (k1 < len) {
          if (kExp != 1) out[o + k1] = v1;
          ring[(o + k1) & RM] = v1;
        }
      } else if ((int64_t)p + len <= (int64_t)wend) {  // from the window
        const uint32_t r = (uint32_t)((int32_t)p - wa);
        for (uint32_t k = lane; k < len; k += 64) {
          const uint8_t x = win[r + k];
          if (kExp != 1) out[o + k] = x;
          ring[(o + k) & RM] = x;
        }
      } else {  // reaches past the window: from global memory
        for (uint32_t k = lane; k < len; k += 64) {
          const uint8_t x = g[p + k];
          out[o + k] = x;
          ring[(o + k) & RM] = x;
        }
      }
      p += len;
    } else {
      len = kind == 1 ? (hi6 & 7u) + 4 : hi6 + 1;
      off = kind == 1 ? ((t >> 5) << 8) | (w & 0xffu) : (w & m);
    if (off == 0 || off > o || len > ulen - o) { flags = kWalkBadStream; break; }
      if (off + len <= kSnappyRing && len <= 64) {  // (every Snappy copy: len <= 64) one lane step
        const uint32_t kk = min(lane, len - 1u);
        uint8_t v;
        if (off >= len) v = ring[(o - off + kk) & RM];  // (scalar branch: no modulo)
        else v = ring[(o - off + kk % off) & RM];
        __builtin_amdgcn_wave_barrier();
        if (lane < len) {
          if (kExp != 1) out[o + lane] = v;
          ring[(o + lane) & RM] = v;
        }
        __builtin_amdgcn_wave_barrier();
      } else if (off + len <= kSnappyRing) {  // out[o + k] = out[o - off + k % off]: sources < o, in the ring
        for (uint32_t k0 = 0; k0 < len; k0 += 64) {
          const uint32_t k = k0 + lane;
          uint8_t v = 0;
          if (k < len) v = ring[(o - off + (off >= len ? k : k % off)) & RM];
          __builtin_amdgcn_wave_barrier();
          if (k < len) {
            if (kExp != 1) out[o + k] = v;
            ring[(o + k) & RM] = v;
          }
          __builtin_amdgcn_wave_barrier();
        }
      } else {
        __builtin_amdgcn_s_waitcnt(0);  // the wave's own stores of the source first
        for (uint32_t k0 = 0; k0 < len; k0 += 64) {
          const uint32_t k = k0 + lane;
          uint8_t v = 0;
          if (k < len) v = *(const volatile uint8_t*)(out + o - off + (off >= len ? k : k % off));
          __builtin_amdgcn_s_waitcnt(0);
          if (k < len) {
            out[o + k] = v;
            ring[(o + k) & RM] = v;
          }
          __builtin_amdgcn_s_waitcnt(0);
        }
      }
    }
    o += len;
    __builtin_amdgcn_wave_barrier();  // one-wave workgroup: LDS ops run in order
  }
  if (!flags && o != ulen) flags = kWalkBadStream;
  if (lane == 0) {
    SnappyWalk w;
    w.count = 0;
    w.flags = flags;
    w.overflow = 0;
    S.walk[b] = w;
  }
}

__global__ void __launch_bounds__(64) k_snappy_global(SnappyParams S) {
  const uint64_t b = S.blk_base + (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= S.blk_base + S.nblk) return;
  const SnappyBlock B = S.blocks[b];
  FlatIn in{S.log + B.data};
  uint32_t p = 0;
  while (in.byte(p) & 0x80u) p++;
  p++;
  uint8_t* out = S.vlog + B.voff;
  const uint32_t flags = snappy_decode<false>(in, B.clen, p, out, B.ulen, 0u, 1u);
  SnappyWalk w;
  w.count = 0;
  w.flags = flags;
  w.overflow = 0;
  S.walk[b] = w;
}

// One lane per decoded block: its records from the virtual log (a lone wave per CU walking from LDS
// paid every load's latency in turn; here the blocks' walks overlap).
__global__ void __launch_bounds__(64) k_snappy_walk(SnappyParams S) {
  const uint64_t b = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= S.nblk || S.walk[b].flags) return;
  const SnappyBlock B = S.blocks[b];
  walk_block(S, b, S.vlog + B.voff, B.ulen);
}

// The last index i in [0, n) with pred(i) (pred true on a prefix), -1 if none: from a guess g, gallop
// away until the answer is bracketed, then bisect.
template <class Pred>
__device__ __forceinline__ int64_t gallop_last(int64_t n, int64_t g, Pred pred) {
  int64_t lo, hi;  // lo == -1 or pred(lo); hi == n or !pred(hi); lo < hi
  int64_t step = 1;
  if (pred(g)) {
    lo = g;
    hi = n;
    while (lo + step < n) {
      if (!pred(lo + step)) {
        hi = lo + step;
        break;
      }
      lo += step;
      step <<= 1;
    }
  } else {
    hi = g;
    lo = -1;
    while (hi - step >= 0) {
      if (pred(hi - step)) {
        lo = hi - step;
        break;
      }
      hi -= step;
      step <<= 1;
    }
  }
  while (hi - lo > 1) {
    const int64_t m = lo + (hi - lo) / 2;
    if (pred(m)) lo = m;
    else hi = m;
  }
  return lo;
}

__global__ void __launch_bounds__(256) k_snappy_rewrite(SnappyParams S) {
  const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (s == 0) {  // the internal build's stats: garbageSize, numEntries, maxDisplacement, hashCollisions, totalDisplacement
    const uint8_t* ih = S.itab - 112;
    uint8_t* oh = S.otab - 112;
    for (int i = 52; i < 68; i++) oh[i] = ih[i];
    for (int i = 84; i < 92; i++) oh[i] = ih[i];
    for (int i = 96; i < 112; i++) oh[i] = ih[i];
  }
  if (s >= S.cap) return;
  const uint8_t* is = S.itab + s * (uint64_t)(S.ihs + S.ias);
  uint8_t* os = S.otab + s * (uint64_t)(S.hs + S.as);
  // 16-byte slots on both sides (8-byte hash and address; tables start 112 bytes into 16-byte
  // aligned buffers): one 16-byte load and store per slot
  const bool wide = S.ihs == 8 && S.ias == 8 && S.hs == 8 && S.as == 8 && !((uintptr_t)S.otab & 15);
  uint64_t h = 0, a = 0;
  if (wide) {
    const uint4 v = *(const uint4*)is;
    h = v.x | ((uint64_t)v.y << 32);
    a = v.z | ((uint64_t)v.w << 32);
  } else {
    for (int i = 0; i < S.ihs; i++) h |= (uint64_t)is[i] << (8 * i);
    for (int i = 0; i < S.ias; i++) a |= (uint64_t)is[S.ihs + i] << (8 * i);
  }
  uint64_t fa = 0;
  if (a != 0) {
    // the block holding virtual offset a: the last block whose voff <= a.  Blocks hold about the same
    // number of bytes, so the search starts at the proportional guess and gallops from there (a few
    // dependent loads where a binary search over every block took ~15)
    const uint64_t vbody = S.vlog_len > 84 ? (uint64_t)S.vlog_len - 84 : 1;
    const int64_t nb = (int64_t)S.nblk;
    const int64_t g0 = min(nb - 1, (int64_t)((double)(a - min(a, (uint64_t)84)) / (double)vbody * (double)nb));
    const int64_t lo = max((int64_t)0, gallop_last(nb, g0, [&](int64_t b) { return (uint64_t)S.blocks[b].voff <= a; }));
    const SnappyBlock B = S.blocks[lo];
    const uint32_t rel = (uint32_t)(a - (uint64_t)B.voff);
    const uint32_t* offs = S.rec_off + lo * S.mepb;
    const uint32_t cnt = min(S.walk[lo].count, S.mepb);
    // entryIndex: the rank of rel among the block's record offsets (records of about one size: the
    // proportional guess again), the first offset >= rel
    uint32_t l = cnt;
    if (cnt) {
      const int64_t g = min((int64_t)cnt - 1, (int64_t)((double)rel / (double)max(B.ulen, 1u) * (double)cnt));
      l = (uint32_t)(gallop_last((int64_t)cnt, g, [&](int64_t i) { return offs[i] < rel; }) + 1);
    }
    if (l >= cnt || offs[l] != rel) atomicOr(S.err, 1);
    fa = ((uint64_t)B.file_pos << S.ebb) | l;
  }
  if (wide) {
    *(uint4*)os = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)fa, (uint32_t)(fa >> 32));
    return;
  }
  for (int i = 0; i < S.hs; i++) os[i] = (uint8_t)(h >> (8 * i));
  for (int i = 0; i < S.as; i++) os[S.hs + i] = (uint8_t)(fa >> (8 * i));
}

// Sharded compressed logs: one rank's blocks [0, nblk), their virtual offsets
// ascending from blocks[0].voff over S.vlog_len decoded bytes, searched as k_snappy_rewrite does.
__global__ void __launch_bounds__(256) k_cz_to_real(SnappyParams S, uint64_t* e, uint64_t n, uint32_t stride,
                                                    int32_t* err) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t* ap = e + (uint64_t)i * stride + 1;  // (the address word of a record: its second)
  const uint64_t del = *ap & (1ull << 63);       // (a DELETE record's mark stays)
  const uint64_t a = *ap & ~(1ull << 63);
  const int64_t nb = (int64_t)S.nblk;
  const uint64_t v0 = nb ? (uint64_t)S.blocks[0].voff : 0;
  const uint64_t span = S.vlog_len > 0 ? (uint64_t)S.vlog_len : 1;
  const int64_t g0 = min(nb - 1, (int64_t)((double)(a - min(a, v0)) / (double)span * (double)nb));
  const int64_t b = nb ? gallop_last(nb, max((int64_t)0, g0), [&](int64_t k) { return (uint64_t)S.blocks[k].voff <= a; }) : -1;
  if (b < 0) {
    atomicOr(err, 1);
    return;
  }
  const SnappyBlock B = S.blocks[b];
  const uint64_t rel = a - (uint64_t)B.voff;
  const uint32_t* offs = S.rec_off + (uint64_t)b * S.mepb;
  const uint32_t cnt = min(S.walk[b].count, S.mepb);
  if (rel >= B.ulen || cnt == 0) {
    atomicOr(err, 1);
    return;
  }
  const int64_t g = min((int64_t)cnt - 1, (int64_t)((double)rel / (double)max(B.ulen, 1u) * (double)cnt));
  const uint32_t l = (uint32_t)(gallop_last((int64_t)cnt, g, [&](int64_t j) { return offs[j] < (uint32_t)rel; }) + 1);
  if (l >= cnt || offs[l] != (uint32_t)rel) {
    atomicOr(err, 1);
    return;
  }
  *ap = del | ((uint64_t)B.file_pos << S.ebb) | l;
}

__global__ void __launch_bounds__(256) k_cz_to_virtual(SnappyParams S, uint64_t* addrs, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = addrs[i] & ~(1ull << 63);
  const int64_t p = (int64_t)(a >> S.ebb);
  const uint32_t idx = (uint32_t)(a & ((1ull << S.ebb) - 1));
  uint64_t v = ~0ull >> 1;
  const int64_t nb = (int64_t)S.nblk;
  if (nb) {
    const int64_t p0 = S.blocks[0].file_pos, p1 = S.blocks[nb - 1].file_pos;
    const int64_t g0 = p1 > p0 ? min(nb - 1, (int64_t)((double)(p - min(p, p0)) / (double)(p1 - p0) * (double)(nb - 1)))
                               : 0;
    const int64_t b = gallop_last(nb, max((int64_t)0, g0), [&](int64_t k) { return S.blocks[k].file_pos <= p; });
    if (b >= 0 && S.blocks[b].file_pos == p && idx < min(S.walk[b].count, S.mepb))
      v = (uint64_t)S.blocks[b].voff + S.rec_off[(uint64_t)b * S.mepb + idx];
  }
  addrs[i] = v;
}

// ------------------------------------------------------------------------------------------------
// Parallel block directory: anchors on the block chain found by speculation, the
// chain between them walked from every anchor at once, every link checked.
// ------------------------------------------------------------------------------------------------
namespace {

// One hop of the chain from p with k_snappy_dir's checks (the same errors): {next, data, clen, ulen}.
// win(p) gives the 16 bytes from p (global memory, or the screen's LDS copy).
struct DirHop {
  int64_t next, data;
  int32_t clen, ulen;
  int32_t err;  // 0, 1 bad framing, 2 larger than the reader's buffers
};

template <class Win>
__device__ __forceinline__ DirHop dir_hop(const SnappyParams& S, int64_t p, const Win& win) {
  DirHop h{0, 0, 0, 0, 0};
  const Window w = win(p);
  int j = 0;
  int32_t err = 0;
  const int32_t clen = dir_vlq(w, j, (int)min<int64_t>(16, S.data_end - p), err);
  const int64_t q = p + j;
  if (err || clen < 0 || q + clen > S.data_end) { h.err = 1; return h; }
  const int32_t ulen = dir_vlq(w, j, (int)min<int64_t>(16, q + clen - p), err);
  if (err || ulen < 0) { h.err = 1; return h; }
  if ((int64_t)ulen > S.max_block || (int64_t)clen > 32 + S.max_block + S.max_block / 6) { h.err = 2; return h; }
  h.next = q + clen;
  h.data = q;
  h.clen = clen;
  h.ulen = ulen;
  return h;
}

// A screen for speculative block starts (never needed for correctness: every link is checked): the
// header hop, then the stream's first ten elements (within 320 bytes) -- a literal first, copy
// offsets within what is already out, nothing past the decompressed size or the stream end.
template <class Win>
__device__ __forceinline__ bool snappy_head_plausible(const SnappyParams& S, const DirHop& h, const Win& win) {
  if (h.err) return false;
  int64_t pos;  // past the preamble's varint
  {
    const Window w = win(h.data);
    int j = 0;
    while (j < 5 && (w.at(j) & 0x80u)) j++;
    pos = h.data + j + 1;
  }
  const int64_t end = h.data + h.clen;
  if (h.ulen == 0) return pos == end;
  const int64_t lim = pos + 320;  // the elements checked start in the next 320 bytes
  uint32_t o = 0;
  for (int e = 0; e < 10; e++) {
    if (pos >= end) return o == (uint32_t)h.ulen;
    if (o >= (uint32_t)h.ulen) return false;  // the output is complete but the stream goes on
    if (pos >= lim) return true;
    const Window w = win(pos);
    const uint32_t t = w.at(0);
    uint32_t len, off = 0;
    if ((t & 3u) == 0) {
      len = (t >> 2) + 1;
      int64_t q = pos + 1;
      if (len > 60) {
        const uint32_t nb = len - 60;
        uint32_t v = 0;
        for (uint32_t k = 0; k < nb; k++) v |= w.at(1 + (int)k) << (8 * k);
        len = v + 1;
        q += nb;
      }
      if (len == 0 || (uint64_t)len > (uint64_t)(h.ulen - o) || q + len > end) return false;
      pos = q + len;
    } else {
      if ((t & 3u) == 1) {
        len = ((t >> 2) & 7u) + 4;
        off = ((t >> 5) << 8) | w.at(1);
        pos += 2;
      } else if ((t & 3u) == 2) {
        len = (t >> 2) + 1;
        off = w.at(1) | (w.at(2) << 8);
        pos += 3;
      } else {
        len = (t >> 2) + 1;
        off = w.at(1) | (w.at(2) << 8) | (w.at(3) << 16) | (w.at(4) << 24);
        pos += 5;
      }
      if (off == 0 || off > o || len > (uint32_t)h.ulen - o || pos > end) return false;
    }
    o += len;
  }
  return true;
}

// One hop of a ZSTD log's chain with k_zstd_dir's checks (its error codes: 1 framing, 2 larger than
// the reader's buffers, 4 no content size): VLQ(compressedSize), then the frame header's magic,
// descriptor, [window], [dictionary id] and Frame_Content_Size (RFC 8878 §3.1.1.1).
template <class Win>
__device__ __forceinline__ DirHop zstd_hop(const SnappyParams& S, int64_t p, const Win& win) {
  DirHop h{0, 0, 0, 0, 0};
  const Window w0 = win(p), w1 = win(p + 16);
  auto at = [&](int j) -> uint32_t { return j < 16 ? w0.at(j) : w1.at(j - 16); };
  const int avail = (int)min<int64_t>(32, S.data_end - p);
  uint32_t v = 0;
  int j = 0;
  int32_t clen = -1;
  for (int i = 0; i < 5; i++) {
    if (j >= avail) { h.err = 1; return h; }
    const uint32_t b = at(j++);
    if (b < 0x80u) { clen = (int32_t)(v | (b << (7 * i))); break; }
    v |= (b & 0x7fu) << (7 * i);
  }
  const int64_t q = p + j;
  if (clen < 0 || q + clen > S.data_end || clen < 6) { h.err = 1; return h; }
  const uint32_t magic = at(j) | (at(j + 1) << 8) | (at(j + 2) << 16) | (at(j + 3) << 24);
  if (magic != 0xFD2FB528u) { h.err = 1; return h; }
  const uint32_t fhd = at(j + 4);
  const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did_flag = fhd & 3;
  const uint32_t did_bytes = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
  const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
  const int f = j + 5 + (single ? 0 : 1) + (int)did_bytes;
  if (fcs_bytes == 0) { h.err = 4; return h; }
  if ((int64_t)p + f + fcs_bytes > q + clen) { h.err = 1; return h; }
  uint64_t fcs = 0;
  for (uint32_t i = 0; i < fcs_bytes; i++) fcs |= (uint64_t)at(f + (int)i) << (8 * i);
  if (fcs_bytes == 2) fcs += 256;
  const int64_t mb = S.max_block;
  const int64_t bound = mb + (mb >> 8) + (mb < (128 << 10) ? (((128 << 10) - mb) >> 11) : 0);
  if ((int64_t)fcs > S.max_block || (int64_t)clen > bound) { h.err = 2; return h; }
  h.next = q + clen;
  h.data = q;
  h.clen = clen;
  h.ulen = (int32_t)fcs;
  return h;
}

// the codec's hop (kCodec 0 SNAPPY, 1 ZSTD) and its screen
template <int kCodec, class Win>
__device__ __forceinline__ DirHop codec_hop(const SnappyParams& S, int64_t p, const Win& win) {
  return kCodec == 1 ? zstd_hop(S, p, win) : dir_hop(S, p, win);
}
template <int kCodec, class Win>
__device__ __forceinline__ bool codec_plausible(const SnappyParams& S, const DirHop& h, const Win& win) {
  return kCodec == 1 ? h.err == 0 : snappy_head_plausible(S, h, win);  // (the ZSTD magic is the screen)
}

// a start that passes the screen, and whose next block (if any) passes it too
template <int kCodec, class Win>
__device__ __forceinline__ bool block_start_plausible(const SnappyParams& S, int64_t p, const Win& win, DirHop& h) {
  h = codec_hop<kCodec>(S, p, win);
  if (!codec_plausible<kCodec>(S, h, win)) return false;
  if (h.next >= S.data_end) return true;
  const DirHop h2 = codec_hop<kCodec>(S, h.next, win);
  return codec_plausible<kCodec>(S, h2, win);
}

struct GlobalWin {
  const SnappyParams* S;
  __device__ __forceinline__ Window operator()(int64_t p) const { return load_window(S->log, p, S->log_len); }
};

// the screen's window: the staged bytes [base, base + n) from LDS (aligned dwords, funnel-shifted),
// anything else from global memory
struct StagedWin {
  const SnappyParams* S;
  const uint32_t* lds;  // base is 16-byte aligned
  int64_t base, n;
  __device__ __forceinline__ Window operator()(int64_t p) const {
    const int64_t r = p - base;
    if (r < 0 || r + 24 > n) return load_window(S->log, p, S->log_len);
    const uint32_t i = (uint32_t)(r >> 2), sh = (uint32_t)(r & 3) * 8u;
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = lds[i + k];
    const uint64_t q0 = d[0] | ((uint64_t)d[1] << 32), q1 = d[2] | ((uint64_t)d[3] << 32);
    const uint64_t q2 = d[4];
    Window w;
    w.lo = sh ? (q0 >> sh) | (q1 << (64 - sh)) : q0;
    w.hi = sh ? (q1 >> sh) | (q2 << (64 - sh)) : q1;
    return w;
  }
};

constexpr int kDirCand = kSdirCand;  // candidate starts per window

}  // namespace

// Window k = [w + k A, w + k A + H) (w = S.win0: 84, or a rank's range start), H = the longest hop
// (so it holds a true start unless it runs past dataEnd): its plausible starts whose next block is
// plausible too, into cand[k].  The window's bytes (and 384 past it, for the screen's look-ahead) are
// staged in LDS first.
template <int kCodec>
__global__ __launch_bounds__(1024) void k_sdir_screen(SnappyParams S, int64_t A, int64_t H, int64_t* cand,
                                                     int32_t* ncand) {
  extern __shared__ __attribute__((aligned(16))) uint32_t stage[];
  __shared__ int32_t n;
  const uint64_t k = blockIdx.x;
  if (threadIdx.x == 0) n = 0;
  const int64_t w0 = S.win0 + (int64_t)k * A;
  const int64_t w1 = min(w0 + H, S.data_end);
  const int64_t base = w0 & ~15LL;
  const int64_t nst = min<int64_t>(((w1 - base + 384 + 15) & ~15LL), ((S.log_len - base) & ~15LL));
  for (int64_t v = threadIdx.x; v < nst / 16; v += blockDim.x)
    reinterpret_cast<uint4*>(stage)[v] = *reinterpret_cast<const uint4*>(S.log + base + 16 * v);
  __syncthreads();
  const StagedWin win{&S, stage, base, nst};
  for (int64_t p = w0 + threadIdx.x; p < w1; p += blockDim.x) {
    DirHop h;
    if (!block_start_plausible<kCodec>(S, p, win, h)) continue;
    const int32_t i = atomicAdd(&n, 1);
    if (i < kDirCand) cand[k * kDirCand + i] = p;
  }
  __syncthreads();
  if (threadIdx.x == 0) ncand[k] = n;
}

// Window k's anchor: the first chain position at or past its end that every candidate chain reaching
// that far (plausible at every hop) agrees on -- the window's true start is a candidate when the
// stream is well formed -- else -1.
template <int kCodec>
__global__ __launch_bounds__(64) void k_sdir_anchor(SnappyParams S, int64_t A, int64_t H, const int64_t* cand,
                                                    const int32_t* ncand, int64_t* anchor) {
  const uint64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t wend = S.win0 + (int64_t)k * A + H;
  const int32_t nc = ncand[k];
  const GlobalWin win{&S};
  int64_t x = -1;
  if (nc <= kDirCand && lane < nc) {
    int64_t p = cand[k * kDirCand + lane];
    while (p < wend && p < S.data_end) {
      DirHop h;
      if (!block_start_plausible<kCodec>(S, p, win, h)) { p = -1; break; }
      p = h.next;
    }
    x = p;
  }
  const unsigned long long alive = __ballot(x >= 0);
  int64_t first = -1;
  if (alive) first = __shfl(x, __ffsll(alive) - 1, 64);
  const bool agree = !__any(x >= 0 && x != first);
  if (lane == 0) anchor[k] = (alive && agree && nc <= kDirCand) ? first : -1;
}

// Link i: the chain from ends[i] to ends[i + 1], every hop with k_snappy_dir's checks.  emit = 0:
// its blocks and decompressed bytes (cnt, usum); emit = 1: its blocks into S.blocks from boff[i],
// virtual offsets from 84 + uoff[i].  fail[0] |= 1 when a link does not land on its end.
template <int kCodec>
__global__ __launch_bounds__(64) void k_sdir_link(SnappyParams S, const int64_t* ends, uint64_t nlinks, int emit,
                                                  uint64_t* cnt, uint64_t* usum, const uint64_t* boff,
                                                  const uint64_t* uoff, int32_t* fail) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= nlinks) return;
  int64_t p = ends[i];
  const int64_t e = ends[i + 1];
  uint64_t nb = 0, us = 0;
  uint64_t bi = emit ? boff[i] : 0;
  const uint64_t v0 = emit ? uoff[i] : 0;
  const GlobalWin win{&S};
  while (p < e) {
    const DirHop h = codec_hop<kCodec>(S, p, win);
    if (h.err) {
      atomicOr(fail, 1 << h.err);
      return;
    }
    if (emit) {
      if (bi >= S.blk_cap) {
        atomicOr(fail, 8);
        return;
      }
      SnappyBlock B;
      B.file_pos = p;
      B.data = h.data;
      B.voff = 84 + (int64_t)(v0 + us);
      B.clen = (uint32_t)h.clen;
      B.ulen = (uint32_t)h.ulen;
      S.blocks[bi++] = B;
    }
    nb++;
    us += (uint64_t)h.ulen;
    p = h.next;
  }
  if (p != e) atomicOr(fail, 1);
  if (!emit) {
    cnt[i] = nb;
    usum[i] = us;
  }
}

void launch_sdir_screen(const SnappyParams& S, hipStream_t s, int codec, int64_t A, int64_t H, uint64_t nwin,
                        int64_t* cand, int32_t* ncand) {
  const size_t lds = sdir_screen_lds(H);
  if (!nwin) return;
  if (codec == 1) {
    (void)hipFuncSetAttribute((const void*)k_sdir_screen<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_sdir_screen<1>, dim3((unsigned)nwin), 1024, lds, s, S, A, H, cand, ncand);
  } else {
    (void)hipFuncSetAttribute((const void*)k_sdir_screen<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_sdir_screen<0>, dim3((unsigned)nwin), 1024, lds, s, S, A, H, cand, ncand);
  }
}

void launch_sdir_anchor(const SnappyParams& S, hipStream_t s, int codec, int64_t A, int64_t H, uint64_t nwin,
                        const int64_t* cand, const int32_t* ncand, int64_t* anchor) {
  if (!nwin) return;
  if (codec == 1) hipLaunchKernelGGL(k_sdir_anchor<1>, dim3((unsigned)nwin), 64, 0, s, S, A, H, cand, ncand, anchor);
  else hipLaunchKernelGGL(k_sdir_anchor<0>, dim3((unsigned)nwin), 64, 0, s, S, A, H, cand, ncand, anchor);
}

void launch_sdir_link(const SnappyParams& S, hipStream_t s, int codec, const int64_t* ends, uint64_t nlinks, int emit,
                      uint64_t* cnt, uint64_t* usum, const uint64_t* boff, const uint64_t* uoff, int32_t* fail) {
  if (!nlinks) return;
  const dim3 g((unsigned)((nlinks + 63) / 64));
  if (codec == 1) hipLaunchKernelGGL(k_sdir_link<1>, g, 64, 0, s, S, ends, nlinks, emit, cnt, usum, boff, uoff, fail);
  else hipLaunchKernelGGL(k_sdir_link<0>, g, 64, 0, s, S, ends, nlinks, emit, cnt, usum, boff, uoff, fail);
}

void launch_snappy_dir(const SnappyParams& S, hipStream_t s) { hipLaunchKernelGGL(k_snappy_dir, 1, 64, 0, s, S); }

void launch_cz_to_real(const SnappyParams& S, hipStream_t s, uint64_t* records, uint64_t n, uint32_t stride_words,
                       int32_t* err) {
  if (n) hipLaunchKernelGGL(k_cz_to_real, dim3((unsigned)((n + 255) / 256)), 256, 0, s, S, records, n, stride_words, err);
}
void launch_cz_to_virtual(const SnappyParams& S, hipStream_t s, uint64_t* addrs, uint64_t n) {
  if (n) hipLaunchKernelGGL(k_cz_to_virtual, dim3((unsigned)((n + 255) / 256)), 256, 0, s, S, addrs, n);
}

hipError_t launch_snappy_decode(const SnappyParams& S, hipStream_t s) {
  if (S.nblk == 0) return hipSuccess;
  const bool gw = !knob_on(Knob::SnappyLds);  // (A/B: the decoded block in LDS)
  if (gw) {
    hipLaunchKernelGGL(k_snappy_gw<0>, dim3((uint32_t)S.nblk), 64, 0, s, S);
  } else if (S.lds_bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_snappy_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)S.lds_bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_snappy_lds, dim3((uint32_t)S.nblk), 64, S.lds_bytes, s, S);
  } else {
    hipLaunchKernelGGL(k_snappy_global, dim3((uint32_t)((S.nblk + 63) / 64)), 64, 0, s, S);
  }
  return hipGetLastError();
}

void launch_snappy_walk(const SnappyParams& S, hipStream_t s) {
  if (S.nblk) hipLaunchKernelGGL(k_snappy_walk, dim3((uint32_t)((S.nblk + 63) / 64)), 64, 0, s, S);
}

void launch_snappy_rewrite(const SnappyParams& S, hipStream_t s) {
  hipLaunchKernelGGL(k_snappy_rewrite, dim3((uint32_t)((S.cap + 255) / 256)), 256, 0, s, S);
}

}  // namespace sk
