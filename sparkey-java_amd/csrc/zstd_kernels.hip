// zstd_kernels.hip -- ZSTD log front end.
//
// A ZSTD log has the layout of a SNAPPY one (snappy.hpp): 84 header bytes, then blocks
// VLQ(compressedSize) || one Zstandard frame of the block's bytes (CompressedOutputStream.flush,
// CompressedOutputStream.java:47-58; the frame from zstd-jni's Zstd.compressByteArray at level 3,
// CompressorType.java:42-56).  These kernels are the ZSTD halves of the SNAPPY front end: the block
// directory (k_zstd_dir: each block's decompressed size from its frame header's Frame_Content_Size)
// and the decode into the virtual log (k_zstd_decode); the record walk, the build over the virtual
// log and the address rewrite are SNAPPY's.
//
// The decoder follows RFC 8878 (Zstandard compression, the format libzstd and so zstd-jni write):
// frames of Raw, RLE and Compressed blocks; literals Raw, RLE, Huffman-coded in 1 or 4 streams (tree
// described directly or by FSE-coded weights) or Treeless; sequences with predefined, RLE, FSE-coded
// or repeated tables; repeat offsets.  One wave decodes one frame: every lane runs the (serial)
// entropy decoding on the same bytes, so control flow stays uniform, and the lanes share the wide
// work -- table fills, the four Huffman streams, and the literal and match copies (64 bytes per
// step; a match whose offset is shorter than the step repeats its period).  Tables live in LDS.
// Literals are Huffman-decoded into the tail of the frame's own output range (the output never
// overtakes them: a block writes at least its literals past its start).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "snappy.hpp"

namespace sk {

namespace {

constexpr uint32_t kZstdMagic = 0xFD2FB528u;
constexpr int kHufMaxBits = 12;  // HUF_TABLELOG_MAX

// literal length / match length codes: baseline and extra bits (RFC 8878 §3.1.1.3.2.1.1)
__constant__ uint32_t kLLBase[36] = {0,  1,  2,   3,   4,   5,    6,    7,    8,    9,     10,    11,
                                     12, 13, 14,  15,  16,  18,   20,   22,   24,   28,    32,    40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,  14,   15,   16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29,  30,  31,  32,   33,   34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (RFC 8878 §3.1.1.3.2.2)
__constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

struct FseE {      // decoding table entry: symbol, bits to read, base of the next state
  uint16_t base;
  uint8_t sym;
  uint8_t nb;
};

// One wave's LDS workspace (per frame).
struct ZWork {
  FseE ll[512];
  FseE ml[512];
  FseE of[256];
  FseE hw[64];              // Huffman weights' FSE table (accuracy <= 6)
  uint16_t huf[1 << kHufMaxBits];  // Huffman decoding table: symbol << 8 | code bits
  int16_t norm[64];
  uint16_t next[64];
  uint8_t w[256];           // Huffman weights
  uint32_t rank[kHufMaxBits + 2];
  // literal / match length codes: baseline | extra bits << 24 (the __constant__ tables, copied here:
  // a constant-memory load indexed by a decoded symbol is a vector memory load, which waits for the
  // wave's outstanding global stores and sat on every sequence's dependent path)
  uint32_t llc[36];
  uint32_t mlc[53];
};

enum : int32_t { kZOk = 0, kZCorrupt = -1, kZUnsupported = -2 };

// bytes from global memory (a frame's bytes; uniform addresses: one load serves the wave)
struct ZIn {
  const uint8_t* p;
  uint32_t n;
  __device__ __forceinline__ uint32_t b(uint32_t i) const { return i < n ? p[i] : 0u; }
  __device__ __forceinline__ uint32_t le16(uint32_t i) const { return b(i) | (b(i + 1) << 8); }
  __device__ __forceinline__ uint32_t le24(uint32_t i) const { return le16(i) | (b(i + 2) << 16); }
  __device__ __forceinline__ uint32_t le32(uint32_t i) const { return le24(i) | (b(i + 3) << 24); }
};

// Backward bit reader over [lo, lo + len) of `in` (RFC 8878 §4.1: the last byte holds the end mark;
// fields are read from the end).  `pos` = unread bits; reading below 0 yields zeros (an overflow
// the callers check where the format requires).  A 64-bit container holds the bits just below the
// position, refilled 7 bytes at a time.
struct RevBits {
  const ZIn* in;
  uint32_t lo;
  int32_t pos;
  uint64_t cont;   // stream bits [cbit, cbit + 56)
  int32_t cbit;
  __device__ __forceinline__ void refill() {
    int32_t s = pos - 56;
    if (s < 0) s = 0;
    const uint32_t byte = (uint32_t)s >> 3;
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) v |= (uint64_t)in->b(lo + byte + i) << (8 * i);
    cont = v;
    cbit = (int32_t)(byte * 8);
  }
  __device__ bool init(const ZIn& src, uint32_t start, uint32_t len) {
    in = &src;
    lo = start;
    if (len == 0) return false;
    const uint32_t last = src.b(start + len - 1);
    if (last == 0) return false;
    pos = (int32_t)((len - 1) * 8 + (31 - __builtin_clz(last)));
    refill();
    return true;
  }
  // the n (<= 25) bits just below bit `at` (bit i of the stream = bit i % 8 of byte i / 8); below
  // the stream start, zeros
  __device__ __forceinline__ uint32_t bits_at(int32_t at, int n) {
    if (n == 0) return 0u;
    int32_t s = at - n;
    uint32_t pad = 0;
    if (s < 0) {
      pad = (uint32_t)(-s);
      s = 0;
      n -= (int)pad;
      if (n <= 0) return 0u;
    }
    if (s < cbit || s + n > cbit + 64) {
      const int32_t keep = pos;
      pos = s + n;
      refill();
      pos = keep;
    }
    const uint32_t x = (uint32_t)((cont >> (s - cbit)) & ((1ull << n) - 1ull));
    return x << pad;
  }
  __device__ __forceinline__ uint32_t read(int n) {
    const uint32_t x = bits_at(pos, n);
    pos -= n;
    return x;
  }
  __device__ __forceinline__ uint32_t peek(int n) { return bits_at(pos, n); }
};

// FSE table description (RFC 8878 §4.1.1) at `at` of `in`: normalized counts into W.norm; returns
// the bytes read (0: corrupt), the accuracy log and the largest symbol.
__device__ uint32_t read_ncount(const ZIn& in, uint32_t at, uint32_t avail, int max_log, int max_sym, int16_t* norm,
                                int& acc_log, int& nsym) {
  uint32_t bitpos = 0;  // forward bits from `at`
  auto bits = [&](int n) -> uint32_t {
    const uint32_t byte = at + (bitpos >> 3);
    const uint64_t v = (uint64_t)in.b(byte) | ((uint64_t)in.b(byte + 1) << 8) | ((uint64_t)in.b(byte + 2) << 16) |
                       ((uint64_t)in.b(byte + 3) << 24);
    return (uint32_t)((v >> (bitpos & 7)) & ((1ull << n) - 1ull));
  };
  acc_log = (int)bits(4) + 5;
  bitpos += 4;
  if (acc_log > max_log) return 0;
  int32_t remaining = (1 << acc_log) + 1;
  int32_t threshold = 1 << acc_log;
  int nb = acc_log + 1;
  int sym = 0;
  bool prev0 = false;
  while (remaining > 1 && sym <= max_sym) {
    if (prev0) {  // repeat flags: 2 bits each, 3 = three more zeros and another flag
      int n0 = sym;
      for (;;) {
        const uint32_t r = bits(2);
        bitpos += 2;
        n0 += (int)r;
        if (r != 3) break;
      }
      if (n0 > max_sym + 1) return 0;
      while (sym < n0) norm[sym++] = 0;
      if (sym > max_sym) break;
    }
    const int32_t mx = (2 * threshold - 1) - remaining;
    const uint32_t v = bits(nb);
    int32_t count;
    if ((int32_t)(v & (uint32_t)(threshold - 1)) < mx) {
      count = (int32_t)(v & (uint32_t)(threshold - 1));
      bitpos += (uint32_t)(nb - 1);
    } else {
      count = (int32_t)(v & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= mx;
      bitpos += (uint32_t)nb;
    }
    count--;  // -1: "less than 1"
    remaining -= count < 0 ? -count : count;
    norm[sym++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      nb--;
      threshold >>= 1;
    }
    if ((bitpos >> 3) > avail) return 0;
  }
  if (remaining != 1 || sym == 0) return 0;
  nsym = sym;
  const uint32_t used = (bitpos + 7) >> 3;
  return used <= avail ? used : 0;
}

// FSE decoding table from normalized counts (RFC 8878 §4.1.1): the symbol spread (lane 0), then
// every state's bits and base (lanes).  `tab` must hold 1 << acc_log entries.
__device__ bool build_fse(ZWork& W, const int16_t* norm, int nsym, int acc_log, FseE* tab, int lane) {
  const int size = 1 << acc_log;
  if (lane == 0) {
    int high = size - 1;
    for (int s = 0; s < nsym; s++) {
      if (norm[s] == -1) {
        tab[high--].sym = (uint8_t)s;
        W.next[s] = 1;
      } else {
        W.next[s] = (uint16_t)max(0, (int)norm[s]);
      }
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int p = 0;
    for (int s = 0; s < nsym; s++)
      for (int i = 0; i < norm[s]; i++) {
        tab[p].sym = (uint8_t)s;
        do {
          p = (p + step) & mask;
        } while (p > high);
      }
    // (every state gets its symbol's next count in state order: serial by nature)
    for (int u = 0; u < size; u++) {
      const int s = tab[u].sym;
      const uint32_t nx = W.next[s]++;
      const int nb = acc_log - (31 - __builtin_clz(nx));
      tab[u].nb = (uint8_t)nb;
      tab[u].base = (uint16_t)((nx << nb) - (uint32_t)size);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  return true;
}

// A one-symbol (RLE mode) table: every read gives `sym`, reads no bits.
__device__ void build_rle(FseE* tab, uint32_t sym, int lane) {
  if (lane == 0) {
    tab[0].sym = (uint8_t)sym;
    tab[0].nb = 0;
    tab[0].base = 0;
  }
  __builtin_amdgcn_wave_barrier();
}

// Huffman tree description (RFC 8878 §4.2.1) at `at`: the decoding table in W.huf; returns the
// description's bytes (0: corrupt) and the table's bits.
__device__ uint32_t read_huffman(ZWork& W, const ZIn& in, uint32_t at, uint32_t avail, int& huf_bits, int lane) {
  const uint32_t hb = in.b(at);
  uint32_t used = 1, nw = 0;
  if (hb < 128) {  // FSE-coded weights, two interleaved states
    if (hb == 0 || 1 + hb > avail) return 0;
    int acc = 0, nsym = 0;
    const uint32_t d = read_ncount(in, at + 1, hb, 6, kHufMaxBits, W.norm, acc, nsym);
    if (!d) return 0;
    build_fse(W, W.norm, nsym, acc, W.hw, lane);
    RevBits br;
    if (!br.init(in, at + 1 + d, hb - d)) return 0;
    uint32_t s1 = br.read(acc), s2 = br.read(acc);
    for (;;) {  // FSE_decompress's tail: stop when a state update reads past the stream start
      if (nw >= 255) return 0;
      W.w[nw++] = W.hw[s1].sym;
      s1 = W.hw[s1].base + br.read(W.hw[s1].nb);
      if (br.pos < 0) {
        W.w[nw++] = W.hw[s2].sym;
        break;
      }
      if (nw >= 255) return 0;
      W.w[nw++] = W.hw[s2].sym;
      s2 = W.hw[s2].base + br.read(W.hw[s2].nb);
      if (br.pos < 0) {
        if (nw >= 255) return 0;
        W.w[nw++] = W.hw[s1].sym;
        break;
      }
    }
    used = 1 + hb;
  } else {  // direct 4-bit weights, two per byte, high nibble first
    nw = hb - 127;
    const uint32_t nbytes = (nw + 1) / 2;
    if (1 + nbytes > avail) return 0;
    for (uint32_t i = 0; i < nw; i++) {
      const uint32_t x = in.b(at + 1 + i / 2);
      W.w[i] = (uint8_t)((i & 1) ? (x & 15) : (x >> 4));
    }
    used = 1 + nbytes;
  }
  // the last symbol's weight completes the sum of 2^(w-1) to a power of two
  uint32_t total = 0;
  for (uint32_t i = 0; i < nw; i++) {
    if (W.w[i] > kHufMaxBits) return 0;
    if (W.w[i]) total += 1u << (W.w[i] - 1);
  }
  if (total == 0) return 0;
  const int bits = 32 - __builtin_clz(total);  // highbit(total) + 1
  if (bits > kHufMaxBits) return 0;
  const uint32_t rest = (1u << bits) - total;
  if (rest & (rest - 1)) return 0;
  W.w[nw] = (uint8_t)((31 - __builtin_clz(rest)) + 1);
  const uint32_t nsym = nw + 1;
  huf_bits = bits;
  // rank starts: weight 1 first (longest codes), symbols in order within a weight
  if (lane == 0) {
    for (int i = 0; i <= kHufMaxBits + 1; i++) W.rank[i] = 0;
    for (uint32_t i = 0; i < nsym; i++) W.rank[W.w[i]]++;
    uint32_t start = 0;
    for (int wgt = 1; wgt <= bits; wgt++) {
      const uint32_t c = W.rank[wgt];
      W.rank[wgt] = start;
      start += c << (wgt - 1);
    }
    for (uint32_t i = 0; i < nsym; i++) {
      const uint32_t wgt = W.w[i];
      if (!wgt) continue;
      const uint32_t len = 1u << (wgt - 1);
      const uint16_t e = (uint16_t)((i << 8) | (uint32_t)(bits + 1 - wgt));
      for (uint32_t u = W.rank[wgt]; u < W.rank[wgt] + len; u++) W.huf[u] = e;
      W.rank[wgt] += len;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  return used;
}

// One Huffman stream [at, at + len) decoding `cnt` literals to out[0, cnt); false when corrupt.
__device__ bool huf_stream(const ZWork& W, const ZIn& in, uint32_t at, uint32_t len, int bits, uint8_t* out,
                           uint32_t cnt) {
  RevBits br;
  if (!br.init(in, at, len)) return false;
  for (uint32_t i = 0; i < cnt; i++) {
    const uint16_t e = W.huf[br.peek(bits)];
    out[i] = (uint8_t)(e >> 8);
    br.pos -= (int32_t)(e & 0xff);
    if (br.pos < 0) return false;
  }
  return br.pos == 0;
}

// the table a mode selects (RFC 8878 §3.1.1.3.2.1): predefined, RLE, FSE-described or repeated
__device__ uint32_t seq_table(ZWork& W, const ZIn& in, uint32_t at, uint32_t avail, int mode, int max_log,
                              int max_sym, const int16_t* def, int def_n, int def_log, FseE* tab, int& log, bool& have,
                              int lane) {
  if (mode == 0) {
    for (int i = 0; i < def_n; i++) W.norm[i] = def[i];
    build_fse(W, W.norm, def_n, def_log, tab, lane);
    log = def_log;
    have = true;
    return 0;
  }
  if (mode == 1) {
    if (avail < 1) return ~0u;
    const uint32_t sym = in.b(at);
    if ((int)sym > max_sym) return ~0u;
    build_rle(tab, sym, lane);
    log = 0;
    have = true;
    return 1;
  }
  if (mode == 2) {
    int acc = 0, nsym = 0;
    const uint32_t d = read_ncount(in, at, avail, max_log, max_sym, W.norm, acc, nsym);
    if (!d) return ~0u;
    build_fse(W, W.norm, nsym, acc, tab, lane);
    log = acc;
    have = true;
    return d;
  }
  return have ? 0u : ~0u;  // repeat: the previous block's table
}

// The output and the literals decoded into it live in LDS (kLds) or, for blocks too large for it,
// in global memory, read back through L2 (volatile: no stale vector-L1 line after the wave's own
// stores).
template <bool kLds>
__device__ __forceinline__ uint8_t out_at(const uint8_t* p) {
  if (kLds) return *p;
  return *(const volatile uint8_t*)p;
}

// XXH64 (seed 0) of n decoded bytes, one lane (only checksummed frames take it; zstd-jni's default
// frames carry no checksum).  The published algorithm: 4 accumulators over 32-byte stripes, merged,
// then the 8/4/1-byte tail and the avalanche.
template <bool kLds>
__device__ uint64_t xxh64_out(const uint8_t* p, uint32_t n) {
  constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                     P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto rd64 = [&](uint32_t i) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)out_at<kLds>(p + i + k) << (8 * k);
    return v;
  };
  auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
  uint32_t i = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= n; i += 32) {
      v1 = round(v1, rd64(i));
      v2 = round(v2, rd64(i + 8));
      v3 = round(v3, rd64(i + 16));
      v4 = round(v4, rd64(i + 24));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) h = (h ^ round(0, v)) * P1 + P4;
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) h = rotl(h ^ round(0, rd64(i)), 27) * P1 + P4;
  if (i + 4 <= n) {
    uint64_t w = 0;
    for (int k = 0; k < 4; k++) w |= (uint64_t)out_at<kLds>(p + i + k) << (8 * k);
    h = rotl(h ^ (w * P1), 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; i++) h = rotl(h ^ (out_at<kLds>(p + i) * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// Copies n bytes src -> dst with the wave, 64 a step (every step's loads complete before its stores;
// a later step only reads below what earlier steps wrote, see the file comment).
template <bool kLds>
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n, int lane, bool src_out) {
  if (!kLds && !src_out) {  // from the frame (never written here): four steps' loads, then one wait
    for (uint32_t i0 = 0; i0 < n; i0 += 256) {
      uint8_t v[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t k = i0 + 64u * q + (uint32_t)lane;
        v[q] = k < n ? src[k] : (uint8_t)0;
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t k = i0 + 64u * q + (uint32_t)lane;
        if (k < n) dst[k] = v[q];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    return;
  }
  for (uint32_t i = 0; i < n; i += 64) {
    const uint32_t k = i + (uint32_t)lane;
    uint8_t v = 0;
    if (k < n) v = src_out ? out_at<kLds>(src + k) : src[k];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (k < n) dst[k] = v;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}

// match: n bytes from `off` back (off may be shorter than a step: the period repeats)
template <bool kLds>
__device__ __forceinline__ void wave_match(uint8_t* dst, uint32_t off, uint32_t n, int lane) {
  if (off >= 64) {
    for (uint32_t i = 0; i < n; i += 64) {
      const uint32_t k = i + (uint32_t)lane;
      const uint8_t v = k < n ? out_at<kLds>(dst + ((int64_t)k - off)) : 0;
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      if (k < n) dst[k] = v;
      __builtin_amdgcn_s_waitcnt(0);  // (the next step may read what this one wrote)
      __builtin_amdgcn_wave_barrier();
    }
  } else {
    for (uint32_t i = 0; i < n; i += 64) {
      const uint32_t k = i + (uint32_t)lane;
      const uint8_t v = k < n ? out_at<kLds>(dst + ((int64_t)(k % off) - off)) : 0;
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      if (k < n) dst[k] = v;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}

// One Zstandard frame (or concatenated frames) in[0, n) -> out[0, cap): the bytes written, or < 0.
template <bool kLds>
__device__ int64_t zstd_decode(ZWork& W, const ZIn& in, uint8_t* out, uint32_t cap, int lane) {
  uint32_t ip = 0, op = 0;
  int ll_log = 0, ml_log = 0, of_log = 0, huf_bits = 0;
  bool have_ll = false, have_ml = false, have_of = false, have_huf = false;
  while (ip < in.n) {
    const uint32_t magic = in.le32(ip);
    if (ip + 4 > in.n) return kZCorrupt;  // a partial frame header
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame: its size must lie inside the block
      if (ip + 8 > in.n) return kZCorrupt;
      const uint32_t skip = in.le32(ip + 4);
      if (skip > in.n - ip - 8) return kZCorrupt;
      ip += 8 + skip;
      continue;
    }
    if (magic != kZstdMagic) return kZCorrupt;
    ip += 4;
    const uint32_t fhd = in.b(ip++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 8) return kZCorrupt;  // reserved bit
    if (!single) ip++;              // Window_Descriptor
    const uint32_t did_bytes = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    uint32_t did = 0;
    for (uint32_t i = 0; i < did_bytes; i++) did |= in.b(ip + i) << (8 * i);
    if (did) return kZUnsupported;  // no dictionaries
    ip += did_bytes;
    const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fcs_bytes; i++) fcs |= (uint64_t)in.b(ip + i) << (8 * i);
    if (fcs_bytes == 2) fcs += 256;
    ip += fcs_bytes;
    const uint32_t frame_start = op;
    // literals are decoded into the tail of the frame's output (see the file comment)
    const uint32_t frame_end = fcs_bytes ? (uint32_t)min<uint64_t>((uint64_t)frame_start + fcs, cap) : cap;
    uint32_t rep[3] = {1, 4, 8};
    have_ll = have_ml = have_of = have_huf = false;
    for (;;) {
      if (ip + 3 > in.n) return kZCorrupt;
      const uint32_t bh = in.le24(ip);
      ip += 3;
      const uint32_t last = bh & 1, btype = (bh >> 1) & 3, bsize = bh >> 3;
      if (btype == 0) {  // Raw
        if (ip + bsize > in.n || op + bsize > cap) return kZCorrupt;
        wave_copy<kLds>(out + op, in.p + ip, bsize, lane, false);
        ip += bsize;
        op += bsize;
      } else if (btype == 1) {  // RLE
        if (ip + 1 > in.n || op + bsize > cap) return kZCorrupt;
        const uint8_t v = (uint8_t)in.b(ip);
        for (uint32_t i = (uint32_t)lane; i < bsize; i += 64) out[op + i] = v;
        ip += 1;
        op += bsize;
      } else if (btype == 2) {  // Compressed
        if (ip + bsize > in.n) return kZCorrupt;
        const uint32_t bend = ip + bsize;
        uint32_t p = ip;
        // ---- literals section ----
        const uint32_t h0 = in.b(p);
        const uint32_t ltype = h0 & 3, sf = (h0 >> 2) & 3;
        uint32_t regen = 0, csize = 0, hlen = 0;
        int nstreams = 1;
        if (ltype <= 1) {
          if ((sf & 1) == 0) { regen = h0 >> 3; hlen = 1; }
          else if (sf == 1) { regen = (h0 >> 4) + (in.b(p + 1) << 4); hlen = 2; }
          else { regen = (h0 >> 4) + (in.b(p + 1) << 4) + (in.b(p + 2) << 12); hlen = 3; }
        } else {
          if (sf <= 1) {
            const uint32_t h = in.le24(p);
            regen = (h >> 4) & 0x3FF;
            csize = (h >> 14) & 0x3FF;
            hlen = 3;
            nstreams = sf == 0 ? 1 : 4;
          } else if (sf == 2) {
            const uint32_t h = in.le32(p);
            regen = (h >> 4) & 0x3FFF;
            csize = (h >> 18) & 0x3FFF;
            hlen = 4;
            nstreams = 4;
          } else {
            const uint64_t h = (uint64_t)in.le32(p) | ((uint64_t)in.b(p + 4) << 32);
            regen = (uint32_t)((h >> 4) & 0x3FFFF);
            csize = (uint32_t)((h >> 22) & 0x3FFFF);
            hlen = 5;
            nstreams = 4;
          }
        }
        p += hlen;
        // where the literals are read from during the sequences
        const uint8_t* lit = nullptr;
        bool lit_out = false;  // the literals were decoded into the output (else: the input's bytes)
        bool lit_rle = false;
        uint8_t lit_v = 0;
        if (ltype == 0) {
          if (p + regen > bend) return kZCorrupt;
          lit = in.p + p;
          p += regen;
        } else if (ltype == 1) {
          if (p + 1 > bend) return kZCorrupt;
          lit_rle = true;
          lit_v = (uint8_t)in.b(p);
          p += 1;
        } else {
          if (p + csize > bend || regen > frame_end - op) return kZCorrupt;
          uint32_t q = p, qend = p + csize;
          if (ltype == 2) {
            const uint32_t d = read_huffman(W, in, q, csize, huf_bits, lane);
            if (!d) return kZCorrupt;
            q += d;
            have_huf = true;
          } else if (!have_huf) {
            return kZCorrupt;
          }
          uint8_t* lbuf = out + (frame_end - regen);
          bool ok = true;
          if (nstreams == 1) {
            ok = huf_stream(W, in, q, qend - q, huf_bits, lbuf, regen);
          } else {
            if (q + 6 > qend) return kZCorrupt;
            const uint32_t s1 = in.le16(q), s2 = in.le16(q + 2), s3 = in.le16(q + 4);
            q += 6;
            if (q + s1 + s2 + s3 > qend) return kZCorrupt;
            const uint32_t s4 = qend - q - s1 - s2 - s3;
            const uint32_t seg = (regen + 3) / 4;
            if (3 * seg > regen) return kZCorrupt;
            const uint32_t so[4] = {q, q + s1, q + s1 + s2, q + s1 + s2 + s3};
            const uint32_t sl[4] = {s1, s2, s3, s4};
            // lanes 0-3: one stream each
            bool mine = true;
            if (lane < 4) mine = huf_stream(W, in, so[lane], sl[lane], huf_bits, lbuf + lane * seg,
                                            lane < 3 ? seg : regen - 3 * seg);
            ok = __all(mine);
          }
          __builtin_amdgcn_s_waitcnt(0);
          __builtin_amdgcn_wave_barrier();
          if (!ok) return kZCorrupt;
          lit = lbuf;
          lit_out = true;
          p = qend;
        }
        // ---- sequences section ----
        uint32_t nseq = 0;
        if (p >= bend) return kZCorrupt;
        const uint32_t s0 = in.b(p);
        if (s0 < 128) { nseq = s0; p += 1; }
        else if (s0 < 255) { nseq = ((s0 - 128) << 8) + in.b(p + 1); p += 2; }
        else { nseq = in.b(p + 1) + (in.b(p + 2) << 8) + 0x7F00; p += 3; }
        uint32_t lpos = 0;  // literals consumed
        if (nseq) {
          const uint32_t modes = in.b(p++);
          if (modes & 3) return kZCorrupt;
          uint32_t d = seq_table(W, in, p, bend - p, (int)(modes >> 6), 9, 35, kLLDef, 36, 6, W.ll, ll_log, have_ll, lane);
          if (d == ~0u) return kZCorrupt;
          p += d;
          d = seq_table(W, in, p, bend - p, (int)((modes >> 4) & 3), 8, 31, kOFDef, 29, 5, W.of, of_log, have_of, lane);
          if (d == ~0u) return kZCorrupt;
          p += d;
          d = seq_table(W, in, p, bend - p, (int)((modes >> 2) & 3), 9, 52, kMLDef, 53, 6, W.ml, ml_log, have_ml, lane);
          if (d == ~0u) return kZCorrupt;
          p += d;
          RevBits br;
          if (!br.init(in, p, bend - p)) return kZCorrupt;
          uint32_t sll = br.read(ll_log), sof = br.read(of_log), sml = br.read(ml_log);
          for (uint32_t k = 0; k < nseq; k++) {
            const FseE eo = W.of[sof], em = W.ml[sml], el = W.ll[sll];
            const uint32_t ofc = eo.sym, mlc = em.sym, llc = el.sym;
            if (ofc > 31 || mlc > 52 || llc > 35) return kZCorrupt;
            uint32_t ofv = (1u << ofc) + br.read((int)ofc);
            const uint32_t mlx = W.mlc[mlc], llx = W.llc[llc];
            const uint32_t ml = (mlx & 0xFFFFFFu) + br.read((int)(mlx >> 24));
            const uint32_t ll = (llx & 0xFFFFFFu) + br.read((int)(llx >> 24));
            uint32_t off;
            if (ofv > 3) {
              off = ofv - 3;
              rep[2] = rep[1];
              rep[1] = rep[0];
              rep[0] = off;
            } else {
              const uint32_t idx = ofv - 1 + (ll == 0 ? 1u : 0u);
              if (idx == 0) {
                off = rep[0];
              } else if (idx == 1) {
                off = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
              } else if (idx == 2) {
                off = rep[2];
                rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
              } else {
                off = rep[0] - 1;
                rep[2] = rep[1];
                rep[1] = rep[0];
                rep[0] = off;
              }
            }
            if (k + 1 < nseq) {  // states: literal length, match length, offset
              sll = el.base + br.read(el.nb);
              sml = em.base + br.read(em.nb);
              sof = eo.base + br.read(eo.nb);
            }
            if (br.pos < 0) return kZCorrupt;
            // execute: ll literals, then ml bytes from off back
            if (lpos + ll > regen || op + ll + ml > frame_end || off == 0 || off > op + ll - frame_start)
              return kZCorrupt;
            if (lit_rle) {
              for (uint32_t i = (uint32_t)lane; i < ll; i += 64) out[op + i] = lit_v;
            } else {
              wave_copy<kLds>(out + op, lit + lpos, ll, lane, lit_out);
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            lpos += ll;
            op += ll;
            wave_match<kLds>(out + op, off, ml, lane);
            op += ml;
          }
          if (br.pos != 0) return kZCorrupt;
        }
        // the literals after the last sequence
        const uint32_t rest = regen - lpos;
        if (op + rest > frame_end) return kZCorrupt;
        if (lit_rle) {
          for (uint32_t i = (uint32_t)lane; i < rest; i += 64) out[op + i] = lit_v;
        } else {
          wave_copy<kLds>(out + op, lit + lpos, rest, lane, lit_out);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        op += rest;
        ip = bend;
      } else {
        return kZCorrupt;
      }
      if (last) break;
    }
    if (fcs_bytes && op - frame_start != fcs) return kZCorrupt;
    if (checksum) {  // Content_Checksum: low 32 bits of XXH64(frame output, seed 0), as libzstd checks it
      if (ip + 4 > in.n) return kZCorrupt;
      uint32_t want = 0;
      if (lane == 0) want = (uint32_t)xxh64_out<kLds>(out + frame_start, op - frame_start);
      want = (uint32_t)__shfl((int)want, 0);
      if (want != in.le32(ip)) return kZCorrupt;
      ip += 4;
    }
  }
  return (int64_t)op;
}

// Util.readUnsignedVLQInt over global bytes
__device__ __forceinline__ int32_t g_vlq(const uint8_t* log, int64_t& p, int64_t end, int32_t& err) {
  uint32_t v = 0;
  for (int i = 0; i < 5; i++) {
    if (p >= end) { err = 1; return 0; }
    const uint32_t b = log[p++];
    if (b < 0x80u) return (int32_t)(v | (b << (7 * i)));
    v |= (b & 0x7fu) << (7 * i);
  }
  err = 1;
  return 0;
}

}  // namespace

// The block chain (as k_snappy_dir): each block's decompressed size from its frame header
// (Frame_Content_Size; a frame without it is not a layout zstd-jni writes: error 4).
__global__ void __launch_bounds__(64) k_zstd_dir(SnappyParams S) {
  if (threadIdx.x != 0) return;
  const SnappyDirResult d0 = *S.dir;
  int64_t p = d0.p ? d0.p : 84;
  uint64_t nb = d0.nblk, total = d0.total;
  int32_t err = 0;
  // ZSTD_compressBound(maxBlockSize): the reader's compressed buffer (CompressorType.java:44-46)
  const int64_t mb = S.max_block;
  const int64_t bound = mb + (mb >> 8) + (mb < (128 << 10) ? (((128 << 10) - mb) >> 11) : 0);
  while (p < S.data_end && nb < S.dir_limit) {
    int64_t q = p;
    const int32_t clen = g_vlq(S.log, q, S.data_end, err);
    if (err || clen < 0 || q + clen > S.data_end) { err = 1; break; }
    // frame header: magic, descriptor, [window], [dictionary id], content size
    if (clen < 6) { err = 1; break; }
    const uint32_t magic = (uint32_t)S.log[q] | ((uint32_t)S.log[q + 1] << 8) | ((uint32_t)S.log[q + 2] << 16) |
                           ((uint32_t)S.log[q + 3] << 24);
    if (magic != kZstdMagic) { err = 1; break; }
    const uint32_t fhd = S.log[q + 4];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did_flag = fhd & 3;
    const uint32_t did_bytes = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
    int64_t f = q + 5 + (single ? 0 : 1) + did_bytes;
    if (fcs_bytes == 0) { err = 4; break; }
    if (f + fcs_bytes > q + clen) { err = 1; break; }
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fcs_bytes; i++) fcs |= (uint64_t)S.log[f + i] << (8 * i);
    if (fcs_bytes == 2) fcs += 256;
    if ((int64_t)fcs > S.max_block || (int64_t)clen > bound) { err = 2; break; }
    const uint32_t ulen = (uint32_t)fcs;
    if (S.vcap >= 0 && (int64_t)(total + (uint64_t)ulen) > S.vcap) { err = 3; break; }
    {
      SnappyBlock B;
      B.file_pos = p;
      B.data = q;
      B.voff = 84 + (int64_t)total;
      B.clen = (uint32_t)clen;
      B.ulen = ulen;
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

// One wave per block: its frame into the virtual log at voff, decoded in LDS when the block fits
// (lds_bytes > 0), then stored 16 bytes a lane; else straight into the virtual log.
// (one instantiation per mode: the global-memory decode alone needs fewer registers, so more waves)
template <bool kInLds>
__global__ void __launch_bounds__(64) k_zstd_decode(SnappyParams S) {
  __shared__ ZWork W;
  if (threadIdx.x < 36) W.llc[threadIdx.x] = kLLBase[threadIdx.x] | ((uint32_t)kLLBits[threadIdx.x] << 24);
  if (threadIdx.x < 53) W.mlc[threadIdx.x] = kMLBase[threadIdx.x] | ((uint32_t)kMLBits[threadIdx.x] << 24);
  __builtin_amdgcn_wave_barrier();
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  const uint64_t b = S.blk_base + blockIdx.x;
  const SnappyBlock B = S.blocks[b];
  const int lane = (int)threadIdx.x;
  ZIn in{S.log + B.data, B.clen};
  int64_t got;
  if (kInLds) {
    // the block at the alignment of its place in the virtual log (16-byte stores out), then its
    // frame's bytes (every bit read of the entropy decoding stays in LDS)
    const int64_t oa = B.voff & ~15LL;
    uint8_t* out = dyn + (B.voff - oa);
    uint8_t* src = dyn + ((16 + ((S.max_block + 15) & ~15LL) + 16));
    {
      const int64_t ia = B.data & ~15LL;
      const int64_t ilo = B.data - ia, ihi = ilo + B.clen;
      const int64_t niv = (ihi + 15) / 16;
      for (int64_t w = lane; w < niv; w += 64) {
        if (ia + 16 * w + 16 <= S.log_len) {
          *(uint4*)(src + 16 * w) = *(const uint4*)(S.log + ia + 16 * w);
        } else {
          for (int i = 0; i < 16; i++) src[16 * w + i] = ia + 16 * w + i < S.log_len ? S.log[ia + 16 * w + i] : 0;
        }
      }
      __syncthreads();
      in.p = src + ilo;
    }
    got = zstd_decode<true>(W, in, out, B.ulen, lane);
    __syncthreads();
    const int64_t lo = B.voff - oa, hi = lo + B.ulen;
    const int64_t nw = (hi + 15) / 16;
    for (int64_t w = lane; w < nw; w += 64) {
      if (16 * w >= lo && 16 * w + 16 <= hi) {
        *(uint4*)(S.vlog + oa + 16 * w) = *(const uint4*)(dyn + 16 * w);
      } else {
        for (int64_t i = max<int64_t>(16 * w, lo); i < min<int64_t>(16 * w + 16, hi); i++) S.vlog[oa + i] = dyn[i];
      }
    }
  } else {
    got = zstd_decode<false>(W, in, S.vlog + B.voff, B.ulen, lane);
  }
  if (lane == 0) {
    SnappyWalk w;
    w.count = 0;
    w.flags = got == (int64_t)B.ulen ? 0u : kWalkBadStream;
    w.overflow = 0;
    S.walk[b] = w;
  }
}

void launch_zstd_dir(const SnappyParams& S, hipStream_t s) { hipLaunchKernelGGL(k_zstd_dir, 1, 64, 0, s, S); }

uint32_t zstd_lds_bytes(int64_t max_block) {
  // the decoded block (+ alignment slack), then the frame: at most ZSTD_compressBound(maxBlockSize)
  // (k_zstd_dir enforces it) + alignment slack
  const int64_t mb = (max_block + 15) & ~15LL;
  const int64_t bound = max_block + (max_block >> 8) + (max_block < (128 << 10) ? (((128 << 10) - max_block) >> 11) : 0);
  const int64_t dyn = 16 + mb + 16 + ((bound + 31) & ~15LL);
  return dyn + (int64_t)sizeof(ZWork) <= 156 * 1024 ? (uint32_t)dyn : 0u;
}

hipError_t launch_zstd_decode(const SnappyParams& S, hipStream_t s) {
  if (S.nblk == 0) return hipSuccess;
  if (S.lds_bytes) {
    hipError_t e = hipFuncSetAttribute((const void*)k_zstd_decode<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)S.lds_bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_zstd_decode<true>, dim3((uint32_t)S.nblk), 64, S.lds_bytes, s, S);
  } else {
    hipLaunchKernelGGL(k_zstd_decode<false>, dim3((uint32_t)S.nblk), 64, 0, s, S);
  }
  return hipGetLastError();
}

}  // namespace sk
