// append_kernels.hip -- the step before the build: LogWriter.put / delete for
// a batch of records on the device, NONE compression (LogWriter.java:96-115,
// UncompressedBlockOutput.java:34-45, LogHeader.java:161-172).
//
//   k_app_keymax   per op: its key length when it is a PUT (else -1), for the prefix max that decides
//                  which DELETEs LogWriter.delete drops (key longer than maxKeyLen at that point)
//   k_app_sizes    per op: kept?, record size; per-workgroup header sums
//   k_app_map      the output seen as aligned 16-byte words: each word's first op
//   k_app_write    one lane per word: its 16 bytes (VLQ headers, key and value bytes), one 16-byte
//                  store
//   k_app_final    the header sums
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "append.hpp"
#include "scan.hpp"

namespace sk {

__device__ __forceinline__ int32_t app_vlq_size(uint64_t v) {  // Util.unsignedVLQSize (Util.java:86-128)
  int32_t n = 1;
  while (n < 10 && v >= (1ull << (7 * n))) n++;
  return n;
}

__global__ __launch_bounds__(256) void k_app_keymax(AppendParams A) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  A.keymax[i] = A.kind[i] ? (int64_t)(A.key_off[i + 1] - A.key_off[i]) : -1;
}

// sizes[i] (0 for a dropped DELETE) and, per workgroup, {numPuts, numDeletes, putSize, deleteSize,
// maxKeyLen, maxValueLen} of its ops
__global__ __launch_bounds__(256) void k_app_sizes(AppendParams A) {
  __shared__ int64_t red[6][4];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t np = 0, nd = 0, ps = 0, ds = 0, mk = -1, mv = -1;
  uint32_t size = 0;
  if (i < A.n) {
    const int64_t klen = (int64_t)(A.key_off[i + 1] - A.key_off[i]);
    if (A.kind[i]) {
      const int64_t vlen = (int64_t)(A.val_off[i + 1] - A.val_off[i]);
      size = (uint32_t)(app_vlq_size((uint64_t)klen + 1) + app_vlq_size((uint64_t)vlen) + klen + vlen);
      np = 1;
      ps = size;
      mk = klen;
      mv = vlen;
    } else {
      const int64_t before = max(A.max_key_len0, A.keymax_pre[i]);  // maxKeyLen when this DELETE runs
      if (klen <= before) {
        size = (uint32_t)(1 + app_vlq_size((uint64_t)klen) + klen);
        nd = 1;
        ds = size;
      }
    }
    A.sizes[i] = size;
  }
  int64_t v[6] = {np, nd, ps, ds, mk, mv};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 6; k++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t t = __shfl_xor(v[k], o, 64);
      v[k] = k < 4 ? v[k] + t : max(v[k], t);
    }
    if (lane == 0) red[k][w] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    int64_t r = red[k][0];
    for (int q = 1; q < 4; q++) r = k < 4 ? r + red[k][q] : max(r, red[k][q]);
    A.partials[(uint64_t)blockIdx.x * 6 + k] = r;
  }
}

// The output as 16-byte words aligned in memory (word w = bytes [16 w - mis, 16 w - mis + 16) of the
// appended range, mis = d_out % 16): map[w] = the op holding the word's first byte (or an earlier op).
__global__ __launch_bounds__(256) void k_app_map(AppendParams A) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  if (i == 0) A.map[0] = 0;
  const uint64_t a = A.off[i], z = a + A.sizes[i];
  if (z == a) return;
  for (uint64_t w = (a + A.mis + 15) >> 4; w <= (z - 1 + A.mis) >> 4; w++) A.map[w] = (uint32_t)i;
}

// A 16-byte aligned window over a source buffer: consecutive bytes cost one 16-byte load per window
// (byte loads only in the last 16 bytes of the buffer, which a 16-byte load could overrun).
struct SrcWin {
  const uint8_t* base = nullptr;
  uint4 v;
  __device__ __forceinline__ uint8_t at(const uint8_t* p, const uint8_t* lim) {
    const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)15);
    if (a != base) {
      if (a + 16 > lim) return *p;
      v = *reinterpret_cast<const uint4*>(a);
      base = a;
    }
    const uint32_t o = (uint32_t)(p - a);
    const uint32_t d = o < 8 ? (o < 4 ? v.x : v.y) : (o < 12 ? v.z : v.w);
    return (uint8_t)(d >> (8 * (o & 3)));
  }
};

// An op's record as the writer sees it: header VLQs, then key bytes, then value bytes.
struct AppRec {
  uint64_t st, en;        // relative output range
  uint64_t vq1, vq2;      // the two header VLQ values
  uint32_t a1, a2;        // their sizes
  const uint8_t* key;
  uint64_t klen;
  const uint8_t* val;
  __device__ __forceinline__ void load(const AppendParams& A, uint64_t op) {
    st = A.off[op];
    en = st + A.sizes[op];
    const int kind = A.kind[op];
    const uint64_t k0 = A.key_off[op];
    klen = A.key_off[op + 1] - k0;
    key = A.keys + k0;
    const uint64_t v0 = kind ? A.val_off[op] : 0;
    val = A.values + v0;
    vq1 = kind ? klen + 1 : 0;
    vq2 = kind ? A.val_off[op + 1] - v0 : klen;
    a1 = (uint32_t)app_vlq_size(vq1);
    a2 = (uint32_t)app_vlq_size(vq2);
  }
  __device__ __forceinline__ uint8_t byte(uint64_t q, SrcWin& kw, SrcWin& vw, const uint8_t* klim,
                                          const uint8_t* vlim) const {
    if (q < a1) return (uint8_t)(((vq1 >> (7 * q)) & 0x7f) | (q + 1 < a1 ? 0x80 : 0));
    if (q < a1 + a2) {
      const uint64_t r = q - a1;
      return (uint8_t)(((vq2 >> (7 * r)) & 0x7f) | (r + 1 < a2 ? 0x80 : 0));
    }
    if (q < a1 + a2 + klen) return kw.at(key + (q - a1 - a2), klim);
    return vw.at(val + (q - a1 - a2 - klen), vlim);
  }
};

// one lane per aligned 16-byte word: its bytes, op by op, then one 16-byte store (byte stores only
// for the two words the range shares with the memory around it)
__global__ __launch_bounds__(256) void k_app_write(AppendParams A) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= A.nwords) return;
  const int64_t r0 = (int64_t)(16 * w) - (int64_t)A.mis;  // relative position of the word's first byte
  const uint64_t total = A.total[0];
  uint64_t op = A.map[w];
  AppRec rec;
  rec.load(A, op);
  SrcWin kw, vw;
  const uint8_t* klim = A.keys + A.key_off[A.n];
  const uint8_t* vlim = A.values + A.val_off[A.n];
  uint8_t b[16];
  const bool full = r0 >= 0 && (uint64_t)r0 + 16 <= total;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int64_t r = r0 + k;
    b[k] = 0;
    if (r < 0 || (uint64_t)r >= total) continue;
    while ((uint64_t)r >= rec.en) rec.load(A, ++op);  // next op (dropped DELETEs have no bytes)
    b[k] = rec.byte((uint64_t)r - rec.st, kw, vw, klim, vlim);
  }
  uint8_t* dst = A.out - A.mis + 16 * w;
  if (full) {
    uint4 v;
    v.x = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    v.y = (uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24);
    v.z = (uint32_t)b[8] | ((uint32_t)b[9] << 8) | ((uint32_t)b[10] << 16) | ((uint32_t)b[11] << 24);
    v.w = (uint32_t)b[12] | ((uint32_t)b[13] << 8) | ((uint32_t)b[14] << 16) | ((uint32_t)b[15] << 24);
    *reinterpret_cast<uint4*>(dst) = v;
  } else {
    for (int k = 0; k < 16; k++) {
      const int64_t r = r0 + k;
      if (r >= 0 && (uint64_t)r < total) dst[k] = b[k];
    }
  }
}

__global__ __launch_bounds__(1024) void k_app_final(AppendParams A, uint32_t nblk) {
  __shared__ int64_t red[6][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t v[6] = {0, 0, 0, 0, -1, -1};
  for (uint32_t b = tid; b < nblk; b += 1024)
    for (int k = 0; k < 6; k++) {
      const int64_t x = A.partials[(uint64_t)b * 6 + k];
      v[k] = k < 4 ? v[k] + x : max(v[k], x);
    }
  for (int k = 0; k < 6; k++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t t = __shfl_xor(v[k], o, 64);
      v[k] = k < 4 ? v[k] + t : max(v[k], t);
    }
    if (lane == 0) red[k][w] = v[k];
  }
  __syncthreads();
  if (tid < 6) {
    int64_t r = red[tid][0];
    for (int q = 1; q < 16; q++) r = tid < 4 ? r + red[tid][q] : max(r, red[tid][q]);
    A.sums[tid] = r;
  }
}

// record sizes, their offsets and the header sums (the caller checks the total against its buffer)
void launch_append_sizes(const AppendParams& A, hipStream_t s) {
  if (A.n == 0) return;
  const unsigned g256 = (unsigned)((A.n + 255) / 256);
  hipLaunchKernelGGL(k_app_keymax, dim3(g256), dim3(256), 0, s, A);
  scan_exclusive<int64_t, int64_t, OpMaxI64>(A.keymax, A.keymax_pre, A.n, A.sums + 8, OpMaxI64(), A.scan_i64, s);
  hipLaunchKernelGGL(k_app_sizes, dim3(g256), dim3(256), 0, s, A);
  scan_exclusive<uint32_t, uint64_t, OpAdd>(A.sizes, A.off, A.n, A.total, OpAdd(), A.scan_u64, s);
  hipLaunchKernelGGL(k_app_final, dim3(1), dim3(1024), 0, s, A, g256);
}

void launch_append_write(const AppendParams& A, hipStream_t s) {
  if (A.n == 0 || A.nwords == 0) return;
  hipLaunchKernelGGL(k_app_map, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, A);
  hipLaunchKernelGGL(k_app_write, dim3((unsigned)((A.nwords + 255) / 256)), dim3(256), 0, s, A);
}

}  // namespace sk
