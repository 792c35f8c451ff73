/*
 * sparkey_oracle.c -- sequential CPU restatement of the reference's hash-file build.
 *
 * TEST INFRASTRUCTURE ONLY (see sparkey_oracle.h).  Every function cites the
 * reference file:line it restates; paths are relative to
 * src/main/java/com/spotify/sparkey/ of spotify/sparkey-java.
 *
 * Scope: CompressionType.NONE logs (the only type on the hot path).
 */
#include "sparkey_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* little-endian helpers (Util.java:46-84, InMemoryData.java:108-124)  */
/* ------------------------------------------------------------------ */
static uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static void wr32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void wr64(uint8_t* p, uint64_t v) { wr32(p, (uint32_t)v); wr32(p + 4, (uint32_t)(v >> 32)); }

static void set_err(char* err, int32_t err_len, const char* msg) {
  if (err && err_len > 0) {
    snprintf(err, (size_t)err_len, "%s", msg);
  }
}

/* ------------------------------------------------------------------ */
/* MurmurHash3.java:18-75                                             */
/* ------------------------------------------------------------------ */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

uint32_t oracle_murmur3_x86_32(const uint8_t* data, int32_t len, int32_t seed) {
  const int32_t nblocks = len / 4;
  uint32_t h1 = (uint32_t)seed;
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  for (int32_t i = 0; i < nblocks; i++) {           /* :29-39 */
    uint32_t k1 = rd32(data + 4 * i);
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const int32_t tail = 4 * nblocks;                 /* :44-61, fall-through tail */
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= (uint32_t)data[tail + 2] << 16; /* fall through */
    case 2: k1 ^= (uint32_t)data[tail + 1] << 8;  /* fall through */
    case 1:
      k1 ^= (uint32_t)data[tail];
      k1 *= c1;
      k1 = rotl32(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= (uint32_t)len;                              /* :66-74 fmix32 */
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}

/* MurmurHash3.java:84-93 */
static uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

/* MurmurHash3.java:100-201: x64_128 with the seed widened unsigned (:103), returns h1 */
uint64_t oracle_murmur3_x64_64(const uint8_t* data, int32_t len, int32_t seed) {
  const int32_t nblocks = len / 16;
  uint64_t h1 = (uint64_t)(uint32_t)seed;
  uint64_t h2 = h1;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int32_t i = 0; i < nblocks; i++) {
    uint64_t k1 = rd64(data + 16 * i);
    uint64_t k2 = rd64(data + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729ULL;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5ULL;
  }
  const uint8_t* t = data + 16 * nblocks;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= (uint64_t)t[14] << 48; /* fall through */
    case 14: k2 ^= (uint64_t)t[13] << 40; /* fall through */
    case 13: k2 ^= (uint64_t)t[12] << 32; /* fall through */
    case 12: k2 ^= (uint64_t)t[11] << 24; /* fall through */
    case 11: k2 ^= (uint64_t)t[10] << 16; /* fall through */
    case 10: k2 ^= (uint64_t)t[9] << 8;   /* fall through */
    case 9:
      k2 ^= (uint64_t)t[8];
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      /* fall through */
    case 8: k1 ^= (uint64_t)t[7] << 56; /* fall through */
    case 7: k1 ^= (uint64_t)t[6] << 48; /* fall through */
    case 6: k1 ^= (uint64_t)t[5] << 40; /* fall through */
    case 5: k1 ^= (uint64_t)t[4] << 32; /* fall through */
    case 4: k1 ^= (uint64_t)t[3] << 24; /* fall through */
    case 3: k1 ^= (uint64_t)t[2] << 16; /* fall through */
    case 2: k1 ^= (uint64_t)t[1] << 8;  /* fall through */
    case 1:
      k1 ^= (uint64_t)t[0];
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

/* HashType.java:44-46 (64-bit) and 70-72 (32-bit, masked to unsigned) */
uint64_t oracle_hash(int32_t hash_size, const uint8_t* key, int32_t len, int32_t seed) {
  if (hash_size == 8) return oracle_murmur3_x64_64(key, len, seed);
  return (uint64_t)oracle_murmur3_x86_32(key, len, seed);
}

/* ------------------------------------------------------------------ */
/* VLQ: Util.java:86-218                                              */
/* ------------------------------------------------------------------ */
int32_t oracle_vlq_size(int64_t value) { /* Util.java:102-128 (long overload) */
  if (value < (1LL << 7)) return 1;
  if (value < (1LL << 14)) return 2;
  if (value < (1LL << 21)) return 3;
  if (value < (1LL << 28)) return 4;
  if (value < (1LL << 35)) return 5;
  if (value < (1LL << 42)) return 6;
  if (value < (1LL << 49)) return 7;
  if (value < (1LL << 56)) return 8;
  return 9;
}

int32_t oracle_vlq_write(uint64_t value, uint8_t* out) { /* Util.java:130-136 */
  int32_t n = 0;
  while (value >= (1u << 7)) {
    out[n++] = (uint8_t)((value & 0x7f) | 0x80);
    value >>= 7;
  }
  out[n++] = (uint8_t)value;
  return n;
}

/* Util.java:146-181: at most 5 bytes, Java int arithmetic (b << 28 may wrap).
 * returns 0 ok, ORACLE_E_CORRUPT_LOG on EOF, ORACLE_E_VLQ on "Too long VLQ value". */
int32_t oracle_vlq_read(const uint8_t* buf, int64_t len, int64_t* pos, int32_t* value) {
  uint32_t v = 0;
  for (int i = 0; i < 5; i++) {
    if (*pos >= len) return ORACLE_E_CORRUPT_LOG;
    uint32_t b = buf[(*pos)++];
    if (b < 0x80) {
      v |= b << (7 * i);
      *value = (int32_t)v;
      return ORACLE_OK;
    }
    v |= (b & 0x7f) << (7 * i);
  }
  return ORACLE_E_VLQ;
}

/* ------------------------------------------------------------------ */
/* Log header: LogHeader.java:55-115                                  */
/* ------------------------------------------------------------------ */
#define LOG_MAGIC 0x49b39c95u
#define LOG_HEADER_SIZE 84
#define INDEX_MAGIC 0x9a11318fu
#define INDEX_HEADER_SIZE 112

typedef struct {
  int32_t major, minor, file_id;
  int64_t num_puts, num_deletes, data_end, max_key_len, max_value_len, delete_size;
  int32_t compression_type, compression_block_size;
  int64_t put_size;
  int32_t max_entries_per_block;
} log_header;

/* ZSTD block decoder (oracle_set_zstd_decoder); NULL: ZSTD logs are unsupported */
static oracle_block_decoder g_zstd = NULL;

void oracle_set_zstd_decoder(oracle_block_decoder fn) { g_zstd = fn; }

static int32_t parse_log_header(const uint8_t* b, int64_t len, log_header* h) {
  if (len < LOG_HEADER_SIZE) return ORACLE_E_NOT_LOG;
  if (rd32(b + 0) != LOG_MAGIC) return ORACLE_E_NOT_LOG;               /* :57-60 */
  h->major = (int32_t)rd32(b + 4);
  if (h->major != 1) return ORACLE_E_VERSION;                           /* :61-64 */
  h->minor = (int32_t)rd32(b + 8);
  if (h->minor > 0) return ORACLE_E_VERSION;                            /* :65-68 */
  h->file_id = (int32_t)rd32(b + 12);
  h->num_puts = (int64_t)rd64(b + 16);
  h->num_deletes = (int64_t)rd64(b + 24);
  h->data_end = (int64_t)rd64(b + 32);
  h->max_key_len = (int64_t)rd64(b + 40);
  h->max_value_len = (int64_t)rd64(b + 48);
  h->delete_size = (int64_t)rd64(b + 56);
  h->compression_type = (int32_t)rd32(b + 64);
  h->compression_block_size = (int32_t)rd32(b + 68);
  h->put_size = (int64_t)rd64(b + 72);
  h->max_entries_per_block = (int32_t)rd32(b + 80);
  if (h->data_end > len) return ORACLE_E_CORRUPT_LOG;                  /* :81-83 */
  if (h->max_key_len > 0x7fffffffLL || h->max_key_len < 0) return ORACLE_E_HEADER; /* CommonHeader.java:38-40 */
  if (h->max_value_len < 0) return ORACLE_E_HEADER;                     /* CommonHeader.java:41-43 */
  if (h->compression_type < 0 || h->compression_type > 2) return ORACLE_E_CORRUPT_LOG; /* values()[ct] */
  if (h->compression_type == 2 && !g_zstd) return ORACLE_E_UNSUPPORTED; /* ZSTD: needs a decoder */
  return ORACLE_OK;
}

static void write_log_header(uint8_t* b, const log_header* h) { /* LogHeader.java:90-115 */
  wr32(b + 0, LOG_MAGIC);
  wr32(b + 4, (uint32_t)h->major);
  wr32(b + 8, (uint32_t)h->minor);
  wr32(b + 12, (uint32_t)h->file_id);
  wr64(b + 16, (uint64_t)h->num_puts);
  wr64(b + 24, (uint64_t)h->num_deletes);
  wr64(b + 32, (uint64_t)h->data_end);
  wr64(b + 40, (uint64_t)h->max_key_len);
  wr64(b + 48, (uint64_t)h->max_value_len);
  wr64(b + 56, (uint64_t)h->delete_size);
  wr32(b + 64, (uint32_t)h->compression_type);
  wr32(b + 68, (uint32_t)h->compression_block_size);
  wr64(b + 72, (uint64_t)h->put_size);
  wr32(b + 80, (uint32_t)h->max_entries_per_block);
}

/* ------------------------------------------------------------------ */
/* Log writer: LogWriter.java:96-115, UncompressedBlockOutput.java:67-87,
 * LogHeader.java:161-172                                             */
/* ------------------------------------------------------------------ */
struct oracle_log {
  log_header h;
  uint8_t* buf;
  int64_t len, cap;
};

static int32_t log_reserve(oracle_log* log, int64_t extra) {
  if (log->len + extra <= log->cap) return 0;
  int64_t nc = log->cap ? log->cap : 4096;
  while (nc < log->len + extra) nc *= 2;
  uint8_t* nb = (uint8_t*)realloc(log->buf, (size_t)nc);
  if (!nb) return ORACLE_E_BUFFER;
  log->buf = nb;
  log->cap = nc;
  return 0;
}

oracle_log* oracle_log_new(int32_t file_identifier, int32_t compression_block_size) {
  oracle_log* log = (oracle_log*)calloc(1, sizeof(oracle_log));
  if (!log) return NULL;
  log->h.major = 1;                     /* LogHeader.java:50-53 */
  log->h.minor = 0;
  log->h.file_id = file_identifier;     /* random in the reference; fixed here */
  log->h.data_end = LOG_HEADER_SIZE;
  log->h.compression_type = 0;
  log->h.compression_block_size = compression_block_size;
  if (log_reserve(log, LOG_HEADER_SIZE)) { free(log); return NULL; }
  log->len = LOG_HEADER_SIZE;
  write_log_header(log->buf, &log->h);
  return log;
}

int32_t oracle_log_put(oracle_log* log, const uint8_t* key, int32_t klen, const uint8_t* val, int64_t vlen) {
  if (klen < 0 || vlen < 0) return ORACLE_E_ARG;
  if (log_reserve(log, 20 + klen + vlen)) return ORACLE_E_BUFFER;
  log->len += oracle_vlq_write((uint64_t)klen + 1, log->buf + log->len);  /* UncompressedBlockOutput.java:68-71 */
  log->len += oracle_vlq_write((uint64_t)vlen, log->buf + log->len);
  memcpy(log->buf + log->len, key, (size_t)klen);
  log->len += klen;
  if (vlen) memcpy(log->buf + log->len, val, (size_t)vlen);
  log->len += vlen;
  log->h.num_puts++;                                                       /* LogHeader.java:161-166 */
  if (klen > log->h.max_key_len) log->h.max_key_len = klen;
  if (vlen > log->h.max_value_len) log->h.max_value_len = vlen;
  log->h.put_size += oracle_vlq_size((int64_t)klen + 1) + oracle_vlq_size(vlen) + klen + vlen;
  return 0;
}

int32_t oracle_log_delete(oracle_log* log, const uint8_t* key, int32_t klen) {
  if (klen < 0) return ORACLE_E_ARG;
  if (klen > log->h.max_key_len) return 0;  /* LogWriter.java:110-115: silently dropped */
  if (log_reserve(log, 10 + klen)) return ORACLE_E_BUFFER;
  log->buf[log->len++] = 0;                 /* UncompressedBlockOutput.java:82-87 */
  log->len += oracle_vlq_write((uint64_t)klen, log->buf + log->len);
  memcpy(log->buf + log->len, key, (size_t)klen);
  log->len += klen;
  log->h.num_deletes++;                     /* LogHeader.java:168-172 */
  log->h.delete_size += 1 + oracle_vlq_size(klen) + klen;
  return 0;
}

int64_t oracle_log_size(const oracle_log* log) { return log->len; }

/* flush(): LogWriter.java:71-80 -- maxEntriesPerBlock = 1 for NONE, dataEnd = file length */
int64_t oracle_log_finish(oracle_log* log, uint8_t* out, int64_t cap) {
  log->h.max_entries_per_block = 1;
  log->h.data_end = log->len;
  write_log_header(log->buf, &log->h);
  if (!out) return log->len;
  if (cap < log->len) return ORACLE_E_BUFFER;
  memcpy(out, log->buf, (size_t)log->len);
  return log->len;
}

void oracle_log_free(oracle_log* log) {
  if (!log) return;
  free(log->buf);
  free(log);
}

/* ------------------------------------------------------------------ */
/* Index build: IndexHash.java:123-350, 454-678                        */
/* ------------------------------------------------------------------ */
typedef struct {
  /* IndexHeader.java:23-38 */
  int32_t file_id, hash_seed;
  int64_t data_end, max_key_len, max_value_len, num_puts;
  int64_t garbage_size, num_entries;
  int32_t address_size, hash_size;
  int64_t capacity, max_displacement;
  int32_t entry_block_bits;
  int64_t hash_collisions, total_displacement;
} index_header;

typedef struct {
  index_header ih;
  uint8_t* table; /* capacity * slot_size, zero initialised (InMemoryData.java:33-52) */
  int32_t slot_size;
  const uint8_t* log;
  int64_t log_len;
  int32_t ebb_mask;
  /* SNAPPY logs: `log` is the virtual stream (84 header bytes, then every block's decompressed bytes
   * back to back); block b starts at file offset blk_pos[b] and at virtual offset blk_voff[b]. */
  int32_t compressed;
  int64_t nblk;
  int64_t* blk_pos;
  int64_t* blk_voff;
} build_ctx;

/* The block that holds virtual offset v (largest b with blk_voff[b] <= v). */
static int64_t block_of(const build_ctx* c, int64_t v) {
  int64_t lo = 0, hi = c->nblk - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) / 2;
    if (c->blk_voff[mid] <= v) lo = mid; else hi = mid - 1;
  }
  return lo;
}

/* CompressedRandomReader.seek to a block start: file position -> virtual offset (<0: no such block). */
static int64_t block_voff(const build_ctx* c, int64_t file_pos) {
  int64_t lo = 0, hi = c->nblk - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    if (c->blk_pos[mid] == file_pos) return c->blk_voff[mid];
    if (c->blk_pos[mid] < file_pos) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

static int32_t calc_entry_block_bits(int32_t max_entries_per_block) { /* IndexHash.java:123-129 */
  int32_t i = 0;
  while ((1 << i) < max_entries_per_block) i++;
  return i;
}

/* Java (long) cast of a double: truncation, NaN -> 0, saturating */
static int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}

static int32_t make_index_header(const log_header* lh, int32_t hash_size, double sparsity,
                                 int32_t seed, index_header* ih) {
  if (sparsity < 1.3) sparsity = 1.3;                                     /* IndexHash.java:135-137 */
  int32_t ebb = calc_entry_block_bits(lh->max_entries_per_block);
  int32_t address_size = lh->data_end <= (1LL << (30 - ebb)) ? 4 : 8;     /* :140, :247-250 */
  if (hash_size == 0) hash_size = lh->num_puts < (1 << 23) ? 4 : 8;       /* :141-143 */
  if (hash_size != 4 && hash_size != 8) return ORACLE_E_ARG;
  int64_t capacity = 1LL | java_d2l((double)lh->num_puts * sparsity);    /* :145 -- the only FP op */
  memset(ih, 0, sizeof(*ih));
  ih->file_id = lh->file_id;
  ih->hash_seed = seed;
  ih->data_end = lh->data_end;
  ih->max_key_len = lh->max_key_len;
  ih->max_value_len = lh->max_value_len;
  ih->num_puts = lh->num_puts;
  ih->address_size = address_size;
  ih->hash_size = hash_size;
  ih->capacity = capacity;
  ih->entry_block_bits = ebb;
  return ORACLE_OK;
}

static void write_index_header(uint8_t* b, const index_header* h) { /* IndexHeader.java:125-155 */
  wr32(b + 0, INDEX_MAGIC);
  wr32(b + 4, 1);
  wr32(b + 8, 1);
  wr32(b + 12, (uint32_t)h->file_id);
  wr32(b + 16, (uint32_t)h->hash_seed);
  wr64(b + 20, (uint64_t)h->data_end);
  wr64(b + 28, (uint64_t)h->max_key_len);
  wr64(b + 36, (uint64_t)h->max_value_len);
  wr64(b + 44, (uint64_t)h->num_puts);
  wr64(b + 52, (uint64_t)h->garbage_size);
  wr64(b + 60, (uint64_t)h->num_entries);
  wr32(b + 68, (uint32_t)h->address_size);
  wr32(b + 72, (uint32_t)h->hash_size);
  wr64(b + 76, (uint64_t)h->capacity);
  wr64(b + 84, (uint64_t)h->max_displacement);
  wr32(b + 92, (uint32_t)h->entry_block_bits);
  wr64(b + 96, (uint64_t)h->hash_collisions);
  wr64(b + 104, (uint64_t)h->total_displacement);
}

/* slot access: HashType.readHash/writeHash (HashType.java:24-36,50-62),
 * AddressSize.readAddress/writeAddress (AddressSize.java:116-158) */
static uint64_t slot_hash(const build_ctx* c, int64_t slot) {
  const uint8_t* p = c->table + slot * c->slot_size;
  return c->ih.hash_size == 8 ? rd64(p) : (uint64_t)rd32(p);
}
static uint64_t slot_addr(const build_ctx* c, int64_t slot) {
  const uint8_t* p = c->table + slot * c->slot_size + c->ih.hash_size;
  return c->ih.address_size == 8 ? rd64(p) : (uint64_t)rd32(p);
}
static void slot_write(build_ctx* c, int64_t slot, uint64_t hash, uint64_t addr) {
  uint8_t* p = c->table + slot * c->slot_size;
  if (c->ih.hash_size == 8) wr64(p, hash); else wr32(p, (uint32_t)hash);
  p += c->ih.hash_size;
  if (c->ih.address_size == 8) wr64(p, addr); else wr32(p, (uint32_t)addr);
}

static uint64_t wanted_slot(uint64_t hash, int64_t cap) { /* IndexHash.java:667-669 */
  return hash % (uint64_t)cap;
}
static int64_t displacement_of(int64_t cap, int64_t slot, uint64_t hash) { /* :671-678 */
  int64_t d = slot - (int64_t)wanted_slot(hash, cap);
  return d >= 0 ? d : d + cap;
}

/* skipStuff (IndexHash.java:550-560) is a no-op for NONE (entryIndex == 0 always). */
static int32_t skip_stuff(const build_ctx* c, int64_t* pos, int32_t entry_index) {
  if (c->compressed) { /* the address names a block; entries are counted from its start */
    int64_t v = block_voff(c, *pos);
    if (v < 0) return ORACLE_E_CORRUPT_LOG;
    *pos = v;
  }
  for (int32_t i = 0; i < entry_index; i++) {
    int32_t k, v;
    int32_t rc = oracle_vlq_read(c->log, c->log_len, pos, &k);
    if (rc) return rc;
    rc = oracle_vlq_read(c->log, c->log_len, pos, &v);
    if (rc) return rc;
    *pos += (k == 0) ? v : (int64_t)k - 1 + v;
  }
  return 0;
}

/* IndexHeader.java:221-228 (Java int arithmetic for the size expression) */
static int64_t garbage_of(int32_t key_len2, int32_t value_len2) {
  int32_t s = (int32_t)((uint32_t)key_len2 + (uint32_t)value_len2 +
                        (uint32_t)oracle_vlq_size((int64_t)key_len2 + 1) + (uint32_t)oracle_vlq_size(value_len2));
  return s;
}

/* Reads the key of the record at `position` (PUT expected): used when keyLen == -1 (SORTING). */
static int32_t read_own_put_key(const build_ctx* c, int64_t position, int32_t entry_index,
                                int32_t* key_len, const uint8_t** key) {
  int64_t pos = position;
  int32_t rc = skip_stuff(c, &pos, entry_index);
  if (rc) return rc;
  int32_t k, v;
  rc = oracle_vlq_read(c->log, c->log_len, &pos, &k);
  if (rc) return rc;
  if (k - 1 == -1) return ORACLE_E_CORRUPT_DATA;                         /* IndexHash.java:611-614 */
  rc = oracle_vlq_read(c->log, c->log_len, &pos, &v);
  if (rc) return rc;
  if (pos + (k - 1) > c->log_len) return ORACLE_E_CORRUPT_LOG;
  *key_len = k - 1;
  *key = c->log + pos;
  return 0;
}

/* IndexHash.put: IndexHash.java:562-665 */
static int32_t idx_put(build_ctx* c, int32_t key_len, const uint8_t* key, uint64_t hash, uint64_t address) {
  const int64_t cap = c->ih.capacity;
  if (c->ih.num_entries >= cap) return ORACLE_E_NO_FREE_SLOTS;           /* :574-576 */
  const int32_t ebb = c->ih.entry_block_bits;
  int64_t slot = (int64_t)wanted_slot(hash, cap);
  int64_t displacement = 0;
  int64_t tries = cap;
  int32_t entry_index = (int32_t)(address & (uint64_t)c->ebb_mask);
  int64_t position = (int64_t)(address >> ebb);
  int might_be_collision = 1;
  while (--tries >= 0) {
    uint64_t hash2 = slot_hash(c, slot);
    uint64_t address2 = slot_addr(c, slot);
    if (address2 == 0) {                                                 /* :594-600 */
      slot_write(c, slot, hash, address);
      c->ih.num_entries++;
      return 0;
    }
    int32_t entry_index2 = (int32_t)(address2 & (uint64_t)c->ebb_mask);
    int64_t position2 = (int64_t)(address2 >> ebb);
    if (might_be_collision && hash == hash2) {                           /* :606-637 */
      int32_t rc;
      if (key_len == -1) {
        rc = read_own_put_key(c, position, entry_index, &key_len, &key);
        if (rc) return rc;
      }
      int64_t pos = position2;
      rc = skip_stuff(c, &pos, entry_index2);
      if (rc) return rc;
      int32_t key_len2, value_len2;
      rc = oracle_vlq_read(c->log, c->log_len, &pos, &key_len2);
      if (rc) return rc;
      rc = oracle_vlq_read(c->log, c->log_len, &pos, &value_len2);
      if (rc) return rc;
      if (key_len2 == 0) return ORACLE_E_CORRUPT_DATA;                   /* "reference to delete entry" */
      key_len2--;
      if (key_len == key_len2) {
        if (pos + key_len > c->log_len) return ORACLE_E_CORRUPT_LOG;
        if (memcmp(c->log + pos, key, (size_t)key_len) == 0) {          /* replace in place */
          slot_write(c, slot, hash, address);
          c->ih.garbage_size += garbage_of(key_len2, value_len2);
          return 0;
        }
      }
    }
    int64_t other = displacement_of(cap, slot, hash2);                    /* :639-653 */
    if (displacement > other || (displacement == other && (int64_t)address < (int64_t)address2)) {
      slot_write(c, slot, hash, address);
      position = position2;
      entry_index = entry_index2;
      address = address2;
      displacement = other;
      hash = hash2;
      might_be_collision = 0;
    }
    displacement++;
    slot++;
    if (slot >= cap) slot = 0;
  }
  return ORACLE_E_NO_FREE_SLOTS;                                          /* :664 */
}

/* IndexHash.delete: IndexHash.java:454-548 */
static int32_t idx_delete(build_ctx* c, int32_t key_len, const uint8_t* key, uint64_t hash, uint64_t address) {
  const int64_t cap = c->ih.capacity;
  const int32_t ebb = c->ih.entry_block_bits;
  int64_t slot = (int64_t)wanted_slot(hash, cap);
  int64_t displacement = 0;
  int32_t entry_index = (int32_t)(address & (uint64_t)c->ebb_mask);
  int64_t position = (int64_t)(address >> ebb);
  for (int64_t guard = 0; guard <= cap; guard++) {
    uint64_t hash2 = slot_hash(c, slot);
    uint64_t address2 = slot_addr(c, slot);
    if (address2 == 0) return 0;
    int32_t entry_index2 = (int32_t)(address2 & (uint64_t)c->ebb_mask);
    int64_t position2 = (int64_t)(address2 >> ebb);
    if (hash == hash2) {
      int32_t rc;
      if (key_len == -1) {                                               /* :479-488 */
        int64_t pos = position;
        rc = skip_stuff(c, &pos, entry_index);
        if (rc) return rc;
        int32_t first;
        rc = oracle_vlq_read(c->log, c->log_len, &pos, &first);
        if (rc) return rc;
        if (first != 0) return ORACLE_E_CORRUPT_DATA;
        rc = oracle_vlq_read(c->log, c->log_len, &pos, &key_len);
        if (rc) return rc;
        if (key_len < 0 || pos + key_len > c->log_len) return ORACLE_E_CORRUPT_LOG;
        key = c->log + pos;
      }
      int64_t pos = position2;
      rc = skip_stuff(c, &pos, entry_index2);
      if (rc) return rc;
      int32_t key_len2;
      rc = oracle_vlq_read(c->log, c->log_len, &pos, &key_len2);
      if (rc) return rc;
      if (key_len2 == 0) return ORACLE_E_CORRUPT_DATA;
      key_len2--;
      if (key_len == key_len2) {
        int32_t value_len2;
        rc = oracle_vlq_read(c->log, c->log_len, &pos, &value_len2);
        if (rc) return rc;
        if (pos + key_len > c->log_len) return ORACLE_E_CORRUPT_LOG;
        if (memcmp(c->log + pos, key, (size_t)key_len) == 0) {
          for (int64_t g2 = 0; g2 < cap; g2++) {                         /* backward shift :503-524 */
            int64_t next_slot = slot + 1;
            if (next_slot == cap) next_slot = 0;
            uint64_t hash3 = slot_hash(c, next_slot);
            uint64_t position3 = slot_addr(c, next_slot);
            if (position3 == 0) break;
            if ((int64_t)wanted_slot(hash3, cap) == next_slot) break;
            slot_write(c, slot, hash3, position3);
            slot = next_slot;
          }
          slot_write(c, slot, 0, 0);
          c->ih.garbage_size += garbage_of(key_len2, value_len2);         /* deletedEntry */
          c->ih.num_entries--;
          return 0;
        }
      }
    }
    int64_t other = displacement_of(cap, slot, hash2);
    if (displacement > other) return 0;
    displacement++;
    slot++;
    if (slot == cap) slot = 0;
  }
  return 0;
}

/* calculateMaxDisplacement: IndexHash.java:195-245 (both quirks kept) */
static void calc_stats(build_ctx* c) {
  const int64_t cap = c->ih.capacity;
  int64_t max_d = 0, collisions = 0, total_d = 0;
  int has_first = 0, has_last = 0, has_prev = 0;
  uint64_t first_hash = 0, last_hash = 0, prev_hash = (uint64_t)-1;
  for (int64_t slot = 0; slot < cap; slot++) {
    uint64_t hash = slot_hash(c, slot);
    if (has_prev && prev_hash == hash) collisions++;  /* compares even an EMPTY slot's 0 hash */
    uint64_t position = slot_addr(c, slot);
    if (position != 0) {
      prev_hash = hash;
      has_prev = 1;
      int64_t d = displacement_of(cap, slot, hash);
      total_d += d;
      if (d > max_d) max_d = d;
      if (slot == 0) { first_hash = hash; has_first = 1; }
      if (slot == cap - 1) { last_hash = hash; has_last = 1; }
    } else {
      has_prev = 0;
    }
  }
  if (has_first && has_last && first_hash == last_hash) collisions++;
  c->ih.total_displacement = total_d;
  c->ih.max_displacement = max_d;
  c->ih.hash_collisions = collisions;
}

/* One framed record (SparkeyLogIterator.java:86-138) */
typedef struct {
  int64_t position;
  int32_t entry_index;
  int32_t is_put;
  int32_t key_len;
  int64_t value_len;
  const uint8_t* key;
} log_rec;

/* Iterates records in [start, end): returns 1 with *r filled, 0 at end, <0 error. */
static int32_t next_record(const build_ctx* c, int64_t* pos, int64_t end, int64_t* prev_pos,
                           int32_t* entry_index, log_rec* r) {
  if (*pos >= end) return 0;
  /* CompressedReader.getBlockPosition (CompressedReader.java:121-126): the block holding the
   * record's first byte; for NONE the record's own offset */
  const int64_t bpos = c->compressed ? c->blk_pos[block_of(c, *pos)] : *pos;
  if (bpos == *prev_pos) (*entry_index)++; else *entry_index = 0;
  *prev_pos = bpos;
  r->position = bpos;
  r->entry_index = *entry_index;
  int64_t p = *pos;
  int32_t first, second, rc;
  /* EOF anywhere inside the first VLQ (its first byte, or after a continuation byte): hasNext catches
   * the EOFException of that read and ends the iteration without an error (SparkeyLogIterator.java:
   * 111-115).  "Too long VLQ value" there is a RuntimeException, not caught (Util.java:217). */
  rc = oracle_vlq_read(c->log, c->log_len, &p, &first);
  if (rc == ORACLE_E_CORRUPT_LOG) return 0;
  if (rc) return rc;
  /* EOF inside the second VLQ: EOFException, wrapped in RuntimeException by hasNext
   * (SparkeyLogIterator.java:117,134-136) */
  rc = oracle_vlq_read(c->log, c->log_len, &p, &second);
  if (rc) return rc == ORACLE_E_CORRUPT_LOG ? ORACLE_E_CORRUPT_RECORD : rc;
  if (first == 0) { r->is_put = 0; r->key_len = second; r->value_len = 0; }
  else { r->is_put = 1; r->key_len = first - 1; r->value_len = second; }
  /* stream.read(keyBuf, 0, keyLen) (:130): IndexOutOfBoundsException for a negative key length or one
   * above maxKeyLen (the buffer's size); a negative value length and a key past the end of the file
   * are not reference-pinned and are rejected the same way */
  if (r->key_len < 0 || r->value_len < 0) return ORACLE_E_CORRUPT_RECORD;
  if (r->key_len > c->ih.max_key_len) return ORACLE_E_CORRUPT_RECORD;
  if (p + r->key_len > c->log_len) return ORACLE_E_CORRUPT_RECORD;
  r->key = c->log + p;
  *pos = p + r->key_len + r->value_len;
  return 1;
}

/* fillFromLog: IndexHash.java:257-303 */
static int32_t fill_from_log(build_ctx* c) {
  int64_t pos = LOG_HEADER_SIZE, prev_pos = -1;
  int32_t entry_index = 0;
  const int32_t ebb = c->ih.entry_block_bits;
  for (;;) {
    log_rec r;
    int32_t rc = next_record(c, &pos, c->compressed ? c->log_len : c->ih.data_end, &prev_pos, &entry_index, &r);
    if (rc < 0) return rc;
    if (rc == 0) return 0;
    uint64_t address = ((uint64_t)r.position << ebb) | (uint64_t)r.entry_index; /* :283 */
    uint64_t hash = oracle_hash(c->ih.hash_size, r.key, r.key_len, c->ih.hash_seed);
    rc = r.is_put ? idx_put(c, r.key_len, r.key, hash, address)
                  : idx_delete(c, r.key_len, r.key, hash, address);
    if (rc) return rc;
  }
}

/* SortHelper.Entry + ENTRY_COMPARATOR (SortHelper.java:42, 153-171) */
typedef struct {
  uint64_t hash;
  int64_t address; /* position << (ebb+1) | entryIndex << 1 | isPut */
  uint64_t wanted;
} sort_entry;

static int cmp_sort_entry(const void* a, const void* b) {
  const sort_entry* x = (const sort_entry*)a;
  const sort_entry* y = (const sort_entry*)b;
  /* Comparator.comparingLong compares signed longs; wanted < cap <= 2^63 */
  if ((int64_t)x->wanted != (int64_t)y->wanted) return (int64_t)x->wanted < (int64_t)y->wanted ? -1 : 1;
  if (x->address != y->address) return x->address < y->address ? -1 : 1;
  return 0;
}

/* fillFromLogSorted: IndexHash.java:305-350 */
static int32_t fill_from_log_sorted(build_ctx* c) {
  int64_t pos = LOG_HEADER_SIZE, prev_pos = -1, n = 0, cap_e = 1024;
  int32_t entry_index = 0;
  const int32_t ebb = c->ih.entry_block_bits;
  sort_entry* es = (sort_entry*)malloc(sizeof(sort_entry) * (size_t)cap_e);
  if (!es) return ORACLE_E_BUFFER;
  for (;;) {
    log_rec r;
    int32_t rc = next_record(c, &pos, c->compressed ? c->log_len : c->ih.data_end, &prev_pos, &entry_index, &r);
    if (rc < 0) { free(es); return rc; }
    if (rc == 0) break;
    if (n == cap_e) {
      cap_e *= 2;
      sort_entry* ne = (sort_entry*)realloc(es, sizeof(sort_entry) * (size_t)cap_e);
      if (!ne) { free(es); return ORACLE_E_BUFFER; }
      es = ne;
    }
    es[n].hash = oracle_hash(c->ih.hash_size, r.key, r.key_len, c->ih.hash_seed);
    es[n].address = (int64_t)(((uint64_t)r.position << (ebb + 1)) | ((uint64_t)r.entry_index << 1) |
                              (uint64_t)(r.is_put ? 1 : 0));
    es[n].wanted = wanted_slot(es[n].hash, c->ih.capacity);
    n++;
  }
  qsort(es, (size_t)n, sizeof(sort_entry), cmp_sort_entry);
  for (int64_t i = 0; i < n; i++) {
    int is_put = (es[i].address & 1) != 0;
    uint64_t address = (uint64_t)es[i].address >> 1;
    int32_t rc = is_put ? idx_put(c, -1, NULL, es[i].hash, address)
                        : idx_delete(c, -1, NULL, es[i].hash, address);
    if (rc) { free(es); return rc; }
  }
  free(es);
  return 0;
}

int64_t oracle_index_size(const uint8_t* log, int64_t log_len, int32_t hash_size, double sparsity) {
  log_header lh;
  int32_t rc = parse_log_header(log, log_len, &lh);
  if (rc) return rc;
  index_header ih;
  rc = make_index_header(&lh, hash_size, sparsity, 1, &ih);
  if (rc) return rc;
  return INDEX_HEADER_SIZE + (int64_t)(ih.hash_size + ih.address_size) * ih.capacity;
}

static const char* err_msg(int32_t rc) {
  switch (rc) {
    case ORACLE_E_NOT_LOG: return "File is not a Sparkey log file";
    case ORACLE_E_VERSION: return "Incompatible version";
    case ORACLE_E_CORRUPT_LOG: return "Corrupt log file";
    case ORACLE_E_NO_FREE_SLOTS: return "No free slots in the hash";
    case ORACLE_E_CORRUPT_DATA: return "Corrupt data";
    case ORACLE_E_VLQ: return "Too long VLQ value";
    case ORACLE_E_HEADER: return "Too large max key len";
    case ORACLE_E_UNSUPPORTED: return "Unsupported compression type";
    case ORACLE_E_BUFFER: return "Buffer too small";
    case ORACLE_E_CORRUPT_RECORD: return "Corrupt log record";
    default: return "Error";
  }
}

/* Snappy raw-format decompression (the published format snappy-java wraps, CompressorType.java:32-34):
 * varint uncompressed length, then literal (tag 00), copy-1 (01), copy-2 (10) and copy-4 (11)
 * elements.  Returns the decompressed length or <0 on a malformed stream or a too-small `out`. */
int64_t oracle_snappy_uncompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  int64_t p = 0, ulen = 0;
  for (int shift = 0;; shift += 7) {
    if (p >= n || shift > 28) return ORACLE_E_CORRUPT_LOG;
    uint8_t b = in[p++];
    ulen |= (int64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if (ulen > cap || ulen > 0xffffffffLL) return ORACLE_E_BUFFER;
  int64_t o = 0;
  while (p < n) {
    const uint8_t t = in[p++];
    int64_t len, off;
    if ((t & 3) == 0) {
      len = (t >> 2) + 1;
      if (len > 60) {
        const int nb = (int)len - 60;
        if (p + nb > n) return ORACLE_E_CORRUPT_LOG;
        len = 0;
        for (int i = 0; i < nb; i++) len |= (int64_t)in[p + i] << (8 * i);
        len += 1;
        p += nb;
      }
      if (p + len > n || o + len > ulen) return ORACLE_E_CORRUPT_LOG;
      memcpy(out + o, in + p, (size_t)len);
      p += len;
      o += len;
      continue;
    }
    if ((t & 3) == 1) {
      if (p + 1 > n) return ORACLE_E_CORRUPT_LOG;
      len = ((t >> 2) & 7) + 4;
      off = ((int64_t)(t >> 5) << 8) | in[p];
      p += 1;
    } else if ((t & 3) == 2) {
      if (p + 2 > n) return ORACLE_E_CORRUPT_LOG;
      len = (t >> 2) + 1;
      off = (int64_t)in[p] | ((int64_t)in[p + 1] << 8);
      p += 2;
    } else {
      if (p + 4 > n) return ORACLE_E_CORRUPT_LOG;
      len = (t >> 2) + 1;
      off = (int64_t)rd32(in + p);
      p += 4;
    }
    if (off == 0 || off > o || o + len > ulen) return ORACLE_E_CORRUPT_LOG;
    for (int64_t i = 0; i < len; i++) out[o + i] = out[o - off + i]; /* overlapping copies repeat */
    o += len;
  }
  return o == ulen ? ulen : ORACLE_E_CORRUPT_LOG;
}

/* ZSTD: every block decoded into a buffer of maxBlockSize bytes (CompressedReader.java:40-49,
 * CompressorType.java:42-56: the decompressed length is what the decoder returns), appended to the
 * virtual stream. */
static int32_t open_zstd(build_ctx* c, const uint8_t* log, int64_t data_end, int64_t max_block, uint8_t** vbuf) {
  int64_t nblk = 0, cap_b = 64, total = 0, vcap = 1 << 16, p = LOG_HEADER_SIZE;
  c->blk_pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap_b);
  c->blk_voff = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap_b);
  uint8_t* v = (uint8_t*)malloc((size_t)vcap);
  uint8_t* tmp = (uint8_t*)malloc((size_t)max_block + 1);
  if (!c->blk_pos || !c->blk_voff || !v || !tmp) { free(v); free(tmp); return ORACLE_E_BUFFER; }
  memcpy(v, log, LOG_HEADER_SIZE);
  while (p < data_end) {
    int64_t q = p;
    int32_t clen;
    int32_t rc = oracle_vlq_read(log, data_end, &q, &clen);
    if (rc) { free(v); free(tmp); return rc; }
    if (clen < 0 || q + clen > data_end) { free(v); free(tmp); return ORACLE_E_CORRUPT_LOG; }
    const int64_t got = g_zstd(log + q, clen, tmp, max_block);
    if (got < 0 || got > max_block) { free(v); free(tmp); return ORACLE_E_CORRUPT_LOG; }
    if (nblk == cap_b) {
      cap_b *= 2;
      c->blk_pos = (int64_t*)realloc(c->blk_pos, sizeof(int64_t) * (size_t)cap_b);
      c->blk_voff = (int64_t*)realloc(c->blk_voff, sizeof(int64_t) * (size_t)cap_b);
      if (!c->blk_pos || !c->blk_voff) { free(v); free(tmp); return ORACLE_E_BUFFER; }
    }
    while (LOG_HEADER_SIZE + total + got + 1 > vcap) {
      vcap *= 2;
      v = (uint8_t*)realloc(v, (size_t)vcap);
      if (!v) { free(tmp); return ORACLE_E_BUFFER; }
    }
    c->blk_pos[nblk] = p;
    c->blk_voff[nblk] = LOG_HEADER_SIZE + total;
    memcpy(v + LOG_HEADER_SIZE + total, tmp, (size_t)got);
    total += got;
    nblk++;
    p = q + clen;
  }
  free(tmp);
  c->compressed = 1;
  c->nblk = nblk;
  c->log = v;
  c->log_len = LOG_HEADER_SIZE + total;
  *vbuf = v;
  return 0;
}

/* The virtual stream of a SNAPPY log: blocks VLQ(compressedSize) || snappy bytes from offset 84 to
 * dataEnd (CompressedOutputStream.flush, CompressedOutputStream.java:47-58; CompressedReader.fetchBlock,
 * CompressedReader.java:66-74). */
static int32_t open_compressed(build_ctx* c, const uint8_t* log, int64_t data_end, int64_t max_block, uint8_t** vbuf) {
  /* the reader's buffers (CompressedReader.java:40-49): compressedBuf holds
   * Snappy.maxCompressedLength(maxBlockSize) = 32 + n + n / 6 bytes, uncompressedBuf maxBlockSize; a
   * block that does not fit fails inside fetchBlock (:51-60) */
  const int64_t max_comp = 32 + max_block + max_block / 6;
  int64_t nblk = 0, cap_b = 64, total = 0, p = LOG_HEADER_SIZE;
  c->blk_pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap_b);
  c->blk_voff = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap_b);
  int64_t* ulens = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap_b);
  if (!c->blk_pos || !c->blk_voff || !ulens) { free(ulens); return ORACLE_E_BUFFER; }
  while (p < data_end) {
    int64_t q = p;
    int32_t clen;
    int32_t rc = oracle_vlq_read(log, data_end, &q, &clen);
    if (rc) { free(ulens); return rc; }
    if (clen < 0 || q + clen > data_end || clen > max_comp) { free(ulens); return ORACLE_E_CORRUPT_LOG; }
    int64_t ulen = 0, r = q;
    for (int shift = 0;; shift += 7) {
      if (r >= q + clen || shift > 28) { free(ulens); return ORACLE_E_CORRUPT_LOG; }
      ulen |= (int64_t)(log[r] & 0x7f) << shift;
      if (!(log[r++] & 0x80)) break;
    }
    if (ulen > max_block) { free(ulens); return ORACLE_E_CORRUPT_LOG; }
    if (nblk == cap_b) {
      cap_b *= 2;
      c->blk_pos = (int64_t*)realloc(c->blk_pos, sizeof(int64_t) * (size_t)cap_b);
      c->blk_voff = (int64_t*)realloc(c->blk_voff, sizeof(int64_t) * (size_t)cap_b);
      ulens = (int64_t*)realloc(ulens, sizeof(int64_t) * (size_t)cap_b);
      if (!c->blk_pos || !c->blk_voff || !ulens) { free(ulens); return ORACLE_E_BUFFER; }
    }
    c->blk_pos[nblk] = p;
    c->blk_voff[nblk] = LOG_HEADER_SIZE + total;
    ulens[nblk] = ulen;
    total += ulen;
    nblk++;
    p = q + clen;
  }
  uint8_t* v = (uint8_t*)malloc((size_t)(LOG_HEADER_SIZE + total + 1));
  if (!v) { free(ulens); return ORACLE_E_BUFFER; }
  memcpy(v, log, LOG_HEADER_SIZE);
  for (int64_t b = 0; b < nblk; b++) {
    int64_t q = c->blk_pos[b];
    int32_t clen;
    (void)oracle_vlq_read(log, data_end, &q, &clen);
    int64_t got = oracle_snappy_uncompress(log + q, clen, v + c->blk_voff[b], ulens[b]);
    if (got != ulens[b]) { free(ulens); free(v); return ORACLE_E_CORRUPT_LOG; }
  }
  free(ulens);
  c->compressed = 1;
  c->nblk = nblk;
  c->log = v;
  c->log_len = LOG_HEADER_SIZE + total;
  *vbuf = v;
  return 0;
}

/* IndexHash.createNew: IndexHash.java:131-167 */
int64_t oracle_build_index(const uint8_t* log, int64_t log_len, int32_t hash_size, double sparsity,
                           int32_t seed, int32_t method, int64_t max_memory,
                           uint8_t* out, int64_t out_cap, char* err, int32_t err_len) {
  log_header lh;
  int32_t rc = parse_log_header(log, log_len, &lh);
  if (rc) { set_err(err, err_len, err_msg(rc)); return rc; }
  build_ctx c;
  memset(&c, 0, sizeof(c));
  rc = make_index_header(&lh, hash_size, sparsity, seed, &c.ih);
  if (rc) { set_err(err, err_len, err_msg(rc)); return rc; }
  c.slot_size = c.ih.hash_size + c.ih.address_size;
  c.log = log;
  c.log_len = log_len;
  c.ebb_mask = (1 << c.ih.entry_block_bits) - 1;
  uint8_t* vbuf = NULL;
  if (lh.compression_type != 0) {
    /* every block is fetched and decoded inside the iterator (CompressedReader.fetchBlock,
     * CompressedReader.java:51-60; a negative maxBlockSize fails in its constructor, :40-49), so a
     * bad block is a RuntimeException there */
    if (lh.compression_block_size < 0) rc = ORACLE_E_CORRUPT_RECORD;
    else if (lh.compression_type == 2) rc = open_zstd(&c, log, lh.data_end, lh.compression_block_size, &vbuf);
    else rc = open_compressed(&c, log, lh.data_end, lh.compression_block_size, &vbuf);
    if (rc == ORACLE_E_CORRUPT_LOG) rc = ORACLE_E_CORRUPT_RECORD;
    if (rc) { free(c.blk_pos); free(c.blk_voff); set_err(err, err_len, err_msg(rc)); return rc; }
  }
  const int64_t hash_length = (int64_t)c.slot_size * c.ih.capacity;
  const int64_t total = INDEX_HEADER_SIZE + hash_length;
  if (out_cap < total) rc = ORACLE_E_BUFFER;
  if (!rc) memset(out, 0, (size_t)total);
  c.table = out + INDEX_HEADER_SIZE;
  int in_memory = method == 0 ? (hash_length <= max_memory) : (method == 1); /* :155-160 */
  if (!rc) rc = in_memory ? fill_from_log(&c) : fill_from_log_sorted(&c);
  free(vbuf);
  free(c.blk_pos);
  free(c.blk_voff);
  if (rc) { set_err(err, err_len, err_msg(rc)); return rc; }
  calc_stats(&c);
  write_index_header(out, &c.ih);
  return total;
}

/* IndexHash.get: IndexHash.java:398-452 (readers validate with this) */
int32_t oracle_get(const uint8_t* index, int64_t index_len, const uint8_t* log, int64_t log_len,
                   const uint8_t* key, int32_t klen, int64_t* value_off, int64_t* value_len) {
  if (index_len < INDEX_HEADER_SIZE || rd32(index) != INDEX_MAGIC) return ORACLE_E_ARG;
  build_ctx c;
  memset(&c, 0, sizeof(c));
  c.ih.hash_seed = (int32_t)rd32(index + 16);
  c.ih.address_size = (int32_t)rd32(index + 68);
  c.ih.hash_size = (int32_t)rd32(index + 72);
  c.ih.capacity = (int64_t)rd64(index + 76);
  c.ih.max_displacement = (int64_t)rd64(index + 84);
  c.ih.entry_block_bits = (int32_t)rd32(index + 92);
  c.slot_size = c.ih.hash_size + c.ih.address_size;
  if (index_len != INDEX_HEADER_SIZE + (int64_t)c.slot_size * c.ih.capacity) return ORACLE_E_ARG; /* :116-121 */
  c.table = (uint8_t*)(index + INDEX_HEADER_SIZE);
  c.log = log;
  c.log_len = log_len;
  c.ebb_mask = (1 << c.ih.entry_block_bits) - 1;
  uint64_t hash = oracle_hash(c.ih.hash_size, key, klen, c.ih.hash_seed);
  int64_t slot = (int64_t)wanted_slot(hash, c.ih.capacity);
  int64_t displacement = 0;
  for (;;) {
    uint64_t hash2 = slot_hash(&c, slot);
    uint64_t position2 = slot_addr(&c, slot);
    if (position2 == 0) return 0;
    int32_t entry_index = (int32_t)(position2 & (uint64_t)c.ebb_mask);
    position2 >>= c.ih.entry_block_bits;
    if (hash == hash2) {
      int64_t pos = (int64_t)position2;
      int32_t rc = skip_stuff(&c, &pos, entry_index);
      if (rc) return rc;
      int32_t key_len2, value_len2;
      rc = oracle_vlq_read(log, log_len, &pos, &key_len2);
      if (rc) return rc;
      if (key_len2 == 0) return ORACLE_E_CORRUPT_DATA;
      key_len2--;
      if (klen == key_len2) {
        rc = oracle_vlq_read(log, log_len, &pos, &value_len2);
        if (rc) return rc;
        if (pos + klen <= log_len && memcmp(log + pos, key, (size_t)klen) == 0) {
          *value_off = pos + klen;
          *value_len = value_len2;
          return 1;
        }
      }
    }
    displacement++;
    if (displacement > c.ih.max_displacement) return 0;
    slot++;
    if (slot == c.ih.capacity) slot = 0;
  }
}
