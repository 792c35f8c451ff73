"""Synthetic Sparkey logs for the BASELINE.json configs, written with numpy in the exact byte layout
LogWriter produces (UncompressedBlockOutput.java:67-72, LogHeader.java:90-115).

  fixed_log(n, 16, 100)      C2: key = LE64(i) || LE64(splitmix64(i ^ seed)) (unique), value = 100 random bytes
  mixed_log(n, 8, 64, 100)   C3: key length uniform in [8, 64], LE64(i) prefix keeps keys unique
  key_value_log(n)           C1: put("key_" + i, "value_" + i) as WriteHashBenchmark.java:52-54
  key_value_log_np(n)        the same bytes built with numpy (WriteHashBenchmark's 10M)
  churn_log(n, pool, p_del)  C2 shape with overwrites and DELETEs: keys drawn from a pool of `pool`
"""
from __future__ import annotations

import numpy as np

from .log_writer import LOG_HEADER_SIZE, LogHeader, vlq_bytes

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return z ^ (z >> np.uint64(31))


def _header(n_puts: int, max_key: int, max_val: int, put_size: int, data_end: int, file_id: int,
            block_size: int, n_deletes: int = 0, delete_size: int = 0) -> bytes:
    h = LogHeader(0, block_size, file_id)
    h.num_puts = n_puts
    h.num_deletes = n_deletes
    h.delete_size = delete_size
    h.max_key_len = max_key
    h.max_value_len = max_val
    h.put_size = put_size
    h.data_end = data_end
    h.max_entries_per_block = 1
    return h.to_bytes()


def fixed_log_range(n: int, lo: int, hi: int, key_len: int = 16, value_len: int = 100, seed: int = 1,
                    file_id: int = 0x5EED5EED, block_size: int = 0):
    """Bytes [lo, hi) of the fixed_log(n, ...) file, generated without the rest of the log (every
    byte is a function of its record index, so each rank of a sharded build makes only its range).
    Returns (84-byte header, uint8 array of hi - lo bytes)."""
    assert key_len >= 16 and key_len + 1 < 128 and value_len < 128
    rec = 2 + key_len + value_len
    total = LOG_HEADER_SIZE + n * rec
    hi = min(hi, total)
    lo = min(lo, hi)
    header = _header(n, key_len, value_len, n * rec, total, file_id, block_size)
    i0 = max(0, (lo - LOG_HEADER_SIZE) // rec)
    i1 = min(n, max(0, (hi - LOG_HEADER_SIZE + rec - 1) // rec))
    m = max(0, i1 - i0)
    body = np.empty((m, rec), dtype=np.uint8)
    i = np.arange(i0, i0 + m, dtype=np.uint64)
    body[:, 0] = key_len + 1
    body[:, 1] = value_len
    body[:, 2:10] = i.view(np.uint8).reshape(m, 8)
    body[:, 10:18] = splitmix64(i ^ np.uint64(seed)).view(np.uint8).reshape(m, 8)
    extra = (key_len - 16) + value_len  # remaining key bytes, then the value: splitmix64 words of (i, j)
    words = (extra + 7) // 8
    base = i * np.uint64(64) + np.uint64((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
    fill = splitmix64(base[:, None] + np.arange(words, dtype=np.uint64)[None, :])
    body[:, 18:] = fill.view(np.uint8).reshape(m, words * 8)[:, :extra]
    start = LOG_HEADER_SIZE + i0 * rec
    buf = np.empty(hi - lo, dtype=np.uint8)
    flat = body.reshape(-1)
    if lo < LOG_HEADER_SIZE:  # the header bytes
        k = min(hi, LOG_HEADER_SIZE) - lo
        buf[:k] = np.frombuffer(header, dtype=np.uint8)[lo: lo + k]
    a = max(lo, start)
    if hi > a:
        buf[a - lo: hi - lo] = flat[a - start: hi - start]
    return header, buf


def fixed_log(n: int, key_len: int = 16, value_len: int = 100, seed: int = 1, file_id: int = 0x5EED5EED,
              block_size: int = 0) -> np.ndarray:
    """n PUTs with fixed-size keys (>= 16 B) and values; returns the whole .spl as a uint8 array."""
    rec = 2 + key_len + value_len
    return fixed_log_range(n, 0, LOG_HEADER_SIZE + n * rec, key_len, value_len, seed, file_id, block_size)[1]


def mixed_log(n: int, min_key: int = 8, max_key: int = 64, value_len: int = 100, seed: int = 3,
              file_id: int = 0x5EED0003, block_size: int = 0) -> np.ndarray:
    """n PUTs, key length uniform in [min_key, max_key] (>= 8), fixed value length (< 128)."""
    assert min_key >= 8 and max_key + 1 < 128 and value_len < 128
    rng = np.random.default_rng(seed)
    klen = rng.integers(min_key, max_key + 1, size=n).astype(np.int64)
    rec = 2 + klen + value_len
    starts = np.empty(n, dtype=np.int64)
    starts[0] = 0
    np.cumsum(rec[:-1], out=starts[1:])
    total = int(rec.sum())
    buf = np.empty(LOG_HEADER_SIZE + total, dtype=np.uint8)
    body = buf[LOG_HEADER_SIZE:]
    body[:] = rng.integers(0, 256, size=total, dtype=np.uint8)
    body[starts] = (klen + 1).astype(np.uint8)
    body[starts + 1] = value_len
    idx = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)
    for b in range(8):
        body[starts + 2 + b] = idx[:, b]
    put_size = total
    buf[:LOG_HEADER_SIZE] = np.frombuffer(
        _header(n, int(klen.max()) if n else 0, value_len if n else 0, put_size, LOG_HEADER_SIZE + total, file_id,
                block_size), dtype=np.uint8)
    return buf


def key_value_log(n: int, file_id: int = 0x0C1C1C1C, block_size: int = 1024) -> bytes:
    """WriteHashBenchmark's data: put("key_" + i, "value_" + i), NONE, block size 1024."""
    parts = []
    max_k = max_v = 0
    put_size = 0
    for i in range(n):
        k = b"key_%d" % i
        v = b"value_%d" % i
        rec = vlq_bytes(len(k) + 1) + vlq_bytes(len(v)) + k + v
        parts.append(rec)
        max_k = max(max_k, len(k))
        max_v = max(max_v, len(v))
        put_size += len(rec)
    body = b"".join(parts)
    return _header(n, max_k, max_v, put_size, LOG_HEADER_SIZE + len(body), file_id, block_size) + body


def key_value_log_np(n: int, file_id: int = 0x0C1C1C1C, block_size: int = 1024) -> np.ndarray:
    """key_value_log(n) built with numpy (the same bytes, fast at WriteHashBenchmark's 10M): records with
    the same number of decimal digits in i have one size, so each digit-count group is one 2-D array."""
    parts = [np.frombuffer(b"", dtype=np.uint8)]
    put_size = max_k = max_v = 0
    lo, d = 0, 1
    while lo < n:
        hi = min(n, 10 ** d)
        m = hi - lo
        kl, vl = 4 + d, 6 + d
        rec = np.empty((m, 2 + kl + vl), dtype=np.uint8)
        rec[:, 0] = kl + 1
        rec[:, 1] = vl
        i = np.arange(lo, hi, dtype=np.int64)
        digits = np.empty((m, d), dtype=np.uint8)
        x = i.copy()
        for k in range(d - 1, -1, -1):
            digits[:, k] = (x % 10 + 48).astype(np.uint8)
            x //= 10
        rec[:, 2:6] = np.frombuffer(b"key_", dtype=np.uint8)
        rec[:, 6:6 + d] = digits
        rec[:, 6 + d:12 + d] = np.frombuffer(b"value_", dtype=np.uint8)
        rec[:, 12 + d:] = digits
        parts.append(rec.reshape(-1))
        put_size += rec.size
        max_k, max_v = max(max_k, kl), max(max_v, vl)
        lo, d = hi, d + 1
    body = np.concatenate(parts)
    out = np.empty(LOG_HEADER_SIZE + body.size, dtype=np.uint8)
    out[:LOG_HEADER_SIZE] = np.frombuffer(_header(n, max_k, max_v, put_size, LOG_HEADER_SIZE + body.size, file_id,
                                                  block_size), dtype=np.uint8)
    out[LOG_HEADER_SIZE:] = body
    return out


def churn_log(n: int, pool: int, p_del: float, key_len: int = 16, value_len: int = 100, seed: int = 5,
              file_id: int = 0x5EED0005, block_size: int = 0) -> np.ndarray:
    """n records of C2 shape whose keys are drawn uniformly from `pool` keys (so later PUTs overwrite
    earlier ones); each record is a DELETE (0x00 VLQ(keyLen) key, UncompressedBlockOutput.java:80-87)
    with probability p_del.  Key j = LE64(j) || LE64(splitmix64(j ^ seed))."""
    assert key_len == 16 and value_len < 128
    rng = np.random.default_rng(seed)
    kidx = rng.integers(0, pool, size=n).astype(np.uint64)
    is_del = rng.random(n) < p_del
    rec = np.where(is_del, 2 + key_len, 2 + key_len + value_len).astype(np.int64)
    starts = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(rec[:-1], out=starts[1:])
    total = int(rec.sum())
    buf = np.empty(LOG_HEADER_SIZE + total, dtype=np.uint8)
    body = buf[LOG_HEADER_SIZE:]
    body[:] = np.frombuffer(rng.bytes(total), dtype=np.uint8)
    body[starts] = np.where(is_del, 0, key_len + 1).astype(np.uint8)
    body[starts + 1] = np.where(is_del, key_len, value_len).astype(np.uint8)
    key = np.concatenate([kidx.view(np.uint8).reshape(n, 8),
                          splitmix64(kidx ^ np.uint64(seed)).view(np.uint8).reshape(n, 8)], axis=1)
    for b in range(key_len):
        body[starts + 2 + b] = key[:, b]
    n_del = int(is_del.sum())
    put_size = int(rec[~is_del].sum())
    buf[:LOG_HEADER_SIZE] = np.frombuffer(
        _header(n - n_del, key_len, value_len if n > n_del else 0, put_size, LOG_HEADER_SIZE + total, file_id,
                block_size, n_del, total - put_size), dtype=np.uint8)
    return buf


def snappy_log(log: np.ndarray, rec: int, block_size: int, codec: str = "snappy") -> np.ndarray:
    """The SNAPPY log a reference writer produces for the same uniform R-byte PUT records (a NONE log
    from fixed_log): CompressedWriter.smartFlush (CompressedWriter.java:111-118) closes a block when
    the next record no longer fits, so every block holds block_size // R records; each block is
    VLQ(compressedSize) || the Snappy stream of its bytes (CompressedOutputStream.java:47-58), here from
    libsnappy through pyarrow.  codec="zstd": a ZSTD log, each block one Zstandard frame from libzstd at
    level 3 (CompressorType.java:42-56).  Records longer than the block size are not handled here."""
    import pyarrow as pa
    from .log_writer import vlq_bytes
    assert 10 <= rec <= block_size
    per = block_size // rec
    hdr = LogHeader.from_bytes(log[:LOG_HEADER_SIZE].tobytes())
    body = log[LOG_HEADER_SIZE:hdr.data_end]
    step = per * rec
    parts = []
    for o in range(0, body.size, step):
        comp = (pa.Codec("zstd", compression_level=3).compress(body[o:o + step], asbytes=True) if codec == "zstd"
                else pa.compress(body[o:o + step], codec="snappy", asbytes=True))
        parts.append(vlq_bytes(len(comp)))
        parts.append(comp)
    data = b"".join(parts)
    hdr.compression_type = 2 if codec == "zstd" else 1
    hdr.compression_block_size = block_size
    hdr.max_entries_per_block = per if body.size else 0
    hdr.data_end = LOG_HEADER_SIZE + len(data)
    out = np.empty(hdr.data_end, dtype=np.uint8)
    out[:LOG_HEADER_SIZE] = np.frombuffer(hdr.to_bytes(), dtype=np.uint8)
    out[LOG_HEADER_SIZE:] = np.frombuffer(data, dtype=np.uint8)
    return out
