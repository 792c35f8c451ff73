"""Test-input generator: SNAPPY- and ZSTD-compressed Sparkey logs, in memory.

Restates the reference's compressed append path so that a log built here has the block layout the
reference writes for the same puts/deletes, block size and file identifier:
  - CompressedWriter.put / delete / smartFlush (CompressedWriter.java:59-124): a record that does not
    fit is pushed to a fresh block when it is smaller than what is pending; a record that still spans
    blocks is followed by an extra flush so that every block starts at a record start;
  - CompressedOutputStream.write / flush (CompressedOutputStream.java:47-110): a block is flushed when
    the buffer fills, as VLQ(compressedSize) || compressed bytes;
  - CompressedWriter.afterFlush (CompressedWriter.java:45-49) and LogWriter.writeHeader
    (LogWriter.java:77-81): maxEntriesPerBlock = the most records started in one block.
The block bytes come from libsnappy through pyarrow (the C++ library snappy-java wraps); any valid
Snappy stream gives the same index, since the index depends only on the decompressed bytes and the
block boundaries.  codec="zstd" writes ZSTD logs: each block one Zstandard frame from libzstd at level 3
(pyarrow), what zstd-jni's Zstd.compress writes (CompressorType.java:42-56).  `literal_only=True` writes raw literal-only Snappy streams instead (the format's
simplest valid encoding), and `encoder=` accepts any callable bytes -> snappy bytes.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sparkey-java_amd"))

from sparkey.log_writer import LOG_HEADER_SIZE, CompressionType, LogHeader, vlq_bytes, vlq_size  # noqa: E402


def snappy_compress(data: bytes) -> bytes:
    import pyarrow as pa
    return pa.compress(data, codec="snappy", asbytes=True)


def snappy_literal_only(data: bytes) -> bytes:
    """A valid Snappy stream with literal elements only (format: varint length, tag 0b00 literals)."""
    out = bytearray(vlq_bytes(len(data)))
    i = 0
    while i < len(data):
        n = min(len(data) - i, 65536)
        if n <= 60:
            out.append((n - 1) << 2)
        elif n <= 256:
            out += bytes([60 << 2, n - 1])
        else:
            out += bytes([61 << 2, (n - 1) & 0xFF, (n - 1) >> 8])
        out += data[i:i + n]
        i += n
    return bytes(out)


def zstd_compress(data: bytes, level: int = 3) -> bytes:
    """One Zstandard frame, as zstd-jni's Zstd.compress at the reference's level 3
    (CompressorType.java:42-56); libzstd through pyarrow."""
    import pyarrow as pa
    return pa.Codec("zstd", compression_level=level).compress(data, asbytes=True)


def zstd_decompress(data: bytes) -> bytes:
    import pyarrow as pa
    return pa.CompressedInputStream(pa.BufferReader(data), "zstd").read()


def snappy_decompress(data: bytes, ulen: int) -> bytes:
    import pyarrow as pa
    return pa.decompress(data, ulen, codec="snappy", asbytes=True)


class CompressedLog:
    """LogWriter over a SNAPPY CompressedWriter, kept in memory; `finish()` returns the .spl bytes."""

    def __init__(self, block_size: int, file_identifier: int = 12345, literal_only: bool = False, encoder=None,
                 codec: str = "snappy"):
        if block_size < 10:  # CompressedOutputStream.java:33-35
            raise OSError("Too small block size - won't be able to fit keylen + valuelen in a single block")
        zstd = codec == "zstd"
        self.header = LogHeader(CompressionType.ZSTD if zstd else CompressionType.SNAPPY, block_size, file_identifier)
        self.block_size = block_size
        self.encoder = encoder or (zstd_compress if zstd else snappy_literal_only if literal_only else snappy_compress)
        self.out = bytearray()
        self.pending = bytearray()
        self.cur_entries = 0
        self.max_entries = 0
        self.flushed = False
        self.block_starts = []  # file offsets of the blocks (for tests)

    # CompressedOutputStream
    def _flush_block(self):
        if not self.pending:
            return
        comp = self.encoder(bytes(self.pending))
        self.block_starts.append(LOG_HEADER_SIZE + len(self.out))
        self.out += vlq_bytes(len(comp))
        self.out += comp
        self.pending = bytearray()
        self.max_entries = max(self.max_entries, self.cur_entries)  # afterFlush
        self.cur_entries = 0
        self.flushed = True

    def _write(self, b: bytes):
        off = 0
        while off < len(b):
            remaining = self.block_size - len(self.pending)
            take = len(b) - off
            if take < remaining:
                self.pending += b[off:]
                return
            self.pending += b[off:off + remaining]
            off += remaining
            self._flush_block()

    # CompressedWriter
    def _smart_flush(self, key_size: int, total_size: int):
        remaining = self.block_size - len(self.pending)
        if remaining < key_size:
            self._flush_block()
        elif remaining < total_size and total_size < self.block_size - remaining:
            self._flush_block()

    def _after_record(self):
        if self.flushed and self.pending:
            self._flush_block()

    def put(self, key: bytes, value: bytes):
        if isinstance(key, str):
            key = key.encode()
        if isinstance(value, str):
            value = value.encode()
        key_size = vlq_size(len(key) + 1) + vlq_size(len(value))
        self._smart_flush(key_size, key_size + len(key) + len(value))
        self.flushed = False
        self.cur_entries += 1
        self._write(vlq_bytes(len(key) + 1) + vlq_bytes(len(value)) + key + value)
        self._after_record()
        self.header.put(len(key), len(value))

    def delete(self, key: bytes):
        if isinstance(key, str):
            key = key.encode()
        if len(key) > self.header.max_key_len:  # LogWriter.java:110-115
            return
        key_size = 1 + vlq_size(len(key) + 1)
        self._smart_flush(key_size, key_size + len(key))
        self.flushed = False
        self.cur_entries += 1
        self._write(b"\x00" + vlq_bytes(len(key)) + key)
        self._after_record()
        self.header.delete(len(key))

    def finish(self) -> bytes:
        self._flush_block()
        self.header.max_entries_per_block = self.max_entries
        self.header.data_end = LOG_HEADER_SIZE + len(self.out)
        return self.header.to_bytes() + bytes(self.out)


def iterate_compressed(log: bytes):
    """Pure-Python restatement of SparkeyLogIterator over a compressed log (SparkeyLogIterator.java:
    86-138, CompressedReader.java:58-130): yields (is_put, key, position, entry_index, value_len) where
    position is the file offset of the block holding the record's first byte.  Small inputs only."""
    hdr = LogHeader.from_bytes(log)
    end = hdr.data_end
    p = LOG_HEADER_SIZE
    stream = bytearray()
    starts = []  # (uncompressed offset, file position)
    while p < end:
        clen, q = _vlq(log, p)
        raw = log[q:q + clen]
        starts.append((len(stream), p))
        if hdr.compression_type == CompressionType.ZSTD:
            stream += zstd_decompress(raw)
        else:
            ulen, _ = _vlq(raw, 0)
            stream += snappy_decompress(raw, ulen)
        p = q + clen
    starts.append((len(stream), end))
    u = 0
    prev = -1
    idx = 0
    bi = 0
    while u < len(stream):
        while starts[bi + 1][0] <= u:
            bi += 1
        pos = starts[bi][1]
        idx = idx + 1 if pos == prev else 0
        prev = pos
        first, u = _vlq(stream, u)
        second, u = _vlq(stream, u)
        if first == 0:
            key = bytes(stream[u:u + second])
            u += second
            yield (False, key, pos, idx, 0)
        else:
            key = bytes(stream[u:u + first - 1])
            u += first - 1 + second
            yield (True, key, pos, idx, second)


def _vlq(b, p):
    v = 0
    s = 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, p
