"""The append path that produces the hash build's input: a Sparkey log (.spl), NONE compression.

Restates LogWriter (LogWriter.java:22-115), LogHeader (LogHeader.java:55-172) and
UncompressedBlockOutput (UncompressedBlockOutput.java:67-106) so that logs written here are byte
for byte what the reference writes for the same puts/deletes and file identifier.
"""
from __future__ import annotations

import os
import random
import struct

LOG_MAGIC = 0x49B39C95
LOG_HEADER_SIZE = 84
_HDR = struct.Struct("<IIIiqqqqqqiiqi")  # LogHeader.java:90-115 field order
assert _HDR.size == LOG_HEADER_SIZE


class CompressionType:
    NONE = 0
    SNAPPY = 1
    ZSTD = 2


def vlq_size(value: int) -> int:
    """Util.unsignedVLQSize (Util.java:86-128)."""
    n = 1
    while n < 9 and value >= 1 << (7 * n):
        n += 1
    return n


def vlq_bytes(value: int) -> bytes:
    """Util.writeUnsignedVLQ (Util.java:130-144)."""
    out = bytearray()
    while value >= 0x80:
        out.append((value & 0x7F) | 0x80)
        value >>= 7
    out.append(value)
    return bytes(out)


class LogHeader:
    def __init__(self, compression_type=CompressionType.NONE, compression_block_size=0, file_identifier=None):
        self.major_version = 1
        self.minor_version = 0
        self.file_identifier = random.getrandbits(31) if file_identifier is None else file_identifier
        self.num_puts = 0
        self.num_deletes = 0
        self.data_end = LOG_HEADER_SIZE
        self.max_key_len = 0
        self.max_value_len = 0
        self.delete_size = 0
        self.compression_type = compression_type
        self.compression_block_size = compression_block_size
        self.put_size = 0
        self.max_entries_per_block = 0

    def to_bytes(self) -> bytes:
        fid = self.file_identifier & 0xFFFFFFFF
        fid = fid - (1 << 32) if fid >= 1 << 31 else fid
        return _HDR.pack(LOG_MAGIC, self.major_version, self.minor_version, fid, self.num_puts, self.num_deletes,
                         self.data_end, self.max_key_len, self.max_value_len, self.delete_size, self.compression_type,
                         self.compression_block_size, self.put_size, self.max_entries_per_block)

    @classmethod
    def from_bytes(cls, b: bytes) -> "LogHeader":
        f = _HDR.unpack(b[:LOG_HEADER_SIZE])
        if f[0] != LOG_MAGIC:
            raise OSError("File is not a Sparkey log file")
        h = cls.__new__(cls)
        (_, h.major_version, h.minor_version, h.file_identifier, h.num_puts, h.num_deletes, h.data_end, h.max_key_len,
         h.max_value_len, h.delete_size, h.compression_type, h.compression_block_size, h.put_size,
         h.max_entries_per_block) = f
        return h

    def put(self, key_len: int, value_len: int) -> None:  # LogHeader.java:161-166
        self.num_puts += 1
        self.max_key_len = max(self.max_key_len, key_len)
        self.max_value_len = max(self.max_value_len, value_len)
        self.put_size += vlq_size(key_len + 1) + vlq_size(value_len) + key_len + value_len

    def delete(self, key_len: int) -> None:  # LogHeader.java:168-172
        self.num_deletes += 1
        self.delete_size += 1 + vlq_size(key_len) + key_len


class LogWriter:
    """Append-only writer of .spl files (only CompressionType.NONE is produced here)."""

    _BUF = 1 << 20

    def __init__(self, path: str, header: LogHeader):
        self.path = path
        self.header = header
        self._buf = bytearray()
        self.closed = False

    @classmethod
    def createNew(cls, path: str, compression_type=CompressionType.NONE, compression_block_size=0,
                  file_identifier=None) -> "LogWriter":
        if compression_type != CompressionType.NONE:
            raise ValueError("only CompressionType.NONE logs are produced by this writer")
        h = LogHeader(compression_type, compression_block_size, file_identifier)
        with open(path, "wb") as f:  # LogWriter.java:27-31: header first, then records
            f.write(h.to_bytes())
        return cls(path, h)

    @classmethod
    def openExisting(cls, path: str) -> "LogWriter":
        """LogWriter(File) (LogWriter.java:33-61): header read, file truncated to dataEnd.  A SNAPPY or
        ZSTD log opens build-only: its header (maxEntriesPerBlock included) is kept as it is, and
        put/delete raise, since this mirror writes no compressed blocks."""
        with open(path, "rb") as f:
            h = LogHeader.from_bytes(f.read(LOG_HEADER_SIZE))
        with open(path, "r+b") as f:  # LogWriter.java:45-55: truncate to dataEnd
            f.truncate(h.data_end)
        return cls(path, h)

    def _check_appendable(self) -> None:
        if self.header.compression_type != CompressionType.NONE:
            raise NotImplementedError("appending to a compressed log is not supported by this writer "
                                      "(only CompressionType.NONE records are produced)")

    def put(self, key: bytes, value: bytes) -> None:
        self._check_appendable()
        if isinstance(key, str):
            key = key.encode("utf-8")
        if isinstance(value, str):
            value = value.encode("utf-8")
        self._buf += vlq_bytes(len(key) + 1)
        self._buf += vlq_bytes(len(value))
        self._buf += key
        self._buf += value
        self.header.put(len(key), len(value))
        if len(self._buf) >= self._BUF:
            self._drain()

    def delete(self, key: bytes) -> None:
        self._check_appendable()
        if isinstance(key, str):
            key = key.encode("utf-8")
        if len(key) > self.header.max_key_len:  # LogWriter.java:110-115
            return
        self._buf += b"\x00"
        self._buf += vlq_bytes(len(key))
        self._buf += key
        self.header.delete(len(key))
        if len(self._buf) >= self._BUF:
            self._drain()

    def _drain(self) -> None:
        if self._buf:
            with open(self.path, "ab") as f:
                f.write(self._buf)
            self._buf = bytearray()

    def flush(self, fsync: bool = False) -> None:
        """LogWriter.flush (LogWriter.java:71-80): data, then the header with dataEnd = file length."""
        self._drain()
        if self.header.compression_type != CompressionType.NONE:
            # nothing was appended (put/delete raise): CompressedWriter keeps maxEntriesPerBlock and
            # the file ends at dataEnd, so the header the reference rewrites is the same bytes
            if fsync:
                with open(self.path, "r+b") as f:
                    os.fsync(f.fileno())
            return
        self.header.max_entries_per_block = 1  # UncompressedBlockOutput.getMaxEntriesPerBlock
        self.header.data_end = os.path.getsize(self.path)
        with open(self.path, "r+b") as f:
            f.seek(0)
            f.write(self.header.to_bytes())
            if fsync:
                f.flush()
                os.fsync(f.fileno())

    def close(self, fsync: bool = False) -> None:
        if self.closed:
            return
        self.closed = True
        self.flush(fsync)
