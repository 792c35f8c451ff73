"""ctypes wrapper for the CPU oracle (oracle/sparkey_oracle.c).

TEST INFRASTRUCTURE ONLY: a sequential restatement of spotify/sparkey-java's
IndexHash.createNew (src/main/java/com/spotify/sparkey/IndexHash.java:131-678).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker.  The product (sparkey-java_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsparkey_oracle.so")
_lib = None

IN_MEMORY = 1
SORTING = 2
AUTO = 0


def zstd_decompress(data: bytes) -> bytes:
    """One ZSTD block through libzstd (pyarrow's bundled copy; zstd-jni wraps the same library,
    CompressorType.java:42-56).  Streaming, so frames without a content size decode too."""
    import pyarrow as pa
    return pa.CompressedInputStream(pa.BufferReader(data), "zstd").read()


_DECODER = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64)


def _zstd_block(src, n, dst, cap):
    try:
        out = zstd_decompress(ctypes.string_at(src, n))
    except Exception:
        return -1
    if len(out) > cap:
        return -1
    ctypes.memmove(dst, out, len(out))
    return len(out)


_zstd_cb = _DECODER(_zstd_block)


def build() -> str:
    """Compiles the oracle with gcc (make); returns the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.oracle_murmur3_x86_32.argtypes = [u8p, ctypes.c_int32, ctypes.c_int32]
        L.oracle_murmur3_x86_32.restype = ctypes.c_uint32
        L.oracle_murmur3_x64_64.argtypes = [u8p, ctypes.c_int32, ctypes.c_int32]
        L.oracle_murmur3_x64_64.restype = ctypes.c_uint64
        L.oracle_hash.argtypes = [ctypes.c_int32, u8p, ctypes.c_int32, ctypes.c_int32]
        L.oracle_hash.restype = ctypes.c_uint64
        L.oracle_vlq_size.argtypes = [ctypes.c_int64]
        L.oracle_vlq_size.restype = ctypes.c_int32
        L.oracle_vlq_write.argtypes = [ctypes.c_uint64, u8p]
        L.oracle_vlq_write.restype = ctypes.c_int32
        L.oracle_vlq_read.argtypes = [u8p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_int32)]
        L.oracle_vlq_read.restype = ctypes.c_int32
        L.oracle_log_new.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.oracle_log_new.restype = ctypes.c_void_p
        L.oracle_log_put.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int32, u8p, ctypes.c_int64]
        L.oracle_log_put.restype = ctypes.c_int32
        L.oracle_log_delete.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int32]
        L.oracle_log_delete.restype = ctypes.c_int32
        L.oracle_log_size.argtypes = [ctypes.c_void_p]
        L.oracle_log_size.restype = ctypes.c_int64
        L.oracle_log_finish.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int64]
        L.oracle_log_finish.restype = ctypes.c_int64
        L.oracle_log_free.argtypes = [ctypes.c_void_p]
        L.oracle_log_free.restype = None
        L.oracle_index_size.argtypes = [u8p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double]
        L.oracle_index_size.restype = ctypes.c_int64
        L.oracle_build_index.argtypes = [u8p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, u8p,
                                         ctypes.c_int64, ctypes.c_char_p, ctypes.c_int32]
        L.oracle_build_index.restype = ctypes.c_int64
        L.oracle_snappy_uncompress.argtypes = [u8p, ctypes.c_int64, u8p, ctypes.c_int64]
        L.oracle_snappy_uncompress.restype = ctypes.c_int64
        L.oracle_get.argtypes = [u8p, ctypes.c_int64, u8p, ctypes.c_int64, u8p, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.oracle_get.restype = ctypes.c_int32
        L.oracle_set_zstd_decoder.argtypes = [_DECODER]
        L.oracle_set_zstd_decoder.restype = None
        L.oracle_set_zstd_decoder(_zstd_cb)
        _lib = L
    return _lib


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else ctypes.c_char_p(b"\0")


def murmur3_x86_32(data: bytes, seed: int) -> int:
    return lib().oracle_murmur3_x86_32(_buf(data), len(data), ctypes.c_int32(seed).value)


def murmur3_x64_64(data: bytes, seed: int) -> int:
    return lib().oracle_murmur3_x64_64(_buf(data), len(data), ctypes.c_int32(seed).value)


def key_hash(hash_size: int, data: bytes, seed: int) -> int:
    return lib().oracle_hash(hash_size, _buf(data), len(data), ctypes.c_int32(seed).value)


def vlq_size(v: int) -> int:
    return lib().oracle_vlq_size(v)


def vlq_write(v: int) -> bytes:
    out = ctypes.create_string_buffer(16)
    n = lib().oracle_vlq_write(v, out)
    return out.raw[:n]


def vlq_read(data: bytes, pos: int = 0):
    """Returns (rc, value, new_pos)."""
    p = ctypes.c_int64(pos)
    v = ctypes.c_int32(0)
    rc = lib().oracle_vlq_read(_buf(data), len(data), ctypes.byref(p), ctypes.byref(v))
    return rc, v.value, p.value


class LogBuilder:
    """LogWriter restatement (append path): produces .spl bytes identical to the reference's."""

    def __init__(self, file_identifier: int = 0x12345678, compression_block_size: int = 0):
        self._h = lib().oracle_log_new(ctypes.c_int32(file_identifier).value, compression_block_size)

    def put(self, key: bytes, value: bytes) -> None:
        rc = lib().oracle_log_put(self._h, _buf(key), len(key), _buf(value), len(value))
        assert rc == 0, rc

    def delete(self, key: bytes) -> None:
        rc = lib().oracle_log_delete(self._h, _buf(key), len(key))
        assert rc == 0, rc

    def finish(self) -> bytes:
        n = lib().oracle_log_finish(self._h, None, 0)
        out = ctypes.create_string_buffer(n)
        lib().oracle_log_finish(self._h, out, n)
        return out.raw

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_log_free(self._h)
            self._h = None


class OracleError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


def _log_arg(log):
    """bytes, or a contiguous uint8 numpy array (large logs without a copy)."""
    if hasattr(log, "ctypes") and hasattr(log, "nbytes"):
        return ctypes.c_void_p(log.ctypes.data), int(log.nbytes)
    return log, len(log)


def index_size(log, hash_size: int = 0, sparsity: float = 0.0) -> int:
    p, n = _log_arg(log)
    return lib().oracle_index_size(p, n, hash_size, sparsity)


def build_index(log: bytes, hash_seed: int, hash_size: int = 0, sparsity: float = 0.0,
                method: int = IN_MEMORY, max_memory: int = 1 << 62) -> bytes:
    """IndexHash.createNew restated; returns the .spi bytes."""
    n = index_size(log, hash_size, sparsity)
    if n < 0:
        raise OracleError(n, "index_size failed")
    out = ctypes.create_string_buffer(n)
    err = ctypes.create_string_buffer(256)
    lp, ln = _log_arg(log)
    rc = lib().oracle_build_index(lp, ln, hash_size, sparsity, ctypes.c_int32(hash_seed).value,
                                  method, max_memory, out, n, err, 256)
    if rc < 0:
        raise OracleError(rc, err.value.decode())
    return out.raw


def snappy_uncompress(data: bytes, cap: int) -> bytes:
    """Snappy raw-format decompression restated (CompressorType.java:32-34)."""
    out = ctypes.create_string_buffer(max(cap, 1))
    rc = lib().oracle_snappy_uncompress(data, len(data), out, cap)
    if rc < 0:
        raise OracleError(rc, "snappy uncompress failed")
    return out.raw[:rc]


def get(index: bytes, log: bytes, key: bytes):
    """IndexHash.get restated; returns the value bytes or None."""
    off = ctypes.c_int64(0)
    ln = ctypes.c_int64(0)
    rc = lib().oracle_get(index, len(index), log, len(log), _buf(key), len(key), ctypes.byref(off),
                          ctypes.byref(ln))
    if rc < 0:
        raise OracleError(rc, "get failed")
    if rc == 0:
        return None
    return log[off.value:off.value + ln.value]
