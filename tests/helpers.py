"""Shared scenario builders and comparison helpers for the parity tests.

Logs are produced by the oracle's LogWriter restatement (byte-identical to the reference's
LogWriter), expected .spi bytes by the oracle's sequential IndexHash restatement.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle

HDR_FIELDS = [("magic", 0, "<I"), ("major", 4, "<I"), ("minor", 8, "<I"), ("fileId", 12, "<i"),
              ("hashSeed", 16, "<i"), ("dataEnd", 20, "<q"), ("maxKeyLen", 28, "<q"), ("maxValueLen", 36, "<q"),
              ("numPuts", 44, "<q"), ("garbageSize", 52, "<q"), ("numEntries", 60, "<q"), ("addressSize", 68, "<i"),
              ("hashSize", 72, "<i"), ("capacity", 76, "<q"), ("maxDisplacement", 84, "<q"),
              ("entryBlockBits", 92, "<i"), ("hashCollisions", 96, "<q"), ("totalDisplacement", 104, "<q")]


def index_header(spi: bytes) -> dict:
    return {name: struct.unpack_from(fmt, spi, off)[0] for name, off, fmt in HDR_FIELDS}


def diff_report(got: bytes, want: bytes) -> str:
    if len(got) != len(want):
        return f"length {len(got)} != {len(want)}"
    hg, hw = index_header(got), index_header(want)
    lines = [f"{k}: got {hg[k]} want {hw[k]}" for k in hg if hg[k] != hw[k]]
    slot = hw["hashSize"] + hw["addressSize"]
    a = np.frombuffer(got[112:], dtype=np.uint8).reshape(-1, slot)
    b = np.frombuffer(want[112:], dtype=np.uint8).reshape(-1, slot)
    bad = np.nonzero((a != b).any(axis=1))[0]
    if len(bad):
        lines.append(f"{len(bad)} slots differ, first {bad[:8].tolist()}")
        s = int(bad[0])
        lines.append(f"slot {s}: got {a[s].tobytes().hex()} want {b[s].tobytes().hex()}")
    return "; ".join(lines) or "identical"


def make_log(puts=(), deletes=(), ops=None, file_id=0x1234567, block_size=0) -> bytes:
    lb = oracle.LogBuilder(file_id, block_size)
    if ops is not None:
        for op, k, v in ops:
            if op == "put":
                lb.put(k, v)
            else:
                lb.delete(k)
    else:
        for k, v in puts:
            lb.put(k, v)
        for k in deletes:
            lb.delete(k)
    return lb.finish()


def key_value_puts(n, kfmt=b"Key%d", vfmt=b"Value%d"):
    return [(kfmt % i, vfmt % i) for i in range(n)]


def random_puts(n, seed=0, kmin=1, kmax=40, vmin=0, vmax=60, unique=True):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kl = int(rng.integers(kmin, kmax + 1))
        key = rng.integers(0, 256, size=kl, dtype=np.uint8).tobytes()
        if unique:
            key = struct.pack("<I", i)[:min(4, kl)] + key[min(4, kl):] if kl >= 4 else key
        vl = int(rng.integers(vmin, vmax + 1))
        out.append((key, rng.integers(0, 256, size=vl, dtype=np.uint8).tobytes()))
    if unique:
        seen = set()
        res = []
        for k, v in out:
            if k not in seen:
                seen.add(k)
                res.append((k, v))
        out = res
    return out


# The reference's exception class per error code (include/sparkey_gpu.h; the JNI shim's mapping)
_RUNTIME = {-5, -6, -10, -13}
_ILLEGAL = {-11, -12}


def java_class(code: int) -> str:
    return "RuntimeException" if code in _RUNTIME else "IllegalArgumentException" if code in _ILLEGAL else "IOException"


def same_error(native, log: bytes, seed: int = 1, **opts_kw):
    """The oracle rejects the log and the GPU build rejects it with the same Java exception class."""
    import oracle
    try:
        oracle.build_index(log, seed, **{k: v for k, v in opts_kw.items() if k in ("hash_size", "method")})
    except oracle.OracleError as e:
        want = e.code
    else:
        raise AssertionError("the oracle accepts the log")
    try:
        native.build_index_mem(log, native.make_opts(hash_seed=seed, **opts_kw))
    except (OSError, RuntimeError, ValueError) as e:
        got = getattr(e, "code", None)
    else:
        raise AssertionError("the GPU build accepts a log the oracle rejects (code %d)" % want)
    assert java_class(got) == java_class(want), (got, want)
    return got, want


def with_trailing_bytes(log: bytes, tail: bytes) -> bytes:
    """The log with `tail` appended and dataEnd moved to the file's end: the iterator then reads `tail`
    as the start of one more record."""
    out = bytearray(log) + tail
    struct.pack_into("<q", out, 32, len(out))
    return bytes(out)
