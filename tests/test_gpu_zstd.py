"""GPU parity for ZSTD logs: the HIP Zstandard front end (block directory from
each frame's Frame_Content_Size, wave-per-block RFC 8878 decode into the virtual log) plus the SNAPPY
path's record walk, build and address rewrite must give .spi bytes identical to the oracle's (libzstd
block decode, CompressedReader block positions, entryIndex addresses; pinned in
test_compressed_oracle.py).  Bit-exact, IN_MEMORY and SORTING, block sizes 10 B - 128 KiB (blocks up
to ~64 KiB decode in LDS, larger ones in global memory).
"""
import random
import struct

import pytest

import oracle

from snappy_log import CompressedLog, zstd_compress
from test_compressed_oracle import _compressed, _ops
from test_gpu_compressed import check

pytestmark = pytest.mark.gpu

IN_MEMORY, SORTING = 1, 2


def _zlog(ops, block_size, level=3):
    cl = CompressedLog(block_size, file_identifier=0x2468, codec="zstd",
                       encoder=None if level == 3 else (lambda d: zstd_compress(d, level)))
    for op, k, v in ops:
        if op == "put":
            cl.put(k, v)
        else:
            cl.delete(k)
    return cl.finish()


@pytest.mark.parametrize("block_size", [10, 16, 100, 1024, 4096, 65536, 131072])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_unique_puts(native, block_size, method):
    rng = random.Random(block_size + 7)
    check(native, _compressed(_ops(rng, 1500, 10 ** 9, 0.0, 200), block_size, codec="zstd"), method=method)


@pytest.mark.parametrize("block_size", [10, 300, 1024, 8192])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_overwrites_and_deletes(native, block_size, method):
    rng = random.Random(block_size + 1)
    check(native, _compressed(_ops(rng, 3000, 800, 0.2, 120), block_size, codec="zstd"), method=method)


def test_spanning_records(native):
    rng = random.Random(3)
    check(native, _compressed(_ops(rng, 400, 10 ** 9, 0.0, 5000), 512, codec="zstd"))


def test_empty_and_single(native):
    check(native, CompressedLog(1024, codec="zstd").finish())
    cl = CompressedLog(1024, codec="zstd")
    cl.put(b"k", b"v")
    check(native, cl.finish())


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
@pytest.mark.parametrize("block_size", [4096, 65536, 131072])
def test_levels(native, level, block_size):
    """Other levels choose other block types and table modes (raw / RLE / Huffman 1 and 4 streams,
    treeless literals, predefined / RLE / FSE / repeated sequence tables, repeat offsets)."""
    rng = random.Random(level * 7 + block_size)
    ops = []
    for i in range(4000):
        kind = i % 4
        if kind == 0:
            v = bytes([rng.randrange(256)]) * rng.randrange(1, 400)          # runs: RLE / long matches
        elif kind == 1:
            v = rng.randbytes(rng.randrange(0, 300))                         # incompressible
        elif kind == 2:
            v = (b"value-%d-" % (i % 37)) * rng.randrange(1, 20)             # short periods, rep offsets
        else:
            v = bytes(rng.choice(b"ACGT") for _ in range(rng.randrange(0, 200)))  # skewed literals
        ops.append(("put", b"key_%d" % rng.randrange(3000), v))
        if rng.random() < 0.05:
            ops.append(("del", b"key_%d" % rng.randrange(3000), b""))
    check(native, _zlog(ops, block_size, level))


@pytest.mark.parametrize("hash_size", [0, 8])
def test_c2_shaped(native, hash_size):
    """C2's record shape (16 B keys, 100 B values), 200K records, 64 KiB blocks."""
    rng = random.Random(9)
    cl = CompressedLog(65536, file_identifier=5, codec="zstd")
    for i in range(200000):
        cl.put(struct.pack("<QQ", i, rng.getrandbits(64)), bytes([i & 0xFF]) * 60 + rng.randbytes(40))
    check(native, cl.finish(), seed=99, hash_size=hash_size)


def test_many_small_blocks(native):
    rng = random.Random(12)
    check(native, _compressed(_ops(rng, 6000, 10 ** 9, 0.0, 40), 12, codec="zstd"))


@pytest.mark.parametrize("delta", [-1000, 0, 5000])
def test_header_put_size_misstated(native, delta):
    rng = random.Random(11)
    log = bytearray(_compressed(_ops(rng, 1200, 10 ** 9, 0.1, 150), 700, codec="zstd"))
    put_size = struct.unpack_from("<q", log, 72)[0]
    struct.pack_into("<q", log, 72, max(0, put_size + delta))
    check(native, bytes(log))


def _streamed_frame(data: bytes) -> bytes:
    """A frame from libzstd's streaming API: no Frame_Content_Size (not what zstd-jni's
    compressByteArray writes)."""
    import pyarrow as pa
    sink = pa.BufferOutputStream()
    with pa.CompressedOutputStream(sink, "zstd") as z:
        z.write(data)
    return sink.getvalue().to_pybytes()


def test_errors(native):
    opts = native.make_opts(hash_seed=1)
    ops = [("put", b"k%d" % i, b"v" * 50) for i in range(200)]
    log = _compressed(ops, 256, codec="zstd")
    bad = bytearray(log)
    bad[84 + 1] ^= 0x01                                           # first frame's magic
    with pytest.raises(OSError):
        native.build_index_mem(bytes(bad), opts)
    bad = bytearray(log)
    struct.pack_into("<i", bad, 68, 16)                           # frames larger than the block size
    with pytest.raises(OSError):
        native.build_index_mem(bytes(bad), opts)
    cl = CompressedLog(256, codec="zstd", encoder=_streamed_frame)
    for _, k, v in ops:
        cl.put(k, v)
    with pytest.raises(OSError, match="content size"):
        native.build_index_mem(cl.finish(), opts)
    # a truncated frame: the last block's frame loses its final byte (dataEnd moves with it)
    bad = bytearray(log[:-1])
    struct.pack_into("<q", bad, 32, len(bad))
    p = 84
    while True:                                                   # the last block's VLQ
        n, q = 0, p
        shift = 0
        while True:
            c = bad[q]
            q += 1
            n |= (c & 0x7F) << shift
            shift += 7
            if c < 0x80:
                break
        if q + n >= len(bad):
            break
        p = q + n
    assert n < 128
    bad[p] = n - 1
    with pytest.raises(OSError):
        native.build_index_mem(bytes(bad), opts)


@pytest.mark.parametrize("block_size", [1024, 16384])
@pytest.mark.parametrize("spacing", ["default", "min"])
def test_parallel_directory_zstd(native, block_size, spacing, monkeypatch, capfd):
    """The parallel block directory on ZSTD logs (frame magic as the screen) equals the serial chain."""
    from sparkey import synth
    log = synth.snappy_log(synth.fixed_log(20000, 16, 100, seed=block_size), 118, block_size, codec="zstd").tobytes()
    if spacing == "min":
        monkeypatch.setenv("SPARKEY_SNAPPY_DIR_A", "1")
    monkeypatch.setenv("SPARKEY_SNAPPY_DIR_DEBUG", "1")
    got, _ = native.build_index_mem(log, native.make_opts(hash_seed=77))
    assert got == oracle.build_index(log, 77)
    assert "[zstd dir] parallel" in capfd.readouterr().err
    monkeypatch.setenv("SPARKEY_SNAPPY_SERIAL_DIR", "1")
    serial, _ = native.build_index_mem(log, native.make_opts(hash_seed=77))
    assert got == serial
