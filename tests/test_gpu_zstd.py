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
from helpers import same_error

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
    same_error(native, bytes(bad))
    bad = bytearray(log)
    struct.pack_into("<i", bad, 68, 16)                           # frames larger than the block size
    same_error(native, bytes(bad))
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
    same_error(native, bytes(bad))


@pytest.mark.parametrize("block_size", [1024, 16384])
@pytest.mark.parametrize("spacing", ["default", "min"])
def test_parallel_directory_zstd(native, block_size, spacing, switch, capfd):
    """The parallel block directory on ZSTD logs (frame magic as the screen) equals the serial chain."""
    from sparkey import synth
    log = synth.snappy_log(synth.fixed_log(20000, 16, 100, seed=block_size), 118, block_size, codec="zstd").tobytes()
    if spacing == "min":
        switch(snappy_dir_a=1)
    switch(snappy_dir_debug=1)
    got, _ = native.build_index_mem(log, native.make_opts(hash_seed=77))
    assert got == oracle.build_index(log, 77)
    assert "[zstd dir] parallel" in capfd.readouterr().err
    switch(snappy_serial_dir=1)
    serial, _ = native.build_index_mem(log, native.make_opts(hash_seed=77))
    assert got == serial


def _checksummed(data: bytes) -> bytes:
    """zstd_compress's frame with Content_Checksum set: FHD bit 2 and the low 32 bits of XXH64(data)
    appended (RFC 8878 §3.1.1), which libzstd verifies on decode."""
    import xxhash
    f = bytearray(zstd_compress(data))
    assert struct.unpack_from("<I", f, 0)[0] == 0xFD2FB528 and not f[4] & 4
    f[4] |= 4
    return bytes(f) + struct.pack("<I", xxhash.xxh64(data).intdigest() & 0xFFFFFFFF)


def _zlog_enc(ops, block_size, encoder):
    cl = CompressedLog(block_size, file_identifier=0x2468, codec="zstd", encoder=encoder)
    for op, k, v in ops:
        if op == "put":
            cl.put(k, v)
        else:
            cl.delete(k)
    return cl.finish()


def _frames(log: bytes):
    """(frame offset, frame length) of every block of a compressed log (VLQ size prefix per block)."""
    data_end = struct.unpack_from("<q", log, 32)[0]
    p, out = 84, []
    while p < data_end:
        n, shift = 0, 0
        while True:
            c = log[p]
            p += 1
            n |= (c & 0x7F) << shift
            shift += 7
            if c < 0x80:
                break
        out.append((p, n))
        p += n
    return out


def _same_outcome(native, log, seed=4321):
    """The GPU build and the oracle (libzstd) either both reject the log or build the same bytes."""
    try:
        want = oracle.build_index(log, seed)
    except oracle.OracleError:
        want = None
    opts = native.make_opts(hash_seed=seed)
    if want is None:
        with pytest.raises((OSError, RuntimeError)):
            native.build_index_mem(log, opts)
    else:
        got, _ = native.build_index_mem(log, opts)
        assert got == want
    return want is not None


@pytest.mark.parametrize("block_size", [512, 8192])
def test_checksummed_frames(native, block_size):
    """Frames carrying Content_Checksum build like the oracle; one flipped checksum byte is rejected
    (libzstd rejects it too)."""
    rng = random.Random(block_size + 3)
    ops = _ops(rng, 800, 10 ** 9, 0.1, 120)
    log = _zlog_enc(ops, block_size, _checksummed)
    check(native, log)
    frames = _frames(log)
    for off, n in (frames[0], frames[len(frames) // 2], frames[-1]):
        bad = bytearray(log)
        bad[off + n - 2] ^= 0x10                      # inside the 4 checksum bytes
        same_error(native, bytes(bad), 4321)


def test_skippable_frames(native):
    """A skippable frame after a block's frame is skipped; one whose size runs past the block (or wraps
    the 32-bit offset: 0xFFFFFFF8) is a corrupt log, not a hang."""
    rng = random.Random(21)
    ops = _ops(rng, 600, 10 ** 9, 0.0, 100)
    good = _zlog_enc(ops, 1024, lambda d: zstd_compress(d) + struct.pack("<II", 0x184D2A53, 3) + b"abc")
    check(native, good)
    for size in (0xFFFFFFF8, 0xFFFFFFFF, 4):
        bad = _zlog_enc(ops, 1024, lambda d, s=size: zstd_compress(d) + struct.pack("<II", 0x184D2A50, s))
        same_error(native, bad, 4321)


def test_byte_flips_inside_frames(native):
    """Single flipped bytes at random positions inside frames: the GPU build rejects exactly the logs
    the oracle (libzstd) rejects, and otherwise builds the oracle's bytes."""
    rng = random.Random(77)
    ops = []
    for i in range(1500):
        v = (b"value-%d-" % (i % 23)) * rng.randrange(1, 12) + rng.randbytes(rng.randrange(0, 40))
        ops.append(("put", b"key_%d" % rng.randrange(1200), v))
    log = _zlog(ops, 4096, level=9)
    frames = _frames(log)
    ok = 0
    for t in range(40):
        off, n = frames[rng.randrange(len(frames))]
        pos = off + rng.randrange(n)
        bad = bytearray(log)
        bad[pos] ^= 1 << rng.randrange(8)
        ok += _same_outcome(native, bytes(bad))
    assert ok < 40  # (most flips break the stream; the point is that both sides agree)
