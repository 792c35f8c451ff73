"""GPU parity for SNAPPY logs: the HIP front end (block directory, wave-per-block
Snappy decode, record walk, address rewrite) plus the normal build must give .spi bytes identical to
the oracle's restatement (CompressedReader block positions, entryIndex addresses; pinned in
test_compressed_oracle.py).  Bit-exact, IN_MEMORY and SORTING.
"""
import random
import struct

import pytest

import oracle
from helpers import same_error
from snappy_log import CompressedLog
from test_compressed_oracle import _compressed, _ops

pytestmark = pytest.mark.gpu

IN_MEMORY, SORTING = 1, 2


def check(native, log, seed=4321, method=IN_MEMORY, hash_size=0):
    want = oracle.build_index(log, seed, hash_size=hash_size, method=method)
    opts = native.make_opts(hash_size=hash_size, hash_seed=seed, method=method)
    got, _ = native.build_index_mem(log, opts)
    assert got == want, "first differing byte %d of %d" % (
        next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), -1), len(want))
    return got


@pytest.mark.parametrize("block_size", [10, 16, 100, 1024, 4096, 65536, 131072])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_unique_puts(native, block_size, method):
    rng = random.Random(block_size)
    check(native, _compressed(_ops(rng, 1500, 10 ** 9, 0.0, 200), block_size), method=method)


@pytest.mark.parametrize("block_size", [10, 300, 1024, 8192])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_overwrites_and_deletes(native, block_size, method):
    rng = random.Random(block_size + 1)
    check(native, _compressed(_ops(rng, 3000, 800, 0.2, 120), block_size), method=method)


@pytest.mark.parametrize("literal_only", [False, True])
def test_spanning_records(native, literal_only):
    rng = random.Random(3)
    log = _compressed(_ops(rng, 400, 10 ** 9, 0.0, 5000), 512, literal_only=literal_only)
    check(native, log)


@pytest.mark.parametrize("hash_size", [4, 8])
def test_write_hash_benchmark_snappy(native, hash_size):
    cl = CompressedLog(1024, file_identifier=77)
    for i in range(1000):
        cl.put(b"key_%d" % i, b"value_%d" % i)
    check(native, cl.finish(), seed=1234, hash_size=hash_size)


def test_empty_and_single(native):
    check(native, CompressedLog(1024).finish())
    cl = CompressedLog(1024)
    cl.put(b"k", b"v")
    check(native, cl.finish())


@pytest.mark.parametrize("hash_size", [0, 8])
def test_c2_shaped(native, hash_size):
    """C2's record shape (16 B keys, 100 B values), 200K records, 64 KiB blocks (8-byte addresses;
    hash_size 8 takes the rewrite's 16-byte slot path)."""
    rng = random.Random(9)
    cl = CompressedLog(65536, file_identifier=5)
    for i in range(200000):
        cl.put(struct.pack("<QQ", i, rng.getrandbits(64)), bytes([i & 0xFF]) * 60 + rng.randbytes(40))
    check(native, cl.finish(), seed=99, hash_size=hash_size)


def test_errors(native):
    """Corrupt blocks fail inside the reference's iterator (CompressedReader.fetchBlock), so they are
    RuntimeExceptions there; the GPU build must raise the class the oracle's code maps to."""
    log = _compressed([("put", b"k%d" % i, b"v" * 50) for i in range(200)], 256)
    bad = bytearray(log)
    bad[64] = 2                                                   # ZSTD
    same_error(native, bytes(bad))
    bad = bytearray(log)
    bad[84] = 0xFF                                                # block size VLQ runs on / past dataEnd
    bad[85] = 0xFF
    same_error(native, bytes(bad))
    bad = bytearray(log)
    struct.pack_into("<i", bad, 68, 16)                           # blocks larger than the block size
    same_error(native, bytes(bad))


@pytest.mark.parametrize("delta", [-1000, -1, 0, 5000])
def test_header_put_size_misstated(native, delta):
    """The virtual log is sized from putSize + deleteSize; a header that understates them takes the
    directory-only pass first (the reference never reads putSize here)."""
    rng = random.Random(11)
    log = bytearray(_compressed(_ops(rng, 1200, 10 ** 9, 0.1, 150), 700))
    put_size = struct.unpack_from("<q", log, 72)[0]
    struct.pack_into("<q", log, 72, max(0, put_size + delta))
    check(native, bytes(log))


def test_many_small_blocks(native):
    """More blocks than the first directory allocation and many 2048-block chunks."""
    rng = random.Random(12)
    check(native, _compressed(_ops(rng, 6000, 10 ** 9, 0.0, 40), 12))


@pytest.mark.parametrize("put_size,delete_size", [(0, 0), (-5, -1), (1 << 62, 1 << 62), (1 << 62, 0)])
def test_header_sizes_zero_or_absurd(native, put_size, delete_size):
    """putSize = deleteSize = 0 on a multi-block log (a zero-sized virtual log must not bound the
    decode at nothing), negative sizes, and sizes no block chain can decompress to (no huge
    allocation): all take the directory-only pass and build what the reference builds, which never
    reads these fields."""
    rng = random.Random(13)
    log = bytearray(_compressed(_ops(rng, 2500, 2000, 0.1, 150), 900))
    struct.pack_into("<q", log, 72, put_size)
    struct.pack_into("<q", log, 56, delete_size)
    check(native, bytes(log))


@pytest.mark.parametrize("block_size", [1024, 4096, 16384])
@pytest.mark.parametrize("spacing", ["default", "min"])
def test_parallel_directory(native, block_size, spacing, switch, capfd):
    """The parallel block directory (windows, anchors, checked links) gives the serial chain's
    directory: the same .spi as the oracle and as the serial chain (snappy_serial_dir), with the anchors as
    dense as the window length allows or at the default spacing."""
    from sparkey import synth
    log = synth.snappy_log(synth.fixed_log(30000, 16, 100, seed=block_size), 118, block_size).tobytes()
    if spacing == "min":
        switch(snappy_dir_a=1)
    switch(snappy_dir_debug=1)
    got = check(native, log, seed=99)
    assert "[snappy dir] parallel" in capfd.readouterr().err
    switch(snappy_serial_dir=1)
    serial, _ = native.build_index_mem(log, native.make_opts(hash_seed=99))
    assert got == serial
