"""Sharded SNAPPY / ZSTD builds through sparkey_build_index_mem with opts.num_gpus = N
(the C++ orchestrator, ranks as threads sharing cuda:0): each rank finds the block chain in its own
byte range of the compressed log, checks its links up to the next rank's entry (induction from 84)
and decodes its blocks into its slice of the virtual log; the NONE steps run over the slices with
the compressed log's addresses ((blockPosition << entryBlockBits) | entryIndex, IndexHash.java:270-283).
Every .spi must equal the oracle's byte for byte; stats.sharded says which path ran (1 sharded, 2 the
sharded exact path for DELETEs and overwrites, 3 the log gathered on every rank: a record spanning two
ranks' blocks, the switch)."""
import random
import struct

import pytest

import oracle
from helpers import diff_report, same_error
from snappy_log import CompressedLog
from test_compressed_oracle import _compressed, _ops

pytestmark = pytest.mark.gpu

IN_MEMORY, SORTING = 1, 2


@pytest.fixture(autouse=True)
def one_device(switch):
    switch(shard_transport=2)


def check(native, log, n, seed=7, method=IN_MEMORY, hash_size=0, sharded=None):
    got, st = native.build_index_mem(log, native.make_opts(hash_size=hash_size, hash_seed=seed, method=method,
                                                            num_gpus=n))
    want = oracle.build_index(log, seed, hash_size=hash_size, method=method)
    assert got == want, diff_report(got, want)
    assert sharded is None or st.sharded == sharded, st.as_dict()
    return st


def uniform(n, block, codec, seed=7):
    from sparkey import synth
    return synth.snappy_log(synth.fixed_log(n, 16, 100, seed=seed, file_id=5), 118, block, codec=codec).tobytes()


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
@pytest.mark.parametrize("n", [2, 3, 4])
def test_uniform_records(native, codec, n):
    st = check(native, uniform(40000, 4096, codec), n, seed=4321, sharded=1)
    assert st.num_entries == 40000


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
@pytest.mark.parametrize("block_size", [1024, 16384])
def test_mixed_records(native, codec, block_size):
    """Records of 10-220 bytes, several per block (entryBlockBits > 0: the entry index in the address)."""
    rng = random.Random(block_size)
    log = _compressed(_ops(rng, 20000, 10 ** 9, 0.0, 200), block_size, codec=codec)
    assert struct.unpack_from("<i", log, 80)[0] > 1
    check(native, log, 3, seed=99, sharded=1)


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_sorting_and_in_memory(native, method):
    check(native, uniform(30000, 8192, "snappy", seed=3), 2, seed=5, method=method, sharded=1)


def test_collision_pairs_32_bit(native):
    """300K keys with 32-bit hashes: the equal-hash pairs' keys are fetched from the ranks holding their
    blocks (compressed-log addresses back to virtual offsets there)."""
    st = check(native, uniform(300000, 65536, "snappy", seed=11), 2, seed=11, hash_size=4, sharded=1)
    assert st.hash_collisions > 0


def test_dense_anchors(native, switch):
    """Windows one hop apart (the snappy_dir_a switch): many anchors per rank, every link checked."""
    switch(snappy_dir_a=1)
    check(native, uniform(20000, 1024, "snappy", seed=8), 4, seed=3, sharded=1)


def test_write_hash_benchmark_shape(native):
    cl = CompressedLog(1024, file_identifier=77)
    for i in range(30000):
        cl.put(b"key_%d" % i, b"value_%d" % i)
    check(native, cl.finish(), 3, seed=1234, sharded=1)


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("n", [2, 3])
def test_deletes_and_overwrites_exact(native, method, n):
    """DELETEs and overwrites: the sharded exact path over the ranks' slices, the
    exchange records' addresses rewritten to the compressed log's."""
    rng = random.Random(5 + n)
    log = _compressed(_ops(rng, 8000, 1500, 0.2, 120), 1024)
    check(native, log, n, seed=4, method=method, sharded=2)


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
def test_churn_shape_exact(native, codec):
    """C2-shaped records drawn from a key pool with 10% DELETEs (bench.py's churn), in 4 KiB blocks."""
    from sparkey import synth
    from snappy_log import CompressedLog
    import numpy as np
    log = synth.churn_log(20000, 15000, 0.1, seed=4).tobytes()
    cl = CompressedLog(4096, file_identifier=9, codec=codec)
    p, end = 84, struct.unpack_from("<q", log, 32)[0]
    while p < end:
        a, b = log[p], log[p + 1]
        if a == 0:
            cl.delete(log[p + 2:p + 2 + b])
            p += 2 + b
        else:
            cl.put(log[p + 2:p + 1 + a], log[p + 1 + a:p + 1 + a + b])
            p += 1 + a + b
    check(native, cl.finish(), 4, seed=5, sharded=2)


def test_gather_switch(native, switch):
    switch(shard_gather_compressed=1)
    check(native, uniform(20000, 4096, "zstd"), 2, seed=4, sharded=3)


@pytest.mark.parametrize("n", [2, 3])
def test_spanning_records(native, n):
    """Values up to 5000 bytes over 512-byte blocks: records span blocks; a rank boundary inside one
    gathers the log (sharded 3), elsewhere the ranks shard it (sharded 1) -- either way the oracle's
    bytes.  The two cases are pinned one by one below."""
    rng = random.Random(3)
    st = check(native, _compressed(_ops(rng, 1500, 10 ** 9, 0.0, 5000), 512), n, seed=21)
    assert st.sharded in (1, 3), st.as_dict()


def test_boundary_between_records_shards(native):
    """Records shorter than the block never span one (CompressedWriter flushes first), so the rank
    boundary falls between records: the ranks shard the log."""
    rng = random.Random(4)
    check(native, _compressed(_ops(rng, 3000, 10 ** 9, 0.0, 100), 512), 2, seed=22, sharded=1)


def test_boundary_inside_spanning_record_gathers(native):
    """One 200 KB record spanning about 400 blocks between a few small ones: the 2-rank boundary falls
    inside it, a record no rank's slice can end, so the ranks gather the log."""
    rng = random.Random(6)
    ops = [("put", b"a%d" % i, b"x%d" % i) for i in range(5)]
    ops.append(("put", b"big", bytes(rng.randrange(256) for _ in range(200000))))
    ops += [("put", b"b%d" % i, b"y%d" % i) for i in range(5)]
    check(native, _compressed(ops, 512), 2, seed=23, sharded=3)


def test_small_and_empty(native):
    """An empty log and a 20-record log (fewer blocks than some ranks' ranges): the oracle's bytes."""
    st = check(native, CompressedLog(1024).finish(), 2)
    print("empty:", st.sharded)
    cl = CompressedLog(1024)
    for i in range(20):
        cl.put(b"k%d" % i, b"v")
    st = check(native, cl.finish(), 3)
    print("20 records:", st.sharded)


def test_corrupt_block_is_the_single_gpu_error(native):
    """A block header in the second rank's range that runs past dataEnd: the ranks' links miss, the
    gathered build raises what one GPU raises."""
    log = bytearray(uniform(20000, 4096, "snappy"))
    p, starts = 84, []
    while p < len(log):
        starts.append(p)
        clen, q, s = 0, p, 0
        while True:
            clen |= (log[q] & 0x7F) << s
            s += 7
            q += 1
            if log[q - 1] < 0x80:
                break
        p = q + clen
    q = starts[len(starts) * 3 // 5]
    log[q:q + 5] = b"\xff\xff\xff\xff\x0f"
    with pytest.raises(RuntimeError) as one:
        native.build_index_mem(bytes(log), native.make_opts(hash_seed=1))
    with pytest.raises(RuntimeError) as two:
        native.build_index_mem(bytes(log), native.make_opts(hash_seed=1, num_gpus=2))
    assert one.value.code == two.value.code


@pytest.mark.parametrize("n", [2, 4])
def test_sharded_device_entry(native, n):
    """sparkey_build_index_sharded_device on a compressed log: each rank reads its range (with the
    geometry's tail for the next range's first anchor) of ONE device log in place."""
    import torch
    log = uniform(50000, 4096, "zstd", seed=9)
    opts = native.make_opts(hash_seed=11, num_gpus=n)
    size = native.index_size(log[:84], opts)
    d_log = torch.frombuffer(bytearray(log), dtype=torch.uint8).to("cuda:0")
    d_spi = torch.empty(size, dtype=torch.uint8, device="cuda:0")
    bufs, outs = [], []
    for r in range(n):
        lo, hi, off, ln = native.shard_geometry(log[:84], len(log), opts, r, n)
        bufs.append(d_log.data_ptr() + lo)
        outs.append(d_spi.data_ptr() + off)
    st = native.build_index_sharded_device(log[:84], len(log), bufs, outs, opts)
    got = d_spi.cpu().numpy().tobytes()
    want = oracle.build_index(log, 11)
    assert got == want, diff_report(got, want)
    assert st.sharded == 1
