"""Sharded build on the GPU: the sparkey_shard_* HIP steps driven by sparkey/sharded.py, 2-4 ranks
sharing cuda:0 as threads of this process (in-process collectives; the RCCL transport is the
bench's N > 1 path).  The assembled .spi must equal the oracle's single-process build byte for
byte, and the single-GPU build of the same log."""
import struct

import numpy as np
import pytest

import oracle
from helpers import diff_report, key_value_puts, make_log, random_puts
from sharded_harness import run_threads

pytestmark = pytest.mark.gpu

IN_MEMORY, SORTING = 1, 2


def check(native, log, world, seed=7, hash_size=0, method=IN_MEMORY, sparsity=0.0):
    kw = dict(hash_size=hash_size, hash_seed=seed, sparsity=sparsity, method=method)
    got, metas = run_threads(log, world, kw)
    want = oracle.build_index(log, seed, hash_size=hash_size, sparsity=sparsity, method=method)
    assert got == want, diff_report(got, want)
    return metas


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_gpu_key_value(native, world):
    metas = check(native, make_log(key_value_puts(20000)), world)
    assert metas[0]["path"] == "sharded"


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_gpu_c2_shape(native, world):
    """C2's record shape (16 B keys, 100 B values, fused framing) at 300K records."""
    from sparkey import synth
    log = synth.fixed_log(300000, 16, 100, seed=5).tobytes()
    metas = check(native, log, world, seed=0x2545F491)
    assert metas[0]["path"] == "sharded"


@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_gpu_wide_table(native, world):
    """More than 64 buckets a coarse digit (sparsity 80: about 19.5K buckets for 250K records): the
    received entries go straight into the fixed bucket regions (k_part2_recv), as at C4's sizes."""
    from sparkey import synth
    log = synth.fixed_log(250000, 16, 100, seed=9).tobytes()
    metas = check(native, log, world, seed=0x51D3, sparsity=80.0)
    assert metas[0]["path"] == "sharded"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sharded_gpu_random_keys(native, seed):
    log = make_log(random_puts(8000, seed=seed, kmin=0, kmax=130, vmax=500))
    check(native, log, 3, seed=seed * 77, hash_size=8)


def test_sharded_gpu_large_values(native):
    """Records longer than 4 KiB: every rank frames with the serial walker."""
    value = b"v" * 6000
    log = make_log([(b"key_%d" % i, value) for i in range(600)])
    check(native, log, 2, seed=17)


def test_sharded_gpu_collision_pairs(native):
    metas = check(native, make_log(key_value_puts(300000)), 2, seed=11, hash_size=4)
    assert metas[0]["n_pairs"] > 0 and metas[0]["path"] == "sharded"


def test_sharded_gpu_small_log(native):
    check(native, make_log(key_value_puts(30)), 3)


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("world", [1, 2, 4])
def test_sharded_gpu_deletes_exact(native, method, world):
    """DELETE records: the sharded exact path (exact ranges replayed by their owners), no gathering."""
    log = make_log(key_value_puts(5000), deletes=[b"Key%d" % i for i in range(0, 5000, 7)])
    metas = check(native, log, world, seed=-5, method=method)
    assert all(m["path"] == "exact" for m in metas)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gpu_duplicates_exact(native, world):
    puts = key_value_puts(5000) + [(b"Key%d" % i, b"again") for i in range(0, 5000, 13)]
    metas = check(native, make_log(puts), world, seed=5)
    assert all(m["path"] == "exact" for m in metas)


def _churn_log(n, keys, seed, del_frac=0.2, vmax=40):
    import random
    rnd = random.Random(seed)
    lb = oracle.LogBuilder(7, 0)
    for _ in range(n):
        k = b"k%d" % rnd.randrange(keys)
        if rnd.random() < del_frac:
            lb.delete(k)
        else:
            lb.put(k, b"v" * rnd.randrange(0, vmax))
    return lb.finish()


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_gpu_churn_exact(native, method, world):
    """Puts, overwrites and deletes over a small key space at sparsity 1.3: long segments crossing the
    slot-range boundaries (and the ring's wrap), equal to the oracle and to the single-GPU build."""
    log = _churn_log(60000, 20000, seed=world, del_frac=0.25)
    metas = check(native, log, world, seed=31, method=method, sparsity=1.3)
    assert all(m["path"] == "exact" for m in metas)
    single, st = native.build_index_mem(log, native.make_opts(hash_seed=31, method=method, sparsity=1.3))
    got, _ = run_threads(log, world, dict(hash_seed=31, method=method, sparsity=1.3))
    assert got == single and st.placement_path == 2


def test_sharded_gpu_c2_shape_overwrites(native):
    """C2's record shape (uniform framing) with every 10th key written twice: the uniform log's exact
    path, 4 ranks."""
    from sparkey import synth
    base = synth.fixed_log(200000, 16, 100, seed=8).tobytes()
    recs = [base[84 + 118 * i: 84 + 118 * (i + 1)] for i in range(0, 200000, 10)]
    lb = oracle.LogBuilder(0x2545F491, 0)
    for i in range(200000):
        r = base[84 + 118 * i: 84 + 118 * (i + 1)]
        lb.put(r[2:18], r[18:])
    for r in recs:
        lb.put(r[2:18], r[18:][::-1])
    metas = check(native, lb.finish(), 4, seed=0x2545F491)
    assert all(m["path"] == "exact" for m in metas)


def test_sharded_gpu_understated_header(native):
    log = bytearray(make_log([(b"k%d" % i, b"v" * (i % 300)) for i in range(6000)]))
    struct.pack_into("<q", log, 48, 10)
    check(native, bytes(log), 3, seed=9)


@pytest.mark.parametrize("world", [1, 4])
def test_sharded_gpu_matches_single(native, world):
    """Mixed record sizes (k_frame, the bin's own partition pass; one rank: entries kept in place)."""
    from sparkey import synth
    log = synth.mixed_log(100000, 8, 64, 100, seed=4).tobytes()
    opts = native.make_opts(hash_seed=99)
    single, _ = native.build_index_mem(log, opts)
    got, metas = run_threads(log, world, dict(hash_seed=99))
    assert got == single, diff_report(got, single)
    assert metas[0]["path"] == "sharded"


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_gpu_snappy_gather(native, world):
    """SNAPPY logs: gathered on every rank, built by the single-GPU SNAPPY path, sliced by slot range."""
    from sparkey import synth
    log = synth.snappy_log(synth.fixed_log(100000, 16, 100, seed=6), 118, 16384).tobytes()
    metas = check(native, log, world, seed=13)
    assert metas[0]["path"] == "gathered"


@pytest.mark.parametrize("world", [1, 3])
def test_sharded_gpu_speculative_retry(native, world, switch):
    """Every speculative frame+bin attempt flagged for a retry (a send buffer of 0 entries): the
    ranks re-frame synchronously and the result is unchanged."""
    switch(shard_sync_frame=1)
    metas = check(native, make_log(key_value_puts(20000)), world)
    assert metas[0]["path"] == "sharded" and metas[0]["rounds"] >= 2


@pytest.mark.parametrize("world", [1, 3])
def test_sharded_gpu_exact_reframe(native, world, switch):
    """The exact path framing its byte range again instead of reusing the canonical step's slabs."""
    switch(exact_reframe=1)
    metas = check(native, _churn_log(30000, 10000, seed=9), world, seed=4, sparsity=1.3)
    assert all(m["path"] == "exact" for m in metas)
