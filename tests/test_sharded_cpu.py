"""Sharded (multi-process) build on CPU: the host orchestration of sparkey/sharded.py over real gloo
collectives (world sizes 2-4), with the device steps simulated on the CPU (tests/shard_sim.py).
The assembled .spi must equal the oracle's single-process IndexHash restatement byte for byte."""
import struct

import numpy as np
import pytest

import oracle
from helpers import diff_report, key_value_puts, make_log, random_puts
from sharded_harness import run_world
from sparkey.sharded import shard_layout

IN_MEMORY, SORTING = 1, 2


def check(log, world, tmp_path, seed=7, hash_size=0, method=IN_MEMORY, sparsity=0.0):
    got, metas = run_world(log, world, dict(hash_size=hash_size, hash_seed=seed, sparsity=sparsity, method=method),
                           str(tmp_path), kind="cpu")
    want = oracle.build_index(log, seed, hash_size=hash_size, sparsity=sparsity, method=method)
    assert got == want, diff_report(got, want)
    return metas


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_key_value(tmp_path, world):
    log = make_log(key_value_puts(3000))
    metas = check(log, world, tmp_path)
    assert all(m["path"] == "sharded" for m in metas)
    assert metas[0]["n_spill"] > 0  # clusters cross the slot-range boundaries


@pytest.mark.parametrize("seed", [1, 2])
def test_sharded_random_keys(tmp_path, seed):
    log = make_log(random_puts(2500, seed=seed, kmin=1, kmax=70, vmax=200))
    metas = check(log, 2, tmp_path, seed=seed * 101, hash_size=8)
    assert metas[0]["path"] == "sharded"


def test_sharded_layout_splits_records(tmp_path):
    """Byte ranges do not follow record boundaries: every rank past 0 has to find its entry."""
    log = make_log(key_value_puts(4000))
    lay = shard_layout(log[:84], len(log), 3)
    assert not lay.small and lay.lo[1] > 84
    check(log, 3, tmp_path, seed=3)


def test_sharded_small_log(tmp_path):
    log = make_log(key_value_puts(40))
    assert shard_layout(log[:84], len(log), 2).small
    check(log, 2, tmp_path)


def test_sharded_hash_collision_pairs(tmp_path):
    """32-bit hashes with many keys: equal-hash pairs of different keys are compared through the
    key fetch exchange and stay on the sharded path."""
    n = 200000
    log = make_log(key_value_puts(n))
    metas = check(log, 2, tmp_path, seed=11, hash_size=4)
    assert metas[0]["n_pairs"] > 0 and metas[0]["path"] == "sharded"


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_duplicates_exact(tmp_path, world):
    """Overwritten keys: the sharded exact path (no gathering), equal to the oracle."""
    puts = key_value_puts(2000) + [(b"Key%d" % i, b"again") for i in range(0, 2000, 17)]
    metas = check(make_log(puts), world, tmp_path, seed=5)
    assert all(m["path"] == "exact" for m in metas)


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_deletes_exact(tmp_path, method, world):
    log = make_log(key_value_puts(2000), deletes=[b"Key%d" % i for i in range(0, 2000, 7)])
    metas = check(log, world, tmp_path, seed=-5, method=method)
    assert all(m["path"] == "exact" for m in metas)
    assert metas[0]["stats"]["garbage_size"] > 0


def test_sharded_churn_exact(tmp_path):
    """Interleaved puts, overwrites and deletes of a small key space (long segments that cross the
    slot-range boundaries), 3 ranks, dense table."""
    import random
    rnd = random.Random(3)
    lb = oracle.LogBuilder(7, 0)
    for i in range(5000):
        k = b"k%d" % rnd.randrange(1500)
        if rnd.random() < 0.2:
            lb.delete(k)
        else:
            lb.put(k, b"v" * rnd.randrange(0, 40))
    metas = check(lb.finish(), 3, tmp_path, seed=77, sparsity=1.3)
    assert all(m["path"] == "exact" for m in metas)


def test_sharded_delete_of_absent_keys(tmp_path):
    """DELETE records of keys never put (no-ops in every state) and deletes before the puts."""
    puts = key_value_puts(1500)
    log = make_log(puts, deletes=[b"Nope%d" % i for i in range(300)] + [b"Key%d" % i for i in range(0, 1500, 5)])
    metas = check(log, 2, tmp_path, seed=12)
    assert all(m["path"] == "exact" for m in metas)


def test_sharded_understated_header(tmp_path):
    """A header understating maxValueLen misleads the entry speculation; the exact exits of the
    previous ranks correct it (re-framing rounds) and the result stays identical."""
    log = bytearray(make_log([(b"k%d" % i, b"v" * (i % 300)) for i in range(3000)]))
    struct.pack_into("<q", log, 48, 10)
    metas = check(bytes(log), 3, tmp_path, seed=9)
    assert metas[0]["rounds"] >= 1


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_snappy_gather(tmp_path, world):
    """SNAPPY logs are built whole on every rank (the single-GPU path) and sliced by slot range."""
    from snappy_log import CompressedLog
    cl = CompressedLog(1024, file_identifier=0x1234567)
    for i in range(3000):
        cl.put(b"Key%d" % i, b"Value%d" % i)
    metas = check(cl.finish(), world, tmp_path, seed=21)
    assert metas[0]["path"] == "gathered"
