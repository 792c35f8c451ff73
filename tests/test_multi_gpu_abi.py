"""Multi-GPU builds through the drop-in boundary: sparkey_build_index_mem / _file with
opts.num_gpus = N (the C++ orchestrator, sparkey-java_amd/csrc/shard_host.cpp, N ranks as threads).
On a one-GPU box the ranks share cuda:0 through the in-process transport
(the shard_transport switch = 2, threads on one device); the RCCL transport runs at N = 1 here (one rank,
sparkey_shard_build over an RCCL communicator) and at N > 1 in the driver's multi-GPU bench.
Every .spi must equal the oracle's (the reference's single-threaded IndexHash.createNew,
IndexHash.java:131-167) byte for byte."""
import os
import random

import pytest

import oracle
from helpers import diff_report, key_value_puts, make_log, random_puts

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


@pytest.mark.parametrize("n", [2, 3, 4])
def test_key_value(native, n):
    check(native, make_log(key_value_puts(20000)), n, sharded=1)


@pytest.mark.parametrize("n", [2, 4])
def test_c2_shape(native, n):
    from sparkey import synth
    log = synth.fixed_log(300000, 16, 100, seed=5).tobytes()
    st = check(native, log, n, seed=0x2545F491, sharded=1)
    assert st.num_entries == 300000


@pytest.mark.parametrize("n", [2, 4])
def test_c3_shape_mixed_keys(native, n):
    from sparkey import synth
    check(native, synth.mixed_log(200000, 8, 64, 100, seed=9).tobytes(), n, seed=99, hash_size=8, sharded=1)


@pytest.mark.parametrize("seed", [1, 2])
def test_random_keys(native, seed):
    check(native, make_log(random_puts(8000, seed=seed, kmin=0, kmax=130, vmax=500)), 3, seed=seed * 77, hash_size=8)


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("n", [2, 4])
def test_deletes_and_overwrites_exact(native, method, n):
    puts = key_value_puts(5000) + [(b"Key%d" % i, b"again") for i in range(0, 5000, 13)]
    log = make_log(puts, deletes=[b"Key%d" % i for i in range(0, 5000, 7)])
    check(native, log, n, seed=-5, method=method, sharded=2)


def test_churn_exact(native):
    from sparkey import synth
    check(native, synth.churn_log(200000, 150000, 0.1, seed=4).tobytes(), 4, seed=5, sharded=2)


def test_collision_pairs_32_bit(native):
    """300K keys with 32-bit hashes: equal-hash pairs checked against the keys across ranks."""
    check(native, make_log(key_value_puts(300000)), 2, seed=11, hash_size=4, sharded=1)


def test_small_log_and_empty(native):
    check(native, make_log(key_value_puts(30)), 3)
    check(native, make_log([]), 2)


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
def test_compressed_logs(native, codec):
    """Compressed logs shard too (each rank decodes its own blocks; test_multi_gpu_compressed.py)."""
    from sparkey import synth
    log = synth.snappy_log(synth.fixed_log(20000, 16, 100, seed=7, file_id=5), 118, 4096, codec=codec).tobytes()
    check(native, log, 2, seed=4321, sharded=1)


def test_large_values_serial_framing(native):
    check(native, make_log([(b"key_%d" % i, b"v" * 6000) for i in range(600)]), 2, seed=17)


def test_error_is_the_single_gpu_error(native):
    """A record the iterator cannot read: the same exception class and code as one GPU and the oracle."""
    import struct
    log = bytearray(make_log(key_value_puts(20000)))
    struct.pack_into("<q", log, 40, 3)
    with pytest.raises(RuntimeError) as e:
        native.build_index_mem(bytes(log), native.make_opts(hash_seed=1, num_gpus=2))
    assert e.value.code == native.E_CORRUPT_RECORD


def test_file_to_file(native, tmp_path):
    from sparkey import synth
    log = synth.mixed_log(100000, 8, 64, 100, seed=3).tobytes()
    lp, sp = str(tmp_path / "m.spl"), str(tmp_path / "m.spi")
    with open(lp, "wb") as f:
        f.write(log)
    st = native.build_index_file(lp, sp, native.make_opts(hash_seed=42, num_gpus=3), fsync=True)
    assert open(sp, "rb").read() == oracle.build_index(log, 42)
    assert st.sharded == 1 and st.num_entries == 100000


def test_rccl_one_rank(native, switch):
    """sparkey_shard_build over an RCCL communicator (world 1 on a one-GPU box): the multi-process path
    bench.py takes at N > 1."""
    import torch
    from sparkey import synth
    switch(shard_transport=None)
    log = synth.fixed_log(200000, 16, 100, seed=6).tobytes()
    opts = native.make_opts(hash_seed=3)
    uid = native.shard_unique_id()
    comm = native.ShardComm(uid, 0, 1, 0)
    plan = native.Plan(0)
    try:
        blo, bhi, ooff, olen = native.shard_geometry(log[:84], len(log), opts, 0, 1)
        assert (blo, bhi, ooff) == (0, len(log), 0)
        d_buf = torch.frombuffer(bytearray(log[blo:bhi]), dtype=torch.uint8).to("cuda:0")
        d_out = torch.empty(olen, dtype=torch.uint8, device="cuda:0")
        for _ in range(2):  # (the communicator and its buffers are reused)
            st = comm.build(plan, log[:84], len(log), d_buf.data_ptr(), blo, bhi, opts, d_out.data_ptr(), olen)
            assert d_out.cpu().numpy().tobytes() == oracle.build_index(log, 3)
        assert st.sharded == 1 and [p for p, _ in comm.phases()][:1] == ["entries"]
    finally:
        plan.close()
        comm.close()


@pytest.mark.parametrize("fail_rank", [0, 2])
def test_one_rank_failing_fails_every_rank(native, switch, fail_rank):
    """One rank fails on its own (its load, forced by the shard_fail_rank switch): every rank returns
    from the same checkpoint with the error (no rank waits in a collective for it), and the next build
    through a fresh group is correct (ranks fail together)."""
    from sparkey import synth
    log = synth.fixed_log(60000, 16, 100, seed=2).tobytes()
    switch(shard_fail_rank=fail_rank)
    with pytest.raises(OSError) as e:
        native.build_index_mem(log, native.make_opts(hash_seed=5, num_gpus=3))
    assert "injected load failure" in str(e.value) or "another rank" in str(e.value)
    switch(shard_fail_rank=None)
    check(native, log, 3, seed=5, sharded=1)


@pytest.mark.parametrize("n", [2, 4])
def test_sharded_device_entry(native, n):
    """sparkey_build_index_sharded_device: every rank reads its range of ONE device log in place and
    writes its part of ONE device .spi in place."""
    import torch
    from sparkey import synth
    for log in (synth.fixed_log(300000, 16, 100, seed=4).tobytes(), make_log(random_puts(50000, seed=3))):
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
