"""Full-size BASELINE.json configurations on the GPU, bit-exact against the oracle:
C2 (10M x 16 B keys / 100 B values), C3 (100M, keys 8-64 B), C5 (C3 with SORTING), and the sharded
build of C2 (4 ranks) against the single-GPU build."""
import numpy as np
import pytest
import torch

import oracle
from helpers import diff_report, index_header

pytestmark = pytest.mark.gpu
IN_MEMORY, SORTING = 1, 2


def device_build(native, log_np, seed, method=IN_MEMORY):
    """Log resident in HBM -> .spi resident in HBM -> host bytes."""
    dev = torch.device("cuda", 0)
    header = log_np[:84].tobytes()
    opts = native.make_opts(hash_seed=seed, method=method)
    n_out = native.index_size(header, opts)
    d_log = torch.from_numpy(log_np).to(dev)
    d_out = torch.empty(n_out, dtype=torch.uint8, device=dev)
    plan = native.Plan(0)
    torch.cuda.synchronize()
    stats = plan.build(header, d_log.data_ptr(), log_np.size, d_out.data_ptr(), n_out, opts)
    out = d_out.cpu().numpy().tobytes()
    plan.close()
    del d_log, d_out
    torch.cuda.empty_cache()
    return out, stats


def test_c2_full_size(native):
    from sparkey import synth
    log = synth.fixed_log(10_000_000, 16, 100, seed=1)
    got, stats = device_build(native, log, 0x2545F491)
    want = oracle.build_index(log, 0x2545F491)
    assert got == want, diff_report(got, want)
    assert stats.placement_path == 0 and stats.framing_path == 2  # uniform records (k_frame_uniform)


def test_c2_full_size_general_framing(native, switch):
    """The same C2 log through the general speculative framing (k_frame3 for its one-byte VLQs)."""
    from sparkey import synth
    switch(no_uniform=1)
    log = synth.fixed_log(10_000_000, 16, 100, seed=1)
    got, stats = device_build(native, log, 0x2545F491)
    want = oracle.build_index(log, 0x2545F491)
    assert got == want, diff_report(got, want)
    assert stats.placement_path == 0 and stats.framing_path in (0, 4)


@pytest.fixture(scope="module")
def c3_log():
    from sparkey import synth
    return synth.mixed_log(100_000_000, 8, 64, 100, seed=3)


@pytest.fixture(scope="module")
def c3_want(c3_log):
    return oracle.build_index(c3_log, 77)


def test_c3_100m_mixed_keys(native, c3_log, c3_want):
    got, stats = device_build(native, c3_log, 77)
    assert got == c3_want, diff_report(got, c3_want)
    h = index_header(got)
    assert h["numEntries"] == 100_000_000 and h["hashSize"] == 8 and h["addressSize"] == 8
    assert stats.framing_path in (0, 4) and stats.placement_path == 0


@pytest.mark.parametrize("sw", [{}, {"no_buckets": 1}, {"no_buckets": 1, "no_frame3": 1}])
def test_mixed_20m_fixed_bucket_regions(native, switch, sw):
    """20M mixed records: 25,391 placement buckets, 100 a digit.  By default k_frame3 writes every entry
    straight into its bucket's fixed region; with the bucket regions off (or k_frame framing), pass 1
    goes to digit regions and pass 2 is k_part2f (past k_part2st's 64 buckets a digit: one read into the
    fixed bucket regions).  The carries are k_summary's."""
    from sparkey import synth
    switch(**sw)
    log = synth.mixed_log(20_000_000, 8, 64, 100, seed=11)
    got, stats = device_build(native, log, 91)
    want = _want_20m(log)
    assert got == want, diff_report(got, want)
    assert stats.placement_path == 0
    assert stats.partition_passes == (2 if sw else 0), stats.as_dict()


_W20 = {}


def _want_20m(log):
    if "w" not in _W20:
        _W20["w"] = oracle.build_index(log, 91)
    return _W20["w"]


def test_c5_100m_sorting(native, c3_log, c3_want):
    """SORTING on the C3 log: identical to IN_MEMORY for unique keys (TestSparkeyWriter.java:9-36)."""
    got, stats = device_build(native, c3_log, 77, method=SORTING)
    assert got == c3_want, diff_report(got, c3_want)


def test_sharded_c2_4_ranks_matches_single(native):
    from sparkey import synth
    from sharded_harness import run_threads
    log = synth.fixed_log(10_000_000, 16, 100, seed=8)
    single, _ = device_build(native, log, 4242)
    got, metas = run_threads(log.tobytes(), 4, dict(hash_seed=4242))
    assert all(m["path"] == "sharded" for m in metas)
    assert got == single, diff_report(got, single)


@pytest.mark.parametrize("method,n", [(IN_MEMORY, 10_000_000), (SORTING, 4_000_000)])
def test_churn_full_size(native, method, n):
    """C2-shaped log with overwrites and DELETEs (keys from a pool of 0.8 n, 10% DELETE records): the
    exact replay over independent slot segments (placement_path 2), bit-exact against the oracle's
    sequential IndexHash.put / delete."""
    from sparkey import synth
    log = synth.churn_log(n, int(n * 0.8), 0.1, seed=5)
    got, stats = device_build(native, log, 0x5EED, method=method)
    want = oracle.build_index(log, 0x5EED, method=method)
    assert got == want, diff_report(got, want)
    assert stats.placement_path == 2 and stats.framing_path in (0, 4)
    h = index_header(got)
    assert h["garbageSize"] > 0 and 0 < h["numEntries"] < n
