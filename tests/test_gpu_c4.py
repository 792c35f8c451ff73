"""C4's sizes on one GPU (BASELINE.json configs[3]: 1B entries, 16 B keys, 100 B values).

- 300M C2-shaped records: 4.8 GB of (hash, address) entries, past 2^32 bytes, a 35 GB log and a 6.2 GB
  .spi, checked byte for byte against the oracle (IndexHash.createNew's sequential restatement).
- 1B records (C4 itself): a 118 GB log made in HBM (sparkey/synth_device.py), built on one GPU, then
  again as 8 ranks of the sharded build (sparkey_build_index_sharded_device, the 8 ranks as threads on
  this GPU: the shard_transport switch), and the two 20.8 GB .spi compared byte for byte on the device
  (both images and the 118 GB log are resident at once: 160 GB of the 288 GB); the header's numEntries,
  and IndexHash.get of every 1000th key through sparkey_get_batch, pin the result against the log itself.  Capacity
  1,300,000,001 slots, a 20.8 GB .spi (IndexHash.java:145; the reference chunks its own tables past
  2 GiB, InMemoryData.java:22-52; LargeFilesTest.java:26-87 is its large-file test).
"""
import numpy as np
import pytest
import torch

import oracle
from helpers import diff_report, index_header

pytestmark = pytest.mark.gpu
SEED = 0x2545F491
DEV = torch.device("cuda", 0)


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_c2_shape_300m_against_oracle(native):
    """300M records: entry buffers past 2^32 bytes, a 35 GB log; the oracle's bytes."""
    from sparkey import synth_device
    n = 300_000_000
    log = synth_device.fixed_log(n, seed=1, device=DEV)
    header = log[:84].cpu().numpy().tobytes()
    opts = native.make_opts(hash_seed=SEED, method=1)
    size = native.index_size(header, opts)
    d_out = torch.empty(size, dtype=torch.uint8, device=DEV)
    plan = native.Plan(0)
    try:
        st = plan.build(header, log.data_ptr(), log.numel(), d_out.data_ptr(), size, opts)
    finally:
        plan.close()
    assert st.num_entries == n and st.placement_path == 0 and st.framing_path == 2, st.as_dict()
    got = d_out.cpu().numpy()
    del d_out
    host_log = log.cpu().numpy()
    del log
    _free()
    want = np.frombuffer(oracle.build_index(host_log, SEED), dtype=np.uint8)
    assert want.size == got.size == size
    if not np.array_equal(got, want):
        raise AssertionError(diff_report(got.tobytes(), want.tobytes()))


def test_c4_1b_single_gpu_equals_8_ranks(native):
    from sparkey import synth_device
    n = 1_000_000_000
    log = synth_device.fixed_log(n, seed=1, device=DEV)
    log_len = log.numel()
    header = log[:84].cpu().numpy().tobytes()
    opts = native.make_opts(hash_seed=SEED, method=1)
    size = native.index_size(header, opts)
    assert size == 112 + 16 * 1_300_000_001
    # one GPU
    spi = torch.empty(size, dtype=torch.uint8, device=DEV)
    plan = native.Plan(0)
    try:
        st = plan.build(header, log.data_ptr(), log_len, spi.data_ptr(), size, opts)
    finally:
        plan.close()
    assert st.num_entries == n and st.capacity == 1_300_000_001 and st.placement_path == 0, st.as_dict()
    single_hdr = spi[:112].cpu().numpy().tobytes()
    h = index_header(single_hdr)
    assert h["numEntries"] == n and h["capacity"] == 1_300_000_001 and h["garbageSize"] == 0
    _free()  # (the single-GPU image stays for the byte comparison)
    # eight ranks of the sharded build on this GPU, each reading its log range in place and writing its
    # part of the .spi in place
    world = 8
    spi8 = torch.empty(size, dtype=torch.uint8, device=DEV)
    opts8 = native.make_opts(hash_seed=SEED, method=1, num_gpus=world)
    bufs, outs = [], []
    for r in range(world):
        lo, hi, off, ln = native.shard_geometry(header, log_len, opts8, r, world)
        bufs.append(log.data_ptr() + lo)
        outs.append(spi8.data_ptr() + off)
    with native.debug(shard_transport=2):
        st8 = native.build_index_sharded_device(header, log_len, bufs, outs, opts8)
    native.release_cached_resources()
    assert st8.sharded == 1 and st8.num_entries == n, st8.as_dict()
    assert spi8[:112].cpu().numpy().tobytes() == single_hdr
    # byte equality of the two 20.8 GB images, on the device (first differing word reported)
    if not torch.equal(spi8, spi):
        w8, w1 = spi8[: size // 8 * 8].view(torch.int64), spi[: size // 8 * 8].view(torch.int64)
        bad = torch.nonzero(w8 != w1)
        first = int(bad[0]) if bad.numel() else -1
        raise AssertionError(f"8-rank .spi differs from the single-GPU .spi: {bad.numel()} words, the first at byte {8 * first}")
    del spi
    # IndexHash.get of every 1000th key finds its record: value at 84 + 118 i + 18, 100 bytes
    idx = torch.arange(0, n, 1000, dtype=torch.int64, device=DEV)
    keys = synth_device.fixed_keys(idx, seed=1).reshape(-1)
    key_off = torch.arange(0, 16 * (idx.numel() + 1), 16, dtype=torch.int64, device=DEV)
    pos = torch.empty(idx.numel(), dtype=torch.int64, device=DEV)
    vlen = torch.empty(idx.numel(), dtype=torch.int64, device=DEV)
    plan = native.Plan(0)
    try:
        plan.get_batch(log.data_ptr(), log_len, spi8.data_ptr(), size, keys.data_ptr(), key_off.data_ptr(),
                       idx.numel(), pos.data_ptr(), vlen.data_ptr())
    finally:
        plan.close()
    assert bool((pos == idx * 118 + 84 + 18).all()) and bool((vlen == 100).all())
    del log, spi8
    _free()
