"""The partition and placement kernels never form an LDS or global index from an entry that lies
outside the buckets their workgroup owns (kGuardForeign, kernel_utils.hpp): such an entry -- a region
whose contents disagree with its count, as a bug or a half-written region would leave it -- fails the
build with a clean SparkeyGpuError instead of a wild store.  IndexHash.put checks its own bounds before
it touches the table (IndexHash.java:574-576).

Round 5's two device faults (an aperture violation in k_part2st<6> during a measurement variant that
cut the framing short) are what these tests pin: the `inject_foreign` switch writes an entry of the
table's last bucket into digit region 0 (before pass 2) or bucket region 0 (before the placement), and
the `frame3_stop` measurement switch cuts k_frame3 short at each phase, after which no later stage may
consume its regions (the host redoes the framing with k_frame).
"""
import pytest

import oracle
from helpers import make_log, random_puts

pytestmark = pytest.mark.gpu

IN_MEMORY = 1


def _uniform_log(n=50000):
    # C2's shape at a small size: every record the same size, so k_frame_uniform writes digit regions
    return make_log([(i.to_bytes(8, "little") * 2, bytes([i % 251]) * 40) for i in range(n)])


def _mixed_log(n=40000, seed=81):
    # C3's shape: one-byte VLQs, mixed key lengths, so k_frame3 writes the bucket regions
    return make_log(random_puts(n, seed=seed, kmin=8, kmax=64, vmin=100, vmax=100))


def _build(native, log, seed=5):
    return native.build_index_mem(log, native.make_opts(hash_size=8, hash_seed=seed, method=IN_MEMORY))


@pytest.mark.parametrize("where,log_fn,framing", [(1, _uniform_log, 2), (2, _uniform_log, 2), (2, _mixed_log, 4)])
def test_foreign_entry_fails_cleanly(native, switch, where, log_fn, framing):
    """A foreign entry in digit region 0 (k_part2st) or bucket region 0 (k_summary / k_place_reg):
    SparkeyGpuError naming the bounds check, no device fault; the next build on the same device, with
    the switch off, is the oracle's bytes."""
    log = log_fn()
    want = oracle.build_index(log, 5, hash_size=8, method=IN_MEMORY)
    got, st = _build(native, log)
    assert got == want and st.framing_path == framing, st.as_dict()
    switch(inject_foreign=where)
    with pytest.raises(native.SparkeyGpuError, match="bounds check"):
        _build(native, log)
    switch(inject_foreign=None)
    got, st = _build(native, log)
    assert got == want and st.framing_path == framing


@pytest.mark.parametrize("stop", [0, 1, 2, 3, 4, 5])
def test_frame3_stop_skips_later_stages(native, switch, stop):
    """frame3_stop (phase cut-offs for measurements) fails k_frame3 after each phase; the partition,
    placement and stats skip that attempt and the host redoes it with k_frame: the oracle's bytes."""
    log = _mixed_log(30000, seed=83)
    want = oracle.build_index(log, 5, hash_size=8, method=IN_MEMORY)
    switch(frame3_stop=stop)
    got, st = _build(native, log)
    assert got == want, st.as_dict()
    assert st.framing_path == 0, st.as_dict()
