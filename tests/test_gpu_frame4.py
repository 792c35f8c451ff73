"""k_frame4 (frame4_kernels.hip, framing path 5): one log chunk per lane, for logs whose VLQs are all
one byte.  The same .spi bytes as the oracle (IndexHash.createNew's sequential restatement) on every
geometry, on logs built to fool its speculation (values whose bytes look like record headers), with
DELETEs and overwrites, and on the cases that fall back to k_frame3 / k_frame / the serial walk.
"""
import numpy as np
import pytest

import oracle
from helpers import diff_report, make_log, random_puts, with_trailing_bytes

pytestmark = pytest.mark.gpu


def build(native, log, seed, hash_size=8, method=1):
    return native.build_index_mem(log, native.make_opts(hash_size=hash_size, hash_seed=seed, method=method))


def check(native, log, seed, hash_size=8, method=1):
    want = oracle.build_index(log, seed, hash_size=hash_size, method=method)
    got, st = build(native, log, seed, hash_size, method)
    assert got == want, diff_report(got, want)
    return st


def header_like_puts(n, seed, kmin=8, kmax=64, vmin=20, vmax=120):
    """PUTs whose value bytes are all small (0x01 .. 0x3f): nearly every byte pair passes the header
    screen, so false record starts survive several steps and chains of false starts form."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kl = int(rng.integers(kmin, kmax + 1))
        key = i.to_bytes(4, "little") + rng.integers(1, 0x40, size=kl - 4, dtype=np.uint8).tobytes()
        vl = int(rng.integers(vmin, vmax + 1))
        out.append((key, rng.integers(1, 0x40, size=vl, dtype=np.uint8).tobytes()))
    return out


SHAPES = [(61, (8, 64, 100, 100), 8), (63, (4, 40, 20, 60), 4), (67, (10, 100, 0, 60), 8),
          (69, (16, 16, 100, 100), 8)]


@pytest.mark.parametrize("sw", [{}, {"frame4_c": 64}, {"frame4_c": 128}, {"frame4_c": 256},
                                {"frame4_c": 512}, {"frame_ticket": 1}])
def test_frame4_geometry(native, switch, sw):
    switch(frame4=1, no_uniform=1, **sw)
    for seed, (kmin, kmax, vmin, vmax), hs in SHAPES:
        puts = random_puts(25000, seed=seed, kmin=kmin, kmax=kmax, vmin=vmin, vmax=vmax)
        st = check(native, make_log(puts), seed, hash_size=hs)
        assert st.framing_path in ((5,) if "frame4_c" not in sw else (0, 4, 5)), st.as_dict()


@pytest.mark.parametrize("c", [0, 64, 128, 256])
def test_frame4_header_like_values(native, switch, c):
    """Values made of header-like bytes: the speculation is wrong often; the bytes are the oracle's."""
    switch(frame4=1, **({"frame4_c": c} if c else {}))
    for seed in (101, 103):
        st = check(native, make_log(header_like_puts(20000, seed)), seed)
        assert st.framing_path in (0, 4, 5), st.as_dict()


def test_frame4_matches_frame3_c3_shape(native, switch):
    """A C3-shaped log (8-64 B keys, 100 B values, 200K records) through k_frame4 and k_frame3."""
    from sparkey import synth
    log = synth.mixed_log(200_000, 8, 64, 100, seed=5).tobytes()
    switch(frame4=1)
    a, sa = build(native, log, 99)
    switch(frame4=0)
    b, sb = build(native, log, 99)
    assert sa.framing_path == 5 and sb.framing_path == 4, (sa.as_dict(), sb.as_dict())
    assert a == b
    want = oracle.build_index(log, 99, hash_size=8)
    assert a == want, diff_report(a, want)


def test_frame4_sorting(native, switch):
    switch(frame4=1)
    puts = random_puts(30000, seed=107, kmin=8, kmax=64, vmin=90, vmax=110)
    st = check(native, make_log(puts), 107, method=2)
    assert st.framing_path == 5, st.as_dict()


def test_frame4_deletes_and_overwrites(native, switch):
    switch(frame4=1)
    rng = np.random.default_rng(109)
    ops = []
    for i in range(60000):
        k = b"k%d" % int(rng.integers(0, 20000))
        k = k + b"x" * max(0, int(rng.integers(8, 41)) - len(k))
        ops.append(("del", k, None) if rng.random() < 0.1 else ("put", k, bytes(int(rng.integers(20, 91)))))
    st = check(native, make_log(ops=ops), 109)
    assert st.framing_path == 5 and st.placement_path == 2, st.as_dict()


def test_frame4_list_caps_fall_back(native, switch):
    """A stretch of 2-3 byte records among long ones: more starts in a chunk than k_frame4's lists
    hold; the build reruns with k_frame3 or k_frame (same bytes)."""
    switch(frame4=1)
    puts = random_puts(4000, seed=111, kmin=30, kmax=60, vmin=100, vmax=120)
    puts += [(bytes([i & 0xFF, i >> 8]), b"") for i in range(3000)]
    puts += random_puts(4000, seed=112, kmin=30, kmax=60, vmin=100, vmax=120)
    seen, uniq = set(), []
    for k, v in puts:
        if k not in seen:
            seen.add(k)
            uniq.append((k, v))
    st = check(native, make_log(uniq), 113)
    assert st.framing_path in (0, 4), st.as_dict()


def test_frame4_understated_header(native, switch):
    """maxValueLen understated: the verified chain breaks the header's maxima; the build reruns down to
    the serial walk and matches the oracle."""
    import struct
    switch(frame4=1)
    log = bytearray(make_log(random_puts(20000, seed=115, kmin=8, kmax=64, vmin=90, vmax=110)))
    struct.pack_into("<q", log, 48, 95)
    check(native, bytes(log), 115)


def test_frame4_wait_timeout(native, switch):
    """No wait at all: a wave whose predecessor has not published yet gives up, and the build reruns
    (down to the serial walk when k_frame3 and k_frame give up too)."""
    switch(frame4=1, frame_spin_ticks=0)
    puts = random_puts(120000, seed=117, kmin=8, kmax=64, vmin=100, vmax=100)
    st = check(native, make_log(puts), 117)
    assert st.framing_path in (1, 5), st.as_dict()


@pytest.mark.parametrize("tail", [b"\x80", b"\xff\xff\xff", b"\x81\x82\x83\x84"])
def test_frame4_eof_inside_first_vlq(native, switch, tail):
    switch(frame4=1)
    base = make_log(random_puts(5000, seed=7, kmin=8, kmax=64, vmin=90, vmax=110))
    check(native, with_trailing_bytes(base, tail), 19)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 10, 63, 64, 65, 100, 1000])
def test_frame4_small_logs(native, switch, n):
    """Logs shorter than a wave, or than one chunk: the frame's first wave alone."""
    switch(frame4=1)
    check(native, make_log(random_puts(n, seed=n, kmin=8, kmax=64, vmin=0, vmax=100)), 5)
