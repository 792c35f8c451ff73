"""GPU parity: the HIP build (through the C-ABI) must produce .spi bytes identical to the oracle's
sequential restatement of IndexHash.createNew (IN_MEMORY and SORTING), on the reference's own test
scenarios (CorrectnessTest, LargeFilesTest, IndexHashTest, WriteHashBenchmark) and on edge cases.
Integer/byte work: the bar is bit-exact.
"""
import numpy as np

import pytest

import oracle
from helpers import diff_report, index_header, key_value_puts, make_log, random_puts, same_error

pytestmark = pytest.mark.gpu

IN_MEMORY, SORTING = 1, 2
SPEC = (0, 4)  # the speculative framings of mixed-size records: k_frame, k_frame3 (one-byte VLQs)


def gpu_build(native, log, seed, hash_size=0, method=IN_MEMORY, sparsity=0.0):
    opts = native.make_opts(hash_size=hash_size, hash_seed=seed, sparsity=sparsity, method=method)
    spi, stats = native.build_index_mem(log, opts)
    return spi, stats


def check(native, log, seed, hash_size=0, method=IN_MEMORY, sparsity=0.0, expect_path=None):
    want = oracle.build_index(log, seed, hash_size=hash_size, sparsity=sparsity, method=method)
    got, stats = gpu_build(native, log, seed, hash_size, method, sparsity)
    assert got == want, diff_report(got, want)
    if expect_path is not None:
        assert stats.placement_path == expect_path, stats.as_dict()
    return got, stats


# --- WriteHashBenchmark (config C1): 1000 x put("key_"+i, "value_"+i), block size 1024 ---
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_c1_write_hash_benchmark(native, method):
    log = make_log(key_value_puts(1000, b"key_%d", b"value_%d"), block_size=1024)
    spi, stats = check(native, log, 1234, method=method, expect_path=0)
    assert len(spi) == 10520 and stats.hash_size == 4 and stats.address_size == 4


# --- CorrectnessTest.SIZES = {0,1,2,3,4,10,100} x hash types (CorrectnessTest.java:38,190-220) ---
@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 10, 100])
@pytest.mark.parametrize("hash_size", [4, 8])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_sizes(native, n, hash_size, method):
    log = make_log(key_value_puts(n))
    check(native, log, 1738868818, hash_size=hash_size, method=method)


# --- testHelperWithDeletes: delete every 7th key (CorrectnessTest.java:109-162) ---
@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 10, 100, 1000])
@pytest.mark.parametrize("hash_size", [4, 8])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_deletes_every_7th(native, n, hash_size, method):
    log = make_log(key_value_puts(n), deletes=[b"Key%d" % i for i in range(n) if i % 7 == 0])
    got, stats = check(native, log, -112683590, hash_size=hash_size, method=method)
    if n:  # PUTs filling every slot (capacity = 1 | (long)(n * 1.3)) leave no segment: the single lane
        assert stats.placement_path == (1 if n >= (int(n * 1.3) | 1) else 2)
    for i in range(n):
        v = oracle.get(got, log, b"Key%d" % i)
        assert v == (None if i % 7 == 0 else b"Value%d" % i)


# --- testCorrectHashLargeFile: 170,000 keys, seed 1234, 32-bit (CorrectnessTest.java:178-200) ---
def test_correct_hash_large_file(native):
    n = 170000
    log = make_log(key_value_puts(n))
    got, stats = check(native, log, 1234, hash_size=4, expect_path=0)
    h = index_header(got)
    assert h["garbageSize"] == 0 and h["hashCollisions"] > 0
    assert oracle.build_index(log, 1234, hash_size=4, method=SORTING) == got
    for i in range(0, n, 997):
        assert oracle.get(got, log, b"Key%d" % i) == b"Value%d" % i


# --- testOverwrite / duplicates: re-put replaces in place (IndexHash.java:606-636) ---
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_overwrite_duplicates(native, method):
    puts = key_value_puts(500) + [(b"Key%d" % i, b"New%d" % i) for i in range(0, 500, 3)]
    log = make_log(puts)
    got, stats = check(native, log, 99, method=method, expect_path=2)
    assert index_header(got)["garbageSize"] > 0


def test_overwrite_single_key(native):
    log = make_log([(b"A", b"B")])
    check(native, log, 5)


@pytest.mark.parametrize("hash_size", [4, 8])
def test_many_equal_wanted_slots(native, hash_size):
    """More than 255 entries wanting one slot (one key put 600 times among 20000 others): k_part2st's
    8-bit slot count would overflow, so the build redoes its partition with dense runs; the exact path
    then replays the overwrites.  The oracle's bytes either way."""
    puts = [(b"k%d" % i, b"v%d" % i) for i in range(20000)]
    puts[5000:5000] = [(b"hot", b"x%d" % i) for i in range(600)]
    got, stats = check(native, make_log(puts), 31, hash_size=hash_size, expect_path=2)
    assert index_header(got)["garbageSize"] > 0


# --- LargeFilesTest: values larger than a framing chunk (LargeFilesTest.java:28-50) ---
def test_large_values(native):
    value = b"value"
    while len(value) < 5 * 1024:
        value += value
    log = make_log([(b"key_%d" % i, value) for i in range(2000)], block_size=1024)
    got, stats = check(native, log, 77, expect_path=0)
    assert oracle.get(got, log, b"key_100") == value


# --- LargeFilesTest.testLargeIndexFileInner: 64-bit hash, value "i % 13" ---
@pytest.mark.parametrize("n", [7000, 150000])
def test_large_index_file(native, n):
    log = make_log([(b"key_%d" % i, b"%d" % (i % 13)) for i in range(n)], block_size=1024)
    check(native, log, 4242, hash_size=8, expect_path=0)


# --- random logs: key lengths 0..300 (multi-block murmur tails), values 0..5000 ---
@pytest.mark.parametrize("seed", range(6))
def test_random_logs(native, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 3000))
    puts = random_puts(n, seed=seed, kmin=0 if seed % 2 else 4, kmax=[16, 40, 130, 300, 8, 64][seed],
                       vmax=[0, 10, 100, 5000, 300, 1][seed])
    log = make_log(puts)
    for hs in (4, 8):
        check(native, log, int(rng.integers(-2**31, 2**31)), hash_size=hs)


# --- sparsity, and a hash seed with the high bit set (unsigned widening, MurmurHash3.java:103) ---
@pytest.mark.parametrize("sparsity", [1.0, 1.3, 2.0, 7.5])
def test_sparsity(native, sparsity):
    log = make_log(key_value_puts(4000))
    check(native, log, -5, hash_size=8, sparsity=sparsity)


# --- nearly full tables: wrap-around clusters (sparsity floor 1.3, small n) ---
@pytest.mark.parametrize("n", [5, 6, 7, 8, 9, 13, 31, 64])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_small_tables_wrap(native, n, seed):
    log = make_log(key_value_puts(n))
    check(native, log, seed, hash_size=4)
    check(native, log, seed, hash_size=8)


# --- mixed puts/deletes/re-puts interleaved ---
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_interleaved_ops(native, method):
    rng = np.random.default_rng(11)
    ops = []
    for i in range(3000):
        k = b"k%d" % int(rng.integers(0, 800))
        if rng.random() < 0.2:
            ops.append(("del", k, None))
        else:
            ops.append(("put", k, b"v%d" % i))
    log = make_log(ops=ops)
    check(native, log, 31337, method=method)


# --- error behaviour (LogHeader.read, CommonHeader, iterator) ---
def test_errors(native):
    log = make_log(key_value_puts(10))
    opts = native.make_opts(hash_seed=1)
    with pytest.raises(OSError):
        native.build_index_mem(b"\0" * 84 + log[84:], opts)       # "File is not a Sparkey log file"
    bad = bytearray(log)
    bad[4] = 2
    with pytest.raises(OSError):
        native.build_index_mem(bytes(bad), opts)                   # major version
    trunc = log[:-5]
    with pytest.raises(OSError):
        native.build_index_mem(trunc, opts)                        # dataEnd > file length
    bad = bytearray(log)
    bad[84] = 0xFF                                                 # corrupt first record header
    same_error(native, bytes(bad))
    bad = bytearray(log)
    bad[64] = 1                                                    # SNAPPY flag over NONE bytes: corrupt blocks
    same_error(native, bytes(bad))


# --- framing edge cases: the speculative framing must fall back to the exact serial walk ---
def test_header_understates_max_value_len(native):
    """The reference never checks valueLen against maxValueLen; speculation prunes with it, so a
    log whose header understates it must still build identically (chunks whose true chain looks
    implausible are walked serially with the reference iterator's rules)."""
    import struct
    log = bytearray(make_log([(b"k%d" % i, b"v" * (i % 300)) for i in range(5000)]))
    struct.pack_into("<q", log, 48, 10)  # maxValueLen := 10
    check(native, bytes(log), 3)


def test_trailing_bytes_after_data_end(native):
    log = make_log(key_value_puts(3000)) + b"\x05garbage" * 1000  # records start < dataEnd only
    check(native, log, 8)


@pytest.mark.parametrize("vlen", [4000, 4096, 9000, 70000])
def test_records_spanning_chunks(native, vlen):
    """Records as long as or longer than a framing chunk; past 4 KiB records the build frames the
    log with the serial walker (few records per byte)."""
    puts = [(b"key%d" % i, bytes([i % 251]) * (vlen + (i % 7))) for i in range(300)]
    got, stats = check(native, make_log(puts), 12, hash_size=8)
    assert stats.framing_path in (SPEC if vlen + 6 + 16 < 4096 else (1,))


def test_understated_max_key_len_is_an_error(native):
    import struct
    log = bytearray(make_log(key_value_puts(100)))
    struct.pack_into("<q", log, 40, 3)  # maxKeyLen := 3 < real key lengths: the reference throws
    got, want = same_error(native, bytes(log))  # IndexOutOfBoundsException (SparkeyLogIterator.java:130)
    assert got == want == native.E_CORRUPT_RECORD
    for sw in ({"no_uniform": 1}, {"no_frame3": 1}, {"serial_framing": 1}):
        with native.debug(**sw):
            got, _ = same_error(native, bytes(log))
        assert got == native.E_CORRUPT_RECORD, sw


def test_header_hides_deletes(native):
    """numDeletes = 0 in a header of a log that holds DELETE records: speculation prunes DELETE
    starts, the verified chain disagrees, the exact path still gives the reference's bytes."""
    import struct
    log = bytearray(make_log(key_value_puts(3000), deletes=[b"Key%d" % i for i in range(0, 3000, 5)]))
    struct.pack_into("<q", log, 24, 0)
    check(native, bytes(log), 21)


# --- tiny records (2-6 bytes): many records per framing chunk; the speculative framing must stay on
#     its fast path (a chunk whose candidate walk does not fit its record is walked exactly) ---
def test_tiny_records_stay_on_fast_framing(native):
    puts = random_puts(60000, seed=5, kmin=0, kmax=3, vmin=0, vmax=2)
    got, stats = check(native, make_log(puts), 17, hash_size=8)
    assert stats.framing_path == 0, stats.as_dict()


# --- k_frame geometry overrides (chunk 256..2048 bytes, region, look-ahead): same bytes, fast path ---
@pytest.mark.parametrize("sw", [{"frame_cmin": 256}, {"frame_cmin": 1024}, {"frame_cmin": 2048},
                                {"frame_region": 16384}, {"frame_look": 16}, {"frame_look": 1024},
                                {"frame_ticket": 1}])
def test_frame_geometry_overrides(native, switch, sw):
    switch(no_uniform=1)  # the fixed-size log would take k_frame_uniform
    switch(no_frame3=1)   # k_frame's geometry (k_frame3: test_frame3_geometry)
    switch(**sw)
    rng = np.random.default_rng(3)
    puts = [(b"%016d" % i, rng.integers(0, 256, 100, dtype=np.uint8).tobytes()) for i in range(40000)]
    got, stats = check(native, make_log(puts), 23, hash_size=8)
    assert stats.framing_path == 0, stats.as_dict()
    puts = random_puts(30000, seed=9, kmin=0, kmax=3, vmin=0, vmax=2)
    got, stats = check(native, make_log(puts), 29, hash_size=4)
    assert stats.framing_path == 0, stats.as_dict()


def test_deletes_take_k_frame(native):
    """A log with DELETEs (0x00 starts a record) and zero-filled values frames speculatively."""
    ops = _churn_ops(60000, 20000, 0.1, 57, klen=(8, 40), vlen=(20, 90))
    got, stats = check(native, make_log(ops=ops), 59, hash_size=8)
    assert stats.framing_path in SPEC and stats.placement_path == 2, stats.as_dict()


# --- k_frame's bounded wait on the previous wave: a tripped wait reruns the build on the serial path ---
def test_frame_wait_timeout_falls_back_to_serial(native, switch):
    switch(no_uniform=1, frame_spin_ticks=0)  # any wait for a predecessor trips at once
    puts = random_puts(120000, seed=31, kmin=1, kmax=40, vmin=0, vmax=60)
    got, stats = check(native, make_log(puts), 37, hash_size=8)
    assert stats.framing_path == 1, stats.as_dict()
    switch(frame_spin_ticks=None)
    got2, stats2 = check(native, make_log(puts), 37, hash_size=8)
    assert stats2.framing_path in SPEC and got2 == got


# --- exact path (DELETEs, overwrites) over independent slot segments vs the single-lane replay ---
def _churn_ops(n, nkeys, p_del, seed, klen=(1, 24), vlen=(0, 40)):
    rng = np.random.default_rng(seed)
    ops = []
    for i in range(n):
        k = b"k%d" % int(rng.integers(0, nkeys))
        k = k + b"x" * max(0, int(rng.integers(klen[0], klen[1] + 1)) - len(k))
        if rng.random() < p_del:
            ops.append(("del", k, None))
        else:
            ops.append(("put", k, bytes(int(rng.integers(vlen[0], vlen[1] + 1)))))
    return ops


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
@pytest.mark.parametrize("n,nkeys,p_del", [(200000, 150000, 0.1), (200000, 20000, 0.3), (100000, 100000, 0.0),
                                           (50000, 500, 0.45)])
def test_exact_segments_churn(native, method, n, nkeys, p_del):
    log = make_log(ops=_churn_ops(n, nkeys, p_del, seed=n + nkeys))
    got, stats = check(native, log, 4711, hash_size=8, method=method)
    assert stats.placement_path == 2, stats.as_dict()


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_exact_segments_equal_serial_replay(native, switch, method):
    log = make_log(ops=_churn_ops(30000, 8000, 0.25, seed=3))
    seg, st1 = gpu_build(native, log, 77, 4, method)
    switch(exact_serial=1)
    ser, st2 = gpu_build(native, log, 77, 4, method)
    assert st1.placement_path == 2 and st2.placement_path == 1
    assert seg == ser, diff_report(seg, ser)
    assert seg == oracle.build_index(log, 77, hash_size=4, method=method)


# small tables: segments that wrap from slot cap-1 to slot 0, DELETEs of keys never put
@pytest.mark.parametrize("n", [3, 5, 8, 13, 31, 64, 200])
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_exact_segments_small_tables(native, n, seed, method):
    ops = _churn_ops(n, max(2, n // 2), 0.3, seed=seed * 1000 + n)
    ops.append(("del", b"never-put", None))
    log = make_log(ops=ops)
    for hs in (4, 8):
        check(native, log, seed, hash_size=hs, method=method)


# one hot key written thousands of times: all its records share a wanted slot, so its segment holds
# more records than a workgroup stages in LDS (the lane-0 HBM replay); warm keys give mid-size ones
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_exact_segments_hot_keys(native, method):
    rng = np.random.default_rng(8)
    ops = []
    for i in range(20000):
        r = rng.random()
        if r < 0.12:
            ops.append(("put", b"hot", b"v%d" % i))
        elif r < 0.14:
            ops.append(("del", b"hot", None))
        elif r < 0.30:
            ops.append(("put", b"warm%d" % int(rng.integers(0, 8)), b"w%d" % i))
        else:
            ops.append(("put", b"cold%d" % int(rng.integers(0, 12000)), b"c"))
    log = make_log(ops=ops)
    for hs in (4, 8):
        got, stats = check(native, log, 1 + hs, hash_size=hs, method=method)
        assert stats.placement_path == 2


# --- uniform records: the header proves every record has the same size (k_frame_uniform) ---
def _uniform_puts(n, klen, vlen, seed=0, dup_every=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        j = i // 2 if dup_every and i % dup_every == 0 else i
        out.append((j.to_bytes(8, "little")[:klen].ljust(klen, b"k"), rng.integers(0, 256, vlen, dtype=np.uint8).tobytes()))
    return out


@pytest.mark.parametrize("klen,vlen", [(16, 100), (8, 0), (4, 1), (64, 63), (126, 127)])
@pytest.mark.parametrize("hash_size", [4, 8])
def test_uniform_records(native, klen, vlen, hash_size):
    log = make_log(_uniform_puts(30000 if klen >= 4 else 250, klen, vlen, seed=klen))
    got, stats = check(native, log, 99 + klen, hash_size=hash_size)
    assert stats.framing_path == 2, stats.as_dict()


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_uniform_records_with_overwrites(native, method):
    log = make_log(_uniform_puts(20000, 16, 20, dup_every=5))
    got, stats = check(native, log, 5, hash_size=8, method=method)
    assert stats.framing_path == 2 and stats.placement_path == 2, stats.as_dict()


def test_uniform_header_but_record_split_differs(native):
    """putSize == numPuts * R, yet one record trades a key byte for a value byte (same size): the
    uniform framing must notice the header mismatch and rerun the general framing."""
    puts = _uniform_puts(5000, 16, 30)
    puts[2500] = (puts[2500][0][:15], puts[2500][1] + b"x")
    import struct
    log = bytearray(make_log(puts))
    struct.pack_into("<q", log, 40, 16)  # maxKeyLen stays 16, maxValueLen stays 31 ...
    struct.pack_into("<q", log, 48, 30)  # ... declare maxValueLen 30 so putSize == n * (2 + 16 + 30)
    got, stats = check(native, bytes(log), 7, hash_size=8)
    assert stats.framing_path in SPEC, stats.as_dict()


def test_uniform_disabled_gives_same_bytes(native, switch):
    log = make_log(_uniform_puts(40000, 16, 100))
    a, sa = gpu_build(native, log, 11, 8)
    switch(no_uniform=1)
    b, sb = gpu_build(native, log, 11, 8)
    assert sa.framing_path == 2 and sb.framing_path in SPEC and a == b


@pytest.mark.parametrize("klen,vlen,hash_size", [(16, 100, 8), (16, 100, 4), (8, 0, 8), (126, 127, 8)])
def test_uniform_compact_entries(native, switch, klen, vlen, hash_size):
    """The uniform staged path carries 12-byte entries (hash, record index) from k_frame_uniform through
    k_part2st to k_place_reg, the address rebuilt from the index (BuildParams.compact); the no_compact
    switch keeps 16-byte entries.  Both give the oracle's bytes."""
    log = make_log(_uniform_puts(60000, klen, vlen, seed=klen + vlen))
    got, stats = check(native, log, 31 + klen, hash_size=hash_size, expect_path=0)
    assert stats.framing_path == 2, stats.as_dict()
    switch(no_compact=1)
    b, _ = gpu_build(native, log, 31 + klen, hash_size)
    assert b == got


@pytest.mark.parametrize("shape", ["uniform", "general", "c3", "hot"])
def test_part2_two_level(native, switch, shape):
    """Pass 2 in two levels (k_part2_sub into sub-digit regions, k_part2_subf into the bucket regions),
    which C4's 4960 buckets a digit take by default, forced on smaller tables: compact entries from the
    uniform framing, 16-byte ones from the slab framings.  The oracle's bytes, and those of the one-level
    pass."""
    if shape == "uniform":
        log = make_log(_uniform_puts(120000, 16, 100, seed=5))
    elif shape == "hot":  # one key 400 times: its slot's 8-bit count wraps (p2_overflow, the dense redo)
        puts = _uniform_puts(120000, 16, 100, seed=8)
        log = make_log(puts + [(puts[7][0], bytes(100))] * 400)
    elif shape == "general":
        log = make_log(_uniform_puts(120000, 16, 100, seed=6) + [(b"short", b"v")])
    else:
        rng = np.random.default_rng(7)
        log = make_log([(rng.integers(0, 256, int(rng.integers(8, 65)), dtype=np.uint8).tobytes(), bytes(100))
                        for _ in range(80000)])
    if shape != "uniform":
        switch(no_buckets=1)  # (k_frame3 would write the bucket regions itself: slabs and pass 1 instead)
    one, _ = gpu_build(native, log, 41, 8)
    switch(part2_two_level=1)
    got, stats = check(native, log, 41, hash_size=8)
    assert got == one, diff_report(got, one)


@pytest.mark.parametrize("region_cap", [60000, 1])
def test_uniform_digit_regions(native, switch, region_cap):
    """k_frame_uniform as partition pass 1 (entries straight into digit regions of ent3): a region
    that fills up (forced with a region capacity of 1) redoes the build with the separate pass; both
    give the reference's bytes, and so does the separate pass by request."""
    log = make_log(_uniform_puts(50000, 16, 40, seed=3))
    want, _ = gpu_build(native, log, 21, 8)
    switch(region_cap=region_cap)
    got, stats = check(native, log, 21, hash_size=8)
    assert stats.framing_path == 2 and got == want
    switch(region_cap=None, no_regions=1)
    b, _ = gpu_build(native, log, 21, 8)
    assert b == want


# --- batched IndexHash.get on the GPU (sparkey_get_batch) against the oracle's get ---
def _reader(log, spi):
    from sparkey.reader import GpuHashReader
    return GpuHashReader(log, spi)


@pytest.mark.parametrize("hash_size", [4, 8])
def test_get_batch_matches_oracle(native, hash_size):
    ops = []
    rng = np.random.default_rng(hash_size)
    for i in range(20000):
        k = b"k%d" % int(rng.integers(0, 6000))
        ops.append(("del", k, None) if rng.random() < 0.15 else ("put", k, b"v%d" % i))
    log = make_log(ops=ops)
    spi, _ = gpu_build(native, log, 321, hash_size)
    keys = [b"k%d" % i for i in range(6500)] + [b"", b"absent", b"k" * 300]
    r = _reader(log, spi)
    got = r.get_batch(keys)
    r.close()
    want = [oracle.get(spi, log, k) for k in keys]
    assert got == want


def test_get_batch_c1_and_errors(native):
    log = make_log(key_value_puts(1000, b"key_%d", b"value_%d"), block_size=1024)
    spi, _ = gpu_build(native, log, 1234)
    r = _reader(log, spi)
    assert r.get_batch([b"key_%d" % i for i in range(1000)]) == [b"value_%d" % i for i in range(1000)]
    assert r.get(b"key_1000") is None
    r.close()
    other = make_log(key_value_puts(10), file_id=0x777)
    with pytest.raises(ValueError):
        _reader(other, spi).get(b"key_1")          # "Log file did not match index file"
    with pytest.raises(RuntimeError):
        _reader(log, spi[:-4]).get(b"key_1")       # "Corrupt index file - incorrect size"


# --- batched LogWriter.put / delete on the GPU (sparkey_log_append) against the oracle's LogBuilder ---
def test_log_append_matches_log_writer(native):
    from sparkey.gpu_log import DELETE, PUT, GpuLogAppender, new_log_header
    rng = np.random.default_rng(17)
    ops = []
    for i in range(30000):
        r = rng.random()
        kl = int(rng.choice([0, 1, 5, 16, 126, 127, 128, 300]))
        key = bytes(rng.integers(0, 256, kl, dtype=np.uint8))
        if r < 0.2:
            ops.append((DELETE, key, None))  # longer than maxKeyLen so far: dropped, as LogWriter.delete does
        else:
            vl = int(rng.choice([0, 1, 100, 127, 128, 16383, 16384]))
            ops.append((PUT, key, bytes(rng.integers(0, 256, vl, dtype=np.uint8))))
    want = make_log(ops=[("put" if k == PUT else "del", key, v) for k, key, v in ops], file_id=0x51)
    app = GpuLogAppender()
    header = new_log_header(0x51)
    body = app.append(header, ops[:12345]) + app.append(header, ops[12345:])
    app.close()
    assert bytes(header) + body == want


def test_log_append_then_build(native):
    """A log written on the GPU builds to the same index as the reference writer's log."""
    from sparkey.gpu_log import PUT, GpuLogAppender, new_log_header
    ops = [(PUT, b"key_%d" % i, b"value_%d" % i) for i in range(1000)]
    app = GpuLogAppender()
    header = new_log_header(0x0C1C1C1C, 1024)
    body = app.append(header, ops)  # updates header in place
    log = bytes(header) + body
    app.close()
    assert log == make_log(key_value_puts(1000, b"key_%d", b"value_%d"), file_id=0x0C1C1C1C, block_size=1024)
    check(native, log, 1234)


# --- k_frame3: the short/long walk framing of one-byte-VLQ logs ---
@pytest.mark.parametrize("sw", [{}, {"frame3_c": 256}, {"frame3_c": 512}, {"frame3_c": 2048},
                                {"frame3_c": 4096}, {"frame3_c": 8192}, {"frame3_c": 8192, "frame_region": 16384},
                                {"frame_region": 16384}, {"frame_region": 4096}, {"frame_region": 6144},
                                {"frame_ticket": 1}, {"frame3_short": 2}, {"frame3_cover": 1},
                                {"frame_look": 16}, {"frame_look": 1024}])
def test_frame3_geometry(native, switch, sw):
    """Chunk sizes, regions, look-aheads and the ticket launch: the same bytes; k_frame3 frames in the
    default geometry (a geometry whose lists cannot hold a chunk's records reruns with k_frame)."""
    switch(**sw)
    env = sw
    for seed, (kmin, kmax, vmin, vmax), hs in [(61, (8, 64, 100, 100), 8), (63, (1, 40, 20, 60), 4),
                                               (67, (10, 100, 0, 60), 8)]:
        puts = random_puts(25000, seed=seed, kmin=kmin, kmax=kmax, vmin=vmin, vmax=vmax)
        got, stats = check(native, make_log(puts), seed, hash_size=hs)
        assert stats.framing_path == 4 if not env else stats.framing_path in SPEC, stats.as_dict()


def test_frame3_matches_k_frame(native, switch):
    """The same mixed log through k_frame3 and k_frame: identical bytes (and the oracle's)."""
    puts = random_puts(60000, seed=71, kmin=8, kmax=64, vmin=100, vmax=100)
    log = make_log(puts)
    a, sa = check(native, log, 71, hash_size=8)
    switch(no_frame3=1)
    b, sb = gpu_build(native, log, 71, 8)
    assert sa.framing_path == 4 and sb.framing_path == 0 and a == b


def test_frame3_with_deletes_and_overwrites(native):
    """DELETE records (0x00 then starts a record) and overwritten keys through k_frame3; the exact
    replay places."""
    ops = _churn_ops(60000, 20000, 0.1, 73, klen=(8, 40), vlen=(20, 90))
    got, stats = check(native, make_log(ops=ops), 73, hash_size=8)
    assert stats.framing_path in SPEC and stats.placement_path == 2, stats.as_dict()


def test_frame3_list_caps_fall_back(native):
    """A stretch of 2-3 byte records in a log of long ones: more records in a chunk than k_frame3's
    lists hold, so the build reruns with k_frame (same bytes)."""
    puts = random_puts(4000, seed=75, kmin=30, kmax=60, vmin=100, vmax=120)
    puts += [(bytes([i & 0xFF, i >> 8]), b"") for i in range(3000)]
    puts += random_puts(4000, seed=76, kmin=30, kmax=60, vmin=100, vmax=120)
    seen, uniq = set(), []
    for k, v in puts:
        if k not in seen:
            seen.add(k)
            uniq.append((k, v))
    got, stats = check(native, make_log(uniq), 77, hash_size=8)
    assert stats.framing_path in SPEC, stats.as_dict()


def test_frame3_understated_header(native):
    """maxValueLen understated: the screen prunes true starts, k_frame3's chain finds no survivor at
    some entry, the build reruns (k_frame, then the serial walk) and still matches the oracle."""
    import struct
    log = bytearray(make_log(random_puts(20000, seed=79, kmin=8, kmax=64, vmin=90, vmax=110)))
    struct.pack_into("<q", log, 48, 95)
    check(native, bytes(log), 79, hash_size=8)


def test_frame3_wait_timeout(native, switch):
    switch(frame_spin_ticks=0)
    puts = random_puts(120000, seed=81, kmin=8, kmax=64, vmin=100, vmax=100)
    got, stats = check(native, make_log(puts), 83, hash_size=8)
    assert stats.framing_path == 1, stats.as_dict()


@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_exact_reframe_wait_timeout(native, switch, method):
    """The exact path frames a log again when k_frame3 wrote the bucket regions (overwritten keys, no
    DELETE in the header).  A wait that runs out only in that second framing (reframe_spin_ticks)
    goes down k_frame and then the serial walk, each attempt from reset status words, and the bytes
    still match the oracle."""
    switch(reframe_spin_ticks=0)
    ops = _churn_ops(60000, 20000, 0.0, 85, klen=(8, 40), vlen=(20, 90))
    got, stats = check(native, make_log(ops=ops), 85, hash_size=8, method=method)
    assert stats.framing_path == 4 and stats.placement_path == 2, stats.as_dict()


# --- EOF inside the last record's first VLQ ends the iteration quietly (SparkeyLogIterator.java:
#     111-115); inside the second VLQ it is a RuntimeException (:117,134-136) ---
@pytest.mark.parametrize("tail", [b"\x80", b"\xff\xff\xff", b"\x81\x82\x83\x84"])
@pytest.mark.parametrize("sw", [{}, {"no_frame3": 1}, {"serial_framing": 1}])
def test_eof_inside_first_vlq(native, switch, tail, sw):
    from helpers import with_trailing_bytes
    switch(**sw)
    for base in (make_log(key_value_puts(3000)), make_log(random_puts(5000, seed=7, kmin=8, kmax=64, vmin=90,
                                                                       vmax=110))):
        check(native, with_trailing_bytes(base, tail), 19, hash_size=8)


def test_eof_inside_second_vlq(native):
    from helpers import with_trailing_bytes
    got, want = same_error(native, with_trailing_bytes(make_log(key_value_puts(300)), b"\x05\x80"))
    assert got == want == native.E_CORRUPT_RECORD


# --- the ring's wrap: runs that spill past the table's last slot into bucket 0 ---
@pytest.mark.parametrize("spill,mixed", [(40, False), (900, False), (900, True), (40, True), (0, True)])
def test_wrap_into_bucket_0(native, switch, spill, mixed):
    """Keys whose wanted slots crowd the last 4-45 slots of the table (and no other key wants the last
    bucket): their run spills past the end into bucket 0 and on (the ring's carry x0 > 0;
    IndexHash.java:562-665 wraps the probe).  Uniform records take k_frame_uniform's digit regions and
    k_part2st's fused carries; mixed ones k_frame3's bucket regions and k_summary's carries, and again
    through the digit regions (no_buckets).  The bytes are the oracle's."""
    n = 3000
    cap = 1 | int(n * 2.0)  # (sparsity 2: every bucket's entries fit its fixed region of 1024)
    seed = 77
    window = max(4, spill // 20)  # (groups of equal wanted slots stay under kGroupMax = 64)
    crowd, rest, i = [], [], 0
    while len(crowd) < spill or len(rest) < n - spill:
        k = b"w%07d" % i
        i += 1
        slot = oracle.key_hash(4, k, seed) % cap
        if slot >= cap - window:
            if len(crowd) < spill:
                crowd.append(k)
        elif slot < cap - 1100 and len(rest) < n - spill:
            rest.append(k)
    keys = rest[: (n - spill) // 2] + crowd + rest[(n - spill) // 2:]
    rng = np.random.default_rng(spill)
    # (mixed: values of 90-110 random bytes, C3's record sizes)
    puts = [(k, b"v%05d" % j + (rng.integers(0, 256, size=int(rng.integers(84, 105)), dtype=np.uint8).tobytes()
                                if mixed else b"")) for j, k in enumerate(keys)]
    log = make_log(puts)
    got, stats = check(native, log, seed, hash_size=4, sparsity=2.0)
    assert stats.capacity == cap and stats.placement_path == 0, stats.as_dict()
    assert stats.framing_path == (4 if mixed else 2), stats.as_dict()
    assert stats.partition_passes == (0 if mixed else 1), stats.as_dict()
    switch(no_buckets=1)
    got2, st2 = gpu_build(native, log, seed, 4, sparsity=2.0)
    assert got2 == got and st2.partition_passes == (2 if mixed else 1), st2.as_dict()
