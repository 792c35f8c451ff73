"""Pins the CPU oracle (oracle/sparkey_oracle.c) to the reference's own known-answer tests and
invariants before anything is compared against it.  CPU only.
"""
import json
import os
import struct

import numpy as np
import pytest

import oracle
from helpers import index_header, key_value_puts, make_log

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# MurmurHash3Test.java:25-177 (150 x86_32 KATs)
def test_murmur3_x86_32_kats(oracle_mod):
    kats = load("murmur3_kat.json")["x86_32"]
    assert len(kats) == 150
    for v in kats:
        assert oracle.murmur3_x86_32(v["key"].encode(), v["seed"]) == v["expected"], v


# MurmurHash3Test.java:179-481 (300 x64_64 KATs, seeds s and s|0x80000000) + :483-487 binary
def test_murmur3_x64_64_kats(oracle_mod):
    k = load("murmur3_kat.json")
    assert len(k["x64_64"]) == 300 and len(k["x64_64_binary"]) == 1
    for v in k["x64_64"]:
        assert oracle.murmur3_x64_64(v["key"].encode(), v["seed"]) == v["expected"], v
    for v in k["x64_64_binary"]:
        assert oracle.murmur3_x64_64(bytes.fromhex(v["key_hex"]), v["seed"]) == v["expected"]


# UtilTest.java:43-87
def test_vlq_kats(oracle_mod):
    k = load("vlq_kat.json")
    for v in k["size"]:
        assert oracle.vlq_size(v["value"]) == v["expected"], v
    for v in k["decode"]:
        rc, val, pos = oracle.vlq_read(bytes(v["bytes"]))
        assert rc == 0 and val == v["expected"] and pos == len(v["bytes"])
        assert oracle.vlq_write(v["expected"]) == bytes(v["bytes"])
    for b in k["too_long"]:
        rc, _, _ = oracle.vlq_read(bytes(b))
        assert rc == -6  # "Too long VLQ value"


# AddressSizeTest.java:16-48 and BytesWrittenTest.java:43-57
def test_format_kats(oracle_mod):
    k = load("format_kat.json")
    a = k["address_size"]
    assert struct.unpack("<Q", bytes(a["long"]["bytes"]))[0] == a["long"]["value"]
    assert struct.unpack("<I", bytes(a["int"]["bytes"]))[0] == a["int"]["value"]
    bw = k["bytes_written"]
    lb = oracle.LogBuilder(1, 20)
    for kl, vl, cnt in bw["puts"]:
        for _ in range(cnt):
            lb.put(b"k" * kl, b"v" * vl)
    for kl, cnt in bw["deletes"]:
        for _ in range(cnt):
            lb.delete(b"k" * kl)
    log = lb.finish()
    put_size, = struct.unpack_from("<q", log, 72)
    delete_size, = struct.unpack_from("<q", log, 56)
    assert put_size == bw["put_size"] and delete_size == bw["delete_size"]


def test_log_writer_python_matches_oracle(tmp_path, oracle_mod):
    """The package's Python LogWriter writes the same bytes as the oracle's LogWriter restatement."""
    from sparkey.log_writer import LogWriter
    p = str(tmp_path / "a.spl")
    lw = LogWriter.createNew(p, 0, 1024, file_identifier=0x1234567)
    lb = oracle.LogBuilder(0x1234567, 1024)
    for i in range(300):
        lw.put(b"key_%d" % i, b"value_%d" % i * (i % 5))
        lb.put(b"key_%d" % i, b"value_%d" % i * (i % 5))
    for i in range(0, 300, 7):
        lw.delete(b"key_%d" % i)
        lb.delete(b"key_%d" % i)
    lw.delete(b"x" * 100)  # longer than maxKeyLen: dropped (LogWriter.java:110-115)
    lb.delete(b"x" * 100)
    lw.close()
    assert open(p, "rb").read() == lb.finish()


def test_synth_logs_match_log_writer(oracle_mod):
    from sparkey import synth
    log = synth.fixed_log(50, 16, 100, seed=9, file_id=77).tobytes()
    body = log[84:]
    lb = oracle.LogBuilder(77, 0)
    for i in range(50):
        rec = body[i * 118:(i + 1) * 118]
        lb.put(rec[2:18], rec[18:])
    assert lb.finish() == log
    log = synth.mixed_log(200, 8, 64, 100, seed=4, file_id=78).tobytes()
    lb = oracle.LogBuilder(78, 0)
    p = 84
    while p < len(log):
        kl = log[p] - 1
        lb.put(log[p + 2:p + 2 + kl], log[p + 2 + kl:p + 2 + kl + 100])
        p += 2 + kl + 100
    assert lb.finish() == log
    assert synth.key_value_log(100) == make_log(key_value_puts(100, b"key_%d", b"value_%d"), file_id=0x0C1C1C1C,
                                                block_size=1024)


# TestSparkeyWriter.java:9-36: IN_MEMORY and SORTING produce byte-identical files, on the
# reference's scenarios (CorrectnessTest SIZES, deletes every 7th, overwrite, large file).
@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 10, 100])
@pytest.mark.parametrize("hash_size", [4, 8])
def test_in_memory_equals_sorting(oracle_mod, n, hash_size):
    log = make_log(key_value_puts(n))
    a = oracle.build_index(log, 1738868818, hash_size=hash_size, method=oracle.IN_MEMORY)
    b = oracle.build_index(log, 1738868818, hash_size=hash_size, method=oracle.SORTING)
    assert a == b
    for i in range(n):
        assert oracle.get(a, log, b"Key%d" % i) == b"Value%d" % i


@pytest.mark.parametrize("n", [1, 10, 100, 1000])
def test_deletes_in_memory_equals_sorting(oracle_mod, n):
    log = make_log(key_value_puts(n), deletes=[b"Key%d" % i for i in range(n) if i % 7 == 0])
    a = oracle.build_index(log, -112683590, method=oracle.IN_MEMORY)
    b = oracle.build_index(log, -112683590, method=oracle.SORTING)
    assert a == b
    for i in range(n):
        assert oracle.get(a, log, b"Key%d" % i) == (None if i % 7 == 0 else b"Value%d" % i)


def test_correct_hash_large_file(oracle_mod):
    """CorrectnessTest.testCorrectHashLargeFile (:178-200)."""
    n = 170000
    log = make_log(key_value_puts(n))
    a = oracle.build_index(log, 1234, hash_size=4, method=oracle.IN_MEMORY)
    h = index_header(a)
    assert h["garbageSize"] == 0 and h["hashCollisions"] > 0 and h["numEntries"] == n
    assert a == oracle.build_index(log, 1234, hash_size=4, method=oracle.SORTING)
    for i in range(0, n, 101):
        assert oracle.get(a, log, b"Key%d" % i) == b"Value%d" % i


def test_index_header_layout(oracle_mod):
    """IndexHeader.asBytes offsets (IndexHeader.java:125-155) and createNew parameters (:135-150)."""
    log = make_log(key_value_puts(1000, b"key_%d", b"value_%d"), block_size=1024)
    spi = oracle.build_index(log, 1234, method=oracle.IN_MEMORY)
    h = index_header(spi)
    assert h["magic"] == 0x9A11318F and h["major"] == 1 and h["minor"] == 1
    assert h["capacity"] == 1301 and h["hashSize"] == 4 and h["addressSize"] == 4
    assert h["numPuts"] == 1000 and h["numEntries"] == 1000 and h["dataEnd"] == len(log) == 17864
    assert len(spi) == 112 + 8 * 1301 == 10520


def test_canonical_layout_matches_sequential(oracle_mod):
    """Independent second algorithm (DESIGN.md "canonical placement"): for unique-key PUT logs the
    Robin-Hood table equals sort-by-(wantedSlot, address) + prefix max + wrap fix-up."""
    from canonical import canonical_table
    for n, hs, seed in [(1000, 4, 1), (5000, 8, 2), (13, 4, 3), (64, 8, 4), (3000, 4, 5)]:
        log = make_log(key_value_puts(n))
        want = oracle.build_index(log, seed, hash_size=hs, method=oracle.IN_MEMORY)
        got = canonical_table(log, seed, hs)
        assert got == want[112:]


@pytest.mark.parametrize("tail", [b"\x80", b"\xff\xff", b"\x81\x82\x83\x84"])
def test_eof_inside_first_vlq_ends_iteration(oracle_mod, tail):
    """dataEnd == file length and the last record's first VLQ cut after continuation bytes: hasNext
    catches the EOFException and ends the iteration (SparkeyLogIterator.java:111-115), so the index
    holds the earlier records and no error is raised."""
    from helpers import index_header, key_value_puts, make_log, with_trailing_bytes
    base = make_log(key_value_puts(500))
    log = with_trailing_bytes(base, tail)
    for method in (oracle.IN_MEMORY, oracle.SORTING):
        got = oracle.build_index(log, 42, method=method)
        want = oracle.build_index(base, 42, method=method)
        assert got[112:] == want[112:]  # the same slots; only the header's dataEnd differs
        assert index_header(got)["dataEnd"] == len(log) and index_header(got)["numEntries"] == 500


def test_eof_inside_second_vlq_is_an_error(oracle_mod):
    """EOF inside the second VLQ is wrapped in a RuntimeException (SparkeyLogIterator.java:117,134-136)."""
    from helpers import key_value_puts, make_log, with_trailing_bytes
    log = with_trailing_bytes(make_log(key_value_puts(50)), b"\x05\x80")
    with pytest.raises(oracle.OracleError) as e:
        oracle.build_index(log, 42)
    assert e.value.code == -13  # ORACLE_E_CORRUPT_RECORD


def test_key_value_log_np_matches_writer(oracle_mod):
    """WriteHashBenchmark's data (put("key_" + i, "value_" + i), block size 1024) from the numpy generator
    equals the LogWriter restatement's bytes across the digit-count boundaries."""
    from sparkey import synth
    for n in (0, 1, 10, 11, 1000, 10001):
        assert synth.key_value_log_np(n).tobytes() == make_log(key_value_puts(n, b"key_%d", b"value_%d"),
                                                               file_id=0x0C1C1C1C, block_size=1024)
