"""The drop-in file -> file entry point and the host-side writer mirror.

`sparkey_build_index_file` is what the JNI shim calls in place of IndexHash.createNew
(IndexHash.java:131-167); SparkeyWriter.writeHash (SingleThreadedSparkeyWriter.java:89-108) wraps it
with the seed / maxMemory resolution, the `-tmp<UUID>` file and Util.renameFile (Util.java:278-315).
The .spi file must hold exactly the oracle's bytes for the same log file and seed: header then slots,
as FileFlushingData.close writes them (FileFlushingData.java:20-34).

CPU tests: the writer mirror's log bytes, renameFile, compressed logs opened build-only, and the
file entry point's error codes that are decided before any device work.  GPU tests: the .spi files.
"""
import os
import random
import struct
import threading

import pytest

import oracle
from helpers import diff_report, key_value_puts, make_log

IN_MEMORY, SORTING = 1, 2


def _write(path, data):
    with open(path, "wb") as f:
        f.write(data)


def _read(path):
    with open(path, "rb") as f:
        return f.read()


# ------------------------------------------------------------------------------------------------
# CPU: host mirror and pre-device error paths
# ------------------------------------------------------------------------------------------------
def test_log_writer_matches_oracle_log_builder(tmp_path):
    from sparkey.log_writer import LogWriter
    lw = LogWriter.createNew(str(tmp_path / "a.spl"), file_identifier=0x1234567)
    ops = [("put", b"Key%d" % i, b"Value%d" % i) for i in range(300)]
    ops += [("delete", b"Key%d" % i, None) for i in range(0, 300, 7)]
    ops += [("put", b"Key5", b"again"), ("delete", b"x" * 100, None)]  # too long a DELETE is dropped
    for op, k, v in ops:
        lw.put(k, v) if op == "put" else lw.delete(k)
    lw.close()
    want = make_log(ops=[(op, k, v) for op, k, v in ops], file_id=0x1234567)
    assert _read(str(tmp_path / "a.spl")) == want


def test_rename_file_replaces_target_and_removes_backup(tmp_path):
    from sparkey.writer import renameFile
    src, dest = tmp_path / "new", tmp_path / "old"
    _write(str(src), b"new")
    _write(str(dest), b"old")
    renameFile(str(src), str(dest))
    assert _read(str(dest)) == b"new" and not src.exists()
    assert [p.name for p in tmp_path.iterdir()] == ["old"]  # the backup is gone
    _write(str(src), b"first")
    renameFile(str(src), str(tmp_path / "fresh"))
    assert _read(str(tmp_path / "fresh")) == b"first"
    with pytest.raises(FileNotFoundError):
        renameFile(str(tmp_path / "missing"), str(dest))


def test_rename_file_rolls_back_on_failure(tmp_path, monkeypatch):
    from sparkey import writer
    src, dest = tmp_path / "new", tmp_path / "old"
    _write(str(src), b"new")
    _write(str(dest), b"old")
    real = os.rename

    def flaky(a, b):
        if a == str(src):
            raise OSError("injected")
        return real(a, b)

    monkeypatch.setattr(writer.os, "rename", flaky)
    with pytest.raises(OSError):
        writer.renameFile(str(src), str(dest))
    monkeypatch.undo()
    assert _read(str(dest)) == b"old" and _read(str(src)) == b"new"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["new", "old"]


def test_open_existing_compressed_log_is_build_only(tmp_path):
    from snappy_log import CompressedLog
    from sparkey.log_writer import LogWriter
    from sparkey.writer import Sparkey
    cl = CompressedLog(1024, file_identifier=99)
    for i in range(500):
        cl.put(b"key_%d" % i, b"value_%d" % i)
    log = cl.finish()
    path = str(tmp_path / "c.spl")
    _write(path, log + b"trailing")  # bytes past dataEnd are cut, as LogWriter.openExisting does
    w = Sparkey.append(path)
    with pytest.raises(NotImplementedError):
        w.put(b"k", b"v")
    with pytest.raises(NotImplementedError):
        w.delete(b"k")
    w.flush()
    w.close()
    assert _read(path) == log  # maxEntriesPerBlock and every other header field unchanged
    lw = LogWriter.openExisting(path)
    assert lw.header.max_entries_per_block == struct.unpack_from("<i", log, 80)[0] > 1


def test_writer_resolves_seed_and_max_memory(tmp_path, monkeypatch):
    """writeHash's seed (0 -> random non-zero) and maxMemory (< 0 -> free/2, floor 10 MiB) reach the
    C-ABI as SingleThreadedSparkeyWriter passes them (SingleThreadedSparkeyWriter.java:95-103)."""
    from sparkey import _native, writer
    seen = []

    def fake_build(log_path, index_path, opts, fsync=False):
        seen.append((opts.hash_seed, opts.max_memory, opts.method, opts.hash_size, fsync))
        _write(index_path, b"spi")
        return _native.BuildStats()

    monkeypatch.setattr(writer._native, "build_index_file", fake_build)
    base = str(tmp_path / "w")
    w = writer.Sparkey.createNew(base)
    w.put(b"a", b"b")
    w.setMaxMemory(5)
    w.writeHash()
    w.setHashSeed(77)
    w.setMaxMemory(-1)
    w.setFsync(True)
    w.setConstructionMethod(writer.ConstructionMethod.SORTING)
    w.writeHash(writer.HashType.HASH_32_BITS)
    w.close()
    (s0, m0, _, h0, f0), (s1, m1, meth1, h1, f1) = seen
    assert s0 != 0 and m0 == 10 * 1024 * 1024 and h0 == 0 and not f0
    assert s1 == 77 and m1 >= 10 * 1024 * 1024 and meth1 == SORTING and h1 == 4 and f1
    assert _read(base + ".spi") == b"spi"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["w.spi", "w.spl"]  # no tmp files left


def test_file_errors_before_device_work(native, tmp_path):
    """Decided from the log file's header and length, before any device allocation."""
    opts = native.make_opts(hash_seed=1)
    out = str(tmp_path / "x.spi")
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "missing.spl"), out, opts)
    assert e.value.code == native.E_IO
    _write(str(tmp_path / "junk.spl"), b"\0" * 200)
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "junk.spl"), out, opts)
    assert e.value.code == native.E_NOT_LOG and "not a Sparkey log" in str(e.value)
    _write(str(tmp_path / "short.spl"), b"\x95\x9c\xb3\x49")
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "short.spl"), out, opts)
    assert e.value.code == native.E_NOT_LOG
    log = make_log(key_value_puts(50))
    _write(str(tmp_path / "cut.spl"), log[:-10])  # dataEnd > file length (LogHeader.java:81-83)
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "cut.spl"), out, opts)
    assert e.value.code == native.E_CORRUPT_LOG and "expected at least" in str(e.value)
    bad = bytearray(log)
    bad[4] = 2  # major version
    _write(str(tmp_path / "ver.spl"), bytes(bad))
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "ver.spl"), out, opts)
    assert e.value.code == native.E_VERSION
    assert not os.path.exists(out)


# ------------------------------------------------------------------------------------------------
# GPU: .spi files
# ------------------------------------------------------------------------------------------------
def _churn_ops(n, pool, p_del, seed):
    rng = random.Random(seed)
    ops = []
    for _ in range(n):
        k = b"K%d" % rng.randrange(pool)
        if ops and rng.random() < p_del:
            ops.append(("delete", k, None))
        else:
            ops.append(("put", k, b"v" * rng.randrange(0, 40)))
    return ops


def _scenarios():
    return {
        "c1": [("put", b"key_%d" % i, b"value_%d" % i) for i in range(1000)],  # WriteHashBenchmark
        "correctness170k": [("put", b"Key%d" % i, b"Value%d" % i) for i in range(170000)],
        "churn": _churn_ops(40000, 15000, 0.15, 11),
    }


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "correctness170k", "churn"])
@pytest.mark.parametrize("fsync", [False, True])
def test_writer_write_hash_file_matches_oracle(native, tmp_path, name, fsync):
    from sparkey.writer import Sparkey
    ops = _scenarios()[name]
    base = str(tmp_path / name)
    w = Sparkey.createNew(base, file_identifier=0x5151)
    for op, k, v in ops:
        w.put(k, v) if op == "put" else w.delete(k)
    w.setHashSeed(1234)
    w.setFsync(fsync)
    w.writeHash()
    log = _read(base + ".spl")
    assert log == make_log(ops=ops, file_id=0x5151)
    want = oracle.build_index(log, 1234)
    got = _read(base + ".spi")
    assert got == want, diff_report(got, want)
    assert sorted(p.name for p in tmp_path.iterdir()) == [name + ".spi", name + ".spl"]
    w.setConstructionMethod(SORTING)  # SORTING over the same log: the same bytes for unique keys
    w.writeHash()
    want_s = oracle.build_index(log, 1234, method=SORTING)
    assert _read(base + ".spi") == want_s
    w.close()


@pytest.mark.gpu
@pytest.mark.parametrize("hash_size", [0, 4, 8])
@pytest.mark.parametrize("fsync", [False, True])
def test_build_index_file_direct(native, tmp_path, hash_size, fsync):
    log = make_log(key_value_puts(20000))
    _write(str(tmp_path / "a.spl"), log)
    opts = native.make_opts(hash_size=hash_size, hash_seed=-7, sparsity=1.7)
    stats = native.build_index_file(str(tmp_path / "a.spl"), str(tmp_path / "a.spi"), opts, fsync)
    want = oracle.build_index(log, -7, hash_size=hash_size, sparsity=1.7)
    assert _read(str(tmp_path / "a.spi")) == want
    assert stats.num_entries == 20000 and stats.capacity == 1 | int(20000 * 1.7)


@pytest.mark.gpu
def test_static_write_hash_and_overwrite_existing_index(native, tmp_path):
    from sparkey.writer import Sparkey
    base = str(tmp_path / "s")
    w = Sparkey.createNew(base)
    for i in range(5000):
        w.put(b"k%d" % i, b"v%d" % i)
    w.close()
    _write(base + ".spi", b"stale index")
    Sparkey.writeHash(base)  # random seed: check through the header's own seed
    spi = _read(base + ".spi")
    seed = struct.unpack_from("<i", spi, 16)[0]
    assert seed != 0
    assert spi == oracle.build_index(_read(base + ".spl"), seed)


@pytest.mark.gpu
def test_write_hash_snappy_log_keeps_header(native, tmp_path):
    from snappy_log import CompressedLog
    from sparkey.writer import Sparkey
    cl = CompressedLog(4096, file_identifier=3)
    for i in range(20000):
        cl.put(b"key_%d" % i, b"value_%d" % i)
    log = cl.finish()
    base = str(tmp_path / "z")
    _write(base + ".spl", log)
    w = Sparkey.append(base)
    w.setHashSeed(99)
    w.writeHash()
    w.close()
    assert _read(base + ".spl") == log
    assert _read(base + ".spi") == oracle.build_index(log, 99)


@pytest.mark.gpu
def test_unwritable_output(native, tmp_path):
    log = make_log(key_value_puts(100))
    _write(str(tmp_path / "a.spl"), log)
    out = str(tmp_path / "no_such_dir" / "a.spi")
    with pytest.raises(OSError) as e:
        native.build_index_file(str(tmp_path / "a.spl"), out, native.make_opts(hash_seed=1))
    assert e.value.code == native.E_IO and "cannot create index file" in str(e.value)


@pytest.mark.gpu
def test_build_failure_leaves_no_file(native, tmp_path):
    log = bytearray(make_log(key_value_puts(100)))
    log[84] = 0xFF  # a first record whose VLQ never ends inside the record bytes
    log[85] = 0xFF
    log[86] = 0xFF
    log[87] = 0xFF
    log[88] = 0xFF
    _write(str(tmp_path / "a.spl"), bytes(log))
    with pytest.raises((OSError, RuntimeError)):
        native.build_index_file(str(tmp_path / "a.spl"), str(tmp_path / "a.spi"), native.make_opts(hash_seed=1))
    assert not os.path.exists(str(tmp_path / "a.spi"))


@pytest.mark.gpu
def test_cached_context_across_sizes_and_release(native, tmp_path):
    """The per-device context grows and is reused: a large, a small and a large log again, then
    released and rebuilt; every .spi equal to the oracle's."""
    sizes = [60000, 300, 0, 90000]
    for i, n in enumerate(sizes):
        log = make_log(key_value_puts(n, kfmt=b"K%d-" + bytes([65 + i]), vfmt=b"V%d"))
        p = str(tmp_path / ("l%d.spl" % i))
        _write(p, log)
        native.build_index_file(p, p[:-1] + "i", native.make_opts(hash_seed=5 + i))
        assert _read(p[:-1] + "i") == oracle.build_index(log, 5 + i), n
        if i == 2:
            native.release_cached_resources()


@pytest.mark.gpu
def test_concurrent_writers(native, tmp_path):
    """Writers on different threads (Sparkey.java:36: one writer per thread): each call gets its own
    context while the cached one is busy."""
    logs = [make_log(key_value_puts(30000 + 1000 * t, kfmt=b"T%d-" + bytes([48 + t]))) for t in range(4)]
    errs = []

    def run(t):
        try:
            p = str(tmp_path / ("t%d.spl" % t))
            _write(p, logs[t])
            for rep in range(3):
                native.build_index_file(p, p[:-1] + "i", native.make_opts(hash_seed=100 + t))
                if _read(p[:-1] + "i") != oracle.build_index(logs[t], 100 + t):
                    errs.append((t, rep))
        except Exception as e:  # noqa: BLE001
            errs.append((t, repr(e)))

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs


@pytest.mark.gpu
def test_build_index_mem_reuses_context(native):
    for n in (100, 50000, 10):
        log = make_log(key_value_puts(n))
        got, _ = native.build_index_mem(log, native.make_opts(hash_seed=42))
        assert got == oracle.build_index(log, 42)
