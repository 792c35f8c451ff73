"""Oracle pinning for SNAPPY and ZSTD logs.

The reference's compressed tests need snappy-java and a JVM, neither of which is here, and the
reference ships no compressed fixture; so the compressed oracle is pinned by two properties:
  - its Snappy decoder against libsnappy (through pyarrow) on random streams;
  - its index for a SNAPPY log against its (golden-vector pinned) index for the NONE log holding the
    same records: the tables must agree slot for slot once every NONE address (the record's offset)
    is replaced by the compressed address (blockPosition << entryBlockBits) | entryIndex that
    iterate_compressed (a pure-Python SparkeyLogIterator over CompressedReader) gives the record.
    Placement depends only on hashes and log order, which compression preserves
    (IndexHash.java:276-283 computes the address; put/delete compare keys read back through it).
"""
import random
import struct

import pytest

import oracle
from helpers import make_log
from snappy_log import CompressedLog, iterate_compressed, snappy_compress, snappy_literal_only

IN_MEMORY, SORTING = 1, 2


def test_snappy_decoder_matches_libsnappy():
    rng = random.Random(7)
    for _ in range(300):
        n = rng.randrange(0, 70000) if rng.random() < 0.1 else rng.randrange(0, 3000)
        alphabet = bytes(rng.sample(range(256), rng.randrange(1, 8)))
        d = bytes(rng.choice(alphabet) if rng.random() < 0.8 else rng.randrange(256) for _ in range(n))
        assert oracle.snappy_uncompress(snappy_compress(d), n) == d
        assert oracle.snappy_uncompress(snappy_literal_only(d), n) == d


def test_snappy_decoder_rejects_bad_streams():
    good = snappy_compress(b"abcabcabcabcabcabcabc" * 20)
    with pytest.raises(oracle.OracleError):
        oracle.snappy_uncompress(good[:-1], 420)          # truncated
    with pytest.raises(oracle.OracleError):
        oracle.snappy_uncompress(b"\x05\x01\x00", 5)       # copy before any output


def _ops(rng, n, nkeys, p_del, vmax):
    ops = []
    for i in range(n):
        k = b"key_%d" % rng.randrange(nkeys)
        if rng.random() < p_del:
            ops.append(("del", k, b""))
        else:
            ops.append(("put", k, b"v%d_" % i + bytes(rng.randrange(256) for _ in range(rng.randrange(vmax)))))
    return ops


def _compressed(ops, block_size, literal_only=False, codec="snappy"):
    cl = CompressedLog(block_size, file_identifier=0x1234567, literal_only=literal_only, codec=codec)
    for op, k, v in ops:
        if op == "put":
            cl.put(k, v)
        else:
            cl.delete(k)
    return cl.finish()


def _slots(spi):
    hs, asz, cap = struct.unpack_from("<i", spi, 72)[0], struct.unpack_from("<i", spi, 68)[0], \
        struct.unpack_from("<q", spi, 76)[0]
    out = []
    for s in range(cap):
        o = 112 + s * (hs + asz)
        out.append((int.from_bytes(spi[o:o + hs], "little"), int.from_bytes(spi[o + hs:o + hs + asz], "little")))
    return out


def _none_offsets(log):
    """Record offsets of a NONE log, in order."""
    p, end, offs = 84, struct.unpack_from("<q", log, 32)[0], []
    while p < end:
        offs.append(p)
        first, p = _vlq(log, p)
        second, p = _vlq(log, p)
        p += second if first == 0 else first - 1 + second
    return offs


def _vlq(b, p):
    v = s = 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, p


def check_equivalent(ops, block_size, method, literal_only=False, hash_size=0, codec="snappy"):
    clog = _compressed(ops, block_size, literal_only, codec)
    nlog = make_log(ops=ops)
    ci = oracle.build_index(clog, 4321, hash_size=hash_size, method=method)
    ni = oracle.build_index(nlog, 4321, hash_size=hash_size, method=method)
    ebb = struct.unpack_from("<i", ci, 92)[0]
    ents = list(iterate_compressed(clog))
    offs = _none_offsets(nlog)
    assert len(ents) == len(offs)
    amap = {0: 0}
    for e, o in zip(ents, offs):
        amap[o] = (e[2] << ebb) | e[3]
    assert [(h, amap[a]) for h, a in _slots(ni)] == _slots(ci)
    for off in (44, 52, 60, 72, 76, 84, 96, 104, 12, 16, 28, 36):   # all header fields but dataEnd/addr/ebb
        assert ci[off:off + 4] == ni[off:off + 4], off
    assert struct.unpack_from("<q", ci, 20)[0] == struct.unpack_from("<q", clog, 32)[0]
    return clog, ci


@pytest.mark.parametrize("block_size", [10, 16, 100, 1024, 4096, 65536])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_unique_puts(block_size, method):
    rng = random.Random(block_size)
    check_equivalent(_ops(rng, 1500, 10 ** 9, 0.0, 200), block_size, method)


@pytest.mark.parametrize("block_size", [10, 300, 1024])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_overwrites_and_deletes(block_size, method):
    rng = random.Random(block_size + 1)
    check_equivalent(_ops(rng, 2000, 600, 0.2, 120), block_size, method)


def test_literal_only_streams_and_spanning_records():
    rng = random.Random(3)
    ops = _ops(rng, 300, 10 ** 9, 0.0, 3000)       # values up to 3 KB over 512-byte blocks
    clog, _ = check_equivalent(ops, 512, IN_MEMORY, literal_only=True)
    assert struct.unpack_from("<i", clog, 80)[0] >= 1


def test_write_hash_benchmark_snappy():
    """WriteHashBenchmark's shape (T/system/WriteHashBenchmark.java:43-54) with SNAPPY, block 1024."""
    ops = [("put", b"key_%d" % i, b"value_%d" % i) for i in range(1000)]
    clog, ci = check_equivalent(ops, 1024, IN_MEMORY)
    mepb = struct.unpack_from("<i", clog, 80)[0]          # ~14-18 B records: 57-73 per 1 KiB block
    assert 50 < mepb < 80
    assert struct.unpack_from("<i", ci, 92)[0] == (mepb - 1).bit_length()


# ---- ZSTD (CompressorType.java:42-56): blocks decoded by libzstd, the library zstd-jni wraps ----

def test_zstd_frames_round_trip():
    """The generator's frames are what zstd-jni writes: single frames with a content size, level 3."""
    from snappy_log import zstd_compress
    rng = random.Random(9)
    for n in (1, 10, 100, 4096, 65536, 131072):
        d = bytes(rng.randrange(4) for _ in range(n // 2)) + bytes(rng.randrange(256) for _ in range(n - n // 2))
        z = zstd_compress(d)
        assert struct.unpack_from("<I", z, 0)[0] == 0xFD2FB528
        assert z[4] >> 6 or z[4] & 0x20                          # Frame_Content_Size present
        assert oracle.zstd_decompress(z) == d


@pytest.mark.parametrize("block_size", [10, 100, 1024, 65536, 131072])
@pytest.mark.parametrize("method", [IN_MEMORY, SORTING])
def test_zstd_unique_puts(block_size, method):
    rng = random.Random(block_size + 7)
    check_equivalent(_ops(rng, 1500, 10 ** 9, 0.0, 200), block_size, method, codec="zstd")


@pytest.mark.parametrize("block_size", [10, 300, 4096])
def test_zstd_overwrites_deletes_and_spanning_records(block_size):
    rng = random.Random(block_size + 8)
    check_equivalent(_ops(rng, 1500, 400, 0.2, 3000 if block_size == 300 else 120), block_size, IN_MEMORY,
                     codec="zstd")


def test_zstd_corrupt_block_is_rejected():
    clog = bytearray(_compressed([("put", b"k%d" % i, b"v" * 50) for i in range(40)], 256, codec="zstd"))
    clog[84 + 1 + 8] ^= 0xFF                                      # inside the first frame's first block
    with pytest.raises(oracle.OracleError):
        oracle.build_index(bytes(clog), 1)


@pytest.mark.parametrize("codec", ["snappy", "zstd"])
@pytest.mark.parametrize("block_size", [118, 500, 4096, 65536])
def test_synth_snappy_log_matches_writer(block_size, codec):
    """bench's SNAPPY / ZSTD generator (synth.snappy_log) writes what CompressedWriter writes."""
    from sparkey import synth
    log = synth.fixed_log(3000, 16, 100, seed=2, file_id=0x777)
    cl = CompressedLog(block_size, file_identifier=0x777, codec=codec)
    body = log[84:].tobytes()
    for i in range(3000):
        r = body[i * 118:(i + 1) * 118]
        cl.put(r[2:18], r[18:])
    assert synth.snappy_log(log, 118, block_size, codec=codec).tobytes() == cl.finish()
