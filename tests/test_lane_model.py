"""A record-for-record model of k_frame_lane (sparkey-java_amd/csrc/frame_lane_kernels.hip), checked
against the log's true record chain (SparkeyLogIterator.java:86-138) on the CPU: the ring entry (the
first surviving candidate of the region's first maxRecLen bytes, and the last point where the later
candidates join its chain, all inside the ring's first 512 bytes), the per-lane walks on to the next
lane's entry, and the fix passes (flags snapshot, one thread per run of disagreeing regions: the run
between the previous exit and a region's first record appended to the previous slab, or a patched
prefix where a false entry's walk meets the true one).  The GPU parity tests check the kernel itself
against the oracle; this model checks the algorithm on many more logs and region sizes than a GPU run
would, and that the kernel's four fix passes settle them."""
import struct

import numpy as np
import pytest

from helpers import make_log, random_puts

PATCH_MAX = 16   # kPatchMax
RING_WIN = 512   # kRingWin
LANE_TAIL = 768  # kLaneTail
CONV_MAX = 12    # kConvMax


def true_chain(log):
    de = struct.unpack_from("<q", log, 32)[0]
    p, out = 84, []
    while p < de:
        b0, b1 = log[p], log[p + 1]
        out.append(p)
        p += 2 + (b0 - 1 if b0 else b1) + (b1 if b0 else 0)
    return out


class LaneModel:
    def __init__(self, log, region):
        self.log = log
        self.mk = struct.unpack_from("<q", log, 40)[0]
        self.mv = struct.unpack_from("<q", log, 48)[0]
        self.nodel = struct.unpack_from("<q", log, 24)[0] == 0
        self.de = struct.unpack_from("<q", log, 32)[0]
        self.mrl = max(2 + self.mk + self.mv, 2 + self.mk)
        cs = 8
        while (1 << cs) < max(region, self.mrl):
            cs += 1
        self.R = 1 << cs
        self.k0 = 84 >> cs
        self.nreg = (self.de + self.R - 1) // self.R - self.k0

    def byte(self, i):
        return self.log[i] if i < len(self.log) else 0

    def plausible_len(self, q):  # plausible_len: one-byte VLQs, the header maxima
        b0, b1 = self.byte(q), self.byte(q + 1)
        if (b0 | b1) & 0x80:
            return 0
        if b0 == 0:
            return 0 if (self.nodel or b1 > self.mk) else 2 + b1
        return 0 if (b0 - 1 > self.mk or b1 > self.mv) else 1 + b0 + b1

    def ring_entry(self, s, e):  # ring_entry: positions relative to the 16-aligned stream base b
        b = s & ~15
        hlim = b + RING_WIN - 16
        cend = min(s + min(self.mrl, e - s), self.de)
        A, mj, ca = -1, -1, []
        for c in range(s, cend):
            if not self.plausible_len(c):
                continue
            if A < 0:
                p, chain, alive = c, [], True
                while p < self.de and p < hlim and len(chain) < CONV_MAX:
                    n = self.plausible_len(p)
                    if not n:
                        alive = False
                        break
                    chain.append(p)
                    p += n
                if alive:
                    A, ca = c, chain
            else:
                p = c
                while True:
                    if p in ca:
                        mj = max(mj, p)
                        break
                    if p >= self.de or p >= hlim or (len(ca) == CONV_MAX and p > ca[-1]):
                        break  # undecided: A, speculatively
                    n = self.plausible_len(p)
                    if not n:
                        break
                    p += n
        return -1 if A < 0 else max(A, mj)

    def walk(self, p, rend, emit):  # walk_records (one-byte VLQ logs; header_valid)
        while p < rend:
            b0, b1 = self.log[p], self.log[p + 1]
            if (b0 | b1) & 0x80:
                return -1
            put = b0 != 0
            klen, vlen = (b0 - 1, b1) if put else (b1, 0)
            if klen > self.mk or vlen > self.mv or (not put and self.nodel) or p + 2 + klen > len(self.log):
                return -1
            if not emit(p):
                return p
            p += 2 + klen + vlen
        return p

    def rend(self, r):
        return min((self.k0 + r + 1) * self.R, self.de)

    def walk_region(self, r, entry):
        recs = []
        ex = self.walk(entry, self.rend(r), lambda p: recs.append(p) or True)
        self.qpos[r], self.exitp[r], self.slab[r] = entry, ex, recs

    def fix_region(self, r, x):
        old = self.slab[r]
        if self.exitp[r] < 0 or self.qpos[r] < 0:
            return self.walk_region(r, x)
        st = {"i": 0, "nb": [], "merged": False, "full": False}

        def emit(p):
            while st["i"] < len(old) and old[st["i"]] < p:
                st["i"] += 1
            if st["i"] < len(old) and old[st["i"]] == p:
                st["merged"] = True
                return False
            if len(st["nb"]) == PATCH_MAX:
                st["full"] = True
                return False
            st["nb"].append(p)
            return True
        ex = self.walk(x, self.rend(r), emit)
        if st["full"] or ex < 0:
            return self.walk_region(r, x)
        if st["merged"] and st["i"] == 0 and r > 0:  # the run before the first record: the previous slab's end
            self.slab[r - 1] = self.slab[r - 1] + st["nb"]
            self.exitp[r - 1] = self.qpos[r]
            return
        if st["merged"]:
            self.slab[r] = st["nb"] + old[st["i"]:]
        else:
            self.slab[r], self.exitp[r] = st["nb"], ex
        self.qpos[r] = x

    def lane_walk(self, r, m, tgt):  # the ring walk: records from m below the region end, then on to tgt
        s = 84 if r == 0 else (self.k0 + r) * self.R
        e, b = self.rend(r), s & ~15
        slim = min(e + LANE_TAIL, len(self.log))
        recs, p, ex = [], m, -1
        while True:
            if p >= e and p >= tgt:
                ex = p
                break
            if (p & ~7) + 16 > slim:
                ex = p if p >= e else -1
                break
            b0, b1 = self.log[p], self.log[p + 1]
            put = b0 != 0
            klen, vlen = (b0 - 1, b1) if put else (b1, 0)
            if (b0 | b1) & 0x80 or klen > self.mk or vlen > self.mv or (not put and self.nodel) or \
                    p + 2 + klen > len(self.log):
                ex = -1
                break
            if p + 2 + klen + 16 > slim and slim < len(self.log):
                ex = p if p >= e else -1
                break
            recs.append(p)
            p += 2 + klen + vlen
        self.qpos[r], self.exitp[r], self.slab[r] = m, ex, recs

    def run(self, passes=4):
        self.qpos, self.exitp, self.slab = [0] * self.nreg, [0] * self.nreg, [[] for _ in range(self.nreg)]
        ms = []
        for r in range(self.nreg):
            s = 84 if r == 0 else (self.k0 + r) * self.R
            ms.append(s if r == 0 else self.ring_entry(s, self.rend(r)))
        for r in range(self.nreg):  # lane r % 64 of wave r // 64
            if ms[r] < 0:
                self.qpos[r], self.exitp[r], self.slab[r] = -2, -1, []
                continue
            nxt = ms[r + 1] if r % 64 != 63 and r + 1 < self.nreg else -1
            self.lane_walk(r, ms[r], nxt if nxt >= 0 else -1)
        bad0 = sum(not f for f in self.flags())
        for _ in range(passes):
            conv = self.flags()  # k_frame_lane_flags: a snapshot
            for r in range(1, self.nreg):  # k_frame_lane_act: one thread per run head
                if conv[r] or not conv[r - 1] or self.exitp[r - 1] < 0:
                    continue
                q = r
                while q < self.nreg:
                    old_exit = self.exitp[q]
                    self.fix_region(q, self.exitp[q - 1])
                    if self.exitp[q] < 0 or q + 1 >= self.nreg:
                        break
                    # on into the next region: it is part of this run, or this fix moved the exit it
                    # agreed with and the region after it is no other run's head
                    if conv[q + 1] and not (self.exitp[q] != old_exit and (q + 2 >= self.nreg or conv[q + 2])):
                        break
                    q += 1
        return bad0, all(self.flags()), [p for recs in self.slab for p in recs]

    def flags(self):
        return [self.exitp[r] >= 0 and (r == 0 or (self.exitp[r - 1] >= 0 and self.exitp[r - 1] == self.qpos[r]))
                for r in range(self.nreg)]


LOGS = [
    ("C3 shape", dict(kmin=8, kmax=64, vmin=100, vmax=100)),
    ("small mixed", dict(kmin=1, kmax=40, vmin=20, vmax=60)),
    ("wide", dict(kmin=0, kmax=126, vmin=0, vmax=127)),
    ("tiny", dict(kmin=0, kmax=3, vmin=0, vmax=2)),
]


@pytest.mark.parametrize("region", [256, 1024, 8192])
@pytest.mark.parametrize("name,kw", LOGS)
def test_lane_model_finds_the_true_chain(name, kw, region):
    log = make_log(random_puts(6000, seed=region + len(name), **kw))
    bad0, clean, recs = LaneModel(log, region).run()
    assert clean, (name, region, bad0)
    assert recs == true_chain(log)


@pytest.mark.parametrize("region", [256, 2048])
def test_lane_model_header_lookalike_values(region):
    """Values of small bytes: nearly every position passes the screen, false entries are common."""
    rng = np.random.default_rng(region)
    puts = [(b"k%d" % i, rng.integers(1, 9, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()) for i in range(8000)]
    log = make_log(puts)
    bad0, clean, recs = LaneModel(log, region).run()
    assert bad0 > 0 and clean
    assert recs == true_chain(log)


def test_lane_model_deletes():
    rng = np.random.default_rng(5)
    keys = [b"key%d" % i for i in range(3000)]
    puts = [(k, rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes()) for k in keys]
    log = make_log(puts, deletes=keys[::3])
    bad0, clean, recs = LaneModel(log, 512).run()
    assert clean and recs == true_chain(log)
