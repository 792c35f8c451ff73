"""CPU simulation of the sparkey_shard_* device steps (test infrastructure only).

sharded.ShardedBuilder drives the same methods on GpuShardSteps (the HIP C-ABI) in production; the
gloo tests on CPU drive this simulation instead, so the host orchestration -- entry verification,
exchange, carry composition, spill routing, key-pair fetches, boundary stats -- runs over real
torch.distributed collectives without a GPU.  Each method restates what its kernel computes, for
small logs, with the oracle's MurmurHash3 (oracle/) as the hash.
"""
from __future__ import annotations

import numpy as np
import torch

import oracle
from sparkey import _native
from sparkey.sharded import INDEX_HEADER_SIZE, LOG_HEADER_SIZE, _capacity, _entry_block_bits, parse_log_header

KBUCKET = 1024
DEL = 1 << 63
M64 = (1 << 64) - 1


def _vlq(buf, p, end):
    v, sh = 0, 0
    for i in range(5):
        if p + i >= end:
            return None, p
        b = buf[p + i]
        v |= (b & 0x7F) << sh
        if b < 0x80:
            return v if v < (1 << 31) else v - (1 << 32), p + i + 1
        sh += 7
    return "vlq", p


class CpuShardSteps:
    def __init__(self):
        self.device = torch.device("cpu")

    def alloc(self, nbytes):
        return torch.zeros(max(16, (nbytes + 15) // 16 * 16), dtype=torch.uint8)

    def begin(self, header, file_len, buf, buf_lo, buf_hi, opts, rank, world):
        self.header = header
        self.h = parse_log_header(header)
        self.opts = opts
        self.buf = buf.numpy()
        self.buf_lo, self.buf_hi = buf_lo, buf_hi
        self.rank, self.world = rank, world
        self.data_end = max(self.h["data_end"], LOG_HEADER_SIZE)
        self.cap = _capacity(self.h, opts)
        self.ebb = _entry_block_bits(self.h)
        self.hs = opts.hash_size or (4 if self.h["num_puts"] < (1 << 23) else 8)
        self.asz = 4 if self.h["data_end"] <= (1 << (30 - self.ebb)) else 8
        self.S = self.hs + self.asz
        self.nb = (self.cap + KBUCKET - 1) // KBUCKET
        self.bpp = max(1, (self.nb + 255) // 256)
        self.seed = opts.hash_seed
        self.slot_lo, self.slot_hi = self.slot_range(rank)
        self.entries = []

    # log access by global position
    def byte(self, p):
        return int(self.buf[p - self.buf_lo])

    def _hdr(self, p):
        """(klen, vlen, hlen, put) of the record at p, or an error string (IndexHash iterator rules)."""
        n = min(12, self.buf_hi - p)
        if n <= 0:
            return "eof"
        raw = self._bytes(p, n)
        first, q = _vlq(raw, 0, n)
        if first is None or first == "vlq":
            return "eof" if first is None else "vlq"
        second, q2 = _vlq(raw, q, n)
        if second is None or second == "vlq":
            return "eof" if second is None else "vlq"
        if first == 0:
            return (second, 0, q2, False)
        return (first - 1, second, q2, True)

    def _bytes(self, p, n):
        lo = p - self.buf_lo
        return self.buf[lo: lo + n].tobytes()

    def slot_range(self, r):
        nd = (self.nb + self.bpp - 1) // self.bpp
        d0, d1 = nd * r // self.world, nd * (r + 1) // self.world
        b0, b1 = min(self.nb, d0 * self.bpp), min(self.nb, d1 * self.bpp)
        return min(self.cap, b0 * KBUCKET), min(self.cap, b1 * KBUCKET)

    def max_record_len(self):
        from sparkey.sharded import max_record_len
        return max_record_len(self.h["max_key_len"], self.h["max_value_len"])

    def _plausible(self, r, p, spec):
        if isinstance(r, str):
            return False
        klen, vlen, hlen, put = r
        if klen < 0 or vlen < 0 or klen > self.h["max_key_len"] or p + hlen + klen > self.buf_hi:
            return False
        if spec and (vlen > self.h["max_value_len"] or (not put and self.h["num_deletes"] == 0)):
            return False
        return True

    def find_entry(self, lo, window):
        L = self.max_record_len()
        cand_end = min(lo + L, self.data_end)
        target = min(lo + L + window, self.data_end)
        exits = set()
        for c in range(lo, cand_end):
            p, alive = c, True
            while p < target:
                r = self._hdr(p)
                if not self._plausible(r, p, True):
                    alive = False
                    break
                p = p + r[2] + r[0] + (r[1] if r[3] else 0)
            if alive:
                exits.add(min(p, self.data_end))
        return exits.pop() if len(exits) == 1 else -1

    def frame(self, entry, frame_end):
        self.entries = []
        p, ndel = entry, 0
        while p < frame_end:
            r = self._hdr(p)
            if not self._plausible(r, p, False):
                code = -6 if r == "vlq" else -3
                self.entries = []
                return {"exit": p, "n": 0, "ndel": 0, "rc": code, "err_pos": p, "framing_path": 1}
            klen, vlen, hlen, put = r
            key = self._bytes(p + hlen, klen)
            hsh = oracle.key_hash(self.hs, key, self.seed) & M64
            addr = p << self.ebb
            if not put:
                addr |= DEL
                ndel += 1
            self.entries.append((hsh, addr))
            p = p + hlen + klen + (vlen if put else 0)
        return {"exit": min(max(p, entry), self.data_end), "n": len(self.entries), "ndel": ndel, "rc": 0,
                "err_pos": 0, "framing_path": 1}

    def _bucket(self, h):
        return (h % self.cap) // KBUCKET

    def bin(self, send, n, world):
        dest = []
        nd = (self.nb + self.bpp - 1) // self.bpp
        for h, a in self.entries:
            d = self._bucket(h) // self.bpp
            dest.append(next(r for r in range(world) if nd * r // world <= d < nd * (r + 1) // world))
        order = sorted(range(len(self.entries)), key=lambda i: dest[i])
        arr = np.array([self.entries[i] for i in order], dtype=np.uint64).reshape(-1, 2)
        send.view(torch.int64)[: 2 * len(order)] = torch.from_numpy(arr.view(np.int64).reshape(-1).copy())
        return [dest.count(r) for r in range(world)]

    def digit_counts(self):
        return [0] * 256  # the simulation's summarize re-sorts what it receives

    def summarize(self, recv, n, digit_counts=None):
        a = recv[: 2 * n].numpy().view(np.uint64).reshape(-1, 2)
        self.mine = sorted(((int(h) % self.cap, int(ad), int(h)) for h, ad in a), key=lambda t: (t[0], t[1] & ~DEL))
        size = self.slot_hi - self.slot_lo
        if size == 0:
            return 0, 0
        n = len(self.mine)
        c = 0
        for j, (w, _, _) in enumerate(self.mine):
            c = max(c, w + n - j - self.slot_hi)
        return c, n - size

    def place(self, carry_in, out, out_off, spill, spill_cap):
        self.out, self.out_off = out, out_off
        nxt = self.slot_lo + carry_in
        sp = []
        for w, addr, h in self.mine:
            pos = max(nxt, w)
            nxt = pos + 1
            if pos < self.slot_hi:
                self._write(pos, h, addr & ~DEL)
            else:
                sp.append((pos % self.cap, h, addr & ~DEL, 0))
        if sp and len(sp) <= spill_cap:
            arr = np.array(sp, dtype=np.uint64)
            spill.view(torch.int64)[: 4 * len(sp)] = torch.from_numpy(arr.view(np.int64).reshape(-1).copy())
        groups = {}
        for w, addr, h in self.mine:
            if not addr & DEL:
                groups.setdefault(h, []).append(addr)
        self._pairs = [(x, y) for g in groups.values() for i, x in enumerate(g) for y in g[i + 1:]]
        return len(sp), len(self._pairs), False

    def _write(self, slot, h, a):
        off = self.out_off + (slot - self.slot_lo) * self.S
        b = (h & ((1 << (8 * self.hs)) - 1)).to_bytes(self.hs, "little") + a.to_bytes(self.asz, "little")
        self.out[off: off + self.S] = torch.frombuffer(bytearray(b), dtype=torch.uint8)

    def _read(self, slot):
        off = self.out_off + (slot - self.slot_lo) * self.S
        b = self.out[off: off + self.S].numpy().tobytes()
        return int.from_bytes(b[: self.hs], "little"), int.from_bytes(b[self.hs:], "little")

    def pairs(self, n):
        return np.array([v for p in self._pairs[:n] for v in p], dtype=np.uint64)

    def key_record_size(self):
        return 8 + ((self.h["max_key_len"] + 7) & ~7)

    def fetch_keys(self, addrs, n, rec, rs):
        for i, a in enumerate(addrs[:n].numpy().view(np.uint64)):
            p = int(a & np.uint64(~DEL & M64)) >> self.ebb
            r = self._hdr(p)
            klen, key = 0xFFFFFFFF, b""
            if self._plausible(r, p, False):
                klen, key = r[0], self._bytes(p + r[2], r[0])
            b = klen.to_bytes(4, "little") + bytes(4) + key
            b = b + bytes(rs - len(b))
            rec[i * rs: (i + 1) * rs] = torch.frombuffer(bytearray(b), dtype=torch.uint8)

    def compare_keys(self, rec, npairs, rs):
        r = rec.numpy()
        for i in range(npairs):
            a, b = r[2 * i * rs: (2 * i + 1) * rs], r[(2 * i + 1) * rs: (2 * i + 2) * rs]
            ka, kb = int.from_bytes(a[:4].tobytes(), "little"), int.from_bytes(b[:4].tobytes(), "little")
            if ka == 0xFFFFFFFF or kb == 0xFFFFFFFF:
                return 2
            if ka == kb and a[8: 8 + ka].tobytes() == b[8: 8 + kb].tobytes():
                return 1
        return 0

    def apply_spill(self, spill, n):
        arr = spill[: 4 * n].numpy().view(np.uint64).reshape(-1, 4)
        for slot, h, a, _ in arr:
            if self.slot_lo <= int(slot) < self.slot_hi:
                self._write(int(slot), int(h), int(a))

    def boundary(self):
        if self.slot_hi <= self.slot_lo:
            return [0, 0, 0, 0]
        h0, a0 = self._read(self.slot_lo)
        h1, a1 = self._read(self.slot_hi - 1)
        return [h0, a0, h1, a1]

    def stats(self, prev_hash, prev_occ):
        mx = col = tot = 0
        ph, po = prev_hash, prev_occ
        for s in range(self.slot_lo, self.slot_hi):
            h, a = self._read(s)
            if po and ph == h:
                col += 1
            if a:
                d = (s - h % self.cap) % self.cap
                tot += d
                mx = max(mx, d)
            ph, po = h, a != 0
        return mx, col, tot

    def index_header(self, opts, num_entries, garbage, max_disp, collisions, total_disp):
        return _native.index_header(self.header, opts, num_entries, garbage, max_disp, collisions, total_disp)

    def full_build(self, log, file_len, out, opts):
        b = log[:file_len].numpy().tobytes()
        method = opts.method if opts.method else 1
        spi = oracle.build_index(b, opts.hash_seed, hash_size=opts.hash_size, sparsity=opts.sparsity, method=method)
        out[: len(spi)] = torch.frombuffer(bytearray(spi), dtype=torch.uint8)
        return {"num_entries": int.from_bytes(spi[60:68], "little"), "placement_path": 1}

    def from_host(self, b, dtype=torch.uint8):
        return torch.frombuffer(bytearray(b), dtype=dtype)
