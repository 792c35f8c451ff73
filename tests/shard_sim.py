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
        self._tab = None

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

    def frame_capacity(self, entry, frame_end):
        return max(0, frame_end - entry) // 2 + 1  # (a record is at least 2 bytes)

    def frame_bin_async(self, entry, frame_end, send, cap, row):
        if entry >= frame_end:
            self.entries = []
            self.bin_row(send, 0, [entry, frame_end, entry, 0, 0, 0, 0, 0], row)
            return
        m = self.frame(entry, frame_end)
        n = m["n"] if not m["rc"] else 0
        self.bin_row(send, n, [entry, frame_end, m["exit"], m["n"], m["ndel"], m["rc"], m["err_pos"], 0], row)

    def bin_row(self, send, n, scalars, row):
        """The bin carries PUT entries only (DELETEs matter to the exact path alone)."""
        world = self.world
        counts = [0] * world
        puts = [e for e in self.entries if not e[1] & DEL] if n else []
        if send is None:  # one rank: the entries stay here
            self.kept = np.array(puts, dtype=np.uint64).reshape(-1, 2)
            counts = [len(puts)]
        elif puts:
            dest = []
            nd = (self.nb + self.bpp - 1) // self.bpp
            for h, a in puts:
                d = self._bucket(h) // self.bpp
                dest.append(next(r for r in range(world) if nd * r // world <= d < nd * (r + 1) // world))
            order = sorted(range(len(puts)), key=lambda i: dest[i])
            arr = np.array([puts[i] for i in order], dtype=np.uint64).reshape(-1, 2)
            send.view(torch.int64)[: 2 * len(order)] = torch.from_numpy(arr.view(np.int64).reshape(-1).copy())
            counts = [dest.count(r) for r in range(world)]
        row.zero_()  # the per-digit counts stay 0: the simulation's summarize re-sorts what it receives
        row[:8] = torch.tensor([int(v) for v in scalars], dtype=torch.int64)
        row[8:8 + world] = torch.tensor(counts, dtype=torch.int64)

    def summarize(self, recv, n, rows, digit_col, fixed):
        a = self.kept[:n] if recv is None else recv[: 2 * n].numpy().view(np.uint64).reshape(-1, 2)
        self.mine = sorted(((int(h) % self.cap, int(ad), int(h)) for h, ad in a), key=lambda t: (t[0], t[1] & ~DEL))
        size = self.slot_hi - self.slot_lo
        if size == 0:
            return torch.zeros(2, dtype=torch.int64)
        n = len(self.mine)
        c = 0
        for j, (w, _, _) in enumerate(self.mine):
            c = max(c, w + n - j - self.slot_hi)
        return torch.tensor([c, n - size], dtype=torch.int64)

    def place(self, funs, out, out_off, spill, spill_cap, flags, inline_cap):
        F = [(int(c), int(a)) for c, a in funs.reshape(-1, 2).tolist()]
        c0, a0 = F[0]
        for fc, fa in F[1:]:
            c0, a0 = max(fc, c0 + fa), a0 + fa
        carry_in = c0
        for r in range(self.rank):
            carry_in = max(F[r][0], carry_in + F[r][1])
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
        if sp:
            arr = np.array(sp[:spill_cap], dtype=np.uint64)
            spill.view(torch.int64)[: 4 * len(arr)] = torch.from_numpy(arr.view(np.int64).reshape(-1).copy())
        groups = {}
        for w, addr, h in self.mine:
            if not addr & DEL:
                groups.setdefault(h, []).append(addr)
        self._pairs = [(x, y) for g in groups.values() for i, x in enumerate(g) for y in g[i + 1:]]
        flags.zero_()
        flags[:4] = torch.tensor([len(sp), len(self._pairs), 0, 0], dtype=torch.int64)
        k = min(len(sp), spill_cap, inline_cap)
        if k:
            arr = np.array(sp[:k], dtype=np.uint64)
            flags[4: 4 + 4 * k] = torch.from_numpy(arr.view(np.int64).reshape(-1).copy())

    def finish(self, rows, inline_cap):
        for row in rows.reshape(self.world, -1):
            n = int(row[0])
            if 0 < n <= inline_cap:
                self.apply_spill(row[4: 4 + 4 * n], n)
        nonempty = int(self.slot_hi > self.slot_lo)
        b = self.boundary()
        mx, col, tot = self.stats(0, 0) if nonempty else (0, 0, 0)
        v = [x - (1 << 64) if x >= (1 << 63) else x for x in b] + [nonempty, mx, col, tot]
        own = [int(x) for x in rows.reshape(self.world, -1)[self.rank, :4]]
        return torch.tensor(own + v, dtype=torch.int64)

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

    def write_header(self, fin, num_entries, out):
        f = fin.reshape(self.world, -1)[:, 4:].tolist()
        mx, col, tot = max(r[5] for r in f), sum(r[6] for r in f), sum(r[7] for r in f)
        prev, last = None, None
        for r, b in enumerate(f):
            if not b[4]:
                continue
            if prev is not None and prev[1] and prev[0] == b[0]:
                col += 1
            prev, last = (b[2], b[3] != 0), r
        if last is not None and f[0][1] != 0 and f[last][3] != 0 and f[0][0] == f[last][2]:
            col += 1
        hdr = self.index_header(self.opts, num_entries, 0, mx, col, tot)
        out[:INDEX_HEADER_SIZE] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8)

    def index_header(self, opts, num_entries, garbage, max_disp, collisions, total_disp):
        return _native.index_header(self.header, opts, num_entries, garbage, max_disp, collisions, total_disp)

    # ---- exact path (DELETEs, duplicate keys) ----
    def first_empty(self):
        for slot in range(self.slot_lo, self.slot_hi):
            if self._read(slot)[1] == 0:
                return slot
        return -1

    def exact_record_size(self):
        k = self.h["max_key_len"]
        return 0 if k > 4096 else 16 + ((10 + k + 7) & ~7)

    def _owner(self, w, starts):
        own, last = -1, -1
        for r, e in enumerate(starts):
            if e < 0:
                continue
            last = r
            if e <= w:
                own = r
        return own if own >= 0 else last

    def exact_frame(self, entry, frame_end, n_records, starts):
        m = self.frame(entry, frame_end)
        assert not m["rc"]
        self._ex = []  # (owner, hash, address, header + key bytes) in log order
        for h, a in self.entries:
            p = (a & ~DEL) >> self.ebb
            klen, vlen, hlen, put = self._hdr(p)
            self._ex.append((self._owner(h % self.cap, starts), h, a, self._bytes(p, hlen + klen)))
        return [sum(1 for e in self._ex if e[0] == r) for r in range(self.world)]

    def exact_pack(self, send):
        rs = self.exact_record_size()
        recs = sorted(self._ex, key=lambda e: e[0])  # stable: log order within each owner
        b = bytearray()
        for _, h, a, body in recs:
            b += int(h).to_bytes(8, "little") + int(a).to_bytes(8, "little") + body + bytes(rs - 16 - len(body))
        if b:
            send[: len(b)] = torch.frombuffer(b, dtype=torch.uint8)

    def exact_build(self, recv, n):
        """IndexHash.put / delete (IndexHash.java:454-665) over the received records, sequentially."""
        rs = self.exact_record_size()
        raw = recv[: n * rs].numpy().tobytes()
        recs = []
        for i in range(n):
            r = raw[i * rs: (i + 1) * rs]
            h, a = int.from_bytes(r[:8], "little"), int.from_bytes(r[8:16], "little")
            first, q = _vlq(r, 16, rs)
            second, q2 = _vlq(r, q, rs)
            put = first != 0
            klen, vlen = (first - 1, second) if put else (second, 0)
            recs.append((h, a & ~DEL, put, klen, vlen, r[q2: q2 + klen]))
        if self.opts.method == 2:  # SORTING: SortHelper's (wantedSlot, address) order
            recs.sort(key=lambda t: (t[0] % self.cap, t[1]))
        info = {t[1]: t for t in recs}
        cap = self.cap
        tab = [None] * cap  # (hash, address)
        st = {"n": 0, "garbage": 0}

        def vsz(v):
            return next(n for n in range(1, 5) if v < 1 << (7 * n)) if v < 1 << 28 else 5

        def gar(k, v):  # IndexHeader.java:221-228
            return k + v + vsz(k + 1) + vsz(v)

        for h, a, put, klen, vlen, key in recs:
            slot, disp = h % cap, 0
            if put:
                hh, aa, might = h, a, True
                for _ in range(cap):
                    cur = tab[slot]
                    if cur is None:
                        tab[slot] = (hh, aa)
                        st["n"] += 1
                        break
                    if might and cur[0] == hh:
                        o = info[cur[1]]
                        if not o[2]:
                            return {"rc": -5, "err_pos": a >> self.ebb, "num_entries": 0, "garbage": 0}
                        if o[3] == klen and o[5] == key:
                            tab[slot] = (hh, aa)
                            st["garbage"] += gar(o[3], o[4])
                            break
                    d2 = (slot - cur[0] % cap) % cap
                    if disp > d2 or (disp == d2 and aa < cur[1]):
                        tab[slot] = (hh, aa)
                        hh, aa = cur
                        disp = d2
                        might = False
                    disp += 1
                    slot = (slot + 1) % cap
            else:
                for _ in range(cap + 1):
                    cur = tab[slot]
                    if cur is None:
                        break
                    if cur[0] == h:
                        o = info[cur[1]]
                        if not o[2]:
                            return {"rc": -5, "err_pos": a >> self.ebb, "num_entries": 0, "garbage": 0}
                        if o[3] == klen and o[5] == key:
                            for _ in range(cap):
                                nx = (slot + 1) % cap
                                c = tab[nx]
                                if c is None or c[0] % cap == nx:
                                    break
                                tab[slot] = c
                                slot = nx
                            tab[slot] = None
                            st["garbage"] += gar(o[3], o[4])
                            st["n"] -= 1
                            break
                    if disp > (slot - cur[0] % cap) % cap:
                        break
                    disp += 1
                    slot = (slot + 1) % cap
        self._tab = tab
        return {"rc": 0, "err_pos": 0, "num_entries": st["n"], "garbage": st["garbage"]}

    def exact_extract(self, a, b, dst=None, dst_off=0):
        for slot in range(a, b):
            cur = self._tab[slot] if self._tab is not None else None
            h, ad = cur if cur is not None else (0, 0)
            bts = (h & ((1 << (8 * self.hs)) - 1)).to_bytes(self.hs, "little") + ad.to_bytes(self.asz, "little")
            o = dst_off + (slot - a) * self.S
            dst[o: o + self.S] = torch.frombuffer(bytearray(bts), dtype=torch.uint8)

    def full_build(self, log, file_len, out, opts):
        b = log[:file_len].numpy().tobytes()
        method = opts.method if opts.method else 1
        spi = oracle.build_index(b, opts.hash_seed, hash_size=opts.hash_size, sparsity=opts.sparsity, method=method)
        out[: len(spi)] = torch.frombuffer(bytearray(spi), dtype=torch.uint8)
        return {"num_entries": int.from_bytes(spi[60:68], "little"), "placement_path": 1}

    def from_host(self, b, dtype=torch.uint8):
        return torch.frombuffer(bytearray(b), dtype=dtype)
