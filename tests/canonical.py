"""Second, independent CPU algorithm for unique-key PUT logs (test infrastructure): the bucketed
max-plus placement the GPU kernels implement (DESIGN.md "canonical placement"), written in numpy.
Used to show that sort + prefix-max + carry composition reproduces the sequential Robin-Hood table.
"""
from __future__ import annotations

import struct

import numpy as np

import oracle

BUCKET = 1024


def parse_puts(log: bytes):
    data_end, = struct.unpack_from("<q", log, 32)
    pos, out = 84, []
    while pos < data_end:
        _, first, p = oracle.vlq_read(log, pos)
        _, second, p = oracle.vlq_read(log, p)
        assert first > 0, "PUT-only logs"
        kl = first - 1
        out.append((pos, log[p:p + kl]))
        pos = p + kl + second
    return out


def canonical_table(log: bytes, seed: int, hash_size: int, sparsity: float = 1.3) -> bytes:
    num_puts, = struct.unpack_from("<q", log, 16)
    data_end, = struct.unpack_from("<q", log, 32)
    cap = 1 | int(num_puts * max(sparsity, 1.3))
    addr_size = 4 if data_end <= 1 << 30 else 8
    recs = parse_puts(log)
    n = len(recs)
    h = np.array([oracle.key_hash(hash_size, k, seed) for _, k in recs], dtype=np.uint64)
    a = np.array([p for p, _ in recs], dtype=np.int64)
    w = (h % np.uint64(cap)).astype(np.int64)
    order = np.lexsort((a, w))                       # (wantedSlot, address)
    w, h, a = w[order], h[order], a[order]
    nb = (cap + BUCKET - 1) // BUCKET
    b = w // BUCKET
    # per-bucket carry functions f(x) = max(c, x + a)
    funs = []
    starts = np.searchsorted(b, np.arange(nb + 1))
    for k in range(nb):
        lo, hi = starts[k], starts[k + 1]
        bsize = min(BUCKET, cap - k * BUCKET)
        cnt = hi - lo
        if cnt:
            j = np.arange(cnt)
            m_last = int(np.max((w[lo:hi] - k * BUCKET) - j))
            c = max(0, cnt + m_last - bsize)
        else:
            c = 0
        funs.append((c, cnt - bsize))
    # ring fixed point: x0 = composite's c (needs n < cap)
    C, A = 0, 0
    for c, aa in funs:
        C, A = max(c, C + aa), A + aa
    assert A < 0
    x = C
    slots = np.zeros((cap, 2), dtype=np.uint64)
    for k in range(nb):
        lo, hi = starts[k], starts[k + 1]
        cnt = hi - lo
        if cnt:
            loc = w[lo:hi] - k * BUCKET
            j = np.arange(cnt)
            pm = np.maximum.accumulate(loc - j)
            p = j + np.maximum(x, pm)
            s = (k * BUCKET + p) % cap
            slots[s, 0] = h[lo:hi]
            slots[s, 1] = a[lo:hi].astype(np.uint64)
        c, aa = funs[k]
        x = max(c, x + aa)
    out = bytearray()
    hs_fmt = "<I" if hash_size == 4 else "<Q"
    as_fmt = "<I" if addr_size == 4 else "<Q"
    for hh, aa in slots:
        out += struct.pack(hs_fmt, int(hh)) + struct.pack(as_fmt, int(aa))
    return bytes(out)
