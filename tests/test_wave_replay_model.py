"""Model of the exact path's wave-parallel replay (csrc/exact_kernels.hip, wave_put / wave_delete):
the chunked probe / shift / backward-shift steps, in local slot indices, checked against the
sequential IndexHash.put / delete (IndexHash.java:454-665) on random segments with repeated keys,
equal hashes of different keys and DELETEs.  Slots hold (hash, address, wanted, record id); keys are
compared by record id.  CPU only: it pins the algorithm the kernel implements, lane for lane."""
import random

import pytest

def seq_put(T, h, a, w, rid, keys):
    slot = w; d = 0; might = True; C = (h, a, w, rid)
    while True:
        o = T[slot]
        if o is None:
            T[slot] = C; return 1, 0
        if might and o[0] == C[0] and keys[o[3]] == keys[C[3]]:
            T[slot] = C; return 0, 1
        d2 = slot - o[2]
        dc = slot - C[2]
        if dc > d2 or (dc == d2 and C[1] < o[1]):
            T[slot] = C; C = o; might = False
        slot += 1

def seq_del(T, h, w, rid, keys):
    slot = w
    while True:
        o = T[slot]
        if o is None: return 0
        if o[0] == h and keys[o[3]] == keys[rid]:
            while True:
                nx = slot + 1
                o3 = T[nx]
                if o3 is None or o3[2] == nx: break
                T[slot] = o3; slot = nx
            T[slot] = None
            return -1
        if slot - w > slot - o[2]: return 0
        slot += 1

W = 64
def wave_put(T, length, h, a, w, rid, keys, lanes=W):
    C = (h, a, w, rid); might = True; s = w
    while True:
        # probe
        found = None
        while found is None:
            evs = []
            for lane in range(lanes):
                i = s + lane; ev = 0
                if i <= length:
                    o = T[i]
                    if o is None: ev = 1
                    else:
                        if might and o[0] == C[0] and keys[o[3]] == keys[C[3]]: ev = 3
                        if not ev:
                            d, d2 = i - C[2], i - o[2]
                            if d > d2 or (d == d2 and C[1] < o[1]): ev = 4
                evs.append(ev)
            ks = [k for k, e in enumerate(evs) if e]
            if ks:
                k = ks[0]; found = (evs[k], s + k, T[s + k])
            else:
                s += lanes
                assert s <= length
        kind, at, occ = found
        if kind == 1: T[at] = C; return 1
        if kind == 3: T[at] = C; return 0
        T[at] = C; C = occ; might = False
        q0 = at + 1
        while True:
            orig = {q: T[q] for q in range(q0, q0 + lanes) if q <= length}
            evs = []; prevs = []
            for lane in range(lanes):
                q = q0 + lane
                prev = C if lane == 0 else (orig[q - 1] if q <= length else C)
                prevs.append(prev); ev = False
                if q <= length:
                    o = orig[q]
                    if o is None: ev = True
                    elif prev is None: ev = True  # garbage lane after an earlier event
                    else:
                        d, d2 = q - prev[2], q - o[2]
                        ev = not (d > d2 or (d == d2 and prev[1] < o[1]))
                evs.append(ev)
            ks = [k for k, e in enumerate(evs) if e]
            k = ks[0] if ks else lanes
            for lane in range(k):
                q = q0 + lane
                if q <= length: T[q] = prevs[lane]
            if k == lanes:
                C = orig[q0 + lanes - 1]; q0 += lanes; assert q0 <= length; continue
            if orig[q0 + k] is None:
                T[q0 + k] = prevs[k]; return 1
            C = prevs[k]; s = q0 + k + 1; break

def wave_del(T, length, h, w, rid, keys, lanes=W):
    s = w
    while True:
        evs = []
        for lane in range(lanes):
            i = s + lane; ev = 0
            if i <= length:
                o = T[i]
                if o is None: ev = 1
                else:
                    if o[0] == h and keys[o[3]] == keys[rid]: ev = 3
                    if not ev and (i - w) > (i - o[2]): ev = 1
            evs.append(ev)
        ks = [k for k, e in enumerate(evs) if e]
        if ks:
            k = ks[0]; kind = evs[k]; at = s + k; break
        s += lanes
        if s > length: return 0
    if kind == 1: return 0
    q0 = at + 1
    while True:
        orig = {q: T[q] for q in range(q0, q0 + lanes) if q <= length}
        stops = []
        for lane in range(lanes):
            q = q0 + lane; stop = True
            if q <= length:
                o = orig[q]; stop = o is None or o[2] == q
            stops.append(stop)
        k = next((j for j, x in enumerate(stops) if x), lanes)
        for lane in range(k): T[q0 + lane - 1] = orig[q0 + lane]
        if k < lanes:
            T[q0 + k - 1] = None; break
        q0 += lanes
    return -1



def _run_trial(rng, trial):
    nops = rng.randint(1, 300)
    span = rng.randint(1, max(1, nops // 2))
    lanes = rng.choice([4, 8, 64])
    nkeys = rng.randint(1, nops)
    ops = [(rng.random() < 0.25, rng.randrange(nkeys)) for _ in range(nops)]
    keys = [k for _, k in ops]
    wk = {}
    for _, key in ops:  # wanted slot and hash are functions of the key; hash 7 collides across keys
        wk.setdefault(key, (rng.randrange(span), rng.randrange(1 << 20) if rng.random() < 0.9 else 7))
    size = nops + span + 2
    t1, t2 = [None] * size, [None] * size
    for idx, (isdel, key) in enumerate(ops):
        w, hsh = wk[key]
        if isdel:
            seq_del(t1, hsh, w, idx, keys)
            wave_del(t2, size - 2, hsh, w, idx, keys, lanes)
        else:
            seq_put(t1, hsh, idx + 1, w, idx, keys)
            wave_put(t2, size - 2, hsh, idx + 1, w, idx, keys, lanes)
        assert t1 == t2, (trial, idx, lanes)


@pytest.mark.parametrize("seed", range(4))
def test_wave_replay_matches_sequential(seed):
    rng = random.Random(seed)
    for trial in range(150):
        _run_trial(rng, trial)
