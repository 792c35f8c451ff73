"""Model of the exact path's segments (csrc/exact_kernels.hip, k_seg_dcount .. k_seg_puts), CPU only.

The claim the kernels rest on: every table state IndexHash.put / delete (IndexHash.java:454-665)
passes through holds each distinct PUT key at most once, so its occupied slots lie inside occ(K), the
slots that the canonical placement of the log's DISTINCT PUT keys occupies.  The runs of occ(K) --
segments -- then replay independently.  Checked here on a small ring with repeated keys, equal
hashes of different keys and DELETEs, in IN_MEMORY (log) and SORTING ((wantedSlot, address),
SortHelper.java:153-171) order:
  - occupancy of every intermediate state lies inside occ(K);
  - replaying each segment on its own gives the whole replay's table;
  - the kernels' arithmetic: distinct counts per wanted slot from the canonical placement of every
    PUT record, the carry scan with its wrap-around, the segment's placed records contiguous in that
    placement (first slot + count), as k_seg_first / k_seg_runs / k_seg_puts compute them.
"""
import random

import pytest


def put(T, cap, rec, keys):
    """IndexHash.put on ring T (slot -> (hash, addr, wanted, rid) or None)."""
    h, a, w, rid = rec
    slot = w; disp = 0; might = True; C = rec
    for _ in range(cap):
        o = T[slot]
        if o is None:
            T[slot] = C
            return
        if might and o[0] == C[0] and keys[o[3]] == keys[C[3]]:
            T[slot] = C
            return
        d2 = (slot - o[2]) % cap
        if disp > d2 or (disp == d2 and C[1] < o[1]):
            T[slot] = C; C = o; disp = d2; might = False
        disp += 1
        slot = (slot + 1) % cap
    raise AssertionError("full")


def delete(T, cap, rec, keys):
    h, a, w, rid = rec
    slot = w; disp = 0
    for _ in range(cap + 1):
        o = T[slot]
        if o is None:
            return
        if o[0] == h and keys[o[3]] == keys[rid]:
            while True:
                nx = (slot + 1) % cap
                o3 = T[nx]
                if o3 is None or o3[2] == nx:
                    break
                T[slot] = o3; slot = nx
            T[slot] = None
            return
        if disp > (slot - o[2]) % cap:
            return
        disp += 1
        slot = (slot + 1) % cap


def occupancy(cap, wanted):
    """occ(S) of a multiset of wanted slots on a ring of cap slots (linear probing)."""
    T = [None] * cap
    for i, w in enumerate(wanted):
        put(T, cap, (i, i, w, i), list(range(len(wanted))))
    return {s for s in range(cap) if T[s] is not None}, T


def make_log(rng, cap, n, pool, hspace, pdel):
    keys = [rng.randrange(pool) for _ in range(n)]
    khash = {}
    for k in range(pool):  # equal hashes of different keys: a small hash space
        khash[k] = rng.randrange(hspace)
    recs = []
    for i, k in enumerate(keys):
        h = khash[k]
        recs.append(dict(h=h, a=i + 1, w=h % cap, key=k, put=rng.random() >= pdel))
    return recs


def replay(cap, recs, order):
    keys = [r["key"] for r in recs]
    T = [None] * cap
    states = []
    for i in order:
        r = recs[i]
        rec = (r["h"], r["a"], r["w"], i)
        (put if r["put"] else delete)(T, cap, rec, keys)
        states.append({s for s in range(cap) if T[s] is not None})
    return T, states


def orders(recs):
    inmem = list(range(len(recs)))
    sort = sorted(inmem, key=lambda i: (recs[i]["w"], recs[i]["a"]))
    return {"in_memory": inmem, "sorting": sort}


def distinct_wanted(recs):
    seen = {}
    for r in recs:
        if r["put"] and r["key"] not in seen:
            seen[r["key"]] = r["w"]
    return list(seen.values())


def runs(cap, occ):
    """Maximal runs of occupied slots around the ring: {start: [slots]}."""
    assert len(occ) < cap
    out = {}
    for s in range(cap):
        if s in occ and (s - 1) % cap not in occ:
            run = []
            t = s
            while t in occ:
                run.append(t); t = (t + 1) % cap
            out[s] = run
    return out


CASES = [(cap, seed) for cap in (23, 64, 97) for seed in range(12)]


@pytest.mark.parametrize("cap,seed", CASES)
def test_states_inside_distinct_occupancy(cap, seed):
    rng = random.Random(cap * 1000 + seed)
    npool = max(3, cap // 3)
    recs = make_log(rng, cap, n=rng.randrange(cap // 2, 2 * cap), pool=npool, hspace=rng.choice([npool, 3 * cap]),
                    pdel=rng.choice([0.0, 0.1, 0.3]))
    if sum(r["put"] for r in recs) >= cap:  # (a full table replays on one lane, not by segments)
        recs = [r for r in recs if not r["put"]] + [r for r in recs if r["put"]][: cap - 1]
        for i, r in enumerate(recs):
            r["a"] = i + 1
    occK, _ = occupancy(cap, distinct_wanted(recs))
    for name, order in orders(recs).items():
        T, states = replay(cap, recs, order)
        for st in states:
            assert st <= occK, name
        # each segment on its own
        T2 = [None] * cap
        keys = [r["key"] for r in recs]
        segs = runs(cap, occK)
        seg_of = {s: st for st, run in segs.items() for s in run}
        for st, run in segs.items():
            L = [None] * cap
            for i in order:
                r = recs[i]
                if seg_of.get(r["w"]) != st:
                    continue
                (put if r["put"] else delete)(L, cap, (r["h"], r["a"], r["w"], i), keys)
            for s in range(cap):
                if L[s] is not None:
                    assert s in run
                    T2[s] = L[s]
        assert T2 == T, name


@pytest.mark.parametrize("cap,seed", CASES)
def test_kernel_arithmetic(cap, seed):
    rng = random.Random(7 + cap * 1000 + seed)
    npool = max(3, cap // 3)
    recs = make_log(rng, cap, n=rng.randrange(cap // 2, cap), pool=npool, hspace=rng.choice([npool, 3 * cap]),
                    pdel=0.2)
    puts = [r for r in recs if r["put"]]
    if not puts or len(puts) >= cap:
        pytest.skip("no segments")
    # the canonical placement of every PUT record (repeats as separate entries), as the fast path leaves it
    _, A = occupancy(cap, [r["w"] for r in puts])
    A = [None if o is None else puts[o[3]] for o in A]
    # k_seg_dcount: distinct keys per wanted slot, a member repeating when an earlier member of its
    # group (consecutive slots with its wanted slot) has its hash and key
    c = [0] * cap
    for t in range(cap):
        if A[t] is None:
            continue
        w = A[t]["w"]; rep = False; j = t
        for _ in range(cap - 1):
            j = (j - 1) % cap
            if A[j] is None or A[j]["w"] != w:
                break
            if A[j]["h"] == A[t]["h"] and A[j]["key"] == A[t]["key"]:
                rep = True
                break
        c[w] += 0 if rep else 1
    want = [0] * cap
    for w in distinct_wanted(recs):
        want[w] += 1
    assert c == want
    # the carry scan (OpMaxPlus, exclusive from slot 0) and k_seg_dmarks' wrap-around
    F = [(0, 0)]
    for s in range(cap):
        fc, fa = F[-1]
        gc, ga = 0, c[s] - 1
        F.append((max(gc, fc + ga), fa + ga))
    tot = F[cap]
    c0 = max(tot[0], tot[1])
    occ = {s for s in range(cap) if max(F[s][0], c0 + F[s][1]) + c[s] >= 1}
    occK, _ = occupancy(cap, distinct_wanted(recs))
    assert occ == occK
    # k_seg_first / k_seg_runs / k_seg_puts: each segment's placed records are consecutive slots
    segs = runs(cap, occK)
    seg_of = {s: st for st, run in segs.items() for s in run}
    D = [None if A[t] is None else seg_of[A[t]["w"]] for t in range(cap)]
    first = {D[t]: t for t in range(cap) if D[t] is not None and D[(t - 1) % cap] != D[t]}
    cnt = {D[t]: (t - first[D[t]]) % cap + 1 for t in range(cap) if D[t] is not None and D[(t + 1) % cap] != D[t]}
    for st in segs:
        members = [t for t in range(cap) if D[t] == st]
        assert cnt.get(st, 0) == len(members)
        if members:
            assert sorted((t - first[st]) % cap for t in members) == list(range(len(members)))


def lane_replay(cap, s0, length, lst, sorted_order):
    """k_seg_lanes on one segment: `lst` = the grouped records (placed PUT records in placement order,
    then DELETEs, each with 'cls' = list index of the first placed PUT record with its key).  Returns the
    segment's slots (local index -> list index or None)."""
    n = len(lst)
    keys = []
    for r in lst:
        l = (r["w"] - s0) % cap
        assert l < length
        k = r["a"]
        if sorted_order:
            k |= (l + (0 if r["w"] < s0 else 32)) << 58
        keys.append((k, l))
    rank = [sum(1 for j in range(n) if keys[j][0] < keys[i][0]) for i in range(n)]
    perm = [None] * n
    for i, rk in enumerate(rank):
        perm[rk] = i
    num = {i: rank[i] for i in range(n)}
    w = [keys[perm[r]][1] for r in range(n)]
    cls = [num[lst[perm[r]]["cls"]] for r in range(n)]
    dele = [not lst[perm[r]]["put"] for r in range(n)]
    slot = [None] * (length + 1)
    for r in range(n):
        s = w[r]
        if not dele[r]:
            C, cw, cc, might = r, s, cls[r], True
            while True:
                o = slot[s]
                if o is None:
                    slot[s] = C; break
                if might and cls[o] == cc:
                    slot[s] = C; break
                d, d2 = s - cw, s - w[o]
                if d > d2 or (d == d2 and C < o):
                    slot[s] = C; C, cw, cc, might = o, w[o], cls[o], False
                s += 1
        else:
            while True:
                o = slot[s]
                if o is None:
                    break
                if cls[o] == cls[r]:
                    while s < length:
                        o3 = slot[s + 1]
                        if o3 is None or w[o3] == s + 1:
                            break
                        slot[s] = o3; s += 1
                    slot[s] = None
                    break
                if s - w[r] > s - w[o]:
                    break
                s += 1
    return [None if o is None else perm[o] for o in slot[:length]]


@pytest.mark.parametrize("sorted_order", [0, 1])
@pytest.mark.parametrize("cap,seed", CASES)
def test_lane_replay_model(cap, seed, sorted_order):
    """k_seg_lanes' numbering and key classes against the sequential replay, segment by segment."""
    rng = random.Random(31 + cap * 1000 + seed)
    npool = max(3, cap // 3)
    recs = make_log(rng, cap, n=rng.randrange(cap // 2, cap), pool=npool, hspace=rng.choice([npool, 3 * cap]),
                    pdel=0.25)
    puts = [r for r in recs if r["put"]]
    if not puts or len(puts) >= cap:
        pytest.skip("no segments")
    order = orders(recs)["sorting" if sorted_order else "in_memory"]
    T, _ = replay(cap, recs, order)
    _, A = occupancy(cap, [r["w"] for r in puts])
    A = [None if o is None else puts[o[3]] for o in A]
    occK, _ = occupancy(cap, distinct_wanted(recs))
    segs = runs(cap, occK)
    seg_of = {s: st for st, run in segs.items() for s in run}
    for st, run in segs.items():
        placed = [t for t in range(cap) if A[t] is not None and seg_of[A[t]["w"]] == st]
        placed.sort(key=lambda t: (t - st) % cap if (t - st) % cap < cap // 2 else (t - st) % cap - cap)
        lst = [dict(A[t]) for t in placed]
        for i, r in enumerate(lst):  # the first placed record of each key (k_seg_dcount / k_seg_puts)
            r["cls"] = next(j for j in range(i + 1) if lst[j]["key"] == r["key"])
        for r in recs:  # DELETEs whose key some PUT record holds (k_seg_assign's delete_class)
            if not r["put"] and seg_of.get(r["w"]) == st:
                c = next((j for j, q in enumerate(lst) if q["key"] == r["key"]), None)
                if c is not None:
                    lst.append(dict(r, cls=c))
        got = lane_replay(cap, st, len(run), lst, sorted_order)
        want = [T[s] for s in run]
        assert [None if g is None else lst[g]["a"] for g in got] == [None if o is None else o[1] for o in want]
