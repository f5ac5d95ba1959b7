"""The wide HNSW kernel's level-0 search (kernels_hnsw.hip k_hnsw_wide)
restated step for step in Python and checked against the reference's
sequential search_from_candidates (faiss/impl/HNSW.cpp:605-741) with its own
data structures: the MinimaxHeap as faiss's 1-based binary CMax heap with
dead slots (:1096-1342, the generic pop_min that takes the highest slot
among equal minima, count_below over every slot), the result heap with
strict admission and heap_replace_top (faiss/utils/Heap.h,
faiss/impl/ResultHandler.h), results by heap_reorder.

The wide form keeps one sorted array of (dis, id, alive) of at most ef
entries, merges a hop's entering arrivals by lower_bound + a backward shift,
derives the results from the array's first k entries and flags the query
(for the sequential kernel) where an equal distance makes the reference's
outcome depend on its heap layout or arrival order.  On random graphs with
frequent equal distances: every unflagged query has the reference's results
and HNSWStats counters, and on distinct distances nothing is flagged.
"""
import random

import numpy as np

FMAX = float(np.finfo(np.float32).max)


# ------------------------------------------------ the reference, restated
def cmax_gt(a, b):
    """CMax::cmp2 on (dis, id) pairs: a above b in the max-heap."""
    return a[0] > b[0] or (a[0] == b[0] and a[1] > b[1])


def heap_push(h, n, e):
    """faiss heap_push<CMax> with the heap h[1..n] (n the new size)."""
    i = n
    while i > 1:
        f = i >> 1
        if not cmax_gt(e, h[f]):
            break
        h[i] = h[f]
        i = f
    h[i] = e


def heap_pop(h, n):
    """faiss heap_pop<CMax> of h[1..n] (the last element sifts from the root)."""
    val = h[n]
    i = 1
    while True:
        i1 = 2 * i
        i2 = i1 + 1
        if i1 > n:
            break
        if i2 == n + 1 or cmax_gt(h[i1], h[i2]):
            if cmax_gt(val, h[i1]):
                break
            h[i] = h[i1]
            i = i1
        else:
            if cmax_gt(val, h[i2]):
                break
            h[i] = h[i2]
            i = i2
    h[i] = h[n]


def heap_replace_top(h, n, e):
    i = 1
    while True:
        i1 = 2 * i
        i2 = i1 + 1
        if i1 > n:
            break
        if i2 == n + 1 or cmax_gt(h[i1], h[i2]):
            if cmax_gt(e, h[i1]):
                break
            h[i] = h[i1]
            i = i1
        else:
            if cmax_gt(e, h[i2]):
                break
            h[i] = h[i2]
            i = i2
    h[i] = e


class MinimaxHeap:
    def __init__(self, n):
        self.n, self.k, self.nvalid = n, 0, 0
        self.h = [None] * (n + 1)  # 1-based (dis, id), id -1 = popped

    def push(self, i, v):
        if self.k == self.n:
            if v >= self.h[1][0]:
                return
            if self.h[1][1] != -1:
                self.nvalid -= 1
            heap_pop(self.h, self.k)
            self.k -= 1
        self.k += 1
        heap_push(self.h, self.k, (v, i))
        self.nvalid += 1

    def pop_min(self):
        i = self.k
        while i >= 1 and self.h[i][1] == -1:
            i -= 1
        if i == 0:
            return -1, None
        imin, vmin = i, self.h[i][0]
        i -= 1
        while i >= 1:
            if self.h[i][1] != -1 and self.h[i][0] < vmin:
                vmin, imin = self.h[i][0], i
            i -= 1
        ret = self.h[imin][1]
        self.h[imin] = (vmin, -1)
        self.nvalid -= 1
        return ret, vmin

    def count_below(self, t):
        return sum(1 for i in range(1, self.k + 1) if self.h[i][0] < t)


def ref_search(nbrs, dist, entry, k, ef, efSearch):
    """search_from_candidates at level 0 seeded with the entry point."""
    res = [None] + [(FMAX, -1)] * k  # heap_heapify<CMax>
    cand = MinimaxHeap(ef)
    cand.push(entry, dist[entry])
    vis = {entry}
    if dist[entry] < res[1][0]:
        heap_replace_top(res, k, (dist[entry], entry))
    ndis = nhops = 0
    while cand.nvalid > 0:
        v0, d0 = cand.pop_min()
        if cand.count_below(d0) >= efSearch:
            break
        for v1 in nbrs[v0]:
            if v1 < 0:
                break
            if v1 in vis:
                continue
            vis.add(v1)
            dis = dist[v1]
            ndis += 1
            if dis < res[1][0]:
                heap_replace_top(res, k, (dis, v1))
            cand.push(v1, dis)
        nhops += 1
    n2 = 1 if cand.nvalid == 0 else 0
    # heap_reorder: ascending by (dis, id), placeholders (FLT_MAX, -1) last
    kept = sorted(e for e in res[1:] if e[1] != -1)
    out = kept + [(FMAX, -1)] * (k - len(kept))
    return out, ndis, nhops, n2


# ------------------------------------------------ the wide form, restated
def wide_search(nbrs, dist, entry, k, ef, efSearch):
    """k_hnsw_wide's level 0: returns (results, tie bits, ndis, nhops, n2).

    The set is a list of (dis, alive, id) sorted by (dis, alive) and, among
    alive entries of equal distance, by id: a dead entry sorts before an
    alive one of its distance, as CMax's cmp2 with the popped slot's id -1
    (HNSW.cpp:1096-1107), and dead entries of one distance in any order (the
    reference cannot tell them apart either)."""
    cs = [(dist[entry], 1, entry)]
    vis = {entry}
    nalive, fa, tie = 1, 0, 0
    ndis = nhops = 0
    n2 = 0
    win = None    # the distance of an open pop-tie window
    dvmin = float("inf")  # (k == ef) smallest distance of an eviction at a tied max
    FL = float("inf")

    def key_lt(e, dv, v):  # entry e below the arrival (dv, alive, v)
        return (e[0], e[1], e[2] if e[1] else -1) < (dv, 1, v)

    def lower_bound(dv, v):
        return sum(1 for e in cs if key_lt(e, dv, v))

    while True:
        S = len(cs)
        if nalive <= 0:
            n2 = 1
            break
        d0, _, v0 = cs[fa]
        # pop_min: the first alive entry.  Another alive one at d0 (right
        # after it: dead entries of a distance sort first): the reference
        # pops the highest heap slot among them — a pop-tie window opens
        if fa + 1 < S and cs[fa + 1][0] == d0:
            win = d0
        cs[fa] = (d0, 0, v0)
        nalive -= 1
        nfa = S
        for i in range(fa + 1, S):
            if cs[i][1]:
                nfa = i
                break
        nb = fa - sum(1 for e in cs[:fa] if e[0] == d0)
        assert nb == sum(1 for e in cs if e[0] < d0)
        if nb >= efSearch:
            n2 = 1 if nalive == 0 else 0
            break
        fa = nfa
        fresh = []
        for v1 in nbrs[v0]:
            if v1 < 0:
                break
            if v1 in vis:
                continue
            vis.add(v1)
            fresh.append(v1)
        ndis += len(fresh)
        nhops += 1
        arr = [(dist[v], v) for v in fresh]
        # inside a window the members' expansion order is the reference's
        # heap layout's: equal as long as no arrival reaches the window's
        # distance (the members are then popped back to back, whatever order)
        if win is not None and any(dv <= win for dv, _ in arr):
            tie |= 1
            break
        full = S == ef
        maxd = cs[ef - 1][0] if full else FL
        # (inside a window: an arrival at the full set's largest distance is
        # dropped here, but may enter in the reference's member order)
        if win is not None and full and any(dv == maxd for dv, _ in arr):
            tie |= 1
            break
        enter = sorted((dv, v) for dv, v in arr if dv < maxd)
        m = len(enter)
        if m:
            lbs = [lower_bound(dv, v) for dv, v in enter]
            kept = sum(1 for j in range(m) if lbs[j] + j < ef)
            if S + m > ef:
                # the kept max after a batch merge: the last kept arrival or
                # the set entry at ef - kept - 1
                cand = []
                if kept:
                    cand.append(enter[kept - 1][0])
                if ef - kept - 1 >= 0:
                    cand.append(cs[ef - kept - 1][0])
                Bd = max(cand)
                na = sum(1 for dv, _ in arr if dv == Bd)
                ns_ = sum(1 for e in cs if e[0] == Bd)
                boundary_tie = na >= 1 and na + ns_ >= 2
            else:
                boundary_tie = False
            if boundary_tie and win is not None:
                tie |= 1
                break
            if boundary_tie:
                # the hop's pushes one at a time, in arrival order
                # (MinimaxHeap::push: drop v >= max by distance, else evict
                # the max by cmp2)
                for dv, v in arr:
                    if len(cs) == ef and dv >= cs[ef - 1][0]:
                        continue
                    p = lower_bound(dv, v)
                    cs.insert(p, (dv, 1, v))
                    nalive += 1
                    if len(cs) > ef:
                        ev = cs.pop()
                        nalive -= ev[1]
                        if ev[0] == cs[ef - 1][0]:
                            dvmin = min(dvmin, ev[0])
                fa = next((i for i, e in enumerate(cs) if e[1]), len(cs))
            else:
                new = list(cs)
                for j, (dv, v) in enumerate(enter):
                    new.insert(lbs[j] + j, (dv, 1, v))
                assert len(new) == S + m and all(x is not None for x in new)
                for ev in new[ef:]:
                    nalive -= ev[1]
                    if ev[0] == new[ef - 1][0]:
                        dvmin = min(dvmin, ev[0])
                nalive += m
                cs = new[:ef]
                fa = next((i for i, e in enumerate(cs) if e[1]), len(cs))
            assert nalive == sum(e[1] for e in cs)
        if win is not None and (nalive == 0 or cs[fa][0] > win):
            win = None
    S = len(cs)
    if tie == 0:
        if k < ef and S > k and cs[k - 1][0] < FMAX and cs[k][0] == cs[k - 1][0]:
            tie |= 8
        if k == ef and S == ef and dvmin == cs[ef - 1][0]:
            tie |= 4
    out = sorted((e[0], e[2]) for e in cs[:k] if e[0] < FMAX)
    out += [(FMAX, -1)] * (k - len(out))
    return out, tie, ndis, nhops, n2


def random_case(rng, n, deg, nlev):
    nbrs = []
    for v in range(n):
        cnt = rng.randint(1, deg)
        nb = rng.sample([u for u in range(n) if u != v], cnt)
        nbrs.append(nb + [-1] * (deg - cnt))
    dist = [float(rng.randrange(nlev)) if nlev else rng.random() * 100 for _ in range(n)]
    return nbrs, dist


def test_wide_set_equals_reference_where_unflagged():
    rng = random.Random(1234)
    checked = flagged = 0
    for it in range(1500):
        n = rng.choice([40, 120, 400])
        deg = rng.choice([4, 8, 16])
        nlev = rng.choice([8, 30, 200, 5000])  # small: frequent equal distances
        nbrs, dist = random_case(rng, n, deg, nlev)
        ef = rng.randint(2, 80)
        k = rng.randint(1, ef)
        efSearch = rng.randint(1, ef)
        entry = rng.randrange(n)
        ref = ref_search(nbrs, dist, entry, k, ef, efSearch)
        out, tie, ndis, nhops, n2 = wide_search(nbrs, dist, entry, k, ef, efSearch)
        if tie:
            flagged += 1
            continue
        checked += 1
        assert out == ref[0], (it, out, ref[0])
        assert (ndis, nhops, n2) == ref[1:], (it, (ndis, nhops, n2), ref[1:])
    assert checked > 500 and flagged > 50, (checked, flagged)


def test_wide_set_distinct_distances_never_flag():
    rng = random.Random(99)
    for it in range(400):
        n = rng.choice([60, 300])
        nbrs, dist = random_case(rng, n, rng.choice([8, 16]), 0)
        ef = rng.randint(2, 100)
        k = rng.randint(1, ef)
        efSearch = rng.randint(1, ef)
        entry = rng.randrange(n)
        ref = ref_search(nbrs, dist, entry, k, ef, efSearch)
        out, tie, ndis, nhops, n2 = wide_search(nbrs, dist, entry, k, ef, efSearch)
        assert tie == 0, it
        assert out == ref[0] and (ndis, nhops, n2) == ref[1:], it
