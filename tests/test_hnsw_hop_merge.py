"""The register HNSW kernel's candidate set (kernels_hnsw.hip CandSet,
hop_merge, CandSet::results) restated lane by lane in Python and checked
against the sequential add_to_heap calls of the reference
(faiss/impl/HNSW.cpp:678-689: per fresh neighbour in arrival order, the
result heap's strict `dis < top` admission and MinimaxHeap::push,
:1096-1107), on random hops with popped (dead) candidates, results smaller
than the candidate set (k < ef) and frequent equal distances:

* the results are never kept separately: they are the set's first k entries
  below FLT_MAX, for every hop the set form accepts;
* the one-merge hop update equals the sequential pushes wherever it accepts
  the hop (it hands equal distances back to the sequential form, which stops
  where the reference's outcome depends on the heap layout or on arrival
  order).
"""
import random

FMAX = 3.4028234663852886e38


def results_of(C, hk, k):
    """CandSet::results: lanes < min(hk, k) with dis < FLT_MAX, then (FMAX, -1)."""
    R = [C[i][:2] for i in range(min(hk, k)) if C[i][0] < FMAX]
    return R + [(FMAX, -1)] * (k - len(R))


def seq_hop(C, hk, R, k, ef, arrivals, nvalid):
    """The reference's order (result heap + MinimaxHeap) and CandSet::push's
    stop rules; None where CandSet stops (the kernel continues with the heap
    layout from a replay)."""
    C = [list(e) for e in C[:hk]]
    R = list(R)
    for dis, vid in arrivals:
        # MinimaxHeap::push, as CandSet::push
        if hk == ef and dis >= C[hk - 1][0]:
            pass  # rejected by the candidates
        else:
            if k < ef and any(e[0] == dis for e in C):
                return None
            if hk == ef:
                if hk >= 2 and C[hk - 2][0] == C[hk - 1][0]:
                    return None
                if C[hk - 1][2]:
                    nvalid -= 1
                C.pop()
            else:
                hk += 1
            C.append([dis, vid, True])
            C.sort(key=lambda e: (e[0], e[1]))
            nvalid += 1
        # the result heap: strict admission, the largest leaves
        if dis < R[k - 1][0]:
            R.append((dis, vid))
            R.sort()
            R = R[:k]
    return [tuple(e) for e in C], hk, R, nvalid


def merge_hop(C, hk, ef, arrivals):
    """hop_merge: ranks by ballots over 64 lanes; None when it declines."""
    cd = [C[i][0] for i in range(hk)]
    fd = [a[0] for a in arrivals]
    m = len(arrivals)
    if hk + m > ef and any(cd[i] == cd[i - 1] for i in range(1, hk)):
        return None
    arr = [0] * 64
    da = set()
    for j, a in enumerate(fd):
        if any(x == a for x in cd) or sum(1 for x in fd if x == a) > 1:
            return None
        ra = sum(1 for x in fd if x < a)
        pc = sum(1 for x in cd if x < a) + ra
        if pc < 64:
            da.add(pc)
        arr[ra] = j
    nh = min(ef, hk + m)
    out = []
    for lane in range(nh):
        na = sum(1 for p in da if p < lane)
        if lane in da:
            dis, vid = arrivals[arr[na]]
            out.append((dis, vid, True))
        else:
            out.append(tuple(C[lane - na]))
    return out, nh, sum(1 for e in out if e[2])


def rand_case(rng, ties):
    ef = rng.choice([1, 2, 5, 16, 40, 64])
    k = rng.choice([1, 3, 10, ef, ef])
    k = min(k, ef)
    val = (lambda: float(rng.randrange(0, 30))) if ties else (lambda: rng.random() * 100)
    ids = iter(rng.sample(range(1, 100000), 400))
    hk = rng.randrange(1, ef + 1)
    C = sorted(((val(), next(ids), rng.random() < 0.7) for _ in range(hk)),
               key=lambda e: (e[0], e[1]))
    nvalid = sum(1 for e in C if e[2])
    R = results_of(C, hk, k)
    nf = rng.randrange(1, 65)
    fresh = [(val(), next(ids)) for _ in range(nf)]
    full0 = hk == ef
    ctop0 = C[hk - 1][0] if full0 else FMAX
    todo = [a for a in fresh if not full0 or a[0] < ctop0]
    return C, hk, R, k, ef, todo, nvalid


def test_results_derived_and_merge_equal_sequential():
    rng = random.Random(11)
    accepted = declined = derived = 0
    for it in range(4000):
        C, hk, R, k, ef, todo, nvalid = rand_case(rng, ties=it % 3 == 0)
        if not todo:
            continue
        s = seq_hop(C, hk, R, k, ef, todo, nvalid)
        if s is not None:
            sC, shk, sR, snv = s
            assert results_of(sC, shk, k) == sR, "results are not the set's first k"
            derived += 1
        g = merge_hop(C, hk, ef, todo)
        if g is None:
            declined += 1
            continue
        accepted += 1
        assert s is not None, "merge accepted a hop the sequential form stops on"
        assert g == (s[0], s[1], s[3])
    assert accepted > 1500 and declined > 200 and derived > 2500
