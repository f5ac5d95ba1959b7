"""The register HNSW kernel's one-merge hop update (kernels_hnsw.hip
hop_merge, CandSet form) restated lane by lane in Python and checked against
the sequential add_to_heap calls it replaces (faiss/impl/HNSW.cpp:678-689:
per fresh neighbour in arrival order, the result heap's `dis < top` admission
and MinimaxHeap::push, :1096-1107), on random hops with dead candidate slots,
result placeholders and frequent equal distances.  Wherever the merge accepts
a hop its outcome must be the sequential one; on equal distances it must hand
the hop back (the kernel then runs the sequential updates).
"""
import random

FMAX = 3.4028234663852886e38
DEAD = -1


def seq_hop(C, hk, R, k, ef, arrivals, nvalid):
    """CandSet::push + SortedQ::insert per arrival; None when CandSet meets a
    layout-dependent eviction (tie of the two largest)."""
    C, R = list(C[:hk]), list(R)
    rmax = R[k - 1][0]
    for dis, vid in arrivals:
        nk = (dis, vid)
        if dis < rmax:
            R.append(nk)
            R.sort()
            R = R[:k]
            rmax = R[k - 1][0]
        if hk == ef:
            top = C[hk - 1]
            if dis >= top[0]:
                continue
            if hk >= 2 and C[hk - 2][0] == top[0]:
                return None
            if top[1] != DEAD:
                nvalid -= 1
            C = C[:hk - 1]
        else:
            hk += 1
        C.append(nk)
        C.sort()
        nvalid += 1
    return C, hk, R, rmax, nvalid


def merge_hop(C, hk, R, k, ef, arrivals):
    """hop_merge: ranks by ballots over 64 lanes; None when it declines."""
    cd = [C[i][0] if i < hk else None for i in range(64)]
    rd = [R[i][0] if i < k else None for i in range(64)]
    fd = [a[0] for a in arrivals]
    m = len(arrivals)
    if hk + m > ef and any(cd[i] == cd[i - 1] for i in range(1, hk)):
        return None
    arr = [0] * 64
    da, dr = set(), set()
    for j, a in enumerate(fd):
        ra = sum(1 for x in fd if x < a)
        pc = sum(1 for i in range(hk) if cd[i] < a) + ra
        pr = sum(1 for i in range(k) if rd[i] < a) + ra
        if any(cd[i] == a for i in range(hk)) or any(rd[i] == a for i in range(k)) \
                or sum(1 for x in fd if x == a) > 1:
            return None
        if pc < 64:
            da.add(pc)
        if pr < 64:
            dr.add(pr)
        arr[ra] = j
    nh = min(ef, hk + m)

    def pull(old, dset, n):
        out = []
        for lane in range(n):
            na = sum(1 for p in dset if p < lane)
            out.append(arrivals[arr[na]] if lane in dset else old[lane - na])
        return out
    NC = pull(C, da, nh)
    NR = pull(R, dr, k)
    return NC, nh, NR, NR[k - 1][0], sum(1 for e in NC if e[1] != DEAD)


def rand_case(rng, ties):
    ef = rng.choice([1, 2, 5, 16, 40, 64])
    k = rng.choice([1, 3, 10, min(ef, 64), 64])
    val = (lambda: float(rng.randrange(0, 30))) if ties else (lambda: rng.random() * 100)
    ids = iter(rng.sample(range(1, 100000), 400))
    hk = rng.randrange(1, ef + 1)
    C = sorted((val(), next(ids) if rng.random() < 0.7 else DEAD) for _ in range(hk))
    nvalid = sum(1 for e in C if e[1] != DEAD)
    nr = rng.randrange(0, k + 1)
    R = sorted((val(), next(ids)) for _ in range(nr)) + [(FMAX, -1)] * (k - nr)
    nf = rng.randrange(1, 65)
    fresh = [(val(), next(ids)) for _ in range(nf)]
    full0 = hk == ef
    ctop0 = C[hk - 1][0] if full0 else FMAX
    rmax0 = R[k - 1][0]
    todo = [a for a in fresh if not full0 or a[0] < rmax0 or a[0] < ctop0]
    return C, hk, R, k, ef, todo, nvalid


def test_hop_merge_equals_sequential_updates():
    rng = random.Random(11)
    accepted = declined = 0
    for it in range(3000):
        C, hk, R, k, ef, todo, nvalid = rand_case(rng, ties=it % 3 == 0)
        if not todo:
            continue
        s = seq_hop(C, hk, R, k, ef, todo, nvalid)
        g = merge_hop(C, hk, R, k, ef, todo)
        if g is None:
            declined += 1
            continue
        accepted += 1
        assert s is not None, "merge accepted a hop whose eviction depends on the layout"
        assert g == s
    assert accepted > 1500 and declined > 200
