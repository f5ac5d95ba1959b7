"""The wave-parallel heap updates of the exact HNSW kernel
(kernels_hnsw.hip LaneHeap::push / sift_place: one lane per heap slot,
ballots + permutes; the GPU parity of the kernel itself is pinned by the
reference fixtures in tests/test_gpu_ref_fixtures.py and the c4 tests)
restated lane by lane in Python and checked against the serial faiss binary
heap loops they replace (faiss/utils/Heap.h:95-149 heap_pop / heap_push /
heap_replace_top with CMax cmp2), including equal distances and the dead
(id -1) slots MinimaxHeap::pop_min leaves behind (faiss/impl/HNSW.cpp:1299-1330),
which can break the heap order the parallel form must not rely on.
"""
import random

def gt(a,b): return a[0]>b[0] or (a[0]==b[0] and a[1]>b[1])
# serial (1-based over list H[0..63] slot p-1)
def s_push(H,k,e):
    p=k
    while p>1:
        f=p>>1
        if not gt(e,H[f-1]): break
        H[p-1]=H[f-1]; p=f
    H[p-1]=e
def s_sift(H,k,e):
    p=1
    while True:
        p1=2*p;p2=p1+1
        if p1>k: break
        if p2==k+1:
            if gt(e,H[p1-1]): break
            H[p-1]=H[p1-1]; p=p1; continue
        if gt(H[p1-1],H[p2-1]):
            if gt(e,H[p1-1]): break
            H[p-1]=H[p1-1]; p=p1
        else:
            if gt(e,H[p2-1]): break
            H[p-1]=H[p2-1]; p=p2
    H[p-1]=e
def clz32(x): return 32-x.bit_length()
# The kernel's form (round 4): heap position p (1-based) lives in lane p & 63
# (position 64 in lane 0), so siblings 2f, 2f + 1 are a DPP lane pair (L ^ 1);
# ballots are rotated right by one so that bit p - 1 is position p.
def pos_of(L): return L if L else 64
def rotr1(m): return ((m >> 1) | (m << 63)) & ((1 << 64) - 1)
def rotl1(m): return ((m << 1) | (m >> 63)) & ((1 << 64) - 1)
def q_push(H,k,e):
    dk=31-clz32(k); nbt=0; anc=[False]*64
    for L in range(64):
        s=pos_of(L); ds=31-clz32(s)
        anc[L]= s<k and (k>>(dk-ds))==s
        if anc[L] and not gt(e,H[L]): nbt|=1<<L
    nbt=rotr1(nbt)
    if nbt==0: p=1
    else:
        f=nbt.bit_length(); df=31-clz32(f); p=k>>(dk-df-1)
    new=list(H)
    for L in range(64):
        s=pos_of(L); par=(s>>1)&63
        if (s==k or anc[L]) and s>p: new[L]=H[par]
        elif s==p: new[L]=e
    H[:]=new
def q_sift(H,k,e):
    lm=0
    for L in range(64):
        s=pos_of(L); sv=H[L^1]; v=H[L]
        lg = (not gt(sv,v)) if (s&1) else (s==k or gt(v,sv))
        if lg and s>=2 and s<=k: lm|=1<<L
    lm=rotr1(lm)
    path=0; c=1
    while 2*c<=k:
        c = 2*c if (lm>>(2*c-1))&1 else 2*c+1
        path|=1<<(c-1)
    pl=rotl1(path); stop=0
    for L in range(64):
        if (pl>>L)&1 and gt(e,H[L]): stop|=1<<L
    stop=rotr1(stop)
    moved = (path & ((stop & -stop)-1)) if stop else path
    p = moved.bit_length() if moved else 1
    new=list(H)
    for L in range(64):
        s=pos_of(L)
        m0 = 2*s<=64 and (moved>>(2*s-1))&1
        m1 = 2*s+1<=64 and (moved>>(2*s))&1
        if m0 or m1: new[L]=H[(2*s+1 if m1 else 2*s)&63]
        elif s==p: new[L]=e
    H[:]=new


def test_lane_mapped_heap_ops_equal_serial_loops():
    """Kernel form: H_lane[p & 63] = H_serial[p - 1]."""
    rng = random.Random(2)
    for trial in range(600):
        ef = rng.choice([1, 2, 3, 5, 7, 16, 31, 32, 33, 63, 64])
        A = [(rng.random(), -1)] * 64
        B = list(A)
        hk = 0
        nval = 8 if trial % 2 else 1000
        def lane(p): return p & 63
        for step in range(200):
            op = rng.random()
            e = (float(rng.randrange(nval)), rng.randrange(-1, 50))
            if op < 0.5 and hk < ef:
                hk += 1
                s_push(A, hk, e)
                q_push(B, hk, e)
            elif op < 0.7 and hk > 0:
                s_sift(A, hk, A[hk - 1])
                q_sift(B, hk, B[lane(hk)])
                hk -= 1
            elif op < 0.9 and hk > 0:
                s_sift(A, hk, e)
                q_sift(B, hk, e)
            elif hk > 0:
                j = rng.randrange(hk)
                A[j] = (A[j][0], -1)
                B[lane(j + 1)] = (B[lane(j + 1)][0], -1)
            assert all(A[p - 1] == B[lane(p)] for p in range(1, hk + 1)), (trial, step, ef, hk)
