"""The wave-parallel heap updates proposed for the exact HNSW kernel
(scripts/experiments/hnsw_wave_heap.patch against kernels_hnsw.hip,
LaneHeap::push_w / sift_place: one lane per heap slot, ballots + permutes;
built with -DHNSW_WAVE_HEAP, not yet the shipped default)
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
def p_push(H,k,e):
    beat=0; anc=[False]*64
    for L in range(64):
        s=L+1
        dk=31-clz32(k); ds=31-clz32(s)
        anc[L]= s<k and (k>>(dk-ds))==s
        if anc[L] and gt(e,H[L]): beat|=1<<L
    p=k
    while p>1 and (beat>>((p>>1)-1))&1: p>>=1
    new=list(H)
    for L in range(64):
        s=L+1; par=(s>>1)-1 if s>=2 else 0
        take=(s==k or anc[L]) and s>p
        if take: new[L]=H[par]
        elif s==p: new[L]=e
    H[:]=new
def p_sift(H,k,e):
    larger=[False]*64
    for L in range(64):
        s=L+1; sib=((s^1)-1)&63
        sv=H[sib]; v=H[L]
        lg = (not gt(sv,v)) if (s&1) else (s==k or gt(v,sv))
        larger[L]=lg and s>=2 and s<=k
    lm=sum(1<<L for L in range(64) if larger[L])|1
    path=0;stop=0
    for L in range(64):
        s=L+1; on=s<=k
        for j in range(6):
            a=s>>j
            on = on and (a<1 or (lm>>(a-1))&1)
        below=on and s>=2
        if below: path|=1<<L
        if below and gt(e,H[L]): stop|=1<<L
    moved = (path & ((stop & -stop)-1)) if stop else path
    p = moved.bit_length() if moved else 1
    new=list(H)
    for L in range(64):
        s=L+1;c0=2*s
        m0 = c0<=64 and (moved>>((c0-1)&63))&1
        m1 = c0<64 and (moved>>(c0&63))&1
        src=min(c0 if m1 else c0-1,63)
        if m0 or m1: new[L]=H[src]
        elif s==p: new[L]=e
    H[:]=new


def test_wave_heap_ops_equal_serial_loops():
    rng = random.Random(1)
    for trial in range(600):
        ef = rng.choice([1, 2, 3, 5, 7, 16, 31, 33, 63, 64])
        A = [(rng.random(), -1)] * 64
        B = list(A)
        hk = 0
        nval = 8 if trial % 2 else 1000  # few distinct values -> many ties
        for step in range(200):
            op = rng.random()
            e = (float(rng.randrange(nval)), rng.randrange(-1, 50))
            if op < 0.5 and hk < ef:
                hk += 1
                s_push(A, hk, e)
                p_push(B, hk, e)
            elif op < 0.7 and hk > 0:  # pop: the last entry sifts from the top
                s_sift(A, hk, A[hk - 1])
                p_sift(B, hk, B[hk - 1])
                hk -= 1
            elif op < 0.9 and hk > 0:  # replace_top
                s_sift(A, hk, e)
                p_sift(B, hk, e)
            elif hk > 0:  # pop_min marks a slot dead in place
                j = rng.randrange(hk)
                A[j] = (A[j][0], -1)
                B[j] = (B[j][0], -1)
            assert A[:hk] == B[:hk], (trial, step, ef, hk)
