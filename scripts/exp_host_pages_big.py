#!/usr/bin/env python3
"""Paged host-buffer search by batch size on c2's index (IVF4096,Flat, 1M,
nprobe 32): faiss_Index_search wall time per call for FAISS_AMD_HOST_PAGES
= 0 (eager host path) / 1 / 2 / 4 / 8 at 10k, 50k and 100k queries beside search_device on the
same batch (graph replay; inputs resident); best and median of 7 calls after
3 warm ones.  Every page count must return the single-page results."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
hip = C.CDLL("libamdhip64.so")
d, nb, k = 128, 1_000_000, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
idx = amd.index_factory(d, "IVF4096,Flat")
idx.train(xb[:200_000])
idx.add(xb)
idx.nprobe = 32
del xb


def timeit(fn, reps=7):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return min(ts) * 1e3, float(np.median(ts)) * 1e3


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


for nq in (10_000, 50_000, 100_000):
    xq = amd.float_rand(nq * d, 5678 + nq).reshape(nq, d)
    px, pd, pi = dmalloc(xq.nbytes), dmalloc(nq * k * 4), dmalloc(nq * k * 8)
    hip.hipMemcpy(px, xq.ctypes.data_as(C.c_void_p), C.c_size_t(xq.nbytes), 1)

    def dev():
        idx.search_device(nq, px.value, k, pd.value, pi.value)
        hip.hipDeviceSynchronize()
    b, m = timeit(dev)
    print("nq %6d search_device      best %.3f ms, median %.3f ms" % (nq, b, m), flush=True)
    ref = None
    for P in (0, 1, 2, 4, 8):
        os.environ["FAISS_AMD_HOST_PAGES"] = str(P)
        D, I = idx.search(xq, k)
        if ref is None:
            ref = (D, I)
        else:
            assert np.array_equal(I, ref[1]) and np.array_equal(D, ref[0]), (nq, P)
        b, m = timeit(lambda: idx.search(xq, k))
        print("nq %6d host pages %d       best %.3f ms, median %.3f ms" % (nq, P, b, m), flush=True)
    os.environ.pop("FAISS_AMD_HOST_PAGES")
    b, m = timeit(lambda: idx.search(xq, k))
    print("nq %6d host default       best %.3f ms, median %.3f ms" % (nq, b, m), flush=True)
    for p in (px, pd, pi):
        hip.hipFree(p)
