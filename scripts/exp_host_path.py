#!/usr/bin/env python3
"""Where the host-pointer search's time goes on c2 (IVF4096,Flat, 1M, 10k
queries, nprobe 32): faiss_Index_search (host buffers) vs search_device
replayed from its graph / eager, and the bare H2D + D2H copies (best and
median of 20 calls, wall clock)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
hip = C.CDLL("libamdhip64.so")
d, nb, nq, k = 128, 1_000_000, 10_000, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
idx = amd.index_factory(d, "IVF4096,Flat")
idx.train(xb[:200_000])
idx.add(xb)
idx.nprobe = 32
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
D = np.empty((nq, k), np.float32)
I = np.empty((nq, k), np.int64)


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


px, pd, pi = dmalloc(xq.nbytes), dmalloc(D.nbytes), dmalloc(I.nbytes)
hip.hipMemcpy(px, xq.ctypes.data_as(C.c_void_p), C.c_size_t(xq.nbytes), 1)


def best(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return "best %.3f ms, median %.3f ms" % (min(ts) * 1e3, float(np.median(ts)) * 1e3)


def host():
    idx.search(xq, k)


def dev():
    idx.search_device(nq, px.value, k, pd.value, pi.value)
    hip.hipDeviceSynchronize()


def copies():
    hip.hipMemcpy(px, xq.ctypes.data_as(C.c_void_p), C.c_size_t(xq.nbytes), 1)
    hip.hipMemcpy(D.ctypes.data_as(C.c_void_p), pd, C.c_size_t(D.nbytes), 2)
    hip.hipMemcpy(I.ctypes.data_as(C.c_void_p), pi, C.c_size_t(I.nbytes), 2)


print("host search (faiss_Index_search):", best(host), flush=True)
print("search_device (graph):", best(dev), flush=True)
os.environ["FAISS_AMD_GRAPH"] = "0"
print("search_device (eager):", best(dev), flush=True)
os.environ.pop("FAISS_AMD_GRAPH")
print("H2D + D2H copies:", best(copies), flush=True)
