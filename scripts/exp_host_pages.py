#!/usr/bin/env python3
"""Host-buffer search on c2 (IVF4096,Flat, 1M, 10k queries, nprobe 32): what
a paged, overlapped faiss_Index_search could give, composed in Python over
the device API before building it in C++.

  host       faiss_Index_search as it is
  composed   H2D + search_device + D2H on one stream, one sync (P = 1)
  paged P    P query pages: page i+1's H2D on a copy stream while page i
             searches on the compute stream, page i-1's D2H behind it
each with pageable and with registered (pinned) caller arrays; best and
median of 20 calls, wall clock."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
d, nb, nq, k = 128, 1_000_000, 10_000, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
idx = amd.index_factory(d, "IVF4096,Flat")
idx.train(xb[:200_000])
idx.add(xb)
idx.nprobe = 32
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
D = np.empty((nq, k), np.float32)
I = np.empty((nq, k), np.int64)
D0, I0 = idx.search(xq, k)


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p.value


def mkstream():
    p = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(p), 1) == 0
    return p.value


def mkevent():
    p = C.c_void_p()
    assert hip.hipEventCreateWithFlags(C.byref(p), 2) == 0  # disable timing
    return p.value


px, pd, pi = dmalloc(xq.nbytes), dmalloc(D.nbytes), dmalloc(I.nbytes)
s, cs = mkstream(), mkstream()
up = [mkevent() for _ in range(16)]
done = [mkevent() for _ in range(16)]
hx, hD, hI = xq.ctypes.data, D.ctypes.data, I.ctypes.data


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


def composed():
    hip.hipMemcpyAsync(px, hx, xq.nbytes, 1, s)
    idx.search_device(nq, px, k, pd, pi, s)
    hip.hipMemcpyAsync(hD, pd, D.nbytes, 2, s)
    hip.hipMemcpyAsync(hI, pi, I.nbytes, 2, s)
    hip.hipStreamSynchronize(s)


def paged(P):
    b = [nq * i // P for i in range(P + 1)]

    def h2d(i):
        hip.hipMemcpyAsync(px + b[i] * d * 4, hx + b[i] * d * 4, (b[i + 1] - b[i]) * d * 4, 1, cs)
        hip.hipEventRecord(up[i], cs)

    def d2h(i):
        hip.hipStreamWaitEvent(cs, done[i], 0)
        hip.hipMemcpyAsync(hD + b[i] * k * 4, pd + b[i] * k * 4, (b[i + 1] - b[i]) * k * 4, 2, cs)
        hip.hipMemcpyAsync(hI + b[i] * k * 8, pi + b[i] * k * 8, (b[i + 1] - b[i]) * k * 8, 2, cs)

    def run():
        h2d(0)
        for i in range(P):
            hip.hipStreamWaitEvent(s, up[i], 0)
            idx.search_device(b[i + 1] - b[i], px + b[i] * d * 4, k, pd + b[i] * k * 4,
                              pi + b[i] * k * 8, s)
            hip.hipEventRecord(done[i], s)
            if i + 1 < P:
                h2d(i + 1)
            if i > 0:
                d2h(i - 1)
        d2h(P - 1)
        hip.hipStreamSynchronize(cs)
    return run


def check():
    assert np.array_equal(I, I0) and np.array_equal(D, D0), "results differ"
    D.fill(0)
    I.fill(0)


def report(tag):
    print("%-28s %s" % ("host search", best(host)), flush=True)
    for name, fn in [("composed", composed)] + [("paged %d" % P, paged(P)) for P in (2, 4, 8)]:
        fn()
        hip.hipDeviceSynchronize()
        check()
        print("%-28s %s" % (name + " " + tag, best(fn)), flush=True)


def copies():
    hip.hipMemcpyAsync(px, hx, xq.nbytes, 1, s)
    hip.hipMemcpyAsync(hD, pd, D.nbytes, 2, s)
    hip.hipMemcpyAsync(hI, pi, I.nbytes, 2, s)
    hip.hipStreamSynchronize(s)


def dev():
    idx.search_device(nq, px, k, pd, pi, s)
    hip.hipStreamSynchronize(s)


print("%-28s %s" % ("search_device", best(dev)), flush=True)
print("%-28s %s" % ("copies pageable", best(copies)), flush=True)
report("pageable")
for a in (xq, D, I):
    assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 0) == 0
print("%-28s %s" % ("copies registered", best(copies)), flush=True)
report("registered")
