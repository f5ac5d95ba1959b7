#!/usr/bin/env python3
"""Host <-> device transfer options for the host-pointer search entry points
(c2 sizes: 10k x 128 fp32 queries in, 10k x 10 x (4 + 8) B results out):
pageable hipMemcpy, hipHostRegister per call (register + copy + unregister),
and a buffer registered once."""
import ctypes as C
import time

import numpy as np

hip = C.CDLL("libamdhip64.so")
nq, d, k = 10_000, 128, 10
x = np.random.default_rng(0).random((nq, d), dtype=np.float32)
out = np.empty(nq * k * 12, np.uint8)


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


dx, dout = dmalloc(x.nbytes), dmalloc(out.nbytes)
st = C.c_void_p()
hip.hipStreamCreate(C.byref(st))
H2D, D2H = 1, 2


def best(fn, reps=20):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return min(ts) * 1e3, float(np.median(ts)) * 1e3


def pageable():
    hip.hipMemcpyAsync(dx, x.ctypes.data_as(C.c_void_p), C.c_size_t(x.nbytes), H2D, st)
    hip.hipMemcpyAsync(out.ctypes.data_as(C.c_void_p), dout, C.c_size_t(out.nbytes), D2H, st)
    hip.hipStreamSynchronize(st)


def reg_per_call():
    for a in (x, out):
        assert hip.hipHostRegister(a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 0) == 0
    pageable()
    for a in (x, out):
        hip.hipHostUnregister(a.ctypes.data_as(C.c_void_p))


print("pageable: best %.3f ms, median %.3f ms" % best(pageable), flush=True)
print("register per call: best %.3f ms, median %.3f ms" % best(reg_per_call), flush=True)
for a in (x, out):
    hip.hipHostRegister(a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 0)
print("registered once: best %.3f ms, median %.3f ms" % best(pageable), flush=True)
for a in (x, out):
    hip.hipHostUnregister(a.ctypes.data_as(C.c_void_p))
