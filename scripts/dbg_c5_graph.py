"""c5 geometry (IVF65536,PQ48, d = 96) through search_device three times
(eager, capture, replay) with the HIP error state checked after each call."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
hip = C.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = C.c_char_p
d, nb, nq, k = 96, int(os.environ.get("NB", "2000000")), 20000, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
idx = amd.index_factory(d, "IVF65536,PQ48")
idx.train(xb[:65536 * 16])
idx.add(xb)
idx.nprobe = 64
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


px, pd, pi = dmalloc(xq.nbytes), dmalloc(nq * k * 4), dmalloc(nq * k * 8)
hip.hipMemcpy(px, xq.ctypes.data_as(C.c_void_p), C.c_size_t(xq.nbytes), 1)
for it in range(4):
    try:
        idx.search_device(nq, px.value, k, pd.value, pi.value)
    except Exception as e:  # noqa: BLE001
        print("call", it, "raised", e, flush=True)
    e1 = hip.hipDeviceSynchronize()
    e2 = hip.hipGetLastError()
    print("call", it, "sync", e1, hip.hipGetErrorString(e1).decode(), "last", e2,
          hip.hipGetErrorString(e2).decode(), flush=True)
