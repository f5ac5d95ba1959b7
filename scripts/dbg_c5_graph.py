"""c5 geometry (IVF65536,PQ48, d = 96) through search_device as bench.py
drives it: eager, capture, replays, with kernel timing on (all stages, then
only the dominant one), on a created stream; the HIP error state is checked
after each call."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
hip = C.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = C.c_char_p
d, k = 96, 10
nb = int(os.environ.get("NB", "2000000"))
nq = int(os.environ.get("NQ", "20000"))
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
idx = amd.index_factory(d, "IVF65536,PQ48")
idx.train(xb[:65536 * 16])
idx.add(xb)
del xb
idx.nprobe = 64
idx.sync_device()
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


st = C.c_void_p()
assert hip.hipStreamCreate(C.byref(st)) == 0
px, pd, pi = dmalloc(xq.nbytes), dmalloc(nq * k * 4), dmalloc(nq * k * 8)
hip.hipMemcpy(px, xq.ctypes.data_as(C.c_void_p), C.c_size_t(xq.nbytes), 1)


def call(tag):
    try:
        idx.search_device(nq, px.value, k, pd.value, pi.value, st.value)
    except Exception as e:  # noqa: BLE001
        print(tag, "raised", e, flush=True)
    e1 = hip.hipDeviceSynchronize()
    e2 = hip.hipGetLastError()
    print(tag, "sync", e1, hip.hipGetErrorString(e1).decode(), "last", e2,
          hip.hipGetErrorString(e2).decode(), flush=True)


call("plain0")
amd.set_kernel_timing(True)
idx.reset_kernel_times()
for i in range(2):
    call(f"timed{i}")
names = idx.kernel_times()
print("stages", [(n, round(t, 3)) for n, t, _ in names], flush=True)
dom = max(names, key=lambda r: r[1])[0]
amd.set_kernel_timing(True, only=dom)
idx.reset_kernel_times()
for i in range(4):
    call(f"only_{dom}{i}")
print("dom times", idx.kernel_times(), flush=True)
amd.set_kernel_timing(False)
call("after")
