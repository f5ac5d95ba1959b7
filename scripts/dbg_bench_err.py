"""Runs bench.py's main() with every library entry point bench calls wrapped:
after each, hipGetLastError is read and reported with the call's name (the
first call that leaves a HIP error behind)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402,F401
import __graft_entry__ as ge  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = C.c_char_p
amd = ge.load_package()


def wrap(owner, name):
    f = getattr(owner, name)

    def w(*a, **kw):
        r = f(*a, **kw)
        e = hip.hipGetLastError()
        if e:
            print(f"HIPERR after {name}: {e} {hip.hipGetErrorString(e).decode()}", flush=True)
        return r
    setattr(owner, name, w)


for cls in {type(c) for c in [amd.Index]} | set(amd.Index.__subclasses__()) | {amd.Index}:
    for nm in ("search_device", "kernel_times", "reset_kernel_times", "quantize_device",
               "sync_device", "add_with_ids", "train", "search_preassigned_device"):
        if nm in cls.__dict__:
            wrap(cls, nm)
wrap(amd, "set_kernel_timing")
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
