#!/usr/bin/env python3
"""Host-buffer search (faiss_Index_search) on c2: pinned staging on / off."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
d, nb, nq, k = 128, 1_000_000, 10_000, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
index = amd.index_factory(d, "IVF4096,Flat")
index.train(xb[:200_000])
index.add(xb)
index.nprobe = 32
index.sync_device()
ref = None
for mode in ["1", "0", "1"]:
    os.environ["FAISS_AMD_STAGING"] = mode
    D, I = index.search(xq, k)
    if ref is None:
        ref = (D, I)
    assert np.array_equal(I, ref[1]) and np.array_equal(D, ref[0])
    ts = []
    for _ in range(10):
        t = time.perf_counter()
        index.search(xq, k)
        ts.append(time.perf_counter() - t)
    print(f"staging={mode}: best {min(ts) * 1e3:.3f} ms, median {np.median(ts) * 1e3:.3f} ms",
          flush=True)
t = time.perf_counter()
for _ in range(10):
    np.copyto(np.empty_like(xq), xq)
print(f"numpy copy of the queries: {(time.perf_counter() - t) / 10 * 1e3:.3f} ms", flush=True)
