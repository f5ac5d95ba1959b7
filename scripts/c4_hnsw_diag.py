#!/usr/bin/env python3
"""c4's HNSW coarse quantizer in isolation (profiling aid, GPU box).

Trains the c4 quantizer (IVF16384_HNSW32,Flat on the 638,976 training rows
of the 10M float_rand set), then searches the 10k bench queries at k = 64
(nprobe) for several efSearch values, printing per call the wall time, the
tie-flag breakdown of the batched kernel (FAISS_AMD_HNSW_STATS) and, from
FAISS_AMD_HNSW_TRACE, the sequential kernel's per-hop phase cycles.
Also times every query through the sequential kernel (FAISS_AMD_HNSW_EXACT=1).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)
amd = ge.load_package()
d, nb, nq = 128, 10_000_000, 10_000
t0 = time.time()
cache = os.path.join(out, "c4_centroids.npy")  # later runs of one GPU call reuse them
if os.path.exists(cache):
    q = amd.IndexHNSWFlat(d, 32)
    q.add(np.load(cache))
else:
    idx = amd.index_factory(d, "IVF16384_HNSW32,Flat")
    xt = amd.float_rand_rows(nb, d, 1234, 0, 1, 638_976)
    idx.train(xt)
    q = idx.quantizer
    np.save(cache, q.storage_vectors())
print(f"trained in {time.time() - t0:.1f}s", flush=True)
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
efs = [int(e) for e in os.environ.get("EFS", "16,64,128").split(",")]
for ef in efs:
    q.efSearch = ef
    q.search(xq, 64)  # warm-up
    tf = os.path.join(out, f"htrace_ef{ef}.bin")
    if os.path.exists(tf):
        os.unlink(tf)
    os.environ["FAISS_AMD_HNSW_STATS"] = "1"
    os.environ["FAISS_AMD_HNSW_TRACE"] = tf
    q.search(xq, 64)
    del os.environ["FAISS_AMD_HNSW_STATS"], os.environ["FAISS_AMD_HNSW_TRACE"]
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        q.search(xq, 64)
        ts.append(time.perf_counter() - t)
    os.environ["FAISS_AMD_HNSW_EXACT"] = "1"
    q.search(xq, 64)
    tx = time.perf_counter()
    q.search(xq, 64)
    tx = time.perf_counter() - tx
    os.environ["FAISS_AMD_HNSW_LAYOUT"] = "1"
    q.search(xq, 64)
    tl = time.perf_counter()
    q.search(xq, 64)
    tl = time.perf_counter() - tl
    del os.environ["FAISS_AMD_HNSW_LAYOUT"]
    ta = os.path.join(out, f"htrace_all_ef{ef}.bin")
    tl_ = os.path.join(out, f"htrace_layout_ef{ef}.bin")
    for f_ in (ta, tl_):
        if os.path.exists(f_):
            os.unlink(f_)
    os.environ["FAISS_AMD_HNSW_TRACE"] = ta
    q.search(xq, 64)
    os.environ["FAISS_AMD_HNSW_TRACE"] = tl_
    os.environ["FAISS_AMD_HNSW_LAYOUT"] = "1"
    q.search(xq, 64)
    del os.environ["FAISS_AMD_HNSW_TRACE"], os.environ["FAISS_AMD_HNSW_LAYOUT"]
    del os.environ["FAISS_AMD_HNSW_EXACT"]
    print(f"ef {ef}: batched+reruns {min(ts) * 1e3:.3f} ms, all-sequential {tx * 1e3:.3f} ms "
          f"(heap layout throughout: {tl * 1e3:.3f} ms)", flush=True)
    for tf in (tf, ta, tl_):
      if os.path.exists(tf):
        tr = np.fromfile(tf, dtype=np.uint64).reshape(-1, 16).astype(np.float64)
        tr = tr[tr[:, 7] > 0]
        if len(tr):
            hops = tr[:, 5].sum()
            ph = ["pop", "nbr ids", "visited", "distances", "heaps"]
            per = " ".join(f"{n} {tr[:, i].sum() / hops:.0f}" for i, n in enumerate(ph))
            print(f"  {os.path.basename(tf)}: traced {len(tr)} queries: {tr[:, 5].mean():.1f} "
                  f"hops, {tr[:, 6].sum() / hops:.1f} fresh/hop, cycles/hop: {per}, "
                  f"query total {tr[:, 7].mean():.0f} cycles (max {tr[:, 7].max():.0f}), "
                  f"{int(tr[:, 8].sum())} continued with the heap layout "
                  f"(replayed log entries: {int(tr[:, 9].sum())}); arrivals that can enter a "
                  f"heap {tr[:, 10].sum() / hops:.1f}/hop, hops before the candidates fill "
                  f"{tr[:, 11].mean():.1f}, fp32 rows after the int8 bound "
                  f"{tr[:, 12].sum() / hops:.1f}/hop; of the heap phase: prediction "
                  f"{tr[:, 13].sum() / hops:.0f}, log {tr[:, 14].sum() / hops:.0f} cycles/hop",
                  flush=True)
