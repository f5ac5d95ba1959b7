#!/usr/bin/env python3
"""c4's HNSW coarse quantizer at wide efSearch (profiling aid, GPU box).

Trains the c4 quantizer (IVF16384_HNSW32,Flat, 638,976 float_rand training
rows), then per (k = nprobe, efSearch) point searches the 10k bench queries:
wall time of the wide kernel + re-runs, the flag breakdown
(FAISS_AMD_HNSW_STATS), the all-sequential time, and from
FAISS_AMD_HNSW_TRACE the wide kernel's per-hop phase cycles.
POINTS="256:768,1024:1024"."""
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
cache = os.path.join(out, "c4_centroids.npy")
if os.path.exists(cache):
    q = amd.IndexHNSWFlat(d, 32)
    q.add(np.load(cache))
else:
    idx = amd.index_factory(d, "IVF16384_HNSW32,Flat")
    idx.train(amd.float_rand_rows(nb, d, 1234, 0, 1, 638_976))
    q = idx.quantizer
    np.save(cache, q.storage_vectors())
print(f"trained in {time.time() - t0:.1f}s", flush=True)
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
PH = ["pop", "nbr", "vis", "q8", "fp32", "sort+lb", "merge"]


def timed(k, reps=3):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        q.search(xq, k)
        ts.append(time.perf_counter() - t)
    return min(ts) * 1e3


for pt in os.environ.get("POINTS", "256:768,1024:1024").split(","):
    k, ef = (int(v) for v in pt.split(":"))
    q.efSearch = ef
    q.search(xq, k)
    t_wide = timed(k)
    if os.environ.get("DIAG_PMC"):  # (under rocprofv3 --pmc: the plain searches only)
        print(f"k {k} ef {ef}: wide+reruns {t_wide:.3f} ms", flush=True)
        continue
    os.environ["FAISS_AMD_HNSW_WIDE_Q8"] = "0"
    t_noq8 = timed(k)
    del os.environ["FAISS_AMD_HNSW_WIDE_Q8"]
    os.environ["FAISS_AMD_HNSW_WIDE_GVIS"] = "1"
    t_gvis = timed(k)
    del os.environ["FAISS_AMD_HNSW_WIDE_GVIS"]
    print(f"  visited bitmap in global scratch: {t_gvis:.3f} ms", flush=True)
    os.environ["FAISS_AMD_HNSW_STATS"] = "1"
    q.search(xq, k)
    del os.environ["FAISS_AMD_HNSW_STATS"]
    tf = os.path.join(out, f"wtrace_k{k}_ef{ef}.bin")
    if os.path.exists(tf):
        os.unlink(tf)
    os.environ["FAISS_AMD_HNSW_TRACE"] = tf
    q.search(xq, k)
    del os.environ["FAISS_AMD_HNSW_TRACE"]
    os.environ["FAISS_AMD_HNSW_WIDE"] = "0"
    t_seq = timed(k, 1)
    # the sequential kernel alone on 2000 queries (every one with an
    # arrival-log slot), with and without the result heap
    x2 = np.ascontiguousarray(xq[:2000])
    ts2 = {}
    for nrb in ("1", "0"):
        os.environ["FAISS_AMD_HNSW_NORB"] = nrb
        q.search(x2, k)
        t = time.perf_counter()
        q.search(x2, k)
        ts2[nrb] = (time.perf_counter() - t) * 1e3
    del os.environ["FAISS_AMD_HNSW_NORB"]
    del os.environ["FAISS_AMD_HNSW_WIDE"]
    print(f"  sequential kernel, 2000 queries: arrival log {ts2['1']:.3f} ms, result heap "
          f"{ts2['0']:.3f} ms", flush=True)
    print(f"k {k} ef {ef}: wide+reruns {t_wide:.3f} ms (no int8 bound {t_noq8:.3f} ms), "
          f"all-sequential {t_seq:.3f} ms", flush=True)
    tr = np.fromfile(tf, dtype=np.uint64).reshape(-1, 16).astype(np.float64)
    un = tr[tr[:, 8] == 0]
    hops = un[:, 9].sum()
    per = " ".join(f"{n} {un[:, i].sum() / hops:.0f}" for i, n in enumerate(PH))
    print(f"  unflagged {len(un)}: {un[:, 9].mean():.1f} hops, cycles/hop: {per}; "
          f"query {un[:, 7].mean():.0f} cycles (max {un[:, 7].max():.0f}); per hop: fresh "
          f"{un[:, 10].sum() / hops:.1f}, enter {un[:, 11].sum() / hops:.1f}, fp32 rows "
          f"{un[:, 12].sum() / hops:.1f}, merge steps {un[:, 13].sum() / hops:.2f}; one-at-a-time "
          f"hops {int(un[:, 14].sum())}, neighbour ids prefetched for {un[:, 15].sum() / hops:.2f} of "
          f"the hops", flush=True)
    fl = tr[tr[:, 8] != 0]
    if len(fl):
        print(f"  flagged {len(fl)}: at hop {fl[:, 9].mean():.1f} on average "
              f"(unflagged queries end at {un[:, 9].mean():.1f})", flush=True)
