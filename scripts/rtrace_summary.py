"""Summarise a re-rank trace (FAISS_AMD_RERANK_TRACE=<file>): per query
s_memrealtime (100 MHz) stamps: start, end, ns | fails << 32, after U, after
the candidate list, after the exact evaluation."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
a = a[a[:, 0] != 0]
t0 = a[:, 0] - a[:, 0].min()
us = 0.01
ph = {"round trip 1 + U": a[:, 3] - a[:, 0], "candidates": a[:, 4] - a[:, 3],
      "exact eval (round trip 2)": a[:, 5] - a[:, 4], "select + write": a[:, 1] - a[:, 5],
      "total": a[:, 1] - a[:, 0]}
print(f"queries {len(a)} span {(a[:, 1].max() - a[:, 0].min()) * us:.1f} us; "
      f"survivors mean {(a[:, 2] & 0xffffffff).mean():.1f}")
for k, v in ph.items():
    v = v[a[:, 5] > 0] * us
    print(f"  {k:28s} mean {v.mean():6.2f} p50 {np.median(v):6.2f} p95 {np.percentile(v, 95):6.2f} us")
end = np.sort(a[:, 1] - a[:, 0].min()) * us
print("  in flight (mean over span):", f"{((a[:, 1] - a[:, 0]).sum() * us) / (end[-1]):.0f}")
st = (a[:, 0] - a[:, 0].min()) * us
en = (a[:, 1] - a[:, 0].min()) * us
bins = np.arange(0, en.max() + 5, 5)
inf = [((st <= b + 2.5) & (en > b + 2.5)).sum() for b in bins]
print("  in flight per 5 us:", " ".join(str(v) for v in inf))
print("  started per 5 us  :", " ".join(str(v) for v in np.histogram(st, bins)[0]))
tot = a[:, 1] - a[:, 0]
o = np.argsort(-tot)[:12]
print("  slowest: total_us ns fails | rt1+U cand exact select (us)")
for i in o:
    print(f"    {tot[i] * us:7.2f} {a[i, 2] & 0xffffffff:5d} {a[i, 2] >> 32:3d} | "
          f"{(a[i, 3] - a[i, 0]) * us:6.2f} {(a[i, 4] - a[i, 3]) * us:6.2f} "
          f"{(a[i, 5] - a[i, 4]) * us:6.2f} {(a[i, 1] - a[i, 5]) * us:6.2f}")
