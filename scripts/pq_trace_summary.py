"""Summary of a FAISS_AMD_PQ_TRACE file (k_ivfpq_filter_w per-task stamps:
start, prologue loads landed, end, info; s_memrealtime at 100 MHz)."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
a = a[a[:, 0] != 0]
ts, tp, te, info = (a[:, i].astype(np.int64) for i in range(4))
tp = np.where(tp > 0, tp, ts)
length = info & 0xFFFF
nq = (info >> 16) & 0xFF
worker = info >> 32
t0, t1 = ts.min(), te.max()
us = 0.01  # ticks -> us
print(f"tasks {len(a)}  span {(t1 - t0) * us:.1f} us  workers {len(np.unique(worker))}")
pro = (tp - ts) * us
body = (te - tp) * us
tiles = (length + 63) // 64
print(f"per task: prologue p50 {np.median(pro):.2f} p90 {np.percentile(pro, 90):.2f} us; "
      f"body p50 {np.median(body):.2f} p90 {np.percentile(body, 90):.2f} us; "
      f"tiles p50 {np.median(tiles):.0f}  body/tile p50 {np.median(body / np.maximum(tiles, 1)):.2f} us")
print(f"sum over tasks: prologue {pro.sum():.0f} us, body {body.sum():.0f} us")
# per worker: busy time, first start, last end
order = np.argsort(worker, kind="stable")
w_sorted = worker[order]
bounds = np.flatnonzero(np.diff(w_sorted)) + 1
groups = np.split(order, bounds)
busy = np.array([((te[g] - ts[g]).sum()) * us for g in groups])
last = np.array([(te[g].max() - t0) * us for g in groups])
first = np.array([(ts[g].min() - t0) * us for g in groups])
print(f"per worker: busy p50 {np.median(busy):.1f} max {busy.max():.1f} us; "
      f"first start p50 {np.median(first):.1f} max {first.max():.1f}; "
      f"last end p10 {np.percentile(last, 10):.1f} p50 {np.median(last):.1f} max {last.max():.1f}")
# busy workers over time
edges = np.linspace(0, (t1 - t0) * us, 11)
cnt = []
for lo, hi in zip(edges[:-1], edges[1:]):
    s = (ts - t0) * us
    e = (te - t0) * us
    ov = np.clip(np.minimum(e, hi) - np.maximum(s, lo), 0, None).sum() / (hi - lo)
    cnt.append(ov)
print("busy tasks per tenth of the span:", " ".join(f"{c:.0f}" for c in cnt))
print("nQ histogram (per task):", np.bincount(np.minimum(nq, 64) // 8, minlength=9).tolist())
