#!/usr/bin/env python3
"""Kernels of the last search step in a rocprofv3 kernel trace: every
dispatch between the last two launches of the step marker kernel.

--window-stats <out.csv>: also write per-kernel statistics (calls, total,
average, min, max in ns, as rocprofv3's kernel_stats.csv) over the search
window only — every dispatch after the first step's end marker up to the last
one — so the index build's launches of the same kernels (k-means assignment,
adds through an HNSW quantizer) do not mix into the averages."""
import csv
import glob
import sys

args = [a for a in sys.argv[1:]]
wstats = None
if "--window-stats" in args:
    i = args.index("--window-stats")
    wstats = args[i + 1]
    del args[i:i + 2]
d = args[0]
marker = args[1] if len(args) > 1 else None
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
if marker is None:  # the step's last kernel: the IVF re-rank (MFMA paths) or the PQ scan
    names = [r["Kernel_Name"] for r in rows]
    marker = next(m for m in ("k_ivf_rerank", "k_ex_select", "k_ivfpq_scan")
                  if any(m in n for n in names))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
# the device-resident steps only: the bench's host-buffer calls (its
# pcie_inclusive leg, paged for large batches) follow them and start with the
# host path's visit-count kernel; cut the window there
host0 = next((i for i in range(idx[0] + 1, len(rows)) if "k_ivf_visit_stats" in rows[i]["Kernel_Name"]),
             len(rows))
idx = [i for i in idx if i < host0]
# the bench's timed steps run back to back: take the consecutive pair of
# step-end kernels with the shortest wall time between them
pairs = list(zip(idx, idx[1:]))
a, b = min(pairs, key=lambda p: int(rows[p[1]]["End_Timestamp"]) - int(rows[p[0]]["End_Timestamp"]))
tot = 0.0
for r in rows[a + 1:b + 1]:
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    print(f"{r['Kernel_Name'][:90]:90s} {us:9.1f} us")
print("step wall", (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3, "us; kernel sum", tot)

if wstats:
    agg = {}
    for r in rows[idx[0] + 1:idx[-1] + 1]:
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(r["Kernel_Name"], [0, 0, None, 0])
        a[0] += 1
        a[1] += ns
        a[2] = ns if a[2] is None else min(a[2], ns)
        a[3] = max(a[3], ns)
    tot = sum(a[1] for a in agg.values()) or 1
    with open(wstats, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                    "MaxNs", "Window"])
        for nm, (c, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([nm, c, t, t / c, 100.0 * t / tot, mn, mx,
                        "device search steps after the first (build and host-buffer calls excluded)"])
