#!/usr/bin/env python3
"""Kernels of the last search step in a rocprofv3 kernel trace: every
dispatch between the last two launches of the step marker kernel."""
import csv
import glob
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else None
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
if marker is None:  # the step's last kernel: the IVF re-rank (MFMA paths) or the PQ scan
    names = [r["Kernel_Name"] for r in rows]
    marker = next(m for m in ("k_ivf_rerank", "k_ex_select", "k_ivfpq_scan")
                  if any(m in n for n in names))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
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
