#!/usr/bin/env python3
"""Kernels of the last search step in a rocprofv3 kernel trace: every
dispatch between the last two launches of the step marker kernel."""
import csv
import glob
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_ivfpq_filter"
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
tot = 0.0
for r in rows[a + 1:b + 1]:
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    print(f"{r['Kernel_Name'][:90]:90s} {us:9.1f} us")
print("step wall", (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3, "us; kernel sum", tot)
