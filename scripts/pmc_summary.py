#!/usr/bin/env python3
"""Per-kernel averages of the rocprofv3 --pmc passes under <dir>/pmc*/.

FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B, see
MI355X_MICROARCH.md "HBM"); sizes are in KB as rocprofv3 reports them.
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection*.csv"),
                          recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (kn, _, cn), v in per.items():
        acc[kn][cn].append(v)
for kn, cs in acc.items():
    print(kn[:110])
    vals = {cn: sum(v) / len(v) for cn, v in cs.items()}
    for cn in sorted(vals):
        v = vals[cn]
        extra = ""
        if cn == "FETCH_SIZE":
            extra = f"   -> HBM read {2 * v / 1e3:.1f} MB/launch (x2 gfx950 correction)"
        if cn == "WRITE_SIZE":
            extra = f"   -> HBM write {v / 1e3:.1f} MB/launch"
        print(f"  {cn:28s} {v:16.1f}  (n={len(cs[cn])}){extra}")
    if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"] > 0:
        wc = vals["SQ_WAVE_CYCLES"]
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if cn in vals:
                print(f"  {cn + ' / WAVE_CYCLES':40s} {vals[cn] / wc:.3f}")
