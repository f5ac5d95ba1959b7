#!/usr/bin/env python3
"""Per-kernel averages of the rocprofv3 --pmc passes under <dir>/pmc*/.

FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B, see
MI355X_MICROARCH.md "HBM"); sizes are in KB as rocprofv3 reports them.
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
json_out = sys.argv[2] if len(sys.argv) > 2 else None  # per-kernel HBM bytes / launch
acc = collections.defaultdict(lambda: collections.defaultdict(list))
last = collections.defaultdict(int)
for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection*.csv"),
                          recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        # one entry per (kernel, grid): the launches of the build (k-means
        # assignment, adds through an HNSW quantizer) stay apart from the
        # search's; "last_dispatch" tells which ran last (the timed steps)
        kn = f'{r["Kernel_Name"]} [grid {r.get("Grid_Size", "?")}]'
        per[(kn, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        last[kn] = max(last[kn], int(r["Dispatch_Id"]))
    for (kn, _, cn), v in per.items():
        acc[kn][cn].append(v)
summary = {}
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
    ent = {"launches": max(len(v) for v in cs.values()), "last_dispatch": last[kn]}
    if "FETCH_SIZE" in vals:
        ent["hbm_read_bytes"] = 2 * vals["FETCH_SIZE"] * 1e3   # KB, x2 (gfx950)
    if "WRITE_SIZE" in vals:
        ent["hbm_write_bytes"] = vals["WRITE_SIZE"] * 1e3
    if "hbm_read_bytes" in ent and "hbm_write_bytes" in ent:
        ent["hbm_bytes"] = ent["hbm_read_bytes"] + ent["hbm_write_bytes"]
    ent["counters"] = vals
    summary[kn] = ent
    if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"] > 0:
        wc = vals["SQ_WAVE_CYCLES"]
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if cn in vals:
                print(f"  {cn + ' / WAVE_CYCLES':40s} {vals[cn] / wc:.3f}")

if json_out:
    with open(json_out, "w") as f:
        json.dump(summary, f, indent=1)
