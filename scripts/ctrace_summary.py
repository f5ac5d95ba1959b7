"""Summarise a coarse-filter trace (FAISS_AMD_COARSE_TRACE=<file>): per work
group s_memtime stamps (shader clock): [0] start, [1] query fragments loaded,
[2 + 2j] before tile j + 1's wait, [3 + 2j] after its barrier."""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 160).astype(np.int64)
a = a[a[:, 0] != 0]
print(f"work groups {len(a)}")
pro = a[:, 1] - a[:, 0]
print(f"prologue cycles: mean {pro.mean():.0f} p50 {np.median(pro):.0f}")
nt = 0
while nt < 78 and (a[:, 3 + 2 * nt] != 0).any():
    nt += 1
if nt:
    waits = np.stack([a[:, 3 + 2 * j] - a[:, 2 + 2 * j] for j in range(nt)], 1)
    comp = [a[:, 2 + 2 * j] - (a[:, 3 + 2 * (j - 1)] if j else a[:, 1]) for j in range(nt)]
    comp = np.stack(comp, 1)
    print(f"tiles traced {nt}: compute (between barriers) mean {comp.mean():.0f} cycles, "
          f"wait+barrier mean {waits.mean():.0f} cycles")
    print("  per tile compute mean:", " ".join(f"{v:.0f}" for v in comp.mean(0)[:12]))
    print("  per tile wait mean   :", " ".join(f"{v:.0f}" for v in waits.mean(0)[:12]))
