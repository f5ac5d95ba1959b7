"""Summarise a per-work-item filter trace (FAISS_AMD_FILTER_TRACE=<file>).

Record per item (8 x u64): t_start, t_loop (query fragments loaded), t_loop_end,
t_end (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32, list, len | nQ << 32.
"""
import sys

import numpy as np

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main(fname):
    a = np.fromfile(fname, dtype=np.uint64).reshape(-1, 8)
    a = a[a[:, 0] != 0]
    t0, t1, t2, t3 = (a[:, i].astype(np.int64) for i in range(4))
    base = t0.min()
    t0, t1, t2, t3 = t0 - base, t1 - base, t2 - base, t3 - base
    hw = a[:, 4] & 0xffffffff
    xcc = (a[:, 4] >> 32) & 0xf
    cu = (hw >> 8) & 0xf
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    ln = (a[:, 6] & 0xffffffff).astype(np.int64)
    nq = (a[:, 6] >> 32).astype(np.int64)
    ntile = (ln + 63) // 64
    span = t3.max() * TICK_US
    print(f"items {len(a)}  span {span:.1f} us  rows {ln.sum()}  queries*lists {nq.sum()}")
    for name, v in [("prologue", t1 - t0), ("loop", t2 - t1), ("epilogue", t3 - t2),
                    ("total", t3 - t0)]:
        v = v * TICK_US
        print(f"  {name:9s} mean {v.mean():6.2f}  p50 {np.median(v):6.2f}  p95 "
              f"{np.percentile(v, 95):6.2f}  max {v.max():6.2f} us")
    per_tile = (t2 - t1) * TICK_US / np.maximum(ntile, 1)
    print(f"  loop per tile: mean {per_tile.mean():.3f} us  p50 {np.median(per_tile):.3f}")
    print(f"  tiles/item mean {ntile.mean():.2f} max {ntile.max()}  nQ mean {nq.mean():.1f} "
          f"max {nq.max()}  active waves mean {np.ceil(nq / 32).mean():.2f}")
    done = np.sort(t3) * TICK_US
    for f in (0.5, 0.9, 0.95, 0.99):
        print(f"  {int(f * 100)}% of items done at {done[int(f * (len(done) - 1))]:.1f} us")
    st = np.sort(t0) * TICK_US
    print(f"  last item starts at {st[-1]:.1f} us")
    # concurrency: items in flight over time
    bins = np.arange(0, t3.max() + 100, 100)  # 1 us bins
    inflight = np.zeros(len(bins))
    for s, e in zip(t0, t3):
        inflight[s // 100:e // 100 + 1] += 1
    print("  in flight per 5 us: " + " ".join(f"{int(inflight[i:i + 5].mean())}"
                                               for i in range(0, len(bins), 5)))
    cuid = ((xcc * 2 + se) * 2 + sh) * 16 + cu  # unique-ish CU key
    ucu = np.unique(cuid)
    per = np.array([(t3[cuid == c].max() - t0[cuid == c].min()) * TICK_US for c in ucu])
    cnt = np.array([(cuid == c).sum() for c in ucu])
    print(f"  CUs used {len(ucu)}  items/CU mean {cnt.mean():.1f} min {cnt.min()} max {cnt.max()}"
          f"  CU busy span mean {per.mean():.1f} max {per.max():.1f} us")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: items {m.sum()} rows {ln[m].sum()} end {t3[m].max() * TICK_US:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
