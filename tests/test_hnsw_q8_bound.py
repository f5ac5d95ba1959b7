"""The int8 lower bound of the register HNSW kernel's level-0 prefilter
(kernels_hnsw.hip q8_query_prep / q8_filter, row image from
IndexHNSW::sync_device) restated in numpy: for random and adversarial rows
and queries (wide and narrow ranges, constant rows, large magnitudes, d not a
multiple of 8) the bound never exceeds the fp32 distance as the reference
evaluates it (faiss/utils/distances_simd.cpp fvec_L2sqr order, ref_arith.h),
so a neighbour it rejects could not have entered either heap."""
import numpy as np

U = 2.0 ** -24


def row_image(y):
    mn, mx = np.float32(y.min()), np.float32(y.max())
    sc = np.float32((float(mx) - float(mn)) / 255.0)
    if not sc > 0 or not np.isfinite(sc):
        sc = np.float32(1.0)
    q = np.clip(np.rint((y.astype(np.float64) - float(mn)) / float(sc)), 0, 255)
    yq = float(sc) * q + float(mn)
    e2 = ((y.astype(np.float64) - yq) ** 2).sum()
    b2 = (yq ** 2).sum()
    ey = np.sqrt(e2) * (1 + 1e-9) + 1e-12 * np.sqrt(b2) + 1e-30
    eyf = np.float32(ey)
    if float(eyf) < ey:
        eyf = np.nextafter(eyf, np.float32(np.inf))
    return q.astype(np.int64), float(mn), float(sc), float(eyf), float(np.float32(b2)), float(q.sum())


def query_image(x):
    ox = float(np.float32(x.min()))
    sx = (float(np.float32(x.max())) - ox) / 255.0
    if not sx > 0:
        sx = 1.0
    q = np.clip(np.rint((x.astype(np.float64) - ox) / sx), 0, 255)
    xh = sx * q + ox
    e2 = ((x.astype(np.float64) - xh) ** 2).sum()
    a2 = (xh ** 2).sum()
    ex = np.sqrt(e2) * (1 + 1e-12) + 1e-12 * np.sqrt(a2) + 1e-300
    return q.astype(np.int64), sx, ox, a2, xh.sum(), ex


def lower_bound(x, y):
    d = x.size
    xq, sx, ox, a2, sa, ex = query_image(x)
    q, o, sc, ey, b2, q1 = row_image(y)
    P = int((xq * q).sum())
    sab = sc * (sx * P + ox * q1) + o * sa
    d2 = a2 + b2 - 2 * sab
    mag = a2 + b2 + 2 * abs(sab)
    d2lo = d2 - 1e-7 * mag
    if not d2lo > 0:
        return 0.0
    t = np.sqrt(d2lo) * (1 - 1e-12) - ex - ey
    if not t > 0:
        return 0.0
    return t * t * (1.0 - (2.0 * d + 16.0) * U)


def ref_l2_fp32(x, y):
    """fvec_L2sqr in the reference's order: 8 fp32 accumulators over the
    first d & ~7 dims (fma of the rounded difference), (j, j+4), (j, j+2),
    (0, 1) reduction, then the tail (ref_arith.h)."""
    x = x.astype(np.float32)
    y = y.astype(np.float32)
    d = x.size
    n8 = d & ~7
    c = np.zeros(8, np.float32)
    for i in range(0, n8, 8):
        t = (x[i:i + 8] - y[i:i + 8]).astype(np.float32)
        c = (np.float64(t) * t + c).astype(np.float32)  # fma: one rounding
    x0, x1, x2, x3 = (np.float32(c[j] + c[j + 4]) for j in range(4))
    r = np.float32(np.float32(x0 + x2) + np.float32(x1 + x3))
    i = n8
    if d - n8 >= 4:
        e = [np.float32(np.float32(x[i + j] - y[i + j]) ** 2) for j in range(4)]
        r = np.float32(r + np.float32(np.float32(e[0] + e[2]) + np.float32(e[1] + e[3])))
        i += 4
    for j in range(i, d):
        t = np.float32(x[j] - y[j])
        r = np.float32(np.float64(t) * t + r)
    return float(r)


def test_q8_lower_bound_never_exceeds_reference_distance():
    rng = np.random.default_rng(7)
    tight = 0
    n = 0
    for case in range(1500):
        d = int(rng.choice([128, 100, 96, 37, 8, 5]))
        kind = case % 5
        if kind == 0:
            x, y = rng.random(d, np.float32), rng.random(d, np.float32)
        elif kind == 1:  # near neighbours: the bound must stay below a small distance
            y = rng.random(d, np.float32)
            x = (y + rng.normal(0, 1e-3, d)).astype(np.float32)
        elif kind == 2:  # wide magnitudes
            x = (rng.normal(0, 1e3, d)).astype(np.float32)
            y = (x + rng.normal(0, 10, d)).astype(np.float32)
        elif kind == 3:  # constant row / identical vectors
            y = np.full(d, np.float32(rng.normal()), np.float32)
            x = y.copy() if case % 2 else (y + np.float32(1e-4)).astype(np.float32)
        else:  # k-means-like centroids: narrow range around 0.5
            y = (0.5 + rng.normal(0, 0.05, d)).astype(np.float32)
            x = rng.random(d, np.float32)
        lb = lower_bound(x, y)
        dis = ref_l2_fp32(x, y)
        assert lb <= dis, (case, d, kind, lb, dis)
        n += 1
        tight += lb >= 0.98 * dis
    assert tight > n // 3  # the bound is useful, not only valid
