#!/usr/bin/env python3
"""Generate tests/golden/ref_fixtures.npz from the reference sources.

Runs only in the build container (needs oracle/_ref/libfaissref.so, which
oracle/ref/Makefile compiles from /root/reference).  Every expected output
below is produced by reference code: faiss::float_rand, fvec_L2sqr /
fvec_inner_product / fvec_norm_L2sqr / fvec_L2sqr_batch_4, the faiss heap
(heap_heapify / heap_replace_top / heap_reorder) driven with the IVF
scanner's admission test, merge_knn_results, HNSW::prepare_level_tab +
add_with_locks (graph build) and HNSW::search.  Inputs are synthetic
(faiss float_rand streams and seeded numpy draws); nothing from the
reference tree is copied into the fixture.

    python oracle/ref/make_golden.py          # rewrites the fixture
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "tests", "golden", "ref_fixtures.npz")

L = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfaissref.so"))
P = C.c_void_p
SZ = C.c_size_t
L.ref_float_rand.argtypes = [P, SZ, C.c_int64]
L.ref_fvec_batch.argtypes = [P, P, SZ, SZ, C.c_int, P]
L.ref_fvec_batch4.argtypes = [P, P, SZ, SZ, P]
L.ref_fvec_norms.argtypes = [P, SZ, SZ, P]
L.ref_heap_stream.argtypes = [P, P, SZ, SZ, C.c_int, P, P]
L.ref_knn_direct.argtypes = [P, SZ, P, SZ, SZ, SZ, C.c_int, P, P]
L.ref_ivf_flat_query.argtypes = [P, SZ, P, P, P, P, P, SZ, SZ, C.c_int, P, P]
L.ref_merge_knn_results.argtypes = [SZ, SZ, C.c_int, P, P, P, P, C.c_int]
L.ref_hnsw_build.argtypes = [P, SZ, SZ, C.c_int, C.c_int]
L.ref_hnsw_build.restype = P
L.ref_hnsw_sizes.argtypes = [P, P]
L.ref_hnsw_copy.argtypes = [P, P, P, P, P, P, C.c_int64]
L.ref_hnsw_free.argtypes = [P]
L.ref_hnsw_search.argtypes = [P, SZ, SZ, P, P, SZ, P, SZ, P, SZ, C.c_int32, C.c_int32, C.c_int,
                              P, SZ, SZ, P, P, P]


def p(a):
    return a.ctypes.data_as(P)


def float_rand(n, seed):
    x = np.empty(n, np.float32)
    L.ref_float_rand(p(x), n, seed)
    return x


def fvec(x, Y, metric_l2):
    out = np.empty(Y.shape[0], np.float32)
    L.ref_fvec_batch(p(x), p(Y), Y.shape[1], Y.shape[0], int(metric_l2), p(out))
    return out


def heap_stream(dis, ids, k, metric_l2):
    D = np.empty(k, np.float32)
    I = np.empty(k, np.int64)
    L.ref_heap_stream(p(dis), p(ids), dis.size, k, int(metric_l2), p(D), p(I))
    return D, I


def knn_direct(x, y, k, metric_l2):
    n = x.shape[0]
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    L.ref_knn_direct(p(x), n, p(y), y.shape[0], x.shape[1], k, int(metric_l2), p(D), p(I))
    return D, I


def main():
    rng = np.random.default_rng(20251015)
    fx = {}

    # ---- float_rand (faiss/utils/random.cpp:95-112): both block regimes
    for n, seed in ((100, 1234), (3000, 5678), (5000, 42)):
        fx[f"float_rand_{n}_{seed}"] = float_rand(n, seed)
    big = float_rand(1 << 20, 1234)
    fx["float_rand_1M_1234_sum"] = np.array([big.astype(np.float64).sum()])
    fx["float_rand_1M_1234_head_tail"] = np.concatenate([big[:16], big[-16:]])

    # ---- fvec_* evaluation order, d covering every epilogue/tail case
    dims = np.array([1, 3, 4, 5, 7, 8, 12, 13, 16, 30, 31, 64, 96, 100, 127, 128, 129, 200])
    fx["fvec_dims"] = dims
    for d in dims:
        q = rng.random(int(d), dtype=np.float32) * 2 - 0.5
        Y = rng.random((24, int(d)), dtype=np.float32) * 2 - 0.5
        fx[f"fvec_q_{d}"] = q
        fx[f"fvec_Y_{d}"] = Y
        fx[f"fvec_l2_{d}"] = fvec(q, Y, True)
        fx[f"fvec_ip_{d}"] = fvec(q, Y, False)
        nr = np.empty(24, np.float32)
        L.ref_fvec_norms(p(Y), int(d), 24, p(nr))
        fx[f"fvec_norm_{d}"] = nr
        b4 = np.empty(24, np.float32)
        L.ref_fvec_batch4(p(q), p(Y), int(d), 24, p(b4))
        fx[f"fvec_b4_{d}"] = b4

    # ---- heap streams with ties: ascending ids and shuffled ids, both metrics
    for case in range(6):
        n = 300
        vals = rng.integers(0, 12, n).astype(np.float32) * np.float32(0.25)
        ids = np.arange(n, dtype=np.int64) * 3 + 7
        if case % 2 == 1:
            ids = rng.permutation(ids)
        for l2 in (1, 0):
            for k in (1, 5, 10, 33):
                D, I = heap_stream(vals, ids, k, l2)
                fx[f"heap_{case}_{l2}_{k}_D"] = D
                fx[f"heap_{case}_{l2}_{k}_I"] = I
        fx[f"heap_{case}_vals"] = vals
        fx[f"heap_{case}_ids"] = ids

    # ---- direct knn (slices below the BLAS threshold)
    d, ny = 30, 700
    xk = float_rand(7 * d, 11).reshape(7, d)
    yk = float_rand(ny * d, 12).reshape(ny, d)
    fx["knn_x"], fx["knn_y"] = xk, yk
    for l2 in (1, 0):
        D, I = knn_direct(xk, yk, 10, l2)
        fx[f"knn_{l2}_D"], fx[f"knn_{l2}_I"] = D, I

    # ---- IVF-Flat: lists from a direct k=1 assignment (vectors whose two
    # nearest centroids are closer than 1e-3 relative are dropped so the
    # list membership is unambiguous under any rounding), duplicated rows
    # (exact ties at the k boundary), ids not monotone across lists
    d, nlist, nb = 32, 16, 2400
    xb = float_rand(nb * d, 21).reshape(nb, d)
    xb = np.concatenate([xb, np.repeat(xb[:40], 6, axis=0)])  # 240 duplicates
    cent = float_rand(nlist * d, 22).reshape(nlist, d)
    for l2 in (1, 0):
        Dk, Ik = knn_direct(xb, cent, 2, l2)
        gap = np.abs(Dk[:, 1] - Dk[:, 0]) / np.maximum(np.abs(Dk[:, 0]), 1e-6)
        keep = gap > 1e-3
        xs = xb[keep]
        ids = (np.arange(xb.shape[0], dtype=np.int64) * 7919 % 100003)[keep]
        assign = Ik[keep, 0]
        order = np.argsort(assign, kind="stable")
        xs, ids, assign = xs[order], ids[order], assign[order]
        list_len = np.bincount(assign, minlength=nlist).astype(np.int64)
        list_off = np.concatenate([[0], np.cumsum(list_len)[:-1]]).astype(np.int64)
        nq, nprobe = 50, 5
        xq = np.concatenate([float_rand(40 * d, 23).reshape(40, d), xb[:10]])
        Dq, Iq = knn_direct(xq, cent, nprobe, l2)
        for k in (1, 10, 25):
            D = np.empty((nq, k), np.float32)
            I = np.empty((nq, k), np.int64)
            for i in range(nq):
                L.ref_ivf_flat_query(p(xq[i]), d, p(xs), p(ids), p(list_off), p(list_len),
                                     p(Iq[i]), nprobe, k, l2, p(D[i]), p(I[i]))
            fx[f"ivf_{l2}_{k}_D"], fx[f"ivf_{l2}_{k}_I"] = D, I
        fx[f"ivf_{l2}_xb"], fx[f"ivf_{l2}_ids"] = xs, ids
        fx[f"ivf_{l2}_list_len"], fx[f"ivf_{l2}_assign"] = list_len, assign
        fx[f"ivf_{l2}_xq"], fx[f"ivf_{l2}_cent"] = xq, cent
        fx[f"ivf_{l2}_Iq"], fx[f"ivf_{l2}_Dq"] = Iq, Dq

    # ---- merge_knn_results with ties across shards and empty slots
    n, k, ns = 30, 10, 3
    allD = np.sort(rng.integers(0, 8, (ns, n, k)).astype(np.float32), axis=2)
    allI = rng.integers(0, 1000, (ns, n, k)).astype(np.int64)
    allI[1, :5, 6:] = -1
    for l2 in (1, 0):
        Dm = allD if l2 else -allD
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        L.ref_merge_knn_results(n, k, ns, p(np.ascontiguousarray(Dm)), p(allI), p(D), p(I), l2)
        fx[f"merge_{l2}_in_D"], fx[f"merge_{l2}_D"], fx[f"merge_{l2}_I"] = Dm, D, I
    fx["merge_in_I"] = allI

    # ---- HNSW: reference build (serial) + reference search
    d, nb, M = 24, 1500, 8
    xh = float_rand(nb * d, 31).reshape(nb, d)
    h = L.ref_hnsw_build(p(xh), nb, d, M, 40)
    sz = np.empty(6, np.int64)
    L.ref_hnsw_sizes(h, p(sz))
    levels = np.empty(sz[0], np.int32)
    offsets = np.empty(sz[1], np.uint64)
    neighbors = np.empty(sz[2], np.int32)
    cum = np.empty(sz[3], np.int32)
    probas = np.empty(64, np.float64)
    L.ref_hnsw_copy(h, p(levels), p(offsets), p(neighbors), p(cum), p(probas), 64)
    L.ref_hnsw_free(h)
    nprob = int(np.count_nonzero(probas[: len(cum) - 1] > 0)) if len(cum) > 1 else 0
    fx["hnsw_xb"], fx["hnsw_levels"], fx["hnsw_offsets"] = xh, levels, offsets
    fx["hnsw_neighbors"], fx["hnsw_cum"] = neighbors, cum
    fx["hnsw_probas"] = probas[: len(cum) - 1]
    fx["hnsw_meta"] = np.array([nb, d, M, sz[4], sz[5], 40], np.int64)
    xq = float_rand(40 * d, 32).reshape(40, d)
    fx["hnsw_xq"] = xq
    for ef in (16, 48):
        for k in (1, 10):
            D = np.empty((40, k), np.float32)
            I = np.empty((40, k), np.int64)
            st = np.zeros(4, np.uint64)
            L.ref_hnsw_search(p(xh), nb, d, p(levels), p(offsets), len(offsets), p(neighbors),
                              len(neighbors), p(cum), len(cum), int(sz[4]), int(sz[5]), ef,
                              p(xq), 40, k, p(D), p(I), p(st))
            fx[f"hnsw_{ef}_{k}_D"], fx[f"hnsw_{ef}_{k}_I"] = D, I
            fx[f"hnsw_{ef}_{k}_stats"] = st  # HNSWStats n1, n2, ndis, nhops
    del nprob

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **fx)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e3:.0f} kB, {len(fx)} arrays)")


if __name__ == "__main__":
    sys.exit(main())
