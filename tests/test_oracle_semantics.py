"""CPU: the oracle's restated semantics (heaps, ties, knn forms, merge)."""
import numpy as np
import pytest

from conftest import rand


def test_heap_strict_admission_and_reorder(orc):
    # ties at the boundary: first-come wins under strict `dis < top` admission
    vals = np.array([5, 3, 5, 1, 3, 5, 2], np.float32)
    ids = np.array([10, 11, 12, 13, 14, 15, 16], np.int64)
    D, I = orc.heap_addn_reorder(3, vals, ids, cmax=True)
    assert D.tolist() == [1, 2, 3] and I.tolist() == [13, 16, 11]
    # fewer candidates than k: padding (FLT_MAX, -1)
    D, I = orc.heap_addn_reorder(4, vals[:2], ids[:2], cmax=True)
    assert I.tolist() == [11, 10, -1, -1]
    assert D[2] == np.finfo(np.float32).max
    # CMin (inner product) keeps the largest, padding -FLT_MAX
    D, I = orc.heap_addn_reorder(2, vals[:3], ids[:3], cmax=False)
    assert D.tolist() == [5, 5] and sorted(I.tolist()) == [10, 12]


def test_equal_keys_keep_smallest_ids_in_increasing_scan(orc):
    # scanning in increasing id order with cmp2 eviction keeps the k smallest
    # (dist, id) pairs — the rule the GPU wave queue implements
    rng = np.random.default_rng(0)
    for _ in range(50):
        vals = rng.integers(0, 4, size=40).astype(np.float32)
        ids = np.arange(40, dtype=np.int64)
        D, I = orc.heap_addn_reorder(7, vals, ids)
        order = np.lexsort((ids, vals))[:7]
        assert I.tolist() == ids[order].tolist()


def test_knn_blas_form_vs_direct(orc):
    x = rand(orc, 50, 32, 1)
    y = rand(orc, 300, 32, 2)
    D1, I1 = orc.knn(x, y, 5, blas_form=True)
    D2, I2 = orc.knn(x, y, 5, blas_form=False)
    np.testing.assert_allclose(D1, D2, rtol=1e-5, atol=1e-5)
    assert (I1 == I2).mean() > 0.99


def test_knn_matches_numpy(orc):
    x = rand(orc, 20, 16, 3)
    y = rand(orc, 100, 16, 4)
    D, I = orc.knn(x, y, 4, blas_form=False)
    ref = ((x[:, None, :].astype(np.float64) - y[None].astype(np.float64)) ** 2).sum(-1)
    np.testing.assert_array_equal(I, np.argsort(ref, axis=1, kind="stable")[:, :4])


def test_float_rand_properties(orc):
    x = orc.float_rand(100000, 1234)
    assert x.dtype == np.float32 and 0 <= x.min() and x.max() <= 1
    assert abs(x.mean() - 0.5) < 0.01
    y = orc.float_rand(100000, 1234)
    assert np.array_equal(x, y)
    assert not np.array_equal(x, orc.float_rand(100000, 1235))


def test_merge_knn_results_semantics(orc):
    # shard 0 and 1 with a distance tie: the lower shard comes first (L2)
    Dall = np.array([[[1, 2, 3]], [[2, 2.5, 9]]], np.float32)
    Iall = np.array([[[10, 11, 12]], [[20, 21, 22]]], np.int64)
    D, I = orc.merge_knn_results(Dall, Iall)
    assert I.tolist() == [[10, 11, 20]]
    # a shard that ran out (-1) is skipped; padding at the end
    Iall2 = np.array([[[10, -1, -1]], [[20, -1, -1]]], np.int64)
    D, I = orc.merge_knn_results(Dall, Iall2)
    assert I.tolist() == [[10, 20, -1]]
    assert D[0, 2] == np.finfo(np.float32).max


def test_oracle_ivf_exhaustive_equals_knn(orc):
    d, nb, nlist = 16, 2000, 8
    xb = rand(orc, nb, d, 5)
    cent = xb[:nlist].copy()
    _, a = orc.knn(xb, cent, 1, blas_form=True)
    a = a[:, 0]
    order = np.argsort(a, kind="stable")
    off = np.zeros(nlist + 1, np.int64)
    off[1:] = np.cumsum(np.bincount(a, minlength=nlist))
    codes = xb[order].view(np.uint8).reshape(nb, d * 4)
    ivf = orc.IVFOracle(d, nlist, 1, off, codes, order.astype(np.int64), centroids=cent)
    xq = rand(orc, 64, d, 6)
    D, I, _, _ = ivf.search(xq, 10, nprobe=nlist)
    Dk, Ik = orc.knn(xq, xb, 10, blas_form=False)
    np.testing.assert_array_equal(I, Ik)
    np.testing.assert_array_equal(D, Dk)


def test_oracle_range_search_restatement(orc):
    """oracle_ivf_range_preassigned against a direct loop over the reference
    semantics (faiss/IndexIVF.cpp:1283-1345, IndexIVFFlat.cpp:181-201):
    probes in order, rows in list order, strict C::cmp(radius, dis)."""
    import numpy as np
    rng = np.random.default_rng(5)
    d, nlist = 12, 7
    sizes = rng.integers(0, 30, nlist)
    off = np.zeros(nlist + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    vecs = rng.random((int(off[-1]), d), dtype=np.float32)
    ids = rng.permutation(int(off[-1])).astype(np.int64) * 3
    xq = rng.random((9, d), dtype=np.float32)
    keys = rng.integers(-1, nlist, (9, 4))
    for metric, radius in ((1, 1.2), (0, 3.0)):
        ref = orc.IVFOracle(d, nlist, metric, off, vecs.view(np.uint8).reshape(len(vecs), -1), ids)
        sel = (ids % 2 == 0).astype(np.uint8)
        for selmask in (None, sel):
            lims, D, I = ref.range_search_preassigned(xq, radius, keys, selmask)
            eD, eI, elims = [], [], [0]
            for i in range(9):
                for key in keys[i]:
                    if key < 0:
                        continue
                    for r in range(off[key], off[key + 1]):
                        if selmask is not None and not selmask[r]:
                            continue
                        dis = (orc.fvec_L2sqr(xq[i], vecs[r]) if metric == 1
                               else orc.fvec_inner_product(xq[i], vecs[r]))
                        if (dis < radius) if metric == 1 else (dis > radius):
                            eD.append(dis)
                            eI.append(ids[r])
                elims.append(len(eI))
            assert lims.tolist() == elims
            assert I.tolist() == eI
            assert np.array_equal(D, np.array(eD, np.float32))
