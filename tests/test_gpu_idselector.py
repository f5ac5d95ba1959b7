"""GPU: IDSelector on the IVF search path (SURVEY §8(f) row 4;
faiss/impl/IDSelector.h, faiss/IndexIVF.cpp:418-430, scanner `use_sel`
faiss/IndexIVFFlat.cpp:165-167 / faiss/IndexIVFPQ.cpp:777-780).

A search restricted to the members of a selector must return exactly what
the same search returns on an index holding only the member vectors, in the
same lists and list order (the reference's tests/test_search_params.py
compares against such a subset index): same ids, same fp32 distances, same
tie order.  Checked for every selector type, both Flat scan paths and the
IVF-PQ path."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu

D_, NB, NLIST = 32, 12000, 48


def selectors(amd, rng):
    ids = np.arange(NB)
    batch = rng.choice(NB, 3000, replace=False)
    arr = rng.choice(NB, 500, replace=False)
    bm = (rng.random(NB) < 0.3)
    bitmap = np.packbits(bm, bitorder="little")
    r1 = amd.IDSelectorRange(2000, 7000)
    out = {
        "range": (amd.IDSelectorRange(2000, 7000), (ids >= 2000) & (ids < 7000)),
        "batch": (amd.IDSelectorBatch(batch), np.isin(ids, batch)),
        "array": (amd.IDSelectorArray(arr), np.isin(ids, arr)),
        "bitmap": (amd.IDSelectorBitmap(bitmap), bm),
        "not": (amd.IDSelectorNot(r1), ~((ids >= 2000) & (ids < 7000))),
        "and": (amd.IDSelectorAnd(amd.IDSelectorRange(0, 9000), amd.IDSelectorBatch(batch)),
                (ids < 9000) & np.isin(ids, batch)),
        "or": (amd.IDSelectorOr(amd.IDSelectorRange(0, 1000), amd.IDSelectorBatch(batch)),
               (ids < 1000) | np.isin(ids, batch)),
        "xor": (amd.IDSelectorXOr(amd.IDSelectorRange(0, 6000), amd.IDSelectorBatch(batch)),
                (ids < 6000) ^ np.isin(ids, batch)),
    }
    return out


@pytest.fixture(scope="module")
def data(amd, orc, gpu):
    xb = rand(orc, NB, D_, 81)
    xq = rand(orc, 300, D_, 82)
    q = amd.IndexFlatL2(D_)
    full = amd.IndexIVFFlat(q, D_, NLIST)
    full.train(xb)
    full.add(xb)
    return q, full, xb, xq


@pytest.mark.parametrize("kind", ["range", "batch", "array", "bitmap", "not", "and", "or", "xor"])
@pytest.mark.parametrize("scan", ["mfma", "exact"])
def test_flat_selector_equals_subset_index(amd, orc, data, monkeypatch, kind, scan):
    q, full, xb, xq = data
    sel, member = selectors(amd, np.random.default_rng(7))[kind]
    monkeypatch.setenv("FAISS_AMD_IVF_SCAN", scan)
    sub = amd.IndexIVFFlat(q, D_, NLIST)
    keep = np.nonzero(member)[0]
    sub.add_with_ids(xb[keep], keep.astype(np.int64))
    for k, nprobe in ((10, 8), (25, 3)):
        full.nprobe = sub.nprobe = nprobe
        D, I = full.search(xq, k, params=amd.SearchParametersIVF(nprobe=nprobe, sel=sel))
        Ds, Is = sub.search(xq, k)
        assert_same_results(D, I, Ds, Is)
        assert np.all(member[I[I >= 0]])


def test_selector_is_member_matches_reference_predicate(amd):
    rng = np.random.default_rng(9)
    for kind, (sel, member) in selectors(amd, rng).items():
        for i in list(range(0, NB, 37)) + [NB - 1]:
            assert sel.is_member(i) == bool(member[i]), (kind, i)
    bm = amd.IDSelectorBitmap(np.array([0b00000101], np.uint8))
    assert [bm.is_member(i) for i in (-1, 0, 1, 2, 8, 1 << 40)] == [False, True, False, True,
                                                                     False, False]


def test_pq_selector_equals_subset_index(amd, orc, gpu, tmp_path):
    d, nb, nlist = 64, 20000, 32
    xb = rand(orc, nb, d, 83)
    xq = rand(orc, 300, d, 84)
    full = amd.index_factory(d, f"IVF{nlist},PQ16")
    full.train(xb)
    full.add(xb)
    fn = tmp_path / "pq.index"
    amd.write_index(full, fn)
    sub = amd.read_index(fn)  # same quantizer and codebooks
    sub.reset()
    keep = np.nonzero(np.random.default_rng(3).random(nb) < 0.4)[0]
    sub.add_with_ids(xb[keep], keep.astype(np.int64))
    sel = amd.IDSelectorBatch(keep)
    for nprobe in (4, 12):
        full.nprobe = sub.nprobe = nprobe
        D, I = full.search(xq, 10, params=amd.SearchParametersIVF(nprobe=nprobe, sel=sel))
        Ds, Is = sub.search(xq, 10)
        assert_same_results(D, I, Ds, Is)


@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("nq,k", [(7, 5), (64, 10), (40, 100)])
def test_flat_index_with_selectors(amd, orc, gpu, metric, nq, k):
    """IndexFlat search with an IDSelector (faiss/IndexFlat.cpp:38-57 ->
    faiss/utils/distances.cpp:840-935, c_api/example_c.c's searches):
    IDSelectorRange searches the rows [imin, imax) in the batch size's form
    (direct below 20 queries, BLAS form above) and shifts the labels; any
    other selector takes the direct form over its members in id order."""
    rng = np.random.default_rng(7 + nq + k + metric)
    xb = rand(orc, NB, D_, 85)
    xq = rand(orc, nq, D_, 86)
    flat = amd.IndexFlatL2(D_) if metric == 1 else amd.IndexFlatIP(D_)
    flat.add(xb)
    for name, (sel, member) in selectors(amd, rng).items():
        D, I = flat.search(xq, k, params=amd.SearchParametersIVF(sel=sel))
        ids = np.nonzero(member)[0]
        if name == "range":
            Dr, Ir = orc.knn(xq, xb[2000:7000], k, metric, blas_form=nq >= 20)
            Ir = np.where(Ir >= 0, Ir + 2000, -1)
        else:
            Dr, Ir = orc.knn(xq, xb[ids], k, metric, blas_form=False)
            Ir = np.where(Ir >= 0, ids[np.maximum(Ir, 0)], -1)
        assert_same_results(D, I, Dr, Ir)


def test_flat_selector_range_outside(amd, orc, gpu):
    """A range past the stored rows selects nothing: (FLT_MAX, -1) rows."""
    xb = rand(orc, 500, 16, 85)
    flat = amd.IndexFlatL2(16)
    flat.add(xb)
    D, I = flat.search(xb[:5], 3, params=amd.SearchParametersIVF(sel=amd.IDSelectorRange(600, 900)))
    assert (I == -1).all() and (D == np.finfo(np.float32).max).all()


def test_pq_selector_keeps_filter_pruning(amd, orc, gpu, monkeypatch, capfd):
    """the code-decoding PQ filter gives a padding row or
    a selector non-member the bias fragment {-inf, 0, 0, 1, 1, 1, 0, 0}
    (kernels_pq_mfma.hip bias_frag), so its key sorts after every real one;
    the round-5 form split -inf into (-inf, NaN, NaN) and its NaN keys made
    streams fail (the re-rank then rescans them: results still exact, the
    pruning lost).  The failing streams per query with a 40 % selector stay
    at the unfiltered search's level (FAISS_AMD_IVF_STATS counters)."""
    import re
    d, nb, nlist = 64, 20000, 32
    xb = rand(orc, nb, d, 83)
    xq = rand(orc, 300, d, 84)
    idx = amd.index_factory(d, f"IVF{nlist},PQ16")
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 8
    keep = np.nonzero(np.random.default_rng(3).random(nb) < 0.4)[0]
    sel = amd.IDSelectorBatch(keep)
    monkeypatch.setenv("FAISS_AMD_IVF_STATS", "1")

    def failing(params):
        capfd.readouterr()
        idx.search(xq, 10, params=params)
        err = capfd.readouterr().err
        m = re.findall(r"ivfpq mfma scan: .*failing streams/q=([0-9.]+)", err)
        assert m, err
        return float(m[-1])

    f0 = failing(None)
    f1 = failing(amd.SearchParametersIVF(nprobe=8, sel=sel))
    assert f1 <= 2.0 * f0 + 0.25, (f0, f1)
