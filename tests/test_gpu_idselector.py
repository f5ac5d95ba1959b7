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


def test_selector_rejected_where_unsupported(amd, orc, gpu):
    xb = rand(orc, 500, 16, 85)
    flat = amd.IndexFlatL2(16)
    flat.add(xb)
    with pytest.raises(amd.FaissError, match="IDSelector"):
        flat.search(xb[:5], 3, params=amd.SearchParametersIVF(nprobe=1,
                                                             sel=amd.IDSelectorRange(0, 10)))
