"""GPU: IVF-Flat range search (faiss/IndexIVF.cpp:1203-1400,
IVFFlatScanner::scan_codes_range faiss/IndexIVFFlat.cpp:181-201).

The GPU result must equal the oracle's restatement bit for bit: the same
lims, the same ids in the same order (probe order, then list order — the
reference's RangeQueryResult order for parallel_mode 0) and the same fp32
distances (reference evaluation order).  Coarse keys are taken from the
library's own quantizer so both sides scan the same lists.  The reference's
own property (tests/test_index.py range tests: an IVF range search with
nprobe = nlist returns the exact range set) is checked too."""
import numpy as np
import pytest

from conftest import rand

pytestmark = pytest.mark.gpu

D_, NB, NLIST = 32, 12000, 48


@pytest.fixture(scope="module")
def flat_ix(amd, orc, gpu):
    xb = rand(orc, NB, D_, 91)
    idx = amd.index_factory(D_, f"IVF{NLIST},Flat")
    idx.train(xb)
    idx.add(xb)
    return idx, xb


def radius_for(idx, xq, k=20):
    D, _ = idx.search(xq, k)
    return float(np.median(D[:, -1]))


def check_equal(got, want):
    lg, Dg, Ig = got
    lw, Dw, Iw = want
    assert np.array_equal(np.asarray(lg, np.int64), np.asarray(lw, np.int64))
    assert np.array_equal(Ig, Iw)
    assert np.array_equal(Dg, Dw)


@pytest.mark.parametrize("nprobe", [1, 5, 16])
def test_range_search_l2_bit_exact(amd, orc, flat_ix, nprobe):
    idx, xb = flat_ix
    idx.nprobe = nprobe
    xq = rand(orc, 300, D_, 92)
    r = radius_for(idx, xq)
    got = idx.range_search(xq, r)
    _, keys = idx.quantizer.search(xq, nprobe)
    want = orc.IVFOracle.from_index(idx).range_search_preassigned(xq, r, keys)
    check_equal(got, want)
    assert got[0][-1] > 300  # a non-trivial result set


def test_range_search_ip_bit_exact(amd, orc, gpu):
    xb = rand(orc, 6000, D_, 93)
    idx = amd.index_factory(D_, "IVF24,Flat", amd.METRIC_INNER_PRODUCT)
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 6
    xq = rand(orc, 200, D_, 94)
    D, _ = idx.search(xq, 30)
    r = float(np.median(D[:, -1]))
    got = idx.range_search(xq, r)
    _, keys = idx.quantizer.search(xq, 6)
    want = orc.IVFOracle.from_index(idx).range_search_preassigned(xq, r, keys)
    check_equal(got, want)
    assert np.all(got[1] > r)


def test_range_search_all_lists_is_exact_range(amd, orc, flat_ix):
    idx, xb = flat_ix
    idx.nprobe = NLIST
    xq = rand(orc, 40, D_, 95)
    r = radius_for(idx, xq, 10)
    lims, D, I = idx.range_search(xq, r)
    for i in range(40):
        dis = np.array([orc.fvec_L2sqr(xq[i], y) for y in xb], np.float32)
        exact = set(np.nonzero(dis < r)[0].tolist())
        assert set(I[lims[i]:lims[i + 1]].tolist()) == exact


def test_range_search_preassigned_keys_edge_cases(amd, orc, flat_ix):
    idx, xb = flat_ix
    xq = rand(orc, 64, D_, 96)
    rng = np.random.default_rng(0)
    keys = rng.integers(0, NLIST, size=(64, 6))
    keys[::3, 2] = -1        # skipped probes (IndexIVF.cpp:1295-1297)
    keys[1::4, 4] = keys[1::4, 0]  # the same list probed twice is scanned twice
    idx.nprobe = 6  # the scan reads nprobe keys per query (IndexIVF.cpp:1253)
    r = radius_for(idx, xq)
    got = idx.range_search_preassigned(xq, r, keys)
    want = orc.IVFOracle.from_index(idx).range_search_preassigned(xq, r, keys)
    check_equal(got, want)
    bad = keys.copy()
    bad[0, 0] = NLIST
    with pytest.raises(amd.FaissError):
        idx.range_search_preassigned(xq, r, bad)


def test_range_search_empty_and_zero_radius(amd, orc, flat_ix):
    idx, _ = flat_ix
    idx.nprobe = 4
    lims, D, I = idx.range_search(np.zeros((0, D_), np.float32), 1.0)
    assert lims.shape == (1,) and lims[0] == 0 and I.size == 0
    xq = rand(orc, 20, D_, 97)
    lims, D, I = idx.range_search(xq, 0.0)  # strict <: nothing at distance >= 0
    assert lims[-1] == 0


def test_range_search_with_selector(amd, orc, flat_ix):
    idx, xb = flat_ix
    idx.nprobe = 8
    xq = rand(orc, 150, D_, 98)
    r = radius_for(idx, xq)
    sel = amd.IDSelectorRange(2000, 9000)
    params = amd.SearchParametersIVF(nprobe=8, sel=sel)
    got = idx.range_search(xq, r, params)
    ref = orc.IVFOracle.from_index(idx)
    mask = ((ref.ids >= 2000) & (ref.ids < 9000)).astype(np.uint8)
    _, keys = idx.quantizer.search(xq, 8)
    want = ref.range_search_preassigned(xq, r, keys, selmask=mask)
    check_equal(got, want)
    assert np.all((got[2] >= 2000) & (got[2] < 9000))


def test_range_search_stats(amd, orc, flat_ix):
    idx, _ = flat_ix
    idx.nprobe = 5
    xq = rand(orc, 100, D_, 99)
    st = amd.cvar.indexIVF_stats
    st.reset()
    idx.range_search(xq, 1.0)
    _, keys = idx.quantizer.search(xq, 5)
    sizes = np.array([idx.get_list_size(int(l)) for l in range(NLIST)])
    assert st.nq == 100
    assert st.nlist == int((sizes[keys] > 0).sum())
    assert st.ndis == int(sizes[keys].sum())


@pytest.fixture(scope="module")
def pq_ix(amd, orc, gpu):
    xb = rand(orc, 8000, 64, 101)
    idx = amd.index_factory(64, "IVF32,PQ16")
    idx.train(xb)
    idx.add(xb)
    return idx


@pytest.mark.parametrize("table", [1, 0])
def test_range_search_pq_bit_exact(amd, orc, pq_ix, table):
    # IVFPQScanner::scan_codes_range (IndexIVFPQ.cpp:1254-1279): the k-NN
    # path's table arithmetic, kept when dis < radius, in scan order
    idx = pq_ix
    xq = rand(orc, 200, 64, 102)
    idx.nprobe = 6
    idx.use_precomputed_table = table
    try:
        D, _ = idx.search(xq, 20)
        r = float(np.median(D[:, -1]))
        Dq, Iq = idx.quantizer.search(xq, 6)
        got_pre = idx.range_search_preassigned(xq, r, Iq, Dq)
        got = idx.range_search(xq, r)
        sel = amd.IDSelectorRange(1000, 5000)
        got_sel = idx.range_search(xq, r, amd.SearchParametersIVF(nprobe=6, sel=sel))
    finally:
        idx.use_precomputed_table = 1
    ref = orc.IVFOracle.from_index(idx)
    ref.s.use_precomputed_table = table
    want = ref.range_search_preassigned(xq, r, Iq, coarse_dis=Dq)
    check_equal(got_pre, want)
    check_equal(got, want)
    assert want[0][-1] > 200
    mask = ((ref.ids >= 1000) & (ref.ids < 5000)).astype(np.uint8)
    check_equal(got_sel, ref.range_search_preassigned(xq, r, Iq, selmask=mask, coarse_dis=Dq))


def test_range_search_pq_ip(amd, orc, gpu):
    """IVF-PQ inner-product range search (dis > radius) equals the oracle
    restatement (pinned to the reference in tests/test_ref_fixtures.py)"""
    xb = rand(orc, 3000, D_, 100)
    idx = amd.index_factory(D_, "IVF16,PQ8", amd.METRIC_INNER_PRODUCT)
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 4
    xq = xb[:20]
    ref = orc.IVFOracle.from_index(idx)
    q = amd.IndexFlat(D_, amd.METRIC_INNER_PRODUCT)
    q.add(idx.quantizer.xb)
    Dq, Iq = q.search(xq, 4)
    radius = float(np.median(ref.search_preassigned(xq, 10, Iq, Dq)[0][:, 5]))
    lims, D, I = idx.range_search(xq, radius)
    lr, Dr, Ir = ref.range_search_preassigned(xq, radius, Iq, coarse_dis=Dq)
    np.testing.assert_array_equal(lims, lr)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
