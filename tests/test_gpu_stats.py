"""GPU: the search-statistics surface of this fork:
IndexIVF::search_stats / search_preassigned_stats with QueryLatencyStats
(faiss/IndexIVF.h:28-32, faiss/IndexIVF.cpp:725-1200), IndexHNSW::search_stats
(faiss/IndexHNSW.cpp:345-366), and the global indexIVF_stats / hnsw_stats
counters (faiss/IndexIVF.h:567-583, faiss/impl/HNSW.h:234-253)."""
import numpy as np
import pytest

from conftest import assert_same_results, rand
from test_oracle_golden import FIX, write_ihnf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def flat_ivf(amd, orc, gpu):
    d, nb, nlist = 32, 20000, 64
    xb = rand(orc, nb, d, 51)
    idx = amd.index_factory(d, f"IVF{nlist},Flat")
    idx.train(xb)
    idx.add(xb)
    return idx, xb


def visit_counts(idx, xq, nprobe):
    """nlist / ndis as faiss counts them: non-empty lists visited, codes scanned."""
    _, Iq = idx.quantizer.search(xq, nprobe)
    sizes = np.array([idx.get_list_size(l) for l in range(idx.nlist)], dtype=np.int64)
    s = np.where(Iq >= 0, sizes[np.maximum(Iq, 0)], 0)
    return int((s > 0).sum()), int(s.sum())


def test_ivf_search_stats_same_results_and_records(amd, orc, flat_ivf):
    idx, _ = flat_ivf
    idx.nprobe = 8
    xq = rand(orc, 300, 32, 52)
    D, I = idx.search(xq, 10)
    st = amd.cvar.indexIVF_stats
    st.reset()
    D2, I2, lat = idx.search_stats(xq, 10)
    assert_same_results(D2, I2, D, I)
    assert lat.shape == (300,)
    assert (lat["quantization_us"] > 0).all() and (lat["list_scan_us"] > 0).all()
    np.testing.assert_allclose(lat["total_us"], lat["quantization_us"] + lat["list_scan_us"])
    # one slice: the amortised coarse time is the same for every query
    assert np.ptp(lat["quantization_us"]) == 0.0
    nl, nd = visit_counts(idx, xq, 8)
    assert (st.nq, st.nlist, st.ndis) == (300, nl, nd)
    # search_stats does not accumulate stage times (reference: commented out)
    assert st.quantization_time == 0.0 and st.search_time == 0.0
    st.reset()
    idx.search(xq, 10)
    assert (st.nq, st.nlist, st.ndis) == (300, nl, nd)
    assert 0.0 < st.quantization_time <= st.search_time


def test_ivf_search_preassigned_stats(amd, orc, flat_ivf):
    idx, _ = flat_ivf
    idx.nprobe = 6
    xq = rand(orc, 120, 32, 53)
    Dq, Iq = idx.quantizer.search(xq, 6)
    D, I = idx.search_preassigned(xq, 5, Iq, Dq)
    own = amd.IndexIVFStats()
    g = amd.cvar.indexIVF_stats
    g.reset()
    D2, I2, lat = idx.search_preassigned_stats(xq, 5, Iq, Dq, ivf_stats=own)
    assert_same_results(D2, I2, D, I)
    assert (lat["list_scan_us"] > 0).all()
    assert (lat["quantization_us"] == 0).all()
    nl, nd = visit_counts(idx, xq, 6)
    assert (own.nq, own.nlist, own.ndis) == (120, nl, nd)
    assert g.nq == 0  # an explicit stats object receives the counts


@pytest.mark.parametrize("desc,k", [("Flat", 10), ("Flat", 100), ("PQ8", 10)])
def test_ivf_search_stats_per_query_latency(amd, orc, gpu, desc, k):
    """list_scan_us is each query's own completion time in the batched scan
    (device clock stamped where its result is emitted: the re-rank wave, or
    the exact path's select), so the per-query values carry the spread the
    author's harness reports as P50 / P95 / P99
    (tutorial/cpp/benchmark-hnsw-ivf/benchmark_hnsw_ivf.cpp:400-404)."""
    import time
    d, nb, nlist = 32, 20000, 64
    xb = rand(orc, nb, d, 54)
    idx = amd.index_factory(d, f"IVF{nlist},{desc}")
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 8
    xq = rand(orc, 2000, d, 55)
    D, I = idx.search(xq, k)
    t = time.perf_counter()
    D2, I2, lat = idx.search_stats(xq, k)
    wall_us = (time.perf_counter() - t) * 1e6
    assert_same_results(D2, I2, D, I)
    ls = lat["list_scan_us"]
    assert (ls > 0).all() and (ls < wall_us).all()
    assert len(np.unique(ls)) > 100  # per-query values, not one batch figure
    p50, p99 = np.percentile(ls, [50, 99])
    assert p50 <= p99
    np.testing.assert_allclose(lat["total_us"], lat["quantization_us"] + ls)
    # search_preassigned_stats: the same per-query stamps
    Dq, Iq = idx.quantizer.search(xq, 8)
    _, _, lat2 = idx.search_preassigned_stats(xq, k, Iq, Dq)
    assert (lat2["list_scan_us"] > 0).all() and len(np.unique(lat2["list_scan_us"])) > 100


def test_ivf_stats_empty_batch(amd, flat_ivf):
    idx, _ = flat_ivf
    D, I, lat = idx.search_stats(np.zeros((0, 32), np.float32), 4)
    assert D.shape == (0, 4) and lat.shape == (0,)


def test_hnsw_search_stats_match_reference_counters(amd, gpu, tmp_path):
    # HNSWStats n1, n2, ndis, nhops of the reference's own HNSW::search on the
    # same graph and queries (fixture from oracle/ref/make_golden.py)
    fx = np.load(FIX, allow_pickle=False)
    p = tmp_path / "g.ihnf"
    write_ihnf(p, fx)
    idx = amd.read_index(str(p))
    hs = amd.cvar.hnsw_stats
    for ef in (16, 48):
        idx.efSearch = ef
        for k in (1, 10):
            hs.reset()
            D, I, lat = idx.search_stats(fx["hnsw_xq"], k)
            assert_same_results(D, I, fx[f"hnsw_{ef}_{k}_D"], fx[f"hnsw_{ef}_{k}_I"])
            got = [hs.n1, hs.n2, hs.ndis, hs.nhops]
            assert got == [int(v) for v in fx[f"hnsw_{ef}_{k}_stats"]], (ef, k, got)
            assert (lat["quantization_us"] == 0).all()
            np.testing.assert_array_equal(lat["total_us"], lat["list_scan_us"])
            # plain search counts the same (faiss always combines hnsw_stats)
            hs.reset()
            idx.search(fx["hnsw_xq"], k)
            assert [hs.n1, hs.n2, hs.ndis, hs.nhops] == got


def test_hnsw_quantizer_stats_through_ivf(amd, orc, gpu):
    # tests/test_graph_based.py:158-164 (ndis > nq * efSearch), with the HNSW
    # graph as the IVF coarse quantizer: its counters reach hnsw_stats too
    d, nb = 32, 20000
    xb = rand(orc, nb, d, 54)
    idx = amd.index_factory(d, "IVF256_HNSW16,Flat")
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 8
    hs = amd.cvar.hnsw_stats
    hs.reset()
    xq = rand(orc, 200, d, 55)
    idx.search(xq, 10)
    assert hs.n1 == 200
    assert hs.ndis > 200 * 16
