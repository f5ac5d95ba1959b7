"""Paged host-buffer search (faiss/gpu/GpuIndex.cu:307-333, searchFromCpuPaged_):
faiss_Index_search on host arrays uploads the queries in pages, page i + 1's
upload overlapping page i's search and page i - 1's download.  Any page
count gives the single-page results bit for bit (and the oracle's), the same
indexIVF_stats counts, stage times, and InterruptCallback behaviour between
pages (faiss/IndexIVF.cpp:627, 707-713)."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu


def _search_pages(amd, idx, xq, k, pages, monkeypatch):
    monkeypatch.setenv("FAISS_AMD_HOST_PAGES", str(pages))
    st = amd.cvar.indexIVF_stats
    st.reset()
    D, I = idx.search(xq, k)
    return D, I, (st.nq, st.nlist, st.ndis), (st.quantization_time, st.search_time)


@pytest.mark.parametrize("d", [32, 30])
def test_flat_pages_bit_exact(amd, orc, gpu, monkeypatch, d):
    xb = rand(orc, 20_000, d, 91)
    idx = amd.index_factory(d, "IVF64,Flat")
    idx.train(xb[:5000])
    idx.add(xb)
    idx.nprobe = 8
    xq = rand(orc, 1000, d, 92)
    D1, I1, c1, _ = _search_pages(amd, idx, xq, 10, 0, monkeypatch)  # the eager path
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 8, nslices=1)
    assert_same_results(D1, I1, Dr, Ir)
    # ragged pages; 50 pages of 20 queries; pages 3 four times: an eager
    # search per page, then the pages' graphs captured, then replayed
    for pages in (1, 1, 1, 2, 3, 7, 50, 3, 3, 3):
        D, I, c, (qt, stt) = _search_pages(amd, idx, xq, 10, pages, monkeypatch)
        assert np.array_equal(I, I1) and np.array_equal(D, D1), pages
        assert c == c1 == (1000, c1[1], c1[2])
        assert 0.0 < qt <= stt
    # a new query batch through the replayed pages' graphs
    xq2 = rand(orc, 1000, d, 99)
    D2, I2, _, _ = _search_pages(amd, idx, xq2, 10, 3, monkeypatch)
    Dr2, Ir2, _, _ = ref.search(xq2, 10, 8, nslices=1)
    assert_same_results(D2, I2, Dr2, Ir2)


def test_pq_pages_and_params(amd, orc, gpu, monkeypatch):
    d = 32
    xb = rand(orc, 20_000, d, 93)
    idx = amd.index_factory(d, "IVF64,PQ8")
    idx.train(xb[:8000])
    idx.add(xb)
    idx.nprobe = 6
    xq = rand(orc, 900, d, 94)
    D1, I1, c1, _ = _search_pages(amd, idx, xq, 7, 1, monkeypatch)
    D4, I4, c4, _ = _search_pages(amd, idx, xq, 7, 4, monkeypatch)
    assert np.array_equal(I4, I1) and np.array_equal(D4, D1)
    assert c4 == c1
    # per-call parameters (nprobe, max_codes) reach every page
    p = amd.SearchParametersIVF(nprobe=12, max_codes=900)
    monkeypatch.setenv("FAISS_AMD_HOST_PAGES", "1")
    Dp1, Ip1 = idx.search(xq, 7, params=p)
    monkeypatch.setenv("FAISS_AMD_HOST_PAGES", "5")
    Dp5, Ip5 = idx.search(xq, 7, params=p)
    assert np.array_equal(Ip5, Ip1) and np.array_equal(Dp5, Dp1)
    assert not np.array_equal(Ip1, I1)


def test_default_pages_large_batch(amd, orc, gpu, monkeypatch):
    # 40000 queries: the default policy takes 2 pages of 20000
    d = 16
    xb = rand(orc, 30_000, d, 95)
    idx = amd.index_factory(d, "IVF128,Flat")
    idx.train(xb[:6000])
    idx.add(xb)
    idx.nprobe = 4
    xq = rand(orc, 40_000, d, 96)
    D1, I1, c1, _ = _search_pages(amd, idx, xq, 5, 0, monkeypatch)
    monkeypatch.delenv("FAISS_AMD_HOST_PAGES")
    amd.cvar.indexIVF_stats.reset()
    for _ in range(3):  # eager, captured, replayed
        amd.cvar.indexIVF_stats.reset()
        D, I = idx.search(xq, 5)
        st = amd.cvar.indexIVF_stats
        assert np.array_equal(I, I1) and np.array_equal(D, D1)
        assert (st.nq, st.nlist, st.ndis) == c1


def test_pages_interrupted_then_exact(amd, orc, gpu, monkeypatch):
    d = 32
    xb = rand(orc, 20_000, d, 97)
    idx = amd.index_factory(d, "IVF64,Flat")
    idx.train(xb[:5000])
    idx.add(xb)
    idx.nprobe = 8
    xq = rand(orc, 600, d, 98)
    monkeypatch.setenv("FAISS_AMD_HOST_PAGES", "3")
    amd.set_interrupt_timeout(1e-9)  # fires at the poll before page 2
    try:
        with pytest.raises(amd.FaissError, match="computation interrupted"):
            idx.search(xq, 10)
        D, I = idx.search(xq, 10)  # fired once: this one runs to the end
    finally:
        amd.set_interrupt_timeout(None)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 8, nslices=1)
    assert_same_results(D, I, Dr, Ir)
