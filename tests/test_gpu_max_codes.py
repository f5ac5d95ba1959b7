"""GPU: max_codes and parallel_mode on the IVF search path (SURVEY §8 row a6,
faiss/IndexIVF.cpp:445-460 and :595-631).  With max_codes > 0 a query scans
its probes in coarse order, cuts the probe that reaches max_codes to the rows
still allowed (scan_one_list's list_size_max, :546-550) and skips the rest.
Checked against the oracle restatement (oracle_ivf_search_preassigned_mc) on
both Flat scan paths and the PQ scan, plus the reference's own property test
(tests/test_search_params.py:351-374)."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu

D_ = 32


@pytest.fixture(scope="module")
def flat_ivf(amd, orc, gpu):
    xb = rand(orc, 20000, D_, 61)
    idx = amd.index_factory(D_, "IVF64,Flat")
    idx.train(xb)
    idx.add(xb)
    return idx


@pytest.fixture(scope="module")
def pq_ivf(amd, orc, gpu):
    xb = rand(orc, 20000, D_, 62)
    idx = amd.index_factory(D_, "IVF64,PQ8")
    idx.train(xb)
    idx.add(xb)
    return idx


def run_preassigned(amd, idx, xq, k, nprobe, max_codes):
    Dq, Iq = idx.quantizer.search(xq, nprobe)
    idx.nprobe = nprobe  # search_preassigned reads nprobe keys per query (faiss)
    idx.max_codes = max_codes
    st = amd.cvar.indexIVF_stats
    st.reset()
    try:
        D, I = idx.search_preassigned(xq, k, Iq, Dq)
    finally:
        idx.max_codes = 0
    return D, I, Iq, Dq, st.ndis


@pytest.mark.parametrize("scan", ["mfma", "exact"])
@pytest.mark.parametrize("max_codes", [1, 150, 700, 2000])
def test_flat_max_codes_matches_oracle(amd, orc, flat_ivf, monkeypatch, scan, max_codes):
    monkeypatch.setenv("FAISS_AMD_IVF_SCAN", scan)
    xq = rand(orc, 300, D_, 63)
    D, I, Iq, Dq, ndis = run_preassigned(amd, flat_ivf, xq, 10, 8, max_codes)
    ref = orc.IVFOracle.from_index(flat_ivf)
    Dr, Ir, ndr = ref.search_preassigned(xq, 10, Iq, Dq, max_codes=max_codes, return_ndis=True)
    assert_same_results(D, I, Dr, Ir)
    assert ndis == ndr <= 300 * max_codes


def test_flat_max_codes_search_params_and_reference_property(amd, orc, flat_ivf):
    # tests/test_search_params.py:351-374: ndis <= target per query, and the
    # unlimited result whenever the cap was not reached
    idx = flat_ivf
    xq = rand(orc, 100, D_, 64)
    st = amd.cvar.indexIVF_stats
    st.reset()
    D0, I0 = idx.search(xq, 10, params=amd.SearchParametersIVF(nprobe=8))
    target = st.ndis // len(xq)
    p = amd.SearchParametersIVF(nprobe=8, max_codes=target)
    Db, Ib = idx.search(xq, 10, params=p)  # batched == per-query below
    hit = 0
    for q in range(len(xq)):
        st.reset()
        Dq, Iq = idx.search(xq[q:q + 1], 10, params=p)
        assert st.ndis <= target
        assert np.array_equal(Iq[0], Ib[q])
        if st.ndis < target:
            hit += 1
            assert np.array_equal(I0[q], Iq[0])
    assert 0 < hit < len(xq)


def test_pq_max_codes_matches_oracle(amd, orc, pq_ivf):
    xq = rand(orc, 200, D_, 65)
    for max_codes in (1, 333, 1200):
        D, I, Iq, Dq, ndis = run_preassigned(amd, pq_ivf, xq, 10, 8, max_codes)
        ref = orc.IVFOracle.from_index(pq_ivf)
        Dr, Ir, ndr = ref.search_preassigned(xq, 10, Iq, Dq, max_codes=max_codes,
                                             return_ndis=True)
        assert ndis == ndr
        # PQ parity: the LUT summation order differs
        assert np.mean(I == Ir) > 0.99
        ok = Ir >= 0
        np.testing.assert_allclose(D[ok], Dr[ok], rtol=1e-4, atol=1e-5)


def test_max_codes_through_parameter_space(amd, orc, flat_ivf):
    xq = rand(orc, 50, D_, 66)
    flat_ivf.nprobe = 8
    amd.ParameterSpace().set_index_parameter(flat_ivf, "max_codes", 400)
    try:
        assert flat_ivf.max_codes == 400
        D, I = flat_ivf.search(xq, 10)
    finally:
        flat_ivf.max_codes = 0
    D2, I2 = flat_ivf.search(xq, 10, params=amd.SearchParametersIVF(nprobe=8, max_codes=400))
    assert_same_results(D, I, D2, I2)


def test_parallel_mode(amd, orc, flat_ivf):
    xq = rand(orc, 100, D_, 67)
    flat_ivf.nprobe = 8
    D0, I0 = flat_ivf.search(xq, 10)
    flat_ivf.parallel_mode = 3  # query-parallel like 0 (IndexIVF.cpp:595)
    try:
        D3, I3 = flat_ivf.search(xq, 10)
        assert_same_results(D3, I3, D0, I0)
        # modes 1 / 2 (probe-parallel in the reference) give mode 0's
        # distances (tests/test_index_accuracy.py:47-60); the GPU computes
        # them as mode 0
        for pm in (1, 2):
            flat_ivf.parallel_mode = pm
            Dp, Ip = flat_ivf.search(xq, 10)
            assert_same_results(Dp, Ip, D0, I0)
        flat_ivf.parallel_mode = 1024  # PARALLEL_MODE_NO_HEAP_INIT: not offered
        with pytest.raises(amd.FaissError, match="parallel_mode"):
            flat_ivf.search(xq, 10)
    finally:
        flat_ivf.parallel_mode = 0
