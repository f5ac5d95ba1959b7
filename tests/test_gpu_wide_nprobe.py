"""nprobe past 64 through the list-centric MFMA filters and the wide
certified re-rank (k_ivf_rerank_wide: probes in chunks of 64 per wave), up to
nprobe 2048 — the reference harness's grid (tutorial/cpp/benchmark-hnsw-ivf/
benchmark.config: nprobe_ratio to 0.128 of nlist).  Ids and distances must
equal the oracle's bit for bit (IVF-Flat L2 and IP, IVF-PQ tables 1 and 0,
duplicated vectors for distance ties at the k boundary), and the filter path
must be the one that ran (its stages in kernel_times(), not the general exact
scan's)."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu


def ran_filter(amd, idx, fn):
    amd.set_kernel_timing(True)
    try:
        idx.reset_kernel_times()
        out = fn()
        names = {nm for nm, _, _ in idx.kernel_times()}
    finally:
        amd.set_kernel_timing(False)
    return out, names


@pytest.fixture(scope="module")
def flat_l2(amd, orc):
    d, nlist = 64, 2048
    base = rand(orc, 150_000, d, 71)
    xb = np.concatenate([base, base[:20_000]])  # duplicates: ties at the k boundary
    idx = amd.index_factory(d, f"IVF{nlist},Flat")
    idx.train(base[:100_000])
    idx.add(xb)
    return idx, base[:40]


@pytest.mark.parametrize("nprobe,k", [(65, 10), (200, 1), (512, 10), (1024, 20), (2048, 10)])
def test_flat_l2_wide_nprobe(amd, orc, gpu, flat_l2, nprobe, k):
    idx, dup = flat_l2
    xq = np.concatenate([rand(orc, 200, 64, 72), dup])
    idx.nprobe = nprobe
    (D, I), names = ran_filter(amd, idx, lambda: idx.search(xq, k))
    assert "ivf_flat_scan" in names and "ivf_rerank" in names, names
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, k, nprobe, nslices=1)
    assert_same_results(D, I, Dr, Ir)


def test_flat_ip_wide_nprobe(amd, orc, gpu):
    d, nlist = 48, 512
    xb = rand(orc, 60_000, d, 73)
    idx = amd.index_factory(d, f"IVF{nlist},Flat", amd.METRIC_INNER_PRODUCT)
    idx.train(xb[:30_000])
    idx.add(np.concatenate([xb, xb[:5000]]))
    xq = rand(orc, 150, d, 74)
    ref = orc.IVFOracle.from_index(idx)
    for nprobe in (100, 400):
        idx.nprobe = nprobe
        (D, I), names = ran_filter(amd, idx, lambda: idx.search(xq, 10))
        assert "ivf_rerank" in names, names
        Dr, Ir, _, _ = ref.search(xq, 10, nprobe, nslices=1)
        assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("table", [1, 0])
def test_pq_wide_nprobe(amd, orc, gpu, table):
    d, nlist = 64, 1024
    base = rand(orc, 80_000, d, 75)
    idx = amd.index_factory(d, f"IVF{nlist},PQ16")
    idx.train(base[:60_000])
    idx.add(np.concatenate([base, base[:8000]]))
    idx.use_precomputed_table = table
    xq = rand(orc, 150, d, 76)
    ref = orc.IVFOracle.from_index(idx)
    ref.s.use_precomputed_table = table
    try:
        for nprobe, k in ((96, 10), (700, 5)):
            idx.nprobe = nprobe
            Dq, Iq = idx.quantizer.search(xq, nprobe)
            (D, I), names = ran_filter(amd, idx,
                                       lambda: idx.search_preassigned(xq, k, Iq, Dq))
            assert "ivfpq_filter" in names and "ivfpq_rerank" in names, names
            Dr, Ir = ref.search_preassigned(xq, k, Iq, Dq)
            assert_same_results(D, I, Dr, Ir)
    finally:
        idx.use_precomputed_table = 1
