"""GPU parity: IVF-PQ, HNSW (standalone and as IVF coarse quantizer), on-disk
format round trips, and IndexShardsIVF, all through the C-ABI."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu


def recall(I, Igt, k):
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(I, Igt)]))


@pytest.fixture(scope="module")
def pq_index(amd, orc, gpu):
    d, nb, nlist, M = 64, 30000, 64, 16
    xb = rand(orc, nb, d, 31)
    idx = amd.index_factory(d, f"IVF{nlist},PQ{M}x8")
    idx.train(xb)
    idx.add(xb)
    return idx, xb


def test_ivfpq_recall_parity_with_oracle(amd, orc, pq_index):
    idx, xb = pq_index
    xq = rand(orc, 500, 64, 32)
    idx.nprobe = 8
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    assert ref.use_precomputed_table == 1
    Dr, Ir, _, _ = ref.search(xq, 10, 8)
    _, Igt = orc.knn(xq, xb, 10, blas_form=False)
    r_gpu, r_ref = recall(I, Igt, 10), recall(Ir, Igt, 10)
    assert abs(r_gpu - r_ref) <= 0.01, (r_gpu, r_ref)
    same = (I == Ir)
    assert same.mean() > 0.97, same.mean()
    # fp32 distances of the same codes agree to 1e-4 relative
    np.testing.assert_allclose(D[same], Dr[same], rtol=1e-4, atol=1e-5)


def test_ivfpq_table0_equals_table1_ids(amd, orc, pq_index):
    # tests/test_index_accuracy.py:496-498: use_precomputed_table 0 vs 1 -> same I
    idx, xb = pq_index
    xq = rand(orc, 300, 64, 33)
    ref1 = orc.IVFOracle.from_index(idx)
    ref0 = orc.IVFOracle.from_index(idx)
    ref0.s.use_precomputed_table = 0
    _, I1, _, _ = ref1.search(xq, 10, 8)
    _, I0, _, _ = ref0.search(xq, 10, 8)
    assert (I1 == I0).mean() > 0.99
    idx.nprobe = 8
    _, Ig = idx.search(xq, 10)
    assert (Ig == I0).mean() > 0.97


@pytest.fixture(scope="module")
def hnsw_index(amd, orc, gpu):
    d, nb = 32, 6000
    xb = rand(orc, nb, d, 41)
    h = amd.IndexHNSWFlat(d, 16)
    h.add(xb)
    return h, xb


@pytest.mark.parametrize("ef", [16, 64, 128])
@pytest.mark.parametrize("k", [1, 10, 32])
def test_hnsw_search_bit_exact(amd, orc, hnsw_index, ef, k):
    h, xb = hnsw_index
    h.efSearch = ef
    xq = rand(orc, 300, 32, 42)
    D, I = h.search(xq, k)
    g = orc.HNSWGraph.from_index(h)
    Dr, Ir = g.search(xq, k, ef)
    assert_same_results(D, I, Dr, Ir)


def test_hnsw_graph_quality(amd, orc, hnsw_index):
    # tests/test_graph_based.py:17-75 style recall floor
    h, xb = hnsw_index
    h.efSearch = 64
    xq = rand(orc, 200, 32, 43)
    _, I = h.search(xq, 1)
    _, Igt = orc.knn(xq, xb, 1, blas_form=False)
    assert (I[:, 0] == Igt[:, 0]).mean() > 0.9


@pytest.mark.parametrize("ef", [16, 64])
def test_ivf_hnsw_quantizer_bit_exact(amd, orc, gpu, ef):
    d, nb, nlist = 32, 20000, 128
    xb = rand(orc, nb, d, 51)
    idx = amd.index_factory(d, f"IVF{nlist}_HNSW16,Flat")
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 16
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
    xq = rand(orc, 300, d, 52)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 16, efSearch=ef)
    assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("desc", ["IVF32,Flat", "IVF32,PQ8", "IVF32_HNSW8,Flat", "Flat"])
def test_write_read_roundtrip(amd, orc, gpu, tmp_path, desc):
    d, nb = 32, 4000
    xb = rand(orc, nb, d, 61)
    idx = amd.index_factory(d, desc)
    idx.train(xb)
    idx.add(xb)
    if hasattr(idx, "nprobe"):
        idx.nprobe = 4
    xq = rand(orc, 100, d, 62)
    D, I = idx.search(xq, 5)
    fn = tmp_path / "x.index"
    amd.write_index(idx, fn)
    idx2 = amd.read_index(fn)
    assert type(idx2).__name__ == type(idx).__name__
    assert idx2.ntotal == nb
    D2, I2 = idx2.search(xq, 5)
    assert_same_results(D2, I2, D, I)
    # writing the re-read index gives the same bytes
    fn2 = tmp_path / "y.index"
    amd.write_index(idx2, fn2)
    assert fn.read_bytes() == fn2.read_bytes()


def test_shards_ivf_equals_unsharded(amd, orc, gpu):
    # tests/test_meta_index.py:128-148 (test_shards_ivf): exact I, close D
    d, nb, nlist = 32, 9000, 40
    xb = rand(orc, nb, d, 71)
    q = amd.IndexFlatL2(d)
    ref = amd.IndexIVFFlat(q, d, nlist)
    ref.train(xb)
    ref.add(xb)
    ref.nprobe = 6
    sh = amd.IndexShardsIVF(q, nlist, False, True)
    parts = [amd.IndexIVFFlat(q, d, nlist) for _ in range(3)]
    for p in parts:
        sh.add_shard(p)
    sh.add(xb)
    sh.nprobe = 6
    xq = rand(orc, 200, d, 72)
    D1, I1 = ref.search(xq, 10)
    D2, I2 = sh.search(xq, 10)
    assert_same_results(D2, I2, D1, I1)


def test_merge_knn_results_device_and_host(amd, orc, gpu):
    rng = np.random.default_rng(3)
    ns, n, k = 5, 200, 10
    Dall = np.sort(rng.integers(0, 50, size=(ns, n, k)).astype(np.float32), axis=2)
    Iall = rng.integers(0, 10**6, size=(ns, n, k)).astype(np.int64)
    Iall[2, :, 6:] = -1
    Dr, Ir = orc.merge_knn_results(Dall, Iall)
    D, I = amd.merge_knn_results(Dall, Iall)
    assert np.array_equal(I, Ir) and np.array_equal(D, Dr)


@pytest.mark.parametrize("table", [1, 0])
@pytest.mark.parametrize("k,nprobe", [(1, 1), (10, 8), (5, 17), (32, 8)])
def test_ivfpq_mfma_bit_exact_vs_oracle(amd, orc, pq_index, monkeypatch, table, k, nprobe):
    # list-centric MFMA filter + re-rank in the reference's table arithmetic
    # (oracle_ivf_search_preassigned: IndexIVFPQ.cpp:560-700) -> the same ids
    # and the same fp32 distances as the restated reference, for both tables
    idx, _ = pq_index
    xq = rand(orc, 400, 64, 34)
    Dq, Iq = idx.quantizer.search(xq, nprobe)
    idx.nprobe = nprobe
    idx.use_precomputed_table = table
    try:
        D, I = idx.search_preassigned(xq, k, Iq, Dq)
        monkeypatch.setenv("FAISS_AMD_PQ_SCAN", "lut")
        Dl, Il = idx.search_preassigned(xq, k, Iq, Dq)
    finally:
        idx.use_precomputed_table = 1
    ref = orc.IVFOracle.from_index(idx)
    ref.s.use_precomputed_table = table
    Dr, Ir = ref.search_preassigned(xq, k, Iq, Dq)
    assert_same_results(D, I, Dr, Ir)
    # the query-centric LUT scan (its own summation order) agrees to 1e-4
    assert (Il == Ir).mean() > 0.97
    ok = Il == Ir
    np.testing.assert_allclose(Dl[ok], Dr[ok], rtol=1e-4, atol=1e-5)


def test_ivfpq_mfma_duplicate_codes_ties(amd, orc, gpu):
    # many identical codes: exact distance ties at the k boundary resolve by
    # the reference's arrival-order rule (the Flat tie machinery)
    d, nlist = 64, 16  # d in {64, 96, 128}: the MFMA path's geometries
    base = rand(orc, 2000, d, 35)
    xb = np.repeat(base[:400], 8, axis=0) + 0.0
    idx = amd.index_factory(d, f"IVF{nlist},PQ16")
    idx.train(base)
    idx.add(xb)
    xq = rand(orc, 200, d, 36)
    idx.nprobe = 4
    Dq, Iq = idx.quantizer.search(xq, 4)
    D, I = idx.search_preassigned(xq, 10, Iq, Dq)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir = ref.search_preassigned(xq, 10, Iq, Dq)
    assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("d", [37, 128])
def test_hnsw_register_kernel_forms_equal_reference(amd, orc, gpu, monkeypatch, d):
    """The register kernel's int8 prefilter (d = 37: padded image dims) and
    its replay continuation, each switched off in turn, on a graph with
    duplicated points (distance ties in the candidate set and the results;
    k < ef and k = ef): every form gives the reference's results."""
    nb = 5000
    xb = rand(orc, nb, d, 61)
    xb[1000:1150] = xb[:150]
    xb[3000:3040] = xb[:40]
    xq = np.concatenate([rand(orc, 300, d, 62), xb[:60]])
    cases = [(16, 10), (64, 64), (40, 5), (64, 1)]
    out = {}
    for q8, rp in (("1", "1"), ("0", "1"), ("1", "0")):
        monkeypatch.setenv("FAISS_AMD_HNSW_Q8", q8)
        monkeypatch.setenv("FAISS_AMD_HNSW_REPLAY", rp)
        h = amd.IndexHNSWFlat(d, 16)
        h.add(xb)
        for ef, k in cases:
            h.efSearch = ef
            out[(q8, rp, ef, k)] = h.search(xq, k)
    g = orc.HNSWGraph.from_index(h)
    for ef, k in cases:
        Dr, Ir = g.search(xq, k, ef)
        for q8, rp in (("1", "1"), ("0", "1"), ("1", "0")):
            D, I = out[(q8, rp, ef, k)]
            assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("d", [37, 128])
def test_hnsw_replay_log_overflow_and_lds_log(amd, orc, gpu, monkeypatch, d):
    """The register kernel's layout-dependent continuations on the
    duplicate-heavy graph: the replay log in HBM (default), in the LDS
    (FAISS_AMD_HNSW_LOG=lds) and both with a 16-entry capacity
    (FAISS_AMD_HNSW_REPLAY_CAP=16), so queries overflow it and search level 0
    again.  Every form gives the reference's results; the counters show each
    continuation was taken, and no replayed log entry ever named a non-node
    (replay_bad == 0: a corrupt log is counted, never silently skipped)."""
    nb = 5000
    xb = rand(orc, nb, d, 61)
    xb[1000:1150] = xb[:150]
    xb[3000:3040] = xb[:40]
    xq = np.concatenate([rand(orc, 300, d, 62), xb[:60]])
    cases = [(16, 10), (64, 64), (40, 5)]
    h = amd.IndexHNSWFlat(d, 16)
    h.add(xb)
    g = orc.HNSWGraph.from_index(h)
    forms = [(None, None), ("lds", None), (None, "16"), ("lds", "16")]
    seen = {}
    for log, cap in forms:
        for var, val in (("FAISS_AMD_HNSW_LOG", log), ("FAISS_AMD_HNSW_REPLAY_CAP", cap)):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        amd.cvar.hnsw_stats.reset()
        for ef, k in cases:
            h.efSearch = ef
            D, I = h.search(xq, k)
            Dr, Ir = g.search(xq, k, ef)
            assert_same_results(D, I, Dr, Ir)
        seen[(log, cap)] = amd.cvar.hnsw_replay_stats
    for form, (replayed, again, bad) in seen.items():
        assert bad == 0, (form, seen)
    # the default log replays every continuation; a 16-entry log overflows
    assert seen[(None, None)][0] > 0 and seen[(None, None)][1] == 0, seen
    assert seen[(None, "16")][1] > 0, seen
    assert seen[("lds", "16")][1] > 0, seen
    assert sum(seen[(None, None)][:2]) == sum(seen[(None, "16")][:2]), seen


@pytest.mark.parametrize("d", [37, 128])
def test_hnsw_sequential_kernel_wide_ef(amd, orc, gpu, d):
    """The sequential kernel (max(efSearch, k) > 64 or k > 64: faiss's heap
    layout in the LDS, or in global scratch past it) on the duplicate-heavy
    graph: heap pops / pushes / replace_top in the reference's layout, ties
    included, for efSearch 100 .. 9000 and k up to 100."""
    nb = 5000
    xb = rand(orc, nb, d, 61)
    xb[1000:1150] = xb[:150]
    xb[3000:3040] = xb[:40]
    xq = np.concatenate([rand(orc, 200, d, 63), xb[:40]])
    h = amd.IndexHNSWFlat(d, 16)
    h.add(xb)
    g = orc.HNSWGraph.from_index(h)
    for ef, k in [(100, 10), (257, 5), (768, 10), (500, 100), (2500, 1), (9000, 10)]:
        h.efSearch = ef
        D, I = h.search(xq, k)
        Dr, Ir = g.search(xq, k, ef)
        assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("nb,ef,k", [(300, 500, 10), (300, 1000, 300), (6000, 200, 200),
                                     (6000, 700, 50), (6000, 2000, 2000)])
@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("mode", ["wide", "wide_inplace", "sequential", "sequential_heap"])
def test_hnsw_wide_edges_bit_exact(amd, orc, gpu, monkeypatch, nb, ef, k, ties, mode):
    """The wide kernel (128 < max(efSearch, k) <= 4096) at its edges: efSearch
    beyond the graph (the candidate set never fills: nalive reaches 0, n2),
    k == ef (the result-heap eviction rule), and heavy exact-distance ties
    (coordinates on a 1/4 grid: many equal fp32 distances, so pop-tie windows,
    one-at-a-time pushes and re-runs all occur) — bit-exact against the
    oracle's HNSW::search, and the wide stage must be the one that ran.
    The same through the sequential kernel for every query
    (FAISS_AMD_HNSW_EXACT=1): with its results selected from the arrival log
    (the result heap rebuilt by a replay where the k-th distance is shared)
    and, FAISS_AMD_HNSW_NORB=0, with the result heap kept throughout; and
    with the flagged queries searched again inside the wide kernel
    (FAISS_AMD_HNSW_INPLACE=1)."""
    if mode.startswith("sequential"):
        monkeypatch.setenv("FAISS_AMD_HNSW_EXACT", "1")
    if mode == "wide_inplace":
        monkeypatch.setenv("FAISS_AMD_HNSW_INPLACE", "1")
    monkeypatch.setenv("FAISS_AMD_HNSW_NORB", "0" if mode == "sequential_heap" else "1")
    d = 32
    xb = rand(orc, nb, d, 71)
    xq = rand(orc, 200, d, 72)
    if ties:
        xb = np.round(xb * 4) / 4
        xq = np.round(xq * 4) / 4
    h = amd.IndexHNSWFlat(d, 16)
    h.add(np.ascontiguousarray(xb, dtype=np.float32))
    h.efSearch = ef
    amd.set_kernel_timing(True)
    try:
        h.reset_kernel_times()
        D, I = h.search(np.ascontiguousarray(xq, dtype=np.float32), k)
        names = {nm for nm, _, _ in h.kernel_times()}
    finally:
        amd.set_kernel_timing(False)
    assert ("hnsw_wide" in names) == mode.startswith("wide"), names
    g = orc.HNSWGraph.from_index(h)
    Dr, Ir = g.search(np.ascontiguousarray(xq, dtype=np.float32), k, ef)
    assert_same_results(D, I, Dr, Ir)
