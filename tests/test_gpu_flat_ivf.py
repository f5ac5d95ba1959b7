"""GPU parity: IndexFlat and IndexIVFFlat (through the C-ABI) vs the oracle.

The GPU path and the oracle evaluate every fp32 distance in the same order
(sequential fma chains; coarse = fma(-2, ip, |x|^2+|y|^2) clamped), so ids AND
distances must match bit for bit on the same index.
"""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("k", [1, 10, 64])
def test_flat_search_bit_exact(amd, orc, gpu, metric, k):
    d, nb, nq = 48, 3000, 300
    xb = rand(orc, nb, d, 11)
    xq = rand(orc, nq, d, 12)
    idx = amd.IndexFlat(d, metric)
    idx.add(xb)
    D, I = idx.search(xq, k)
    Dr, Ir = orc.knn(xq, xb, k, metric=metric, blas_form=True)
    assert_same_results(D, I, Dr, Ir)


def test_flat_fewer_vectors_than_k(amd, orc, gpu):
    d = 8
    xb = rand(orc, 5, d, 1)
    idx = amd.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(rand(orc, 3, d, 2), 10)
    assert (I[:, 5:] == -1).all() and (D[:, 5:] == np.finfo(np.float32).max).all()
    empty = amd.IndexFlatL2(d)
    D, I = empty.search(rand(orc, 3, d, 2), 4)
    assert (I == -1).all()


def build_ivf(amd, orc, d, nb, nlist, desc="Flat", seed=1234):
    xb = rand(orc, nb, d, seed)
    idx = amd.index_factory(d, f"IVF{nlist},{desc}")
    idx.train(xb)
    idx.add(xb)
    return idx, xb


@pytest.fixture(scope="module")
def cfg1(amd, orc, gpu):
    # BASELINE.json configs[0]: IVF256,Flat d=64, 100k vectors, nq=1k, nprobe=8
    idx, xb = build_ivf(amd, orc, 64, 100_000, 256)
    xq = rand(orc, 1000, 64, 5678)
    return idx, xb, xq


def test_cfg1_ivfflat_bit_exact(amd, orc, cfg1):
    idx, xb, xq = cfg1
    idx.nprobe = 8
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 8, nslices=1)
    assert_same_results(D, I, Dr, Ir)
    # recall sanity against exact search
    _, Igt = orc.knn(xq, xb, 10, blas_form=False)
    rec = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(I, Igt)])
    assert rec > 0.2


def test_cfg1_lowlevel_decomposition(amd, orc, cfg1):
    # tests/test_lowlevel_ivf.cpp:150-213: quantizer->search + search_preassigned == search
    idx, xb, xq = cfg1
    idx.nprobe = 8
    Dq, Iq = idx.quantizer.search(xq, 8)
    D1, I1 = idx.search_preassigned(xq, 10, Iq, Dq)
    D2, I2 = idx.search(xq, 10)
    assert_same_results(D1, I1, D2, I2)
    # and the coarse step equals the oracle's flat knn
    Dqr, Iqr = orc.knn(xq, idx.quantizer.xb, 8, blas_form=True)
    assert_same_results(Dq, Iq, Dqr, Iqr)


@pytest.mark.parametrize("nprobe", [1, 3, 17, 64, 100, 256])
@pytest.mark.parametrize("k", [1, 5, 37, 64, 100, 1024])
def test_ivfflat_nprobe_k_grid(amd, orc, cfg1, nprobe, k):
    idx, xb, xq = cfg1
    idx.nprobe = nprobe
    D, I = idx.search(xq[:200], k)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq[:200], k, nprobe, nslices=1)
    assert_same_results(D, I, Dr, Ir)


def test_ivfflat_exhaustive_equals_exact(amd, orc, cfg1):
    """nprobe = nlist visits every list: the result is the exact k-NN of the
    whole base, as a flat index (direct form of fvec_L2sqr) computes it"""
    idx, xb, xq = cfg1
    idx.nprobe = idx.nlist
    q = xq[:50]
    D, I = idx.search(q, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(q, 10, idx.nlist, nslices=1)
    assert_same_results(D, I, Dr, Ir)
    De, Ie = orc.knn(q, xb, 10, metric=1, blas_form=False)
    assert_same_results(D, I, De, Ie)


def test_ivfflat_edge_cases(amd, orc, gpu):
    # ragged / tiny / empty lists, d not a multiple of 4, nq = 1, ids given
    d, nb, nlist = 30, 700, 40
    xb = rand(orc, nb, d, 7)
    q = amd.IndexFlatL2(d)
    idx = amd.IndexIVFFlat(q, d, nlist)
    idx.train(xb)
    ids = (np.arange(nb, dtype=np.int64) * 7919) % 100003
    idx.add_with_ids(xb[:300], ids[:300])
    idx.nprobe = 6
    ref = orc.IVFOracle.from_index(idx)
    for nq in (1, 7, 129):
        xq = rand(orc, nq, d, 100 + nq)
        D, I = idx.search(xq, 12)
        Dr, Ir, _, _ = ref.search(xq, 12, 6, nslices=1)
        assert_same_results(D, I, Dr, Ir)
    # empty index: all padding
    idx.reset()
    D, I = idx.search(rand(orc, 4, d, 3), 5)
    assert (I == -1).all()


def test_ivfflat_inner_product(amd, orc, gpu):
    d, nb, nlist = 32, 5000, 32
    xb = rand(orc, nb, d, 21)
    q = amd.IndexFlatIP(d)
    idx = amd.IndexIVFFlat(q, d, nlist, amd.METRIC_INNER_PRODUCT)
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 4
    xq = rand(orc, 100, d, 22)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 4, nslices=1)
    assert_same_results(D, I, Dr, Ir)


def test_search_params_override(amd, orc, cfg1):
    # tests/test_params_override.cpp: per-call nprobe overrides index.nprobe
    idx, xb, xq = cfg1
    idx.nprobe = 1
    p = amd.SearchParametersIVF(nprobe=8)
    D1, I1 = idx.search(xq[:100], 10, params=p)
    idx.nprobe = 8
    D2, I2 = idx.search(xq[:100], 10)
    assert_same_results(D1, I1, D2, I2)


def test_device_entry_points_match_host(amd, orc, cfg1):
    import ctypes
    idx, xb, xq = cfg1
    idx.nprobe = 8
    D, I = idx.search(xq, 10)
    # device buffers through hipMalloc of the HIP runtime in the library's process
    hip = ctypes.CDLL("libamdhip64.so")
    def dmalloc(nbytes):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
        return p
    n = xq.shape[0]
    px, pd, pi = dmalloc(xq.nbytes), dmalloc(n * 10 * 4), dmalloc(n * 10 * 8)
    hip.hipMemcpy(px, xq.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(xq.nbytes), 1)
    idx.search_device(n, px.value, 10, pd.value, pi.value)
    hip.hipDeviceSynchronize()
    D2 = np.empty((n, 10), np.float32)
    I2 = np.empty((n, 10), np.int64)
    hip.hipMemcpy(D2.ctypes.data_as(ctypes.c_void_p), pd, ctypes.c_size_t(D2.nbytes), 2)
    hip.hipMemcpy(I2.ctypes.data_as(ctypes.c_void_p), pi, ctypes.c_size_t(I2.nbytes), 2)
    for p in (px, pd, pi):
        hip.hipFree(p)
    assert_same_results(D2, I2, D, I)


# --- the two IVF-Flat scan algorithms (direct exact VALU scan, fp32-MFMA
# filter + exact re-rank + flagged fallback) must give identical results.
@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 10, 16, 24])
@pytest.mark.parametrize("nprobe", [8, 32])
def test_scan_modes_identical(amd, orc, cfg1, monkeypatch, k, nprobe):
    idx, xb, xq = cfg1
    idx.nprobe = nprobe
    q = xq[:300]
    monkeypatch.setenv("FAISS_AMD_IVF_SCAN", "mfma")
    Dm, Im = idx.search(q, k)
    monkeypatch.setenv("FAISS_AMD_IVF_SCAN", "exact")
    De, Ie = idx.search(q, k)
    assert_same_results(Dm, Im, De, Ie)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(q, k, nprobe, nslices=1)
    assert_same_results(Dm, Im, Dr, Ir)


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["l2", "ip"])
@pytest.mark.parametrize("mode", ["mfma", "exact"])
def test_scan_duplicates_reference_tie_rule(amd, orc, gpu, monkeypatch, metric, mode):
    # 25 copies of every vector: long runs of equal distances cross the k
    # boundary.  The reference heap (strict admission, eviction by (dis, id))
    # keeps an arrival-order-dependent subset of the tied candidates (for IP
    # not the lexicographic one); both scan paths must reproduce it.
    d, nu, copies, nlist = 64, 160, 25, 8
    base = rand(orc, nu, d, 31)
    perm = np.random.default_rng(0).permutation(nu * copies)
    xb = np.ascontiguousarray(np.repeat(base, copies, axis=0)[perm])
    if metric == "l2":
        quant, mt = amd.IndexFlatL2(d), amd.METRIC_L2
    else:
        quant, mt = amd.IndexFlatIP(d), amd.METRIC_INNER_PRODUCT
    idx = amd.IndexIVFFlat(quant, d, nlist, mt)
    idx.train(xb)
    idx.add(xb)
    idx.nprobe = 3
    xq = np.ascontiguousarray(np.concatenate([base[:40], rand(orc, 40, d, 32)]))
    ref = orc.IVFOracle.from_index(idx)
    monkeypatch.setenv("FAISS_AMD_IVF_SCAN", mode)
    for k in (5, 10, 20, 40):
        D, I = idx.search(xq, k)
        Dr, Ir, _, _ = ref.search(xq, k, 3, nslices=1)
        assert_same_results(D, I, Dr, Ir)


@pytest.mark.gpu
def test_mfma_scan_d128_bench_shape(amd, orc, gpu):
    # the bench's shape (d=128, k=10, nprobe=32) at a size the oracle finishes fast
    idx, xb = build_ivf(amd, orc, 128, 200_000, 1024)
    idx.nprobe = 32
    xq = rand(orc, 2000, 128, 5678)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 32, nslices=1)
    assert_same_results(D, I, Dr, Ir)


@pytest.mark.gpu
@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("ny,k", [(256, 8), (1024, 32), (4096, 32), (4096, 64), (5000, 1)])
def test_coarse_bf3_equals_f32_tile_and_oracle(amd, orc, gpu, monkeypatch, metric, ny, k):
    # bf16x3 filter + exact re-rank vs the f32 MFMA tile + select; duplicated
    # rows make exact distance ties at the k boundary
    d = 64
    y = rand(orc, ny, d, 41)
    y[ny // 2: ny // 2 + 40] = y[:40]
    x = np.ascontiguousarray(np.concatenate([rand(orc, 180, d, 42), y[:20]]))
    idx = amd.IndexFlat(d, metric)
    idx.add(y)
    monkeypatch.setenv("FAISS_AMD_COARSE", "f32")
    Df, If = idx.search(x, k)
    monkeypatch.setenv("FAISS_AMD_COARSE", "bf3")
    Db, Ib = idx.search(x, k)
    assert_same_results(Db, Ib, Df, If)
    Dr, Ir = orc.knn(x, y, k, metric=metric, blas_form=True)
    assert_same_results(Db, Ib, Dr, Ir)


@pytest.mark.gpu
@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("k,nsplit", [(64, 16), (40, 16), (64, 0), (10, 0)])
def test_coarse_bf3_failing_streams(amd, orc, gpu, monkeypatch, metric, k, nsplit):
    # 16 splits x 4 thread streams (c5's coarse plan at k = 64: KT = 8).  A
    # tight cluster inside the first split puts far more than KT of a nearby
    # query's top-k in single streams (those streams fail and are re-scanned
    # exactly); duplicated rows give ties at the k boundary.
    d, ny = 64, 65536
    y = rand(orc, ny, d, 43)
    rng = np.random.default_rng(7)
    y[:300] = y[0] + 1e-3 * rng.standard_normal((300, d)).astype(np.float32)
    y[ny // 2: ny // 2 + 40] = y[1000:1040]
    x = np.ascontiguousarray(np.concatenate([rand(orc, 150, d, 44), y[:10] + 1e-3, y[1000:1010]]))
    idx = amd.IndexFlat(d, metric)
    idx.add(y)
    if nsplit:
        monkeypatch.setenv("FAISS_AMD_COARSE_NSPLIT", str(nsplit))
    monkeypatch.setenv("FAISS_AMD_COARSE", "bf3")
    Db, Ib = idx.search(x, k)
    Dr, Ir = orc.knn(x, y, k, metric=metric, blas_form=True)
    assert_same_results(Db, Ib, Dr, Ir)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 10, 32])
def test_filter_precisions_identical(amd, orc, cfg1, monkeypatch, k):
    # bf16x2 / bf16x3 filters and the direct exact scan return the same result
    idx, xb, xq = cfg1
    idx.nprobe = 16
    q = xq[:256]
    out = {}
    for mode, prec in (("mfma", "bf16x2"), ("mfma", "bf16x3"), ("exact", "bf16x2")):
        monkeypatch.setenv("FAISS_AMD_IVF_SCAN", mode)
        monkeypatch.setenv("FAISS_AMD_IVF_PREC", prec)
        out[(mode, prec)] = idx.search(q, k)
    ref = out[("exact", "bf16x2")]
    for key, (D, I) in out.items():
        assert_same_results(D, I, *ref)


@pytest.mark.gpu
def test_ivf_many_lists_bucketing(amd, orc, gpu):
    # nlist > 16384: the bucket count runs one LDS histogram per list range
    # (c5's IVF65536 geometry), the scan walks the counts in 4096-list chunks
    d, nlist = 16, 20000
    xb = rand(orc, 2 * nlist, d, 71)
    idx = amd.index_factory(d, f"IVF{nlist},Flat")
    idx.train(xb)
    idx.add(xb)
    xq = rand(orc, 3000, d, 72)
    idx.nprobe = 16
    Dq, Iq = idx.quantizer.search(xq, 16)
    D, I = idx.search_preassigned(xq, 10, Iq, Dq)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir = ref.search_preassigned(xq, 10, Iq, Dq)
    assert_same_results(D, I, Dr, Ir)


@pytest.mark.gpu
@pytest.mark.parametrize("desc", ["Flat", "PQ4"])
@pytest.mark.parametrize("k", [10, 100])
def test_preassigned_duplicate_probes(amd, orc, gpu, desc, k):
    """A caller-supplied assignment may name a list more than once; the
    reference then scans it once per probe (faiss/IndexIVF.cpp:595-631) and
    its heap holds such vectors more than once.  One list holds most of the
    base, so a query whose probes all name it has more candidates than the
    arena has rows (the exact path's per-query slot must still hold them)."""
    d, nlist, nq, np_ = 16, 8, 40, 8
    xt = rand(orc, 2000, d, 81)
    idx = amd.index_factory(d, f"IVF{nlist},{desc}")
    idx.train(xt)
    crowd = xt[:1] + 0.01 * rand(orc, 2500, d, 83)   # ~2500 rows in one list
    xb = np.ascontiguousarray(np.concatenate([xt[:700], crowd]), np.float32)
    idx.add(xb)
    idx.nprobe = np_  # search_preassigned reads nprobe (<= nlist) columns
    xq = rand(orc, nq, d, 82)
    Dq, Iq = idx.quantizer.search(xq, nlist)
    big = int(np.argmax([idx.get_list_size(l) for l in range(nlist)]))
    assert idx.get_list_size(big) * np_ > idx.ntotal
    keys = np.full((nq, np_), big, dtype=np.int64)     # the crowded list, 8 times
    keys[nq // 2:, 1::2] = Iq[nq // 2:, :1]             # half the queries: two lists
    by_list = np.empty_like(Dq)
    np.put_along_axis(by_list, Iq, Dq, axis=1)        # coarse distance of every list
    cdis = np.ascontiguousarray(np.take_along_axis(by_list, keys, axis=1), np.float32)
    D, I = idx.search_preassigned(xq, k, keys, cdis)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir = ref.search_preassigned(xq, k, keys, cdis)
    assert_same_results(D, I, Dr, Ir)


@pytest.mark.parametrize("nq,t", [(40, 3), (40, 2), (59, 3), (12, 4)])
def test_search_slices_emulate_reference_threads(amd, orc, gpu, nq, t):
    """set_search_slices(t) = a reference run on t OpenMP threads: slices of
    fewer than 20 queries take the direct coarse form (faiss/IndexIVF.cpp:
    359-368, faiss/utils/distances.cpp:807-823); the oracle slices the same."""
    d = 32
    xb = amd.float_rand(50_000 * d, 1234).reshape(-1, d)
    idx = amd.index_factory(d, "IVF256,Flat")
    idx.train(xb[:20_000])
    idx.add(xb)
    idx.nprobe = 8
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 8, nslices=min(t, nq))
    amd.set_search_slices(t)
    try:
        D, I = idx.search(xq, 10)
    finally:
        amd.set_search_slices(1)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
