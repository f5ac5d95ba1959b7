"""Pin the CPU oracle (and the product's host-side pieces) to the reference.

tests/golden/ref_fixtures.npz holds outputs of the reference's own code,
compiled from /root/reference by oracle/ref/Makefile and driven by
oracle/ref/make_golden.py (see that script for what each array is).  These
tests run on the CPU and check bit-for-bit equality with the fixtures; when
the compiled reference is present (the build container), a few cases are
also re-run live against it.
"""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "ref_fixtures.npz")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libfaissref.so")


@pytest.fixture(scope="module")
def fx():
    return np.load(FIX, allow_pickle=False)


def test_float_rand_matches_reference(orc, amd, fx):
    # faiss/utils/random.cpp:95-112
    for key in fx.files:
        if key.startswith("float_rand_") and key.count("_") == 3 and "1M" not in key:
            _, _, n, seed = key.split("_")
            ref = fx[key]
            assert np.array_equal(orc.float_rand(int(n), int(seed)), ref), key
            assert np.array_equal(amd.float_rand(int(n), int(seed)), ref), key
    big = orc.float_rand(1 << 20, 1234)
    assert big.astype(np.float64).sum() == fx["float_rand_1M_1234_sum"][0]
    assert np.array_equal(np.concatenate([big[:16], big[-16:]]),
                          fx["float_rand_1M_1234_head_tail"])


def test_float_rand_rows_is_strided_slice(orc, amd):
    # bench.py draws a shard's rows (rank, rank + nshards, ...) of the global
    # float_rand matrix without materialising it; both block-size regimes
    for n_rows, d in ((300, 3), (20000, 96)):
        full = orc.float_rand(n_rows * d, 77).reshape(n_rows, d)
        for row0, step in ((0, 1), (3, 8), (n_rows - 1, 5)):
            nout = (n_rows - 1 - row0) // step + 1
            got = amd.float_rand_rows(n_rows, d, 77, row0=row0, step=step, nout=nout)
            assert np.array_equal(got, full[row0::step]), (n_rows, row0, step)


def test_fvec_evaluation_order_matches_reference(orc, fx):
    # faiss/utils/distances_simd.cpp:220-300 as compiled with the reference's
    # AVX2 flags; the oracle restates that order (oracle.c ref_dist_)
    L = orc.lib()
    for d in fx["fvec_dims"]:
        q, Y = fx[f"fvec_q_{d}"], fx[f"fvec_Y_{d}"]
        l2 = np.array([orc.fvec_L2sqr(q, y) for y in Y], np.float32)
        ip = np.array([orc.fvec_inner_product(q, y) for y in Y], np.float32)
        nr = np.array([L.oracle_fvec_norm_L2sqr(y.ctypes.data_as(C.c_void_p), int(d))
                       for y in Y], np.float32)
        assert np.array_equal(l2, fx[f"fvec_l2_{d}"]), f"fvec_L2sqr d={d}"
        assert np.array_equal(ip, fx[f"fvec_ip_{d}"]), f"fvec_inner_product d={d}"
        assert np.array_equal(nr, fx[f"fvec_norm_{d}"]), f"fvec_norm_L2sqr d={d}"
        # fvec_L2sqr_batch_4 (the HNSW distance computer) has the same order
        assert np.array_equal(fx[f"fvec_b4_{d}"], fx[f"fvec_l2_{d}"]), f"batch_4 d={d}"


def test_heap_streams_match_reference(orc, fx):
    # heap_heapify / strict admission / heap_replace_top / heap_reorder
    for case in range(6):
        vals, ids = fx[f"heap_{case}_vals"], fx[f"heap_{case}_ids"]
        for l2 in (1, 0):
            for k in (1, 5, 10, 33):
                D, I = orc.heap_addn_reorder(k, vals, ids, cmax=bool(l2))
                assert np.array_equal(D, fx[f"heap_{case}_{l2}_{k}_D"]), (case, l2, k)
                assert np.array_equal(I, fx[f"heap_{case}_{l2}_{k}_I"]), (case, l2, k)


def test_direct_knn_matches_reference(orc, fx):
    for l2 in (1, 0):
        D, I = orc.knn(fx["knn_x"], fx["knn_y"], 10, metric=l2, blas_form=False)
        assert np.array_equal(D, fx[f"knn_{l2}_D"]) and np.array_equal(I, fx[f"knn_{l2}_I"])


def ivf_fixture_oracle(orc, fx, l2):
    xs, ids = fx[f"ivf_{l2}_xb"], fx[f"ivf_{l2}_ids"]
    list_len = fx[f"ivf_{l2}_list_len"]
    off = np.concatenate([[0], np.cumsum(list_len)]).astype(np.int64)
    codes = np.ascontiguousarray(xs).view(np.uint8).reshape(xs.shape[0], -1)
    return orc.IVFOracle(xs.shape[1], len(list_len), l2, off, codes, ids, fx[f"ivf_{l2}_cent"])


@pytest.mark.parametrize("l2", [1, 0])
def test_ivf_flat_scan_matches_reference(orc, fx, l2):
    # faiss/IndexIVFFlat.cpp:155-179 driven by faiss/IndexIVF.cpp:595-631 on
    # lists with duplicated vectors (ties at the k boundary)
    ref = ivf_fixture_oracle(orc, fx, l2)
    xq, Iq, Dq = fx[f"ivf_{l2}_xq"], fx[f"ivf_{l2}_Iq"], fx[f"ivf_{l2}_Dq"]
    for k in (1, 10, 25):
        D, I = ref.search_preassigned(xq, k, Iq, Dq)
        assert np.array_equal(I, fx[f"ivf_{l2}_{k}_I"]), k
        assert np.array_equal(D, fx[f"ivf_{l2}_{k}_D"]), k
        # full search with slices below the BLAS threshold = direct coarse path
        D2, I2, _, CI = ref.search(xq, k, Iq.shape[1], nslices=xq.shape[0])
        assert np.array_equal(CI, Iq)
        assert np.array_equal(I2, fx[f"ivf_{l2}_{k}_I"]) and np.array_equal(D2, D)


def test_merge_knn_results_matches_reference(orc, amd, fx):
    # faiss/utils/Heap.cpp:159-230 (ties -> lower shard, -1 slots skipped)
    for l2 in (1, 0):
        Din, Iin = fx[f"merge_{l2}_in_D"], fx["merge_in_I"]
        D, I = orc.merge_knn_results(Din, Iin, metric=l2)
        assert np.array_equal(D, fx[f"merge_{l2}_D"]) and np.array_equal(I, fx[f"merge_{l2}_I"])
        D2, I2 = amd.merge_knn_results(Din, Iin, keep_max=not l2)
        assert np.array_equal(D2, fx[f"merge_{l2}_D"]) and np.array_equal(I2, fx[f"merge_{l2}_I"])


def hnsw_fixture_graph(orc, fx):
    nb, d, M, ep, ml, efc = (int(v) for v in fx["hnsw_meta"])
    return orc.HNSWGraph(ep, ml, fx["hnsw_levels"], fx["hnsw_offsets"], fx["hnsw_neighbors"],
                         fx["hnsw_cum"], fx["hnsw_xb"])


def test_hnsw_search_matches_reference(orc, fx):
    # faiss/impl/HNSW.cpp:943-996 on a graph the reference built
    g = hnsw_fixture_graph(orc, fx)
    for ef in (16, 48):
        for k in (1, 10):
            D, I = g.search(fx["hnsw_xq"], k, ef)
            assert np.array_equal(I, fx[f"hnsw_{ef}_{k}_I"]), (ef, k)
            assert np.array_equal(D, fx[f"hnsw_{ef}_{k}_D"]), (ef, k)


def test_hnsw_build_matches_reference(amd, fx):
    # product host build (hnsw.cpp) vs faiss HNSW::prepare_level_tab +
    # add_with_locks in hnsw_add_vertices order, run serially
    nb, d, M, ep, ml, efc = (int(v) for v in fx["hnsw_meta"])
    idx = amd.IndexHNSWFlat(d, M)
    idx.efConstruction = efc
    idx.add(fx["hnsw_xb"])
    gep, gml, levels, offsets, neighbors, cum = idx.graph()
    assert (gep, gml) == (ep, ml)
    assert np.array_equal(levels, fx["hnsw_levels"])
    assert np.array_equal(np.asarray(offsets, np.uint64), fx["hnsw_offsets"])
    assert np.array_equal(cum, fx["hnsw_cum"])
    assert np.array_equal(neighbors, fx["hnsw_neighbors"])


def write_ihnf(path, fx):
    """An IHNf file (faiss/impl/index_write.cpp:300-316,760-778) of the fixture graph."""
    nb, d, M, ep, ml, efc = (int(v) for v in fx["hnsw_meta"])

    def header(f):
        f.write(struct.pack("<iqqqBi", d, nb, 1 << 20, 1 << 20, 1, 1))

    def vec(f, a, fmt):
        a = np.ascontiguousarray(a)
        f.write(struct.pack("<Q", a.size))
        f.write(a.astype(fmt).tobytes())

    with open(path, "wb") as f:
        f.write(b"IHNf")
        header(f)
        vec(f, fx["hnsw_probas"], "<f8")
        vec(f, fx["hnsw_cum"], "<i4")
        vec(f, fx["hnsw_levels"], "<i4")
        vec(f, fx["hnsw_offsets"], "<u8")
        vec(f, fx["hnsw_neighbors"], "<i4")
        f.write(struct.pack("<iiiii", ep, ml, efc, 16, 1))
        f.write(b"IxF2")
        header(f)
        xb = np.ascontiguousarray(fx["hnsw_xb"], "<f4")
        f.write(struct.pack("<Q", xb.size))
        f.write(xb.tobytes())


def test_ihnf_file_roundtrip_host(amd, fx, tmp_path):
    # reader accepts a reference-layout file; the graph comes back unchanged
    p = tmp_path / "g.ihnf"
    write_ihnf(p, fx)
    idx = amd.read_index(str(p))
    gep, gml, levels, offsets, neighbors, cum = idx.graph()
    assert np.array_equal(neighbors, fx["hnsw_neighbors"]) and np.array_equal(levels,
                                                                             fx["hnsw_levels"])
    q = tmp_path / "g2.ihnf"
    amd.write_index(idx, str(q))
    assert p.read_bytes() == q.read_bytes()


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="compiled reference only in the build "
                                                       "container (oracle/ref/Makefile)")
def test_live_reference_fvec_random_dims(orc):
    L = C.CDLL(REF_SO)
    L.ref_fvec_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int,
                                 C.c_void_p]
    rng = np.random.default_rng(7)
    for d in rng.integers(1, 300, 25):
        q = rng.standard_normal(int(d)).astype(np.float32)
        Y = rng.standard_normal((16, int(d))).astype(np.float32)
        for l2 in (1, 0):
            out = np.empty(16, np.float32)
            L.ref_fvec_batch(q.ctypes.data_as(C.c_void_p), Y.ctypes.data_as(C.c_void_p), int(d),
                             16, l2, out.ctypes.data_as(C.c_void_p))
            f = orc.fvec_L2sqr if l2 else orc.fvec_inner_product
            mine = np.array([f(q, y) for y in Y], np.float32)
            assert np.array_equal(mine, out), (int(d), l2)
