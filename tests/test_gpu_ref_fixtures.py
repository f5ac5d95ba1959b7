"""HIP path vs reference-run fixtures (tests/golden/ref_full*, produced by the
reference library compiled from source; see tests/test_ref_fixtures.py).

Every comparison is bit-exact: ids and distances equal the reference's own
search over the reference-written index files.  Covers IVF-Flat L2/IP and
IVF-PQ (M = 4, 8, 12, 16, 24, 32, 48; dsub 2, 4, 8, 16; tables 0 and 1; IP)
search_preassigned with k up to 300 and nprobe up to nlist, end-to-end
search, store_pairs, parallel_mode 1/2, max_codes + IDSelector, range search,
the add path (coarse assignment + PQ codes), HNSW-IVF for efSearch 16..200 /
nprobe 8..100, and a standalone HNSW over duplicated vectors.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GDIR = os.path.join(HERE, "golden", "ref_full")
FX = np.load(os.path.join(HERE, "golden", "ref_full.npz"))
PQ_TAGS = ["pq_m32d128", "pq_m48d96", "pq_m16d64", "pq_m24d96", "pq_m8d64", "pq_m4d64",
           "pq_m12d48", "pq_ip_m16d64"]


def path(tag):
    return os.path.join(GDIR, tag + ".faiss")


def eq(D, I, key):
    np.testing.assert_array_equal(I, FX[key + "_I"], err_msg=key)
    np.testing.assert_array_equal(D, FX[key + "_D"], err_msg=key)


def pre_cases(tag):
    for key in FX.files:
        if not (key.startswith(tag + "_") and "_pre_" in key and key.endswith("_D")):
            continue
        parts = key[len(tag) + 1:-2].split("_")
        if parts[0].startswith("t"):
            yield key[:-2], int(parts[0][1:]), int(parts[2]), int(parts[3])
        else:
            yield key[:-2], None, int(parts[1]), int(parts[2])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"] + PQ_TAGS)
def test_gpu_preassigned_equals_reference(amd, gpu, tag):
    idx = amd.read_index(path(tag))
    xq = FX[tag + "_xq"]
    for key, table, nprobe, k in pre_cases(tag):
        if table is not None and FX[tag + "_info"][2] == 1:
            idx.use_precomputed_table = table
        # the probe count of search_preassigned is the index's nprobe
        # (faiss/IndexIVF.cpp:417-420), as in the reference run
        idx.nprobe = nprobe
        D, I = idx.search_preassigned(xq, k, FX[f"{tag}_q{nprobe}_I"], FX[f"{tag}_q{nprobe}_D"])
        eq(D, I, key)


@pytest.mark.parametrize("tag", ["pq_m32d128", "pq_m48d96", "pq_m16d64"])
@pytest.mark.parametrize("cdis", ["null", "garbage"])
def test_gpu_preassigned_table0_ignores_centroid_dis(amd, gpu, tag, cdis):
    """Precomputed table 0 never reads coarse_dis (faiss/IndexIVFPQ.cpp:634-700):
    NULL or unrelated centroid_dis must give the reference's table-0 result
    (the list filter keys on |x - y_C|^2 and computes it itself)."""
    idx = amd.read_index(path(tag))
    xq = FX[tag + "_xq"]
    ran = 0
    for key, table, nprobe, k in pre_cases(tag):
        if table != 0:
            continue
        idx.use_precomputed_table = 0
        idx.nprobe = nprobe
        cd = FX[f"{tag}_q{nprobe}_D"]
        cd = None if cdis == "null" else (np.random.default_rng(7).random(cd.shape) * 50.0 - 20.0)
        D, I = idx.search_preassigned(xq, k, FX[f"{tag}_q{nprobe}_I"], cd)
        eq(D, I, key)
        ran += 1
    assert ran > 0


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip", "pq_m32d128", "pq_m48d96", "pq_m16d64",
                                 "pq_ip_m16d64"])
def test_gpu_search_equals_reference(amd, gpu, tag):
    idx = amd.read_index(path(tag))
    xq = FX[tag + "_xq"]
    for key in [k for k in FX.files if k.startswith(tag + "_full_") and k.endswith("_D")]:
        nprobe, k = map(int, key[len(tag) + 6:-2].split("_"))
        idx.nprobe = nprobe
        D, I = idx.search(xq, k)
        eq(D, I, key[:-2])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"])
def test_gpu_store_pairs_equals_reference(amd, gpu, tag):
    idx = amd.read_index(path(tag))
    idx.nprobe = 4
    D, I = idx.search_preassigned(FX[tag + "_xq"], 10, FX[f"{tag}_q4_I"], FX[f"{tag}_q4_D"],
                                  store_pairs=True)
    eq(D, I, tag + "_sp")


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"])
@pytest.mark.parametrize("pm", [1, 2])
def test_gpu_parallel_mode_equals_reference(amd, gpu, tag, pm):
    """parallel_mode 1/2 (probe-parallel heaps + merge in the reference):
    the reference's own test asserts D equal to mode 0 (test_index_accuracy.py:47-60)"""
    idx = amd.read_index(path(tag))
    idx.nprobe = 8
    idx.parallel_mode = pm
    D, I = idx.search(FX[tag + "_xq"], 10)
    eq(D, I, f"{tag}_pm{pm}")


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"])
def test_gpu_params_max_codes_selector_equals_reference(amd, gpu, tag):
    idx = amd.read_index(path(tag))
    sel = amd.IDSelectorBatch(FX[tag + "_params_sel"])
    sp = amd.SearchParametersIVF(nprobe=8, max_codes=300, sel=sel)
    D, I = idx.search(FX[tag + "_xq"], 10, params=sp)
    eq(D, I, tag + "_params")


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"] + PQ_TAGS)
def test_gpu_range_equals_reference(amd, gpu, tag):
    idx = amd.read_index(path(tag))
    idx.nprobe = 8 if tag.startswith("flat") else 5
    lims, D, I = idx.range_search(FX[tag + "_xq"], float(FX[tag + "_range_radius"][0]))
    np.testing.assert_array_equal(lims, FX[tag + "_range_lims"])
    np.testing.assert_array_equal(I, FX[tag + "_range_I"])
    np.testing.assert_array_equal(D, FX[tag + "_range_D"])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"] + PQ_TAGS)
def test_gpu_add_path_equals_reference(amd, gpu, tag):
    """IndexIVF::add_with_ids on the GPU: coarse assignment (quantizer->assign)
    and, for PQ, the codes of IndexIVFPQ::encode_vectors, as the reference
    computed them for the same vectors."""
    idx = amd.read_index(path(tag))
    xa = FX[tag + "_xa"]
    n0 = idx.ntotal
    ids = np.arange(10 ** 9, 10 ** 9 + xa.shape[0], dtype=np.int64)
    idx.add_with_ids(xa, ids)
    assert idx.ntotal == n0 + xa.shape[0]
    got_list = np.full(xa.shape[0], -1, np.int64)
    got_code = {}
    for l in range(idx.nlist):
        lid = idx.list_ids(l)
        codes = idx.list_codes(l)
        for j in np.nonzero(lid >= 10 ** 9)[0]:
            i = int(lid[j] - 10 ** 9)
            got_list[i] = l
            got_code[i] = np.asarray(codes[j]).reshape(-1)
    np.testing.assert_array_equal(got_list, FX[tag + "_assign"])
    if tag.startswith("pq"):
        C = np.stack([got_code[i] for i in range(xa.shape[0])]).astype(np.uint8)
        np.testing.assert_array_equal(C, FX[tag + "_codes"])
    else:
        for i in range(xa.shape[0]):
            np.testing.assert_array_equal(got_code[i].view(np.float32), xa[i])


@pytest.mark.parametrize("ef", [16, 64, 200])
@pytest.mark.parametrize("nprobe", [8, 100])
@pytest.mark.parametrize("path_", ["batched", "sequential"])
def test_gpu_hnsw_ivf_equals_reference(amd, gpu, monkeypatch, ef, nprobe, path_):
    if path_ == "sequential":
        monkeypatch.setenv("FAISS_AMD_HNSW_EXACT", "1")
    idx = amd.read_index(path("hnswivf"))
    q = idx.quantizer
    q.efSearch = ef
    idx.nprobe = nprobe
    xq = FX["hnswivf_xq"]
    Dq, Iq = q.search(xq, nprobe)
    np.testing.assert_array_equal(Iq, FX[f"hnswivf_ef{ef}_q{nprobe}_I"])
    np.testing.assert_array_equal(Dq, FX[f"hnswivf_ef{ef}_q{nprobe}_D"])
    D, I = idx.search(xq, 10)
    eq(D, I, f"hnswivf_ef{ef}_{nprobe}")


@pytest.mark.parametrize("ef", [16, 64])
@pytest.mark.parametrize("nprobe", [8, 100])
@pytest.mark.parametrize("defer", ["1", "0"])
def test_gpu_hnsw_ivf_device_equals_reference(amd, gpu, monkeypatch, ef, nprobe, defer):
    """The device entry point (bench.py's step): the HNSW quantizer's tie
    re-runs overlapped with the scan of the other queries (defer=1, the
    default) or run before it (FAISS_AMD_HNSW_DEFER=0); both equal the
    reference's IndexIVF::search."""
    from conftest import device_search
    monkeypatch.setenv("FAISS_AMD_HNSW_DEFER", defer)
    idx = amd.read_index(path("hnswivf"))
    idx.quantizer.efSearch = ef
    idx.nprobe = nprobe
    D, I = device_search(idx, FX["hnswivf_xq"], 10)
    eq(D, I, f"hnswivf_ef{ef}_{nprobe}")


@pytest.mark.parametrize("ef", [8, 32, 200])
@pytest.mark.parametrize("k", [1, 10, 40])
@pytest.mark.parametrize("path_", ["batched", "sequential"])
def test_gpu_hnsw_duplicates_equal_reference(amd, gpu, monkeypatch, ef, k, path_):
    """exact distance ties in the MinimaxHeap and the result heap; the
    sequential kernel (register heaps for ef, k <= 64) on every query too"""
    if path_ == "sequential":
        monkeypatch.setenv("FAISS_AMD_HNSW_EXACT", "1")
    idx = amd.read_index(path("hnsw_dup"))
    idx.efSearch = ef
    D, I = idx.search(FX["hnsw_dup_xq"], k)
    eq(D, I, f"hnsw_dup_ef{ef}_{k}")


def test_gpu_flat_index_equals_reference(amd, gpu):
    idx = amd.read_index(path("flat"))
    D, I = idx.search(FX["flat_xq"], 10)
    eq(D, I, "flat_10")
