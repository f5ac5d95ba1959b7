"""CPU checks against reference-run fixtures (tests/golden/ref_full*).

The fixtures were produced by the reference library itself, compiled from
/root/reference by oracle/ref/Makefile (`full`), with
oracle/ref/make_golden_full.py: index files written by faiss::write_index and
the D/I / lims / codes of the reference's own searches over them.  Here:
  * the product's reader parses every reference-written file, its lists equal
    the reference's (sizes + sha256 of codes and ids), and its writer gives the
    file back byte for byte;
  * the oracle restatement reproduces every reference output bit for bit
    (IVF-Flat and IVF-PQ search_preassigned / search / range search, PQ
    encoding, HNSW-IVF search, standalone HNSW with duplicated vectors).
The GPU path is checked against the same arrays in test_gpu_ref_fixtures.py.
"""
import hashlib
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GDIR = os.path.join(HERE, "golden", "ref_full")
FX = np.load(os.path.join(HERE, "golden", "ref_full.npz"))

IVF_TAGS = ["flat_l2", "flat_ip", "pq_m32d128", "pq_m48d96", "pq_m16d64", "pq_m24d96",
            "pq_m8d64", "pq_m4d64", "pq_m12d48", "pq_ip_m16d64", "hnswivf"]
PQ_TAGS = [t for t in IVF_TAGS if t.startswith("pq_")]


def path(tag):
    return os.path.join(GDIR, tag + ".faiss")


def lists_digest(idx):
    sizes = np.array([idx.get_list_size(l) for l in range(idx.nlist)], np.int64)
    sha = hashlib.sha256()
    for l in range(idx.nlist):
        sha.update(np.ascontiguousarray(idx.list_codes(l), np.uint8).tobytes())
        sha.update(np.ascontiguousarray(idx.list_ids(l), np.int64).tobytes())
    return sizes, np.frombuffer(sha.digest(), np.uint8)


@pytest.mark.parametrize("tag", IVF_TAGS)
def test_read_reference_file(amd, tag):
    idx = amd.read_index(path(tag))
    info = FX[tag + "_info"]
    assert idx.d == info[0] and idx.ntotal == info[1]
    assert idx.metric_type == (1 if info[2] else 0)
    assert idx.nlist == info[3] and idx.code_size == info[5]
    if tag in PQ_TAGS:
        pi = idx.pq_info()
        assert pi["M"] == info[6] and pi["nbits"] == info[7]
        assert pi["by_residual"] == info[8]
    sizes, sha = lists_digest(idx)
    np.testing.assert_array_equal(sizes, FX[tag + "_sizes"])
    np.testing.assert_array_equal(sha, FX[tag + "_sha"])


@pytest.mark.parametrize("tag", IVF_TAGS + ["flat", "hnsw_dup"])
def test_rewrite_reference_file_byte_identical(amd, tag, tmp_path):
    idx = amd.read_index(path(tag))
    out = str(tmp_path / "re.faiss")
    amd.write_index(idx, out)
    with open(path(tag), "rb") as f1, open(out, "rb") as f2:
        assert f1.read() == f2.read()


def _pre_cases(tag):
    for key in FX.files:
        if not (key.startswith(tag + "_") and "_pre_" in key and key.endswith("_D")):
            continue
        parts = key[len(tag) + 1:-2].split("_")
        if parts[0].startswith("t"):
            yield key[:-2], int(parts[0][1:]), int(parts[2]), int(parts[3])
        else:
            yield key[:-2], None, int(parts[1]), int(parts[2])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"] + PQ_TAGS)
def test_oracle_preassigned_equals_reference(amd, orc, tag):
    idx = amd.read_index(path(tag))
    ref = orc.IVFOracle.from_index(idx)
    xq = FX[tag + "_xq"]
    n = 0
    for key, table, nprobe, k in _pre_cases(tag):
        if table is not None and FX[tag + "_info"][2] == 1:
            ref.use_precomputed_table = table
        D, I = ref.search_preassigned(xq, k, FX[f"{tag}_q{nprobe}_I"], FX[f"{tag}_q{nprobe}_D"])
        np.testing.assert_array_equal(I, FX[key + "_I"], err_msg=key)
        np.testing.assert_array_equal(D, FX[key + "_D"], err_msg=key)
        n += 1
    assert n >= 4


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip", "pq_m32d128", "pq_ip_m16d64"])
def test_oracle_search_equals_reference(amd, orc, tag):
    """IndexIVF::search end to end (one slice, BLAS-form coarse)."""
    idx = amd.read_index(path(tag))
    ref = orc.IVFOracle.from_index(idx)
    xq = FX[tag + "_xq"]
    for key in [k for k in FX.files if k.startswith(tag + "_full_") and k.endswith("_D")]:
        nprobe, k = map(int, key[len(tag) + 6:-2].split("_"))
        D, I, _, _ = ref.search(xq, k, nprobe, nslices=1)
        np.testing.assert_array_equal(I, FX[key[:-2] + "_I"], err_msg=key)
        np.testing.assert_array_equal(D, FX[key], err_msg=key)


@pytest.mark.parametrize("ef", [16, 64, 200])
def test_oracle_hnsw_ivf_equals_reference(amd, orc, ef):
    idx = amd.read_index(path("hnswivf"))
    ref = orc.IVFOracle.from_index(idx)
    xq = FX["hnswivf_xq"]
    for nprobe in (8, 100):
        D, I, CD, CI = ref.search(xq, 10, nprobe, efSearch=ef, nslices=1)
        np.testing.assert_array_equal(CI, FX[f"hnswivf_ef{ef}_q{nprobe}_I"])
        np.testing.assert_array_equal(CD, FX[f"hnswivf_ef{ef}_q{nprobe}_D"])
        np.testing.assert_array_equal(I, FX[f"hnswivf_ef{ef}_{nprobe}_I"])
        np.testing.assert_array_equal(D, FX[f"hnswivf_ef{ef}_{nprobe}_D"])


def test_oracle_hnsw_duplicates_equal_reference(amd, orc):
    """IndexHNSWFlat over duplicated vectors: exact distance ties in both
    heaps (MinimaxHeap pop_min / push rules, faiss/impl/HNSW.cpp:1096-1342)."""
    idx = amd.read_index(path("hnsw_dup"))
    g = orc.HNSWGraph.from_index(idx)
    xq = FX["hnsw_dup_xq"]
    for ef in (8, 32, 200):
        for k in (1, 10, 40):
            D, I = g.search(xq, k, ef)
            np.testing.assert_array_equal(I, FX[f"hnsw_dup_ef{ef}_{k}_I"], err_msg=f"{ef} {k}")
            np.testing.assert_array_equal(D, FX[f"hnsw_dup_ef{ef}_{k}_D"])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip", "pq_m32d128", "pq_m48d96",
                                 "pq_ip_m16d64"])
def test_oracle_range_equals_reference(amd, orc, tag):
    idx = amd.read_index(path(tag))
    ref = orc.IVFOracle.from_index(idx)
    xq = FX[tag + "_xq"]
    nprobe = 8 if tag.startswith("flat") else 5
    lims, D, I = ref.range_search_preassigned(
        xq, float(FX[tag + "_range_radius"][0]), FX[f"{tag}_q{nprobe}_I"]
        if f"{tag}_q{nprobe}_I" in FX.files else _coarse(ref, xq, nprobe)[1],
        coarse_dis=FX[f"{tag}_q{nprobe}_D"] if f"{tag}_q{nprobe}_D" in FX.files
        else _coarse(ref, xq, nprobe)[0])
    np.testing.assert_array_equal(lims, FX[tag + "_range_lims"])
    np.testing.assert_array_equal(I, FX[tag + "_range_I"])
    np.testing.assert_array_equal(D, FX[tag + "_range_D"])


def _coarse(ref, xq, nprobe):
    _, _, CD, CI = ref.search(xq, 1, nprobe, nslices=1)
    return CD, CI


@pytest.mark.parametrize("tag", PQ_TAGS)
def test_oracle_pq_encode_equals_reference(amd, orc, tag):
    idx = amd.read_index(path(tag))
    ref = orc.IVFOracle.from_index(idx)
    codes = ref.encode(FX[tag + "_xa"], FX[tag + "_assign"])
    np.testing.assert_array_equal(codes, FX[tag + "_codes"])


@pytest.mark.parametrize("tag", ["flat_l2", "flat_ip"] + PQ_TAGS)
def test_oracle_assign_equals_reference(amd, orc, tag):
    """add-path coarse assignment = quantizer->assign (BLAS form, k = 1)"""
    idx = amd.read_index(path(tag))
    ref = orc.IVFOracle.from_index(idx)
    _, CI = _coarse(ref, FX[tag + "_xa"], 1)
    np.testing.assert_array_equal(CI[:, 0], FX[tag + "_assign"])
