"""Every BASELINE.json config at its own geometry on the HIP path, checked
against the oracle restatement (itself pinned to the reference library in
tests/test_ref_fixtures.py).

  c2  IVF4096,Flat d=128, nb = 1M, nq = 10k, nprobe 32        (full size)
  c3  IVF4096,PQ32x8 d=128, nb = 1M, nq = 10k, nprobe 32      (full size)
  c4  IVF16384_HNSW32,Flat d=128, efSearch 16 / 64 / 128, nprobe 64
      (quantizer geometry of c4; nb = 1M of its 10M, nq = 2000)
  c5  IVF65536,PQ48 d=96, nprobe 64 (one shard's geometry; nb = 2M of the
      12.5M of an 8-GPU shard, nq = 2000)
and at their real sizes (the bench's batches searched whole on the GPU, a
subset of the queries re-derived by the oracle):
  c4  10M vectors, the 10k-query batch, efSearch 64 through search() and
      16 / 64 / 128 through search_device() (400 queries checked)
  c5  one 12.5M-vector shard of the 100M set (ids == 0 mod 8, as bench.py
      --shard-of 8), the 100k-query batch (400 queries checked): ~190 rows
      per list, the PQ filter's long-list work items at full length
Ids and distances must be equal bit for bit (data: faiss float_rand streams,
xb seed 1234, xq seed 5678, as bench.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def build(amd, desc, d, nb, ntrain, seed=1234):
    xb = amd.float_rand(nb * d, seed).reshape(nb, d)
    idx = amd.index_factory(d, desc)
    idx.train(xb[:ntrain])
    idx.add(xb)
    return idx


def check(D, I, Dr, Ir, what):
    bad = np.nonzero((I != Ir).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} queries differ, first {bad[:4]}"
    assert np.array_equal(D, Dr), f"{what}: max |dD| {np.abs(D - Dr).max()}"


def test_c2_ivf4096_flat_full(amd, orc, gpu):
    d, nq = 128, 10_000
    idx = build(amd, "IVF4096,Flat", d, 1_000_000, 200_000)
    idx.nprobe = 32
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 32, nslices=1)
    check(D, I, Dr, Ir, "c2")


def test_c2_host_pages_full(amd, orc, gpu, monkeypatch):
    # c2's index, a 60k-query host batch: the default pages it (2 pages of
    # 30k, uploads overlapping searches); equal to the eager one-call path
    # and, on queries around the page boundary and a spread, to the oracle
    d, nq = 128, 60_000
    idx = build(amd, "IVF4096,Flat", d, 1_000_000, 200_000)
    idx.nprobe = 32
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    monkeypatch.delenv("FAISS_AMD_HOST_PAGES", raising=False)
    for _ in range(3):  # eager pages, captured, replayed
        D, I = idx.search(xq, 10)
    monkeypatch.setenv("FAISS_AMD_HOST_PAGES", "0")
    D0, I0 = idx.search(xq, 10)
    check(D, I, D0, I0, "c2 pages vs eager")
    sel = np.r_[0:50, 29_950:30_050, 59_950:60_000, 1_000:60_000:300]
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[sel]), 10, 32, nslices=1)
    check(D[sel], I[sel], Dr, Ir, "c2 pages vs oracle")


def test_c3_ivf4096_pq32_full(amd, orc, gpu):
    d, nq = 128, 10_000
    idx = build(amd, "IVF4096,PQ32", d, 1_000_000, 200_000)
    assert idx.use_precomputed_table == 1  # 4096 x 32 x 256 x 4 B <= 2 GiB
    idx.nprobe = 32
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 32, nslices=1)
    check(D, I, Dr, Ir, "c3")


@pytest.fixture(scope="module")
def c4_index(amd):
    return build(amd, "IVF16384_HNSW32,Flat", 128, 1_000_000, 638_976)


@pytest.mark.parametrize("ef", [16, 64])
def test_c4_device_entry_point(amd, orc, gpu, c4_index, ef):
    """c4 through Index::search_device (bench.py's step), where the HNSW
    quantizer's tie re-runs overlap the scan of the other queries."""
    from conftest import device_search
    d, nq = 128, 2000
    idx = c4_index
    idx.nprobe = 64
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = device_search(idx, xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 64, efSearch=ef, nslices=1)
    check(D, I, Dr, Ir, f"c4 device efSearch {ef}")


def test_c4_pipelined_chunks(amd, orc, gpu, c4_index, monkeypatch):
    """IndexIVF::scan_hnsw_pipelined: the batch in 1 / 2 / 3 chunks (each
    chunk's quantizer search on a side stream overlapping the previous chunk's
    scan) gives one result, the reference's."""
    from conftest import device_search
    d, nq = 128, 4099
    idx = c4_index
    idx.nprobe = 64
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", 64)
    xq = amd.float_rand(nq * d, 777).reshape(nq, d)
    out = {}
    for p in ("1", "2", "3"):
        monkeypatch.setenv("FAISS_AMD_HNSW_PIPE", p)
        out[p] = device_search(idx, xq, 10)
    for p in ("2", "3"):
        check(out[p][0], out[p][1], out["1"][0], out["1"][1], f"c4 pipelined {p} chunks")
    rows = np.arange(0, nq, 41)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), 10, 64, efSearch=64, nslices=1)
    check_subset(out["3"][0], out["3"][1], Dr, Ir, rows, "c4 pipelined vs oracle")


@pytest.mark.parametrize("ef", [16, 64, 128])
def test_c4_hnsw32_ivf16384(amd, orc, gpu, c4_index, ef):
    d, nq = 128, 2000
    idx = c4_index
    idx.nprobe = 64
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 64, efSearch=ef, nslices=1)
    check(D, I, Dr, Ir, f"c4 efSearch {ef}")


@pytest.mark.parametrize("nprobe,ef", [(256, 768), (2500, 2500), (6400, 19200)])
def test_c4_harness_grid_corners(amd, orc, gpu, c4_index, nprobe, ef):
    """The reference harness's (nprobe, efSearch) grid reaches nprobe 6400 and
    efSearch 3 nprobe (tutorial/cpp/benchmark-hnsw-ivf/benchmark.config):
    wide HNSW heaps (LDS, then global scratch past the LDS), nprobe past the
    MFMA filters (the general exact scan)."""
    d, nq = 128, 64
    idx = c4_index
    idx.nprobe = nprobe
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
    try:
        xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
        D, I = idx.search(xq, 10)
        ref = orc.IVFOracle.from_index(idx)
        Dr, Ir, _, _ = ref.search(xq, 10, nprobe, efSearch=ef, nslices=1)
        check(D, I, Dr, Ir, f"c4 nprobe {nprobe} efSearch {ef}")
    finally:
        idx.nprobe = 64
        amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", 64)


@pytest.mark.parametrize("nprobe,ef", [(64, 200), (128, 384), (256, 768), (1024, 1024),
                                       (2048, 4096)])
def test_c4_wide_hnsw_grid(amd, orc, gpu, c4_index, nprobe, ef):
    """128 < max(efSearch, nprobe) <= 4096: the wide kernel (k_hnsw_wide, the
    candidate set sorted in the LDS) + sequential re-runs of the queries it
    flags, bit-exact against the oracle, through search() and the device
    entry point (IndexIVF::scan_hnsw_split overlaps the re-runs with the
    scan); the wide stage must be the one that ran."""
    from conftest import device_search
    d, nq = 128, 500
    idx = c4_index
    idx.nprobe = nprobe
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
    try:
        xq = amd.float_rand(nq * d, 4242).reshape(nq, d)
        q = idx.quantizer
        amd.set_kernel_timing(True)
        try:
            q.reset_kernel_times()
            D, I = idx.search(xq, 10)
            names = {nm for nm, _, _ in q.kernel_times()}
        finally:
            amd.set_kernel_timing(False)
        assert "hnsw_wide" in names, names
        ref = orc.IVFOracle.from_index(idx)
        Dr, Ir, _, _ = ref.search(xq, 10, nprobe, efSearch=ef, nslices=1)
        check(D, I, Dr, Ir, f"c4 wide nprobe {nprobe} efSearch {ef}")
        D2, I2 = device_search(idx, xq, 10)
        check(D2, I2, Dr, Ir, f"c4 wide device nprobe {nprobe} efSearch {ef}")
    finally:
        idx.nprobe = 64
        amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", 64)


@pytest.mark.parametrize("nprobe", [2049, 4096])
def test_flat_coarse_nprobe_beyond_2048(amd, orc, gpu, nprobe):
    """A flat quantizer's top-nprobe beyond 2048 (the global-scratch select)."""
    d, nq = 32, 40
    idx = build(amd, "IVF4096,Flat", d, 200_000, 200_000)
    idx.nprobe = nprobe
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, nprobe, nslices=1)
    check(D, I, Dr, Ir, f"IVF4096 nprobe {nprobe}")


def test_c5_ivf65536_pq48_shard(amd, orc, gpu):
    d, nq = 96, 2000
    idx = build(amd, "IVF65536,PQ48", d, 2_000_000, 65536 * 16)
    assert idx.use_precomputed_table == 0  # 65536 x 48 x 256 x 4 B > 2 GiB
    idx.nprobe = 64
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 64, nslices=1)
    check(D, I, Dr, Ir, "c5")


def check_subset(D, I, Dr, Ir, rows, what):
    check(D[rows], I[rows], Dr, Ir, what)


@pytest.fixture(scope="module")
def c4_10m(amd):
    d, nb = 128, 10_000_000
    idx = amd.index_factory(d, "IVF16384_HNSW32,Flat")
    xt = amd.float_rand_rows(nb, d, 1234, 0, 1, 638_976)
    idx.train(xt)
    del xt
    for c0 in range(0, nb, 2_000_000):
        idx.add(amd.float_rand_rows(nb, d, 1234, c0, 1, 2_000_000))
    idx.nprobe = 64
    return idx


def test_c4_full_10m(amd, orc, gpu, c4_10m):
    d, nq = 128, 10_000
    idx = c4_10m
    amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", 64)
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    rows = np.arange(0, nq, nq // 400)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), 10, 64, efSearch=64, nslices=1)
    check_subset(D, I, Dr, Ir, rows, "c4 10M efSearch 64")


def test_c4_full_10m_device(amd, orc, gpu, c4_10m):
    """The bench's step: the 10k-query batch through Index::search_device on
    the 10M index (register HNSW kernel at efSearch 16 / 64, the batched
    kernel with the overlapped tie re-runs at 128), a 400-query oracle
    subset bit-exact."""
    from conftest import device_search
    d, nq = 128, 10_000
    idx = c4_10m
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    rows = np.arange(0, nq, nq // 400)
    ref = orc.IVFOracle.from_index(idx)
    try:
        for ef in (16, 64, 128):
            amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
            D, I = device_search(idx, xq, 10)
            Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), 10, 64, efSearch=ef,
                                      nslices=1)
            check_subset(D, I, Dr, Ir, rows, f"c4 10M device efSearch {ef}")
    finally:
        amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", 64)


def test_c5_full_shard(amd, orc, gpu):
    d, nb, nshard, nq = 96, 100_000_000, 8, 100_000
    idx = amd.index_factory(d, "IVF65536,PQ48")
    xt = amd.float_rand_rows(nb, d, 1234, 0, 1, 65536 * 16)
    idx.train(xt)
    del xt
    ids = np.arange(0, nb, nshard, dtype=np.int64)
    for c0 in range(0, len(ids), 2_500_000):
        cid = ids[c0:c0 + 2_500_000]
        idx.add_with_ids(amd.float_rand_rows(nb, d, 1234, c0 * nshard, nshard, len(cid)), cid)
    assert idx.ntotal == 12_500_000
    idx.nprobe = 64
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    D, I = idx.search(xq, 10)
    rows = np.arange(0, nq, nq // 400)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), 10, 64, nslices=1)
    check_subset(D, I, Dr, Ir, rows, "c5 12.5M shard")
