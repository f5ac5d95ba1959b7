"""IndexShardsIVF built by the IVF shard cloner (faiss/gpu/GpuCloner.cpp:283-420,
shard_type 1 / 2 / 4) searched on the GPU: the merged result equals the
unsharded index's search (IndexShardsIVF.cpp:158-245: one coarse pass, the
shards' search_preassigned, merge_knn_results).  Three forms:
  single  — every shard on the quantizer's device, one stream;
  rccl1   — the multi-device path as a one-rank RCCL communicator;
  ranks   — the multi-rank composition with one rank per shard on the box's
            one GPU (FAISS_AMD_SHARDS_RANKS=shard): query-split coarse pass
            on each rank's copy of the quantizer, all-gather of the coarse
            results, per-rank merge of its query slice, gather to rank 0 —
            over the copy transport (RCCL refuses a device twice in one
            communicator; with distinct devices the same grouped operations
            go through RCCL).
Random data (no distance ties), so ids and distances must be equal.
"""
import contextlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODES = {"single": {"FAISS_AMD_SHARDS_RCCL": "0"},
         "rccl1": {"FAISS_AMD_SHARDS_RCCL": "1"},
         "ranks": {"FAISS_AMD_SHARDS_RCCL": "1", "FAISS_AMD_SHARDS_RANKS": "shard"}}


@contextlib.contextmanager
def env(values):
    keys = ("FAISS_AMD_SHARDS_RCCL", "FAISS_AMD_SHARDS_RANKS")
    old = {k: os.environ.get(k) for k in keys}
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(values)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=["IVF64,Flat", "IVF64,PQ8", "IVF64_HNSW16,Flat"])
def src(request, amd):
    d, nb = 32, 20000
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, request.param)
    idx.train(xb[:10000])
    idx.add(xb)
    idx.nprobe = 8
    return idx


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("shard_type", [1, 2, 4])
def test_shards_equal_unsharded(amd, gpu, src, shard_type, mode):
    xq = amd.float_rand(300 * src.d, 5678).reshape(300, src.d)
    D0, I0 = src.search(xq, 10)
    sh = amd.index_ivf_to_shards(src, 3, shard_type, devices=[0, 0, 0])
    sh.nprobe = src.nprobe
    assert sh.ntotal == src.ntotal
    with env(MODES[mode]):
        D, I = sh.search(xq, 10)
    np.testing.assert_array_equal(I, I0)
    np.testing.assert_array_equal(D, D0)


@pytest.mark.parametrize("nq", [1, 10, 19, 20, 59, 301])
def test_shard_ranks_ragged_slices(amd, gpu, src, nq):
    """Batches that do not split evenly over the ranks (the last slices short
    or empty), and batches below 20 queries: the coarse form follows the
    whole batch size (direct below 20), not the slice size."""
    xq = amd.float_rand(nq * src.d, 91).reshape(nq, src.d)
    D0, I0 = src.search(xq, 7)
    sh = amd.index_ivf_to_shards(src, 4, 1, devices=[0, 0, 0, 0])
    sh.nprobe = src.nprobe
    with env(MODES["ranks"]):
        D, I = sh.search(xq, 7)
        D2, I2 = sh.search(xq, 7)  # the cached exchange state serves a second call
    np.testing.assert_array_equal(I, I0)
    np.testing.assert_array_equal(D, D0)
    np.testing.assert_array_equal(I2, I0)
