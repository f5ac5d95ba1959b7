"""IndexShardsIVF built by the IVF shard cloner (faiss/gpu/GpuCloner.cpp:283-420,
shard_type 1 / 2 / 4) searched on the GPU: the merged result equals the
unsharded index's search (IndexShardsIVF.cpp:158-245: one coarse pass, the
shards' search_preassigned, merge_knn_results), in the single-device form and
through the RCCL multi-device form (FAISS_AMD_SHARDS_RCCL=1 forces it on the
one device of the box: a one-rank communicator; with several devices the same
code broadcasts the batch and gathers the shards' tables point to point).
Random data (no distance ties), so ids and distances must be equal.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["IVF64,Flat", "IVF64,PQ8"])
def src(request, amd):
    d, nb = 32, 20000
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, request.param)
    idx.train(xb[:10000])
    idx.add(xb)
    idx.nprobe = 8
    return idx


@pytest.mark.parametrize("rccl", [False, True])
@pytest.mark.parametrize("shard_type", [1, 2, 4])
def test_shards_equal_unsharded(amd, gpu, src, shard_type, rccl):
    xq = amd.float_rand(300 * src.d, 5678).reshape(300, src.d)
    D0, I0 = src.search(xq, 10)
    sh = amd.index_ivf_to_shards(src, 3, shard_type, devices=[0, 0, 0])
    sh.nprobe = src.nprobe
    assert sh.ntotal == src.ntotal
    old = os.environ.get("FAISS_AMD_SHARDS_RCCL")
    os.environ["FAISS_AMD_SHARDS_RCCL"] = "1" if rccl else "0"
    try:
        D, I = sh.search(xq, 10)
    finally:
        if old is None:
            del os.environ["FAISS_AMD_SHARDS_RCCL"]
        else:
            os.environ["FAISS_AMD_SHARDS_RCCL"] = old
    np.testing.assert_array_equal(I, I0)
    np.testing.assert_array_equal(D, D0)
