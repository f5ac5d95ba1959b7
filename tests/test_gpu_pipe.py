"""The flat quantizer's pipelined batch (FAISS_AMD_PIPE=<chunks>,
IndexIVF::scan_flat_pipelined): each chunk's coarse search on a second
stream overlapping the previous chunk's list scan.  Every chunking must give
the one-chunk result bit for bit — eager, captured and replayed as a
hipGraph, and through the host entry point — and the one-chunk result is
the oracle's (faiss/IndexIVF.cpp:303-397)."""
import numpy as np
import pytest

from test_gpu_search_graph import Bufs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("desc", ["IVF512,Flat", "IVF512,PQ32"])
def test_pipelined_chunks_equal_one_chunk(amd, orc, gpu, monkeypatch, desc):
    d, nb, nq, k = 128, 120_000, 5000, 10
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, desc)
    idx.train(xb[:60_000])
    idx.add(xb)
    idx.nprobe = 24
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    b = Bufs(xq, k)
    try:
        monkeypatch.setenv("FAISS_AMD_PIPE", "1")
        D0, I0 = b.search(idx)
        for P in ("2", "3", "4"):
            monkeypatch.setenv("FAISS_AMD_PIPE", P)
            for _ in range(4):  # eager, capture, replays
                D, I = b.search(idx)
                assert np.array_equal(I, I0) and np.array_equal(D, D0), P
            Dh, Ih = idx.search(xq, k)
            assert np.array_equal(Ih, I0) and np.array_equal(Dh, D0), P
    finally:
        b.close()
    if desc.endswith("Flat"):
        sub = np.arange(0, nq, 25)
        ref = orc.IVFOracle.from_index(idx)
        Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[sub]), k, 24, nslices=1)
        assert np.array_equal(I0[sub], Ir) and np.array_equal(D0[sub], Dr)
