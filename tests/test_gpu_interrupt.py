"""InterruptCallback / TimeoutCallback (faiss/impl/AuxIndexStructures.h:135-170):
a host search that polls an installed callback after it fires raises
"computation interrupted" (faiss/IndexIVF.cpp:627, 707-713; IndexHNSW.cpp:315),
k-means polls it per iteration (Clustering.cpp:487); a TimeoutCallback fires
once, and searches after it (or after clear_instance) return the oracle's
results."""
import numpy as np
import pytest

from conftest import assert_same_results, rand

pytestmark = pytest.mark.gpu


@pytest.fixture
def interrupt(amd):
    yield amd.set_interrupt_timeout
    amd.set_interrupt_timeout(None)


def test_ivf_search_interrupted_then_exact(amd, orc, gpu, interrupt):
    d = 32
    xb = rand(orc, 20_000, d, 81)
    idx = amd.index_factory(d, "IVF64,Flat")
    idx.train(xb[:5000])
    idx.add(xb)
    idx.nprobe = 8
    xq = rand(orc, 300, d, 82)
    interrupt(1e-9)  # fires at the first poll
    with pytest.raises(amd.FaissError, match="computation interrupted"):
        idx.search(xq, 10)
    D, I = idx.search(xq, 10)  # fired once: this one runs to the end
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(xq, 10, 8, nslices=1)
    assert_same_results(D, I, Dr, Ir)
    interrupt(1e-9)
    Dq, Iq = idx.quantizer.search(xq, 8)
    with pytest.raises(amd.FaissError, match="computation interrupted"):
        idx.search_preassigned(xq, 10, Iq, Dq)
    interrupt(None)
    D2, I2 = idx.search(xq, 10)
    assert_same_results(D2, I2, Dr, Ir)
    interrupt(3600.0)  # not due: no effect
    D3, I3 = idx.search(xq, 10)
    assert_same_results(D3, I3, Dr, Ir)


def test_hnsw_search_and_kmeans_interrupted(amd, orc, gpu, interrupt):
    d = 24
    xb = rand(orc, 4000, d, 83)
    h = amd.IndexHNSWFlat(d, 16)
    h.add(xb)
    xq = rand(orc, 100, d, 84)
    D0, I0 = h.search(xq, 5)
    interrupt(1e-9)
    with pytest.raises(amd.FaissError, match="computation interrupted"):
        h.search(xq, 5)
    D1, I1 = h.search(xq, 5)
    assert np.array_equal(I0, I1) and np.array_equal(D0, D1)
    idx = amd.index_factory(d, "IVF32,Flat")
    interrupt(1e-9)
    with pytest.raises(amd.FaissError, match="computation interrupted"):
        idx.train(xb)
    interrupt(None)
    idx.train(xb)
    assert idx.is_trained
