import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and runs the HIP path")


@pytest.fixture(scope="session")
def amd():
    return ge.load_package()


@pytest.fixture(scope="session")
def orc():
    return ge.load_oracle()


@pytest.fixture(scope="session")
def gpu(amd):
    # GPU tests fail loudly (never skip) when the device is missing
    n = amd.device_count()
    assert n >= 1, "no HIP device visible: GPU tests need an MI355X"
    return n


def rand(orc, n, d, seed):
    return orc.float_rand(n * d, seed).reshape(n, d)


def assert_same_results(D, I, Dr, Ir, rtol=0.0):
    """Bit-exact ids; distances equal (rtol=0) or within rtol."""
    assert D.shape == Dr.shape and I.shape == Ir.shape
    bad = np.nonzero((I != Ir).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} queries with different ids, first {bad[:5]}: " \
                          f"{I[bad[0]]} vs {Ir[bad[0]]} / {D[bad[0]]} vs {Dr[bad[0]]}"
    if rtol == 0.0:
        assert np.array_equal(D, Dr), f"max |dD| = {np.abs(D - Dr).max()}"
    else:
        np.testing.assert_allclose(D, Dr, rtol=rtol, atol=0)


def device_search(idx, xq, k):
    """Index::search_device (the device entry point bench.py times) on
    hipMalloc'd copies of xq; returns host (D, I)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def dmalloc(nbytes):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 4))) == 0
        return p
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    n = xq.shape[0]
    px, pd, pi = dmalloc(xq.nbytes), dmalloc(n * k * 4), dmalloc(n * k * 8)
    try:
        hip.hipMemcpy(px, xq.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(xq.nbytes), 1)
        idx.search_device(n, px.value, k, pd.value, pi.value)
        assert hip.hipDeviceSynchronize() == 0
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        hip.hipMemcpy(D.ctypes.data_as(ctypes.c_void_p), pd, ctypes.c_size_t(D.nbytes), 2)
        hip.hipMemcpy(I.ctypes.data_as(ctypes.c_void_p), pi, ctypes.c_size_t(I.nbytes), 2)
    finally:
        for p in (px, pd, pi):
            hip.hipFree(p)
    return D, I
