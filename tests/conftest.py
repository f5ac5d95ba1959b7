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
