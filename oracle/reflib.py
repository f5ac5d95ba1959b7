"""ctypes access to oracle/_ref/libfaissfull.so — the reference CPU library
compiled in place from /root/reference by oracle/ref/Makefile (`full`).

TEST INFRASTRUCTURE ONLY: bench.py's `cpu_baseline` leg times the
reference's own IndexIVF::search with it (kind "reference"); the fixture
generator (oracle/ref/make_golden_full.py) drives it directly.  Never used by
the product path.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libfaissfull.so")
_L = None


def lib():
    """Load the library (RTLD_GLOBAL: MKL's dispatch libraries resolve symbols
    of libmkl_core through the global scope); raises OSError if absent."""
    global _L
    if _L is None:
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        P, I64 = C.c_void_p, C.c_int64
        L.reff_last_error.restype = C.c_char_p
        L.reff_read_index.restype = P
        L.reff_read_index.argtypes = [C.c_char_p, C.c_int]
        L.reff_free.argtypes = [P]
        L.reff_set_threads.argtypes = [C.c_int]
        L.reff_set_nprobe.argtypes = [P, I64]
        L.reff_set_quantizer_efsearch.argtypes = [P, C.c_int]
        L.reff_search.argtypes = [P, I64, P, I64, P, P]
        _L = L
    return _L


def available():
    try:
        lib()
        return True
    except OSError:
        return False


class RefIndex:
    """A reference faiss::Index read from a file written by write_index."""

    def __init__(self, fname, io_flags=0):
        self.h = lib().reff_read_index(fname.encode(), io_flags)
        if not self.h:
            raise RuntimeError(lib().reff_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().reff_free(self.h)
            self.h = None

    def _ok(self, rc):
        if rc != 0:
            raise RuntimeError(lib().reff_last_error().decode())

    def set_nprobe(self, nprobe):
        self._ok(lib().reff_set_nprobe(self.h, nprobe))

    def set_quantizer_efsearch(self, ef):
        self._ok(lib().reff_set_quantizer_efsearch(self.h, ef))

    def search(self, x, k, nthreads):
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        lib().reff_set_threads(int(nthreads))
        self._ok(lib().reff_search(self.h, n, x.ctypes.data_as(C.c_void_p), k,
                                   D.ctypes.data_as(C.c_void_p), I.ctypes.data_as(C.c_void_p)))
        return D, I
