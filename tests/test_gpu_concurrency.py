"""Concurrent searches through shared state.

The reference's Index::search is const and reentrant; faiss lets
several IVF indexes share one coarse quantizer.  Here two IVF-Flat indexes
share one HNSW quantizer whose efSearch (100) takes the batched kernel with
the overlapped tie re-runs (IndexHNSW::split_begin / split_finish), and two
threads search them at once on their own HIP streams; every result must equal
the single-threaded one.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Dev:
    """hipMalloc'd buffers + a stream for one thread's device searches."""

    def __init__(self, xq, k):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.n, self.k = xq.shape[0], k
        self.st = ctypes.c_void_p()
        assert self.hip.hipStreamCreate(ctypes.byref(self.st)) == 0
        self.bufs = []
        self.px = self._alloc(xq.nbytes)
        self.pd = self._alloc(self.n * k * 4)
        self.pi = self._alloc(self.n * k * 8)
        x = np.ascontiguousarray(xq, dtype=np.float32)
        self.hip.hipMemcpy(self.px, x.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(x.nbytes), 1)

    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 4))) == 0
        self.bufs.append(p)
        return p

    def search(self, idx):
        idx.search_device(self.n, self.px.value, self.k, self.pd.value, self.pi.value,
                          self.st.value)
        assert self.hip.hipStreamSynchronize(self.st) == 0
        D = np.empty((self.n, self.k), np.float32)
        I = np.empty((self.n, self.k), np.int64)
        self.hip.hipMemcpy(D.ctypes.data_as(ctypes.c_void_p), self.pd, ctypes.c_size_t(D.nbytes), 2)
        self.hip.hipMemcpy(I.ctypes.data_as(ctypes.c_void_p), self.pi, ctypes.c_size_t(I.nbytes), 2)
        return D, I

    def close(self):
        for p in self.bufs:
            self.hip.hipFree(p)
        self.hip.hipStreamDestroy(self.st)


def test_two_ivf_sharing_one_hnsw_quantizer_two_threads(amd, gpu):
    d, nlist, nb, nq, k = 64, 1024, 200_000, 2000, 10
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    q = amd.IndexHNSWFlat(d, 32)
    a = amd.IndexIVFFlat(q, d, nlist)
    a.train(xb[:60_000])
    a.add(xb[: nb // 2])
    b = amd.IndexIVFFlat(q, d, nlist)  # the trained quantizer, shared
    assert b.is_trained
    b.add(xb[nb // 2:])
    for ix in (a, b):
        ix.nprobe = 64
    q.efSearch = 100  # batched HNSW kernel + overlapped re-runs (split)
    xa = amd.float_rand(nq * d, 5678).reshape(nq, d)
    xbq = amd.float_rand(nq * d, 777).reshape(nq, d)
    da, db = Dev(xa, k), Dev(xbq, k)
    try:
        ra, rb = da.search(a), db.search(b)
        out, errs = {"a": [], "b": []}, []

        def run(name, dev, ix):
            try:
                for _ in range(6):
                    out[name].append(dev.search(ix))
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ts = [threading.Thread(target=run, args=("a", da, a)),
              threading.Thread(target=run, args=("b", db, b))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        for D, I in out["a"]:
            np.testing.assert_array_equal(I, ra[1])
            np.testing.assert_array_equal(D, ra[0])
        for D, I in out["b"]:
            np.testing.assert_array_equal(I, rb[1])
            np.testing.assert_array_equal(D, rb[0])
    finally:
        da.close()
        db.close()
