"""ctypes bindings of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (see oracle.h).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker / the CPU baseline, never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None
_P = C.c_void_p


class HNSWStruct(C.Structure):
    _fields_ = [("entry_point", C.c_int32), ("max_level", C.c_int32), ("ntotal", C.c_int64),
                ("levels", _P), ("offsets", _P), ("neighbors", _P),
                ("cum_nneighbor_per_level", _P), ("storage", _P), ("d", C.c_int)]


class IVFStruct(C.Structure):
    _fields_ = [("d", C.c_int), ("nlist", C.c_int64), ("metric", C.c_int),
                ("centroids", _P), ("hnsw", C.POINTER(HNSWStruct)), ("list_off", _P),
                ("codes", _P), ("code_size", C.c_size_t), ("ids", _P), ("pq_M", C.c_int),
                ("pq_nbits", C.c_int), ("pq_centroids", _P), ("by_residual", C.c_int),
                ("use_precomputed_table", C.c_int), ("precomputed_table", _P)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        L.oracle_float_rand.argtypes = [_P, C.c_size_t, C.c_int64]
        for f in ("oracle_fvec_L2sqr", "oracle_fvec_inner_product"):
            getattr(L, f).argtypes = [_P, _P, C.c_size_t]
            getattr(L, f).restype = C.c_float
        L.oracle_fvec_norm_L2sqr.argtypes = [_P, C.c_size_t]
        L.oracle_fvec_norm_L2sqr.restype = C.c_float
        L.oracle_heap_heapify.argtypes = [C.c_int, C.c_size_t, _P, _P]
        L.oracle_heap_replace_top.argtypes = [C.c_int, C.c_size_t, _P, _P, C.c_float, C.c_int64]
        L.oracle_heap_addn.argtypes = [C.c_int, C.c_size_t, _P, _P, _P, _P, C.c_size_t]
        L.oracle_heap_reorder.argtypes = [C.c_int, C.c_size_t, _P, _P]
        L.oracle_heap_reorder.restype = C.c_size_t
        L.oracle_knn.argtypes = [_P, _P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int,
                                 C.c_int, _P, _P, C.c_int]
        L.oracle_hnsw_search.argtypes = [C.POINTER(HNSWStruct), _P, C.c_size_t, C.c_size_t,
                                         C.c_int, _P, _P, C.c_int]
        L.oracle_ivfpq_prepare.argtypes = [C.POINTER(IVFStruct)]
        L.oracle_ivf_search_preassigned.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P,
                                                    C.c_size_t, C.c_size_t, _P, _P, _P, _P,
                                                    C.c_int]
        L.oracle_ivf_search_preassigned_mc.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P,
                                                       C.c_size_t, C.c_size_t, _P, _P,
                                                       C.c_int64, _P, _P, _P, C.c_int]
        L.oracle_ivf_search.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P, C.c_size_t,
                                        C.c_size_t, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int]
        L.oracle_ivf_search_fast.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P, C.c_size_t,
                                             C.c_size_t, _P, _P, C.c_int]
        L.oracle_merge_knn_results.argtypes = [C.c_size_t, C.c_size_t, C.c_int, _P, _P, _P, _P,
                                               C.c_int]
        L.oracle_ivf_range_preassigned.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P,
                                                   C.c_size_t, _P, _P, C.c_float, _P, _P, _P,
                                                   _P, C.c_int64]
        L.oracle_ivf_range_preassigned.restype = C.c_int64
        L.oracle_max_threads.restype = C.c_int
        L.oracle_ivfpq_encode.argtypes = [C.POINTER(IVFStruct), C.c_size_t, _P, _P, _P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def nthreads_default():
    return lib().oracle_max_threads()


def float_rand(n, seed):
    x = np.empty(n, dtype=np.float32)
    lib().oracle_float_rand(_p(x), n, seed)
    return x


def fvec_L2sqr(x, y):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    return lib().oracle_fvec_L2sqr(_p(x), _p(y), x.size)


def fvec_inner_product(x, y):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    return lib().oracle_fvec_inner_product(_p(x), _p(y), x.size)


def heap_addn_reorder(k, vals, ids, cmax=True):
    """heapify(k) + heap_addn(vals, ids) + heap_reorder, as faiss does."""
    bv = np.empty(k, np.float32)
    bi = np.empty(k, np.int64)
    vals = np.ascontiguousarray(vals, np.float32)
    ids = np.ascontiguousarray(ids, np.int64)
    L = lib()
    L.oracle_heap_heapify(int(cmax), k, _p(bv), _p(bi))
    L.oracle_heap_addn(int(cmax), k, _p(bv), _p(bi), _p(vals), _p(ids), vals.size)
    L.oracle_heap_reorder(int(cmax), k, _p(bv), _p(bi))
    return bv, bi


def knn(x, y, k, metric=1, blas_form=True, nthreads=None):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    n = x.shape[0]
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    lib().oracle_knn(_p(x), _p(y), x.shape[1], n, y.shape[0], k, metric, int(blas_form), _p(D),
                     _p(I), nthreads or nthreads_default())
    return D, I


class HNSWGraph:
    """Holds the arrays of an HNSW graph for the oracle."""

    def __init__(self, entry_point, max_level, levels, offsets, neighbors, cum, storage):
        self.levels = np.ascontiguousarray(levels, np.int32)
        self.offsets = np.ascontiguousarray(offsets, np.uint64)
        self.neighbors = np.ascontiguousarray(neighbors, np.int32)
        self.cum = np.ascontiguousarray(cum, np.int32)
        self.storage = np.ascontiguousarray(storage, np.float32)
        self.s = HNSWStruct(entry_point, max_level, self.storage.shape[0], _p(self.levels),
                            _p(self.offsets), _p(self.neighbors), _p(self.cum),
                            _p(self.storage), self.storage.shape[1])

    @classmethod
    def from_index(cls, idx):
        ep, ml, levels, offsets, neighbors, cum = idx.graph()
        storage = idx_storage(idx)
        return cls(ep, ml, levels, offsets, neighbors, cum, storage)

    def search(self, x, k, efSearch, nthreads=None):
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        lib().oracle_hnsw_search(C.byref(self.s), _p(x), n, k, efSearch, _p(D), _p(I),
                                 nthreads or nthreads_default())
        return D, I


def idx_storage(hidx):
    """Vectors of an IndexHNSWFlat (via reconstruct of its flat storage)."""
    return hidx.storage_vectors()


class IVFOracle:
    """Oracle view of an IVF index exported from the GPU library (same data)."""

    def __init__(self, d, nlist, metric, list_off, codes, ids, centroids=None, hnsw=None,
                 pq=None):
        self.d, self.nlist, self.metric = d, nlist, metric
        self.list_off = np.ascontiguousarray(list_off, np.int64)
        self.codes = np.ascontiguousarray(codes, np.uint8)
        self.ids = np.ascontiguousarray(ids, np.int64)
        self.centroids = (np.ascontiguousarray(centroids, np.float32) if centroids is not None
                          else None)
        self.hnsw = hnsw
        code_size = self.codes.shape[1] if self.codes.ndim == 2 else d * 4
        s = IVFStruct()
        s.d, s.nlist, s.metric = d, nlist, metric
        s.centroids = _p(self.centroids) if self.centroids is not None else None
        s.hnsw = C.pointer(hnsw.s) if hnsw is not None else C.POINTER(HNSWStruct)()
        s.list_off, s.codes, s.code_size, s.ids = (_p(self.list_off), _p(self.codes), code_size,
                                                   _p(self.ids))
        if pq is not None:
            self.pq_centroids = np.ascontiguousarray(pq["centroids"], np.float32)
            s.pq_M, s.pq_nbits = pq["M"], pq["nbits"]
            s.pq_centroids = _p(self.pq_centroids)
            s.by_residual = int(pq["by_residual"])
            s.use_precomputed_table = 0
            s.precomputed_table = None
        else:
            s.pq_M = 0
        self.s = s
        if pq is not None:
            lib().oracle_ivfpq_prepare(C.byref(self.s))

    @property
    def use_precomputed_table(self):
        return self.s.use_precomputed_table

    @use_precomputed_table.setter
    def use_precomputed_table(self, t):
        """0 (per-list residual tables) or 1 (needs the table prepare() built)."""
        if t == 1 and not self.s.precomputed_table:
            raise ValueError("no precomputed table for this index")
        self.s.use_precomputed_table = int(t)

    @classmethod
    def from_index(cls, idx):
        """Export an hnsw-ivf_amd IndexIVFFlat / IndexIVFPQ (host mirrors)."""
        off, codes, ids = idx.invlists_arrays()
        q = idx.quantizer
        hnsw = None
        centroids = None
        if type(q).__name__ == "IndexHNSWFlat":
            hnsw = HNSWGraph.from_index(q)
        else:
            centroids = q.xb
        pq = None
        if type(idx).__name__ == "IndexIVFPQ":
            info = idx.pq_info()
            pq = dict(M=info["M"], nbits=info["nbits"], by_residual=info["by_residual"],
                      centroids=idx.pq_centroids)
        return cls(idx.d, idx.nlist, idx.metric_type, off, codes, ids, centroids, hnsw, pq)

    def search(self, x, k, nprobe, efSearch=16, nslices=1, nthreads=None):
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        nprobe = min(nprobe, self.nlist)
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        CI = np.empty((n, nprobe), np.int64)
        CD = np.empty((n, nprobe), np.float32)
        lib().oracle_ivf_search(C.byref(self.s), n, _p(x), k, nprobe, efSearch, nslices, _p(D),
                                _p(I), _p(CI), _p(CD), nthreads or nthreads_default())
        return D, I, CD, CI

    def search_preassigned(self, x, k, keys, coarse_dis, nthreads=None, max_codes=0,
                           return_ndis=False):
        x = np.ascontiguousarray(x, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        coarse_dis = np.ascontiguousarray(coarse_dis, np.float32)
        n, nprobe = keys.shape
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        nd = np.zeros(1, np.int64)
        lib().oracle_ivf_search_preassigned_mc(C.byref(self.s), n, _p(x), k, nprobe, _p(keys),
                                               _p(coarse_dis), max_codes, _p(D), _p(I), _p(nd),
                                               nthreads or nthreads_default())
        return (D, I, int(nd[0])) if return_ndis else (D, I)

    def encode(self, x, list_nos):
        """IndexIVFPQ::encode_vectors: [n, M] uint8 codes (dsub < 16)."""
        x = np.ascontiguousarray(x, np.float32)
        ln = np.ascontiguousarray(list_nos, np.int64)
        codes = np.empty((x.shape[0], self.s.pq_M), np.uint8)
        lib().oracle_ivfpq_encode(C.byref(self.s), x.shape[0], _p(x), _p(ln), _p(codes))
        return codes

    def range_search_preassigned(self, x, radius, keys, selmask=None, coarse_dis=None):
        """IVF range search (faiss/IndexIVF.cpp:1243-1400): (lims, D, I).
        selmask: per concatenated row uint8 membership (IDSelector), or None;
        coarse_dis: [n, nprobe] (IVF-PQ with precomputed tables)."""
        x = np.ascontiguousarray(x, np.float32)
        keys = np.ascontiguousarray(keys, np.int64)
        n, nprobe = keys.shape
        cd = (np.zeros((n, nprobe), np.float32) if coarse_dis is None
              else np.ascontiguousarray(coarse_dis, np.float32))
        lims = np.zeros(n + 1, np.uint64)
        sm = None if selmask is None else np.ascontiguousarray(selmask, np.uint8)
        args = (C.byref(self.s), n, _p(x), nprobe, _p(keys), _p(cd), float(radius),
                _p(sm) if sm is not None else None, _p(lims))
        tot = lib().oracle_ivf_range_preassigned(*args, None, None, 0)
        D = np.empty(tot, np.float32)
        I = np.empty(tot, np.int64)
        lib().oracle_ivf_range_preassigned(*args, _p(D), _p(I), tot)
        return lims.astype(np.int64), D, I

    def search_fast(self, x, k, nprobe, nthreads=None):
        x = np.ascontiguousarray(x, np.float32)
        n = x.shape[0]
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        lib().oracle_ivf_search_fast(C.byref(self.s), n, _p(x), k, nprobe, _p(D), _p(I),
                                     nthreads or nthreads_default())
        return D, I


def merge_knn_results(Dall, Iall, metric=1):
    Dall = np.ascontiguousarray(Dall, np.float32)
    Iall = np.ascontiguousarray(Iall, np.int64)
    ns, n, k = Dall.shape
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    lib().oracle_merge_knn_results(n, k, ns, _p(Dall), _p(Iall), _p(D), _p(I), metric)
    return D, I
