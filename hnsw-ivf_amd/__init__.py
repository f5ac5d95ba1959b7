"""hnsw-ivf_amd — Python host mirror of the MI355X-native IVF search path.

Mirrors the reference's Python surface for this path (faiss SWIG API as used
by the reference's tests and tutorials: ``index.train/add/add_with_ids/
search``, ``index.nprobe``, ``index_factory``, ``read_index``/``write_index``,
``ParameterSpace().set_index_parameter``) on top of the C-ABI library
``lib/libfaiss_amd.so`` (include/faiss_amd_c.h).  Every compute call goes to
the HIP kernels; there is no CPU fallback: if the library or a GPU is missing
the calls raise.

The package directory name contains a hyphen, so it is loaded by path:
``load_package()`` in ``__graft_entry__`` / tests / bench.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FAISS_AMD_LIB") or os.path.join(_HERE, "lib", "libfaiss_amd.so")

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
IO_FLAG_ONDISK_SAME_DIR = 4  # reference faiss/index_io.h:51
IO_FLAG_SKIP_IVF_DATA = 8  # :53
IO_FLAG_MMAP = 8 | 0x646F0000  # :64 — lists mapped from the file, streamed to HBM

_lib = None


class FaissError(RuntimeError):
    pass


def lib():
    """Load the C-ABI library (raises when it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FaissError(
                f"{LIB_PATH} missing: build it with `make -C hnsw-ivf_amd` "
                "(the search path has no CPU fallback)")
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


_P = C.c_void_p
_I64 = C.c_int64


class IndexIVFStats(C.Structure):
    """faiss/IndexIVF.h:567-583 (faiss.cvar.indexIVF_stats); aliases the
    library's global, so reset() / field reads act on it directly."""
    _fields_ = [("nq", C.c_size_t), ("nlist", C.c_size_t), ("ndis", C.c_size_t),
                ("nheap_updates", C.c_size_t), ("quantization_time", C.c_double),
                ("search_time", C.c_double)]

    def reset(self):
        lib().faiss_IndexIVFStats_reset(C.byref(self))


class HNSWStats(C.Structure):
    """faiss/impl/HNSW.h:234-253 (faiss.cvar.hnsw_stats), aliases the global."""
    _fields_ = [("n1", C.c_size_t), ("n2", C.c_size_t), ("ndis", C.c_size_t),
                ("nhops", C.c_size_t)]

    def reset(self):
        lib().faiss_amd_HNSWStats_reset()


# faiss/IndexIVF.h:28-32 QueryLatencyStats, one record per query (microseconds)
QUERY_LATENCY_DTYPE = np.dtype([("total_us", np.float64), ("quantization_us", np.float64),
                                ("list_scan_us", np.float64)])


class _CVar:
    """faiss.cvar: the library's global statistics."""

    @property
    def indexIVF_stats(self):
        return lib().faiss_get_indexIVF_stats().contents

    @property
    def hnsw_stats(self):
        return lib().faiss_amd_get_hnsw_stats().contents

    @property
    def hnsw_row_stats(self):
        """(fp32 rows, int8-image rows) the GPU HNSW kernels read (not in the
        reference; reset with hnsw_stats)."""
        a, b = C.c_uint64(), C.c_uint64()
        lib().faiss_amd_get_hnsw_row_stats(C.byref(a), C.byref(b))
        return a.value, b.value

    @property
    def hnsw_replay_stats(self):
        """(replayed, searched again, corrupt logs) of the register HNSW
        kernel's layout-dependent continuations (not in the reference)."""
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        lib().faiss_amd_get_hnsw_replay_stats(C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value


cvar = _CVar()


def set_interrupt_timeout(seconds):
    """faiss.TimeoutCallback.reset(seconds) (seconds >= 0) /
    InterruptCallback.clear_instance() (None or < 0): a host search that polls
    the callback after it fires raises FaissError("computation interrupted")."""
    lib().faiss_amd_set_interrupt_timeout(-1.0 if seconds is None else float(seconds))


def _declare(L):
    sig = {
        "faiss_get_last_error": (C.c_char_p, []),
        "faiss_Index_free": (None, [_P]),
        "faiss_Index_d": (C.c_int, [_P]),
        "faiss_Index_is_trained": (C.c_int, [_P]),
        "faiss_Index_ntotal": (_I64, [_P]),
        "faiss_Index_metric_type": (C.c_int, [_P]),
        "faiss_Index_verbose": (C.c_int, [_P]),
        "faiss_Index_set_verbose": (None, [_P, C.c_int]),
        "faiss_Index_train": (C.c_int, [_P, _I64, _P]),
        "faiss_Index_add": (C.c_int, [_P, _I64, _P]),
        "faiss_Index_add_with_ids": (C.c_int, [_P, _I64, _P, _P]),
        "faiss_Index_search": (C.c_int, [_P, _I64, _P, _I64, _P, _P]),
        "faiss_Index_search_with_params": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P]),
        "faiss_RangeSearchResult_new": (C.c_int, [C.POINTER(_P), _I64]),
        "faiss_RangeSearchResult_free": (None, [_P]),
        "faiss_RangeSearchResult_nq": (C.c_size_t, [_P]),
        "faiss_RangeSearchResult_buffer_size": (C.c_size_t, [_P]),
        "faiss_RangeSearchResult_lims": (None, [_P, C.POINTER(C.POINTER(C.c_size_t))]),
        "faiss_RangeSearchResult_labels": (None, [_P, C.POINTER(C.POINTER(C.c_int64)),
                                                  C.POINTER(C.POINTER(C.c_float))]),
        "faiss_Index_range_search": (C.c_int, [_P, _I64, _P, C.c_float, _P]),
        "faiss_amd_Index_range_search_with_params": (C.c_int, [_P, _I64, _P, C.c_float, _P, _P]),
        "faiss_IndexIVF_range_search_preassigned": (C.c_int, [_P, _I64, _P, C.c_float, _P, _P,
                                                              _P]),
        "faiss_Index_reset": (C.c_int, [_P]),
        "faiss_SearchParametersIVF_new": (C.c_int, [C.POINTER(_P)]),
        "faiss_SearchParametersIVF_new_with": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, C.c_size_t]),
        "faiss_SearchParametersIVF_free": (None, [_P]),
        "faiss_SearchParametersIVF_nprobe": (C.c_size_t, [_P]),
        "faiss_SearchParametersIVF_set_nprobe": (None, [_P, C.c_size_t]),
        "faiss_amd_SearchParametersIVF_set_quantizer_efSearch": (None, [_P, C.c_int]),
        "faiss_IndexFlat_new_with": (C.c_int, [C.POINTER(_P), _I64, C.c_int]),
        "faiss_IndexFlatL2_new_with": (C.c_int, [C.POINTER(_P), _I64]),
        "faiss_IndexFlatIP_new_with": (C.c_int, [C.POINTER(_P), _I64]),
        "faiss_IndexFlat_xb": (None, [_P, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_size_t)]),
        "faiss_IndexIVF_nlist": (C.c_size_t, [_P]),
        "faiss_IndexIVF_nprobe": (C.c_size_t, [_P]),
        "faiss_IndexIVF_set_nprobe": (None, [_P, C.c_size_t]),
        "faiss_SearchParametersIVF_max_codes": (C.c_size_t, [_P]),
        "faiss_IDSelector_is_member": (C.c_int, [_P, _I64]),
        "faiss_IDSelector_free": (None, [_P]),
        "faiss_IDSelectorRange_new": (C.c_int, [C.POINTER(_P), _I64, _I64]),
        "faiss_IDSelectorBatch_new": (C.c_int, [C.POINTER(_P), C.c_size_t, _P]),
        "faiss_amd_IDSelectorArray_new": (C.c_int, [C.POINTER(_P), C.c_size_t, _P]),
        "faiss_IDSelectorBitmap_new": (C.c_int, [C.POINTER(_P), C.c_size_t, _P]),
        "faiss_IDSelectorNot_new": (C.c_int, [C.POINTER(_P), _P]),
        "faiss_IDSelectorAnd_new": (C.c_int, [C.POINTER(_P), _P, _P]),
        "faiss_IDSelectorOr_new": (C.c_int, [C.POINTER(_P), _P, _P]),
        "faiss_IDSelectorXOr_new": (C.c_int, [C.POINTER(_P), _P, _P]),
        "faiss_SearchParameters_new": (C.c_int, [C.POINTER(_P), _P]),
        "faiss_SearchParameters_free": (None, [_P]),
        "faiss_SearchParametersIVF_set_max_codes": (None, [_P, C.c_size_t]),
        "faiss_amd_IndexIVFPQ_set_use_precomputed_table": (C.c_int, [_P, C.c_int]),
        "faiss_amd_IndexIVF_max_codes": (C.c_size_t, [_P]),
        "faiss_amd_IndexIVF_set_max_codes": (None, [_P, C.c_size_t]),
        "faiss_amd_IndexIVF_parallel_mode": (C.c_int, [_P]),
        "faiss_amd_IndexIVF_set_parallel_mode": (None, [_P, C.c_int]),
        "faiss_IndexIVF_quantizer": (_P, [_P]),
        "faiss_IndexIVF_own_fields": (C.c_int, [_P]),
        "faiss_IndexIVF_set_own_fields": (None, [_P, C.c_int]),
        "faiss_IndexIVF_search_preassigned": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P, C.c_int]),
        "faiss_IndexIVF_get_list_size": (C.c_size_t, [_P, C.c_size_t]),
        "faiss_IndexIVF_invlists_get_ids": (None, [_P, C.c_size_t, _P]),
        "faiss_amd_IndexIVF_invlists_get_codes": (None, [_P, C.c_size_t, _P]),
        "faiss_amd_IndexIVF_code_size": (C.c_size_t, [_P]),
        "faiss_IndexIVFStats_reset": (None, [_P]),
        "faiss_get_indexIVF_stats": (C.POINTER(IndexIVFStats), []),
        "faiss_amd_IndexIVF_search_stats": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P]),
        "faiss_amd_IndexIVF_search_preassigned_stats": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P, C.c_int, _P, _P, _P]),
        "faiss_amd_IndexHNSW_search_stats": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _P]),
        "faiss_amd_get_hnsw_stats": (C.POINTER(HNSWStats), []),
        "faiss_amd_HNSWStats_reset": (None, []),
        "faiss_amd_get_hnsw_row_stats": (None, [C.c_void_p, C.c_void_p]),
        "faiss_amd_get_hnsw_replay_stats": (None, [C.c_void_p, C.c_void_p, C.c_void_p]),
        "faiss_amd_fold_device_stats": (C.c_int, [_P]),
        "faiss_amd_set_interrupt_timeout": (None, [C.c_double]),
        "faiss_IndexIVFFlat_new_with": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, C.c_size_t]),
        "faiss_IndexIVFFlat_new_with_metric": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, C.c_size_t, C.c_int]),
        "faiss_amd_IndexIVFPQ_new_with": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]),
        "faiss_amd_IndexIVFPQ_pq_centroids": (None, [_P, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_size_t)]),
        "faiss_amd_IndexIVFPQ_info": (C.c_int, [_P, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "faiss_amd_IndexHNSWFlat_new_with": (C.c_int, [C.POINTER(_P), C.c_int, C.c_int, C.c_int]),
        "faiss_amd_IndexHNSW_efSearch": (C.c_int, [_P]),
        "faiss_amd_IndexHNSW_set_efSearch": (None, [_P, C.c_int]),
        "faiss_amd_IndexHNSW_efConstruction": (C.c_int, [_P]),
        "faiss_amd_IndexHNSW_set_efConstruction": (None, [_P, C.c_int]),
        "faiss_amd_IndexHNSW_storage": (_P, [_P]),
        "faiss_amd_IndexHNSW_graph": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.POINTER(C.c_size_t)), C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.POINTER(C.c_int32))]),
        "faiss_amd_IndexShardsIVF_new": (C.c_int, [C.POINTER(_P), _P, C.c_size_t, C.c_int, C.c_int]),
        "faiss_amd_IndexShardsIVF_add_shard": (C.c_int, [_P, _P]),
        "faiss_amd_IndexShardsIVF_count": (C.c_int, [_P]),
        "faiss_amd_IndexShardsIVF_shard": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
        "faiss_amd_IndexIVF_copy_subset_to": (C.c_int, [_P, _P, C.c_int, C.c_int64, C.c_int64,
                                                        C.POINTER(C.c_size_t)]),
        "faiss_amd_index_ivf_to_shards": (C.c_int, [_P, C.c_int, C.c_int, _P, C.POINTER(_P)]),
        "faiss_write_index": (C.c_int, [_P, _P]),
        "faiss_write_index_fname": (C.c_int, [_P, C.c_char_p]),
        "faiss_amd_write_index_ondisk": (C.c_int, [_P, C.c_char_p, C.c_char_p]),
        "faiss_read_index": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
        "faiss_read_index_fname": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_P)]),
        "faiss_index_factory": (C.c_int, [C.POINTER(_P), C.c_int, C.c_char_p, C.c_int]),
        "faiss_ParameterSpace_new": (C.c_int, [C.POINTER(_P)]),
        "faiss_ParameterSpace_free": (None, [_P]),
        "faiss_ParameterSpace_set_index_parameter": (C.c_int, [_P, _P, C.c_char_p, C.c_double]),
        "faiss_amd_merge_knn_results": (C.c_int, [C.c_size_t, C.c_size_t, C.c_int, _P, _P, _P, _P, C.c_int]),
        "faiss_amd_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "faiss_amd_set_device": (C.c_int, [C.c_int]),
        "faiss_amd_Index_sync_device": (C.c_int, [_P]),
        "faiss_amd_Index_search_device": (C.c_int, [_P, _I64, _P, _I64, _P, _P, _P]),
        "faiss_amd_IndexIVF_search_preassigned_device": (C.c_int, [_P, _I64, _P, _I64, C.c_int, _P, _P, _P, _P, _P]),
        "faiss_amd_IndexIVF_quantize_device": (C.c_int, [_P, _I64, _P, C.c_int, _P, _P, _P]),
        "faiss_amd_merge_knn_results_device": (C.c_int, [C.c_size_t, C.c_size_t, C.c_int, _P, _P, _P, _P, C.c_int, _P]),
        "faiss_amd_set_kernel_timing": (C.c_int, [C.c_int]),
        "faiss_amd_set_search_slices": (C.c_int, [C.c_int]),
        "faiss_amd_set_kernel_timing_filter": (C.c_int, [C.c_char_p]),
        "faiss_amd_Index_type": (C.c_char_p, [_P]),
        "faiss_amd_reset_kernel_times": (C.c_int, [_P]),
        "faiss_amd_float_rand": (C.c_int, [_P, C.c_size_t, C.c_int64]),
        "faiss_amd_float_rand_rows": (C.c_int, [_P, _I64, C.c_int, C.c_int64, _I64, _I64, _I64]),
        "faiss_amd_last_kernel_times": (C.c_int, [_P, C.POINTER(C.c_int), _P, _P, _P]),
        "faiss_amd_IndexIVF_debug_rows": (C.c_int, [_P, C.c_int, _I64, _I64, _P,
                                                    C.POINTER(C.c_size_t), C.POINTER(C.c_int64)]),
        "faiss_clone_index": (C.c_int, [_P, C.POINTER(_P)]),
        "faiss_Index_reconstruct": (C.c_int, [_P, _I64, _P]),
        "faiss_Index_reconstruct_n": (C.c_int, [_P, _I64, _I64, _P]),
        "faiss_Index_assign": (C.c_int, [_P, _I64, _P, _P, _I64]),
        "faiss_IndexIVF_imbalance_factor": (C.c_double, [_P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


EXPORTED_SYMBOLS = None  # filled lazily by exported_symbols()


def exported_symbols():
    """Names declared in include/faiss_amd_c.h (parsed from the header)."""
    import re
    hdr = os.path.join(_HERE, "..", "include", "faiss_amd_c.h")
    txt = open(hdr).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(faiss_\w+)\s*\(", txt)))


def _check(rc):
    if rc != 0:
        msg = lib().faiss_get_last_error().decode(errors="replace")
        raise FaissError(f"faiss_amd error {rc}: {msg}")


def _f32(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    assert x.ndim == 2
    return x


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------- Index
class Index:
    """Wraps a FaissIndex* handle (owned unless `owner` is another Index)."""

    def __init__(self, handle, owner=None):
        self.h = C.c_void_p(handle) if not isinstance(handle, C.c_void_p) else handle
        self._owner = owner
        self._keep = []

    def __del__(self):
        try:
            if self._owner is None and self.h and self.h.value and _lib is not None:
                _lib.faiss_Index_free(self.h)
                self.h = C.c_void_p(None)
        except Exception:
            pass

    def release(self):
        """Give up ownership (e.g. after handing the handle to an owner)."""
        self._owner = True

    @property
    def d(self):
        return lib().faiss_Index_d(self.h)

    @property
    def ntotal(self):
        return lib().faiss_Index_ntotal(self.h)

    @property
    def is_trained(self):
        return bool(lib().faiss_Index_is_trained(self.h))

    @property
    def metric_type(self):
        return lib().faiss_Index_metric_type(self.h)

    @property
    def verbose(self):
        return bool(lib().faiss_Index_verbose(self.h))

    @verbose.setter
    def verbose(self, v):
        lib().faiss_Index_set_verbose(self.h, int(bool(v)))

    def train(self, x):
        x = _f32(x)
        _check(lib().faiss_Index_train(self.h, x.shape[0], _ptr(x)))

    def add(self, x):
        x = _f32(x)
        _check(lib().faiss_Index_add(self.h, x.shape[0], _ptr(x)))

    def add_with_ids(self, x, ids):
        x = _f32(x)
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        _check(lib().faiss_Index_add_with_ids(self.h, x.shape[0], _ptr(x), _ptr(ids)))

    def search(self, x, k, params=None):
        x = _f32(x)
        n = x.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        if params is None:
            _check(lib().faiss_Index_search(self.h, n, _ptr(x), k, _ptr(D), _ptr(I)))
        else:
            _check(lib().faiss_Index_search_with_params(self.h, n, _ptr(x), k, params.h,
                                                        _ptr(D), _ptr(I)))
        return D, I

    def range_search(self, x, radius, params=None):
        """faiss Index.range_search: (lims [n+1], D, I) in the reference's scan order."""
        x = _f32(x)
        n = x.shape[0]
        return _range_call(n, lambda r: (
            lib().faiss_Index_range_search(self.h, n, _ptr(x), float(radius), r)
            if params is None else
            lib().faiss_amd_Index_range_search_with_params(self.h, n, _ptr(x), float(radius),
                                                           params.h, r)))

    def reset(self):
        _check(lib().faiss_Index_reset(self.h))

    # ---- device-resident extensions (pointers are ints, e.g. tensor.data_ptr())
    def sync_device(self):
        _check(lib().faiss_amd_Index_sync_device(self.h))

    def search_device(self, n, x_ptr, k, D_ptr, I_ptr, stream=None):
        _check(lib().faiss_amd_Index_search_device(self.h, n, C.c_void_p(x_ptr), k,
                                                   C.c_void_p(D_ptr), C.c_void_p(I_ptr),
                                                   C.c_void_p(stream or 0)))

    def fold_device_stats(self):
        """Fold device-side counters (hnsw_stats) of device-API searches."""
        _check(lib().faiss_amd_fold_device_stats(self.h))

    def reset_kernel_times(self):
        _check(lib().faiss_amd_reset_kernel_times(self.h))

    def kernel_times(self):
        n = C.c_int(0)
        _check(lib().faiss_amd_last_kernel_times(self.h, C.byref(n), None, None, None))
        cnt = n.value
        names = C.create_string_buffer(32 * max(cnt, 1))
        ms = (C.c_double * max(cnt, 1))()
        un = (C.c_double * max(cnt, 1))()
        _check(lib().faiss_amd_last_kernel_times(self.h, C.byref(n), names, ms, un))
        out = []
        for i in range(cnt):
            nm = names.raw[32 * i:32 * (i + 1)].split(b"\0")[0].decode()
            out.append((nm, ms[i], un[i]))
        return out


class IndexFlat(Index):
    def __init__(self, d=None, metric=METRIC_L2, handle=None, owner=None):
        if handle is None:
            p = C.c_void_p()
            _check(lib().faiss_IndexFlat_new_with(C.byref(p), d, metric))
            handle = p
        super().__init__(handle, owner)

    @property
    def xb(self):
        p = C.POINTER(C.c_float)()
        n = C.c_size_t(0)
        lib().faiss_IndexFlat_xb(self.h, C.byref(p), C.byref(n))
        if n.value == 0:
            return np.zeros((0, self.d), dtype=np.float32)
        return np.ctypeslib.as_array(p, shape=(n.value,)).reshape(-1, self.d).copy()


class IndexFlatL2(IndexFlat):
    def __init__(self, d):
        super().__init__(d, METRIC_L2)


class IndexFlatIP(IndexFlat):
    def __init__(self, d):
        super().__init__(d, METRIC_INNER_PRODUCT)


class IndexHNSW(Index):
    @property
    def efSearch(self):
        return lib().faiss_amd_IndexHNSW_efSearch(self.h)

    @efSearch.setter
    def efSearch(self, v):
        lib().faiss_amd_IndexHNSW_set_efSearch(self.h, int(v))

    @property
    def efConstruction(self):
        return lib().faiss_amd_IndexHNSW_efConstruction(self.h)

    @efConstruction.setter
    def efConstruction(self, v):
        lib().faiss_amd_IndexHNSW_set_efConstruction(self.h, int(v))

    def search_stats(self, x, k):
        """IndexHNSW::search_stats: (D, I, per-query QueryLatencyStats records)."""
        x = _f32(x)
        n = x.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        st = np.zeros(n, dtype=QUERY_LATENCY_DTYPE)
        _check(lib().faiss_amd_IndexHNSW_search_stats(self.h, n, _ptr(x), k, None, _ptr(D),
                                                      _ptr(I), _ptr(st)))
        return D, I, st

    def storage_vectors(self):
        h = lib().faiss_amd_IndexHNSW_storage(self.h)
        return IndexFlat(handle=h, owner=self).xb

    def graph(self):
        """(entry_point, max_level, levels, offsets, neighbors, cum_nneighbor_per_level)."""
        ep, ml = C.c_int(), C.c_int()
        nn, nc = C.c_size_t(), C.c_size_t()
        lv = C.POINTER(C.c_int32)()
        of = C.POINTER(C.c_size_t)()
        nb = C.POINTER(C.c_int32)()
        cu = C.POINTER(C.c_int32)()
        _check(lib().faiss_amd_IndexHNSW_graph(self.h, C.byref(ep), C.byref(ml), C.byref(nn),
                                               C.byref(nc), C.byref(lv), C.byref(of),
                                               C.byref(nb), C.byref(cu)))
        nt = self.ntotal
        levels = np.ctypeslib.as_array(lv, shape=(nt,)).copy() if nt else np.zeros(0, np.int32)
        offsets = np.ctypeslib.as_array(of, shape=(nt + 1,)).copy()
        neighbors = (np.ctypeslib.as_array(nb, shape=(nn.value,)).copy() if nn.value
                     else np.zeros(0, np.int32))
        cum = np.ctypeslib.as_array(cu, shape=(nc.value,)).copy()
        return ep.value, ml.value, levels, offsets, neighbors, cum


class IndexHNSWFlat(IndexHNSW):
    def __init__(self, d=None, M=32, metric=METRIC_L2, handle=None, owner=None):
        if handle is None:
            p = C.c_void_p()
            _check(lib().faiss_amd_IndexHNSWFlat_new_with(C.byref(p), d, M, metric))
            handle = p
        super().__init__(handle, owner)


class IndexIVF(Index):
    @property
    def nlist(self):
        return lib().faiss_IndexIVF_nlist(self.h)

    @property
    def nprobe(self):
        return lib().faiss_IndexIVF_nprobe(self.h)

    @nprobe.setter
    def nprobe(self, v):
        lib().faiss_IndexIVF_set_nprobe(self.h, int(v))

    @property
    def max_codes(self):
        return lib().faiss_amd_IndexIVF_max_codes(self.h)

    @max_codes.setter
    def max_codes(self, v):
        lib().faiss_amd_IndexIVF_set_max_codes(self.h, int(v))

    @property
    def parallel_mode(self):
        return lib().faiss_amd_IndexIVF_parallel_mode(self.h)

    @parallel_mode.setter
    def parallel_mode(self, v):
        lib().faiss_amd_IndexIVF_set_parallel_mode(self.h, int(v))

    @property
    def code_size(self):
        return lib().faiss_amd_IndexIVF_code_size(self.h)

    @property
    def quantizer(self):
        h = lib().faiss_IndexIVF_quantizer(self.h)
        return _wrap(h, owner=self)

    def get_list_size(self, l):
        return lib().faiss_IndexIVF_get_list_size(self.h, l)

    def list_ids(self, l):
        n = self.get_list_size(l)
        out = np.empty(n, dtype=np.int64)
        if n:
            lib().faiss_IndexIVF_invlists_get_ids(self.h, l, _ptr(out))
        return out

    def list_codes(self, l):
        n = self.get_list_size(l)
        out = np.empty(n * self.code_size, dtype=np.uint8)
        if n:
            lib().faiss_amd_IndexIVF_invlists_get_codes(self.h, l, _ptr(out))
        return out.reshape(n, self.code_size)

    def debug_rows(self, what, row0=0, n=None):
        """HBM arena rows [row0, row0 + n) as bytes [n][row_bytes] (diagnostic):
        what 0 = code rows, 1 = row -> list table, 2 = the filter's stream image.
        n = None returns (row_bytes, arena_rows) only."""
        rb, rows = C.c_size_t(), C.c_int64()
        _check(lib().faiss_amd_IndexIVF_debug_rows(self.h, int(what), 0, 0, None, C.byref(rb),
                                                   C.byref(rows)))
        if n is None:
            return rb.value, rows.value
        out = np.empty((int(n), rb.value), dtype=np.uint8)
        _check(lib().faiss_amd_IndexIVF_debug_rows(self.h, int(what), int(row0), int(n),
                                                   _ptr(out), None, None))
        return out

    def search_preassigned(self, x, k, assign, centroid_dis, store_pairs=False):
        """centroid_dis may be None (NULL), as the reference allows where its
        scanner does not read it."""
        x = _f32(x)
        n = x.shape[0]
        assign = np.ascontiguousarray(assign, dtype=np.int64)
        if centroid_dis is not None:
            centroid_dis = np.ascontiguousarray(centroid_dis, dtype=np.float32)
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        _check(lib().faiss_IndexIVF_search_preassigned(
            self.h, n, _ptr(x), k, _ptr(assign),
            _ptr(centroid_dis) if centroid_dis is not None else None, _ptr(D), _ptr(I),
            int(store_pairs)))
        return D, I

    def range_search_preassigned(self, x, radius, assign, centroid_dis=None):
        x = _f32(x)
        n = x.shape[0]
        assign = np.ascontiguousarray(assign, dtype=np.int64)
        if assign.shape != (n, min(self.nprobe, self.nlist)):
            raise ValueError("assign must be [n, nprobe] (the index's nprobe)")
        cd = (np.zeros(assign.shape, np.float32) if centroid_dis is None
              else np.ascontiguousarray(centroid_dis, dtype=np.float32))
        return _range_call(n, lambda r: lib().faiss_IndexIVF_range_search_preassigned(
            self.h, n, _ptr(x), float(radius), _ptr(assign), _ptr(cd), r))

    def search_stats(self, x, k, params=None):
        """IndexIVF::search_stats: (D, I, per-query QueryLatencyStats records)."""
        x = _f32(x)
        n = x.shape[0]
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        st = np.zeros(n, dtype=QUERY_LATENCY_DTYPE)
        _check(lib().faiss_amd_IndexIVF_search_stats(self.h, n, _ptr(x), k,
                                                     params.h if params is not None else None,
                                                     _ptr(D), _ptr(I), _ptr(st)))
        return D, I, st

    def search_preassigned_stats(self, x, k, assign, centroid_dis, ivf_stats=None):
        """IndexIVF::search_preassigned_stats: (D, I, per-query records)."""
        x = _f32(x)
        n = x.shape[0]
        assign = np.ascontiguousarray(assign, dtype=np.int64)
        centroid_dis = np.ascontiguousarray(centroid_dis, dtype=np.float32)
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        st = np.zeros(n, dtype=QUERY_LATENCY_DTYPE)
        _check(lib().faiss_amd_IndexIVF_search_preassigned_stats(
            self.h, n, _ptr(x), k, _ptr(assign), _ptr(centroid_dis), _ptr(D), _ptr(I), 0, None,
            C.byref(ivf_stats) if ivf_stats is not None else None, _ptr(st)))
        return D, I, st

    def quantize_device(self, n, x_ptr, nprobe, cdis_ptr, assign_ptr, stream=None):
        _check(lib().faiss_amd_IndexIVF_quantize_device(self.h, n, C.c_void_p(x_ptr), nprobe,
                                                        C.c_void_p(cdis_ptr),
                                                        C.c_void_p(assign_ptr),
                                                        C.c_void_p(stream or 0)))

    def search_preassigned_device(self, n, x_ptr, k, nprobe, assign_ptr, cdis_ptr, D_ptr,
                                  I_ptr, stream=None):
        _check(lib().faiss_amd_IndexIVF_search_preassigned_device(
            self.h, n, C.c_void_p(x_ptr), k, nprobe, C.c_void_p(assign_ptr),
            C.c_void_p(cdis_ptr), C.c_void_p(D_ptr), C.c_void_p(I_ptr),
            C.c_void_p(stream or 0)))

    def invlists_arrays(self):
        """(list_offsets[nlist+1], codes[ntotal, code_size] u8, ids[ntotal] i64)."""
        nl = self.nlist
        sizes = np.array([self.get_list_size(l) for l in range(nl)], dtype=np.int64)
        off = np.zeros(nl + 1, dtype=np.int64)
        off[1:] = np.cumsum(sizes)
        codes = np.empty((int(off[-1]), self.code_size), dtype=np.uint8)
        ids = np.empty(int(off[-1]), dtype=np.int64)
        for l in range(nl):
            if sizes[l]:
                codes[off[l]:off[l + 1]] = self.list_codes(l)
                ids[off[l]:off[l + 1]] = self.list_ids(l)
        return off, codes, ids


class IndexIVFFlat(IndexIVF):
    def __init__(self, quantizer=None, d=None, nlist=None, metric=METRIC_L2, handle=None,
                 owner=None):
        if handle is None:
            p = C.c_void_p()
            _check(lib().faiss_IndexIVFFlat_new_with_metric(C.byref(p), quantizer.h, d, nlist,
                                                            metric))
            handle = p
            self._q = quantizer  # quantizer must outlive the index (own_fields = false)
        super().__init__(handle, owner)


class IndexIVFPQ(IndexIVF):
    def __init__(self, quantizer=None, d=None, nlist=None, M=None, nbits=8, metric=METRIC_L2,
                 handle=None, owner=None):
        if handle is None:
            p = C.c_void_p()
            _check(lib().faiss_amd_IndexIVFPQ_new_with(C.byref(p), quantizer.h, d, nlist, M,
                                                       nbits, metric))
            handle = p
            self._q = quantizer
        super().__init__(handle, owner)

    def pq_info(self):
        M, nb = C.c_size_t(), C.c_size_t()
        br, up = C.c_int(), C.c_int()
        _check(lib().faiss_amd_IndexIVFPQ_info(self.h, C.byref(M), C.byref(nb), C.byref(br),
                                               C.byref(up)))
        return dict(M=M.value, nbits=nb.value, by_residual=bool(br.value),
                    use_precomputed_table=up.value)

    @property
    def use_precomputed_table(self):
        return self.pq_info()["use_precomputed_table"]

    @use_precomputed_table.setter
    def use_precomputed_table(self, v):
        _check(lib().faiss_amd_IndexIVFPQ_set_use_precomputed_table(self.h, int(v)))

    @property
    def pq_centroids(self):
        p = C.POINTER(C.c_float)()
        n = C.c_size_t(0)
        lib().faiss_amd_IndexIVFPQ_pq_centroids(self.h, C.byref(p), C.byref(n))
        info = self.pq_info()
        dsub = self.d // info["M"]
        return np.ctypeslib.as_array(p, shape=(n.value,)).reshape(
            info["M"], 1 << info["nbits"], dsub).copy()


class IndexShardsIVF(IndexIVF):
    """faiss/IndexShardsIVF.h: shards sharing one coarse quantizer; shards on
    other devices than the quantizer are searched over RCCL (shards.cpp)."""

    def __init__(self, quantizer, nlist, threaded=False, successive_ids=True):
        p = C.c_void_p()
        _check(lib().faiss_amd_IndexShardsIVF_new(C.byref(p), quantizer.h, nlist, int(threaded),
                                                  int(successive_ids)))
        self._q = quantizer
        self._shards = []
        super().__init__(p, None)

    def add_shard(self, idx):
        _check(lib().faiss_amd_IndexShardsIVF_add_shard(self.h, idx.h))
        self._shards.append(idx)

    def count(self):
        return lib().faiss_amd_IndexShardsIVF_count(self.h)

    def shard(self, i):
        """Shard i (a view owned by this index)."""
        s = C.c_void_p()
        _check(lib().faiss_amd_IndexShardsIVF_shard(self.h, i, C.byref(s)))
        return _wrap(s, owner=self)


class IDSelector:
    """faiss/impl/IDSelector.h selectors (membership evaluated on the GPU for
    every inverted-list row; non-members are skipped by the IVF scans)."""

    def __init__(self, h, keep=()):
        self.h = h
        self._keep = keep  # borrowed arrays / child selectors stay alive

    def is_member(self, i):
        return bool(lib().faiss_IDSelector_is_member(self.h, int(i)))

    def __del__(self):
        try:
            lib().faiss_IDSelector_free(self.h)
        except Exception:
            pass


def IDSelectorRange(imin, imax):
    p = C.c_void_p()
    _check(lib().faiss_IDSelectorRange_new(C.byref(p), int(imin), int(imax)))
    return IDSelector(p)


def IDSelectorBatch(ids):
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    p = C.c_void_p()
    _check(lib().faiss_IDSelectorBatch_new(C.byref(p), len(ids), _ptr(ids)))
    return IDSelector(p)


def IDSelectorArray(ids):
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    p = C.c_void_p()
    _check(lib().faiss_amd_IDSelectorArray_new(C.byref(p), len(ids), _ptr(ids)))
    return IDSelector(p, (ids,))


def IDSelectorBitmap(bitmap):
    bm = np.ascontiguousarray(bitmap, dtype=np.uint8)
    p = C.c_void_p()
    _check(lib().faiss_IDSelectorBitmap_new(C.byref(p), len(bm), _ptr(bm)))
    return IDSelector(p, (bm,))


def IDSelectorNot(sel):
    p = C.c_void_p()
    _check(lib().faiss_IDSelectorNot_new(C.byref(p), sel.h))
    return IDSelector(p, (sel,))


def _sel_binary(fn, a, b):
    p = C.c_void_p()
    _check(fn(C.byref(p), a.h, b.h))
    return IDSelector(p, (a, b))


def IDSelectorAnd(a, b):
    return _sel_binary(lib().faiss_IDSelectorAnd_new, a, b)


def IDSelectorOr(a, b):
    return _sel_binary(lib().faiss_IDSelectorOr_new, a, b)


def IDSelectorXOr(a, b):
    return _sel_binary(lib().faiss_IDSelectorXOr_new, a, b)


class SearchParametersIVF:
    def __init__(self, nprobe=1, max_codes=0, quantizer_efSearch=0, sel=None):
        p = C.c_void_p()
        _check(lib().faiss_SearchParametersIVF_new_with(C.byref(p), sel.h if sel else None,
                                                        nprobe, max_codes))
        self.h = p
        self._sel = sel
        if quantizer_efSearch:
            lib().faiss_amd_SearchParametersIVF_set_quantizer_efSearch(self.h,
                                                                       int(quantizer_efSearch))

    def __del__(self):
        try:
            lib().faiss_SearchParametersIVF_free(self.h)
        except Exception:
            pass


class ParameterSpace:
    def __init__(self):
        p = C.c_void_p()
        _check(lib().faiss_ParameterSpace_new(C.byref(p)))
        self.h = p

    def set_index_parameter(self, index, name, value):
        _check(lib().faiss_ParameterSpace_set_index_parameter(self.h, index.h, name.encode(),
                                                              float(value)))

    def __del__(self):
        try:
            lib().faiss_ParameterSpace_free(self.h)
        except Exception:
            pass


# ---------------------------------------------------------------- helpers
def _range_call(n, fn):
    """Run a range-search C call on a fresh RangeSearchResult and copy it out."""
    r = C.c_void_p()
    _check(lib().faiss_RangeSearchResult_new(C.byref(r), n))
    try:
        _check(fn(r))
        lp = C.POINTER(C.c_size_t)()
        lib().faiss_RangeSearchResult_lims(r, C.byref(lp))
        lims = np.ctypeslib.as_array(lp, shape=(n + 1,)).copy()
        tot = int(lims[-1])
        I = np.empty(tot, np.int64)
        D = np.empty(tot, np.float32)
        if tot:
            ip, dp = C.POINTER(C.c_int64)(), C.POINTER(C.c_float)()
            lib().faiss_RangeSearchResult_labels(r, C.byref(ip), C.byref(dp))
            I[:] = np.ctypeslib.as_array(ip, shape=(tot,))
            D[:] = np.ctypeslib.as_array(dp, shape=(tot,))
        return lims, D, I
    finally:
        lib().faiss_RangeSearchResult_free(r)


def _wrap(h, owner=None):
    """Wrap a raw FaissIndex* in the Python class of its dynamic type."""
    h = C.c_void_p(h) if not isinstance(h, C.c_void_p) else h
    t = lib().faiss_amd_Index_type(h).decode()
    if t == "IndexShardsIVF":
        return IndexShardsIVF.__new__(IndexShardsIVF)._init_from(h, owner)
    cls = {"IndexIVFPQ": IndexIVFPQ, "IndexIVFFlat": IndexIVFFlat,
           "IndexHNSWFlat": IndexHNSWFlat, "IndexFlat": IndexFlat}.get(t)
    if cls is None:
        return Index(h, owner)
    return cls(handle=h, owner=owner)


def index_factory(d, description, metric=METRIC_L2):
    p = C.c_void_p()
    _check(lib().faiss_index_factory(C.byref(p), d, description.encode(), metric))
    return _wrap(p)


def read_index(fname, io_flags=0):
    p = C.c_void_p()
    _check(lib().faiss_read_index_fname(str(fname).encode(), io_flags, C.byref(p)))
    return _wrap(p)


def write_index(index, fname):
    _check(lib().faiss_write_index_fname(index.h, str(fname).encode()))


def clone_index(index):
    """faiss.clone_index (c_api/clone_index_c.h): a deep copy."""
    p = C.c_void_p()
    _check(lib().faiss_clone_index(index.h, C.byref(p)))
    return _wrap(p)


def write_index_ondisk(index, fname, lists_fname):
    """IVF index file whose lists live in `lists_fname` (OnDiskInvertedLists
    layout, faiss/invlists/OnDiskInvertedLists.cpp:683-704)."""
    _check(lib().faiss_amd_write_index_ondisk(index.h, str(fname).encode(),
                                               str(lists_fname).encode()))


def merge_knn_results(Dall, Iall, keep_max=False):
    """faiss.merge_knn_results: Dall/Iall [nshard, n, k]."""
    Dall = np.ascontiguousarray(Dall, dtype=np.float32)
    Iall = np.ascontiguousarray(Iall, dtype=np.int64)
    ns, n, k = Dall.shape
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    _check(lib().faiss_amd_merge_knn_results(n, k, ns, _ptr(Dall), _ptr(Iall), _ptr(D), _ptr(I),
                                             METRIC_INNER_PRODUCT if keep_max else METRIC_L2))
    return D, I


def merge_knn_results_device(n, k, nshard, all_d_ptr, all_i_ptr, d_ptr, i_ptr, metric=METRIC_L2,
                             stream=None):
    _check(lib().faiss_amd_merge_knn_results_device(n, k, nshard, C.c_void_p(all_d_ptr),
                                                    C.c_void_p(all_i_ptr), C.c_void_p(d_ptr),
                                                    C.c_void_p(i_ptr), metric,
                                                    C.c_void_p(stream or 0)))


def float_rand(n, seed):
    """faiss.float_rand (bit-exact restatement, host)."""
    x = np.empty(n, dtype=np.float32)
    _check(lib().faiss_amd_float_rand(_ptr(x), n, seed))
    return x


def float_rand_rows(n_rows, d, seed, row0=0, step=1, nout=None):
    """Rows row0, row0+step, ... of float_rand(n_rows * d, seed) as [n_rows][d]."""
    if nout is None:
        nout = (n_rows - row0 + step - 1) // step
    x = np.empty((nout, d), dtype=np.float32)
    _check(lib().faiss_amd_float_rand_rows(_ptr(x), n_rows, d, seed, row0, step, nout))
    return x


def device_count():
    n = C.c_int(0)
    _check(lib().faiss_amd_device_count(C.byref(n)))
    return n.value


def set_device(dev):
    _check(lib().faiss_amd_set_device(int(dev)))


def set_search_slices(t):
    """Emulate a reference IndexIVF::search on t OpenMP threads: the batch is
    quantized in min(t, n) slices, each in the form its size selects
    (faiss/IndexIVF.cpp:359-368); 1 (the default) = one slice."""
    _check(lib().faiss_amd_set_search_slices(int(t)))


def set_kernel_timing(enable=True, only=None):
    """HIP-event timing of the kernel stages of later searches; `only`
    restricts it to the stage of that name (kernel_times() names)."""
    _check(lib().faiss_amd_set_kernel_timing_filter(only.encode() if only else None))
    _check(lib().faiss_amd_set_kernel_timing(int(bool(enable))))


def _shards_init_from(self, h, owner):
    Index.__init__(self, h, owner)
    self._shards = []
    return self


IndexShardsIVF._init_from = _shards_init_from

# faiss/invlists/InvertedLists.h:36-43
SUBSET_TYPE_ID_RANGE, SUBSET_TYPE_ID_MOD, SUBSET_TYPE_ELEMENT_RANGE = 0, 1, 2
SUBSET_TYPE_INVLIST_FRACTION, SUBSET_TYPE_INVLIST = 3, 4


def copy_subset_to(src, dst, subset_type, a1, a2):
    """IndexIVF::copy_subset_to (faiss/IndexIVF.cpp:1732-1739): entries of
    src selected by (subset_type, a1, a2) appended to dst; returns the count."""
    n = C.c_size_t()
    _check(lib().faiss_amd_IndexIVF_copy_subset_to(src.h, dst.h, int(subset_type), int(a1),
                                                    int(a2), C.byref(n)))
    return n.value


def index_ivf_to_shards(src, nshard, shard_type=1, devices=None):
    """GpuCloner.cpp:283-420 for IVF: nshard shards of src (shard_type 1 id
    modulo, 2 id range, 4 list range), shard i on devices[i]."""
    p = C.c_void_p()
    dv = None
    if devices is not None:
        dv = (C.c_int * nshard)(*[int(x) for x in devices])
    _check(lib().faiss_amd_index_ivf_to_shards(src.h, int(nshard), int(shard_type),
                                                C.cast(dv, C.c_void_p) if dv is not None else None,
                                                C.byref(p)))
    return _wrap(p)
