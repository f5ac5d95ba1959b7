"""CPU: the C-ABI library loads and exports every symbol include/*.h declares."""
import ctypes
import os
import subprocess


def test_library_exports_all_header_symbols(amd):
    L = amd.lib()
    syms = amd.exported_symbols()
    assert len(syms) >= 60
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_nm_dynamic_symbols(amd):
    out = subprocess.run(["nm", "-D", "--defined-only", amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    defined = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for s in amd.exported_symbols():
        assert s in defined, s


def test_library_has_gfx950_code_object(amd):
    blob = open(amd.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_errors_are_reported_without_gpu(amd):
    # factory parsing error is a pure host-side FaissException -> rc -2
    p = ctypes.c_void_p()
    rc = amd.lib().faiss_index_factory(ctypes.byref(p), 16, b"LSH", 1)
    assert rc == -2
    assert b"unsupported" in amd.lib().faiss_get_last_error()


def test_factory_and_type_query_without_gpu(amd):
    idx = amd.index_factory(32, "IVF16,Flat")
    assert type(idx).__name__ == "IndexIVFFlat"
    assert idx.nlist == 16 and idx.d == 32 and not idx.is_trained
    pq = amd.index_factory(32, "IVF16,PQ8x8np")
    assert type(pq).__name__ == "IndexIVFPQ"
    assert pq.pq_info()["M"] == 8 and pq.code_size == 8
    h = amd.index_factory(32, "IVF16_HNSW32,Flat")
    assert type(h.quantizer).__name__ == "IndexHNSWFlat"
    f = amd.index_factory(32, "Flat")
    assert type(f).__name__ == "IndexFlat"
