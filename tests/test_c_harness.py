"""Compiled consumers of the drop-in boundary.

tests/c/harness.c is the reference benchmark harness's search sequence
(tutorial/cpp/benchmark-hnsw-ivf/benchmark_hnsw_ivf.cpp:361-404: read_index
with IO_FLAG_MMAP -> nprobe / quantizer efSearch / parallel_mode ->
IndexIVF::search_stats -> QPS and latency percentiles) written against
include/faiss_amd_c.h and built by a plain C compiler; tests/c/harness.cpp is
the same sequence against the C++ mirror include/faiss_amd.h.  The CPU tests
compile and link both with warnings as errors (header drift, C-vs-C++
breakage); the GPU test runs them on a reference-shaped HNSW -> IVF index and
checks their results against the Python mirror and the oracle, bit for bit.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "hnsw-ivf_amd", "lib")


def compile_c(out):
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", f"-I{INC}",
                    os.path.join(ROOT, "tests", "c", "harness.c"), "-o", out, f"-L{LIBDIR}",
                    "-lfaiss_amd", f"-Wl,-rpath,{LIBDIR}"], check=True, capture_output=True)


def compile_cpp(out):
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", f"-I{INC}",
                    os.path.join(ROOT, "tests", "c", "harness.cpp"), "-o", out, f"-L{LIBDIR}",
                    "-lfaiss_amd", f"-Wl,-rpath,{LIBDIR}", "-L/opt/rocm/lib", "-lamdhip64"],
                   check=True, capture_output=True)


def test_c_harness_compiles(tmp_path):
    compile_c(str(tmp_path / "harness_c"))
    # a bad index file name comes back as the reference's -2 / last-error path
    r = subprocess.run([str(tmp_path / "harness_c"), str(tmp_path / "missing.faiss"), "10", "10",
                        "8", "16", "1", str(tmp_path / "o.bin")], capture_output=True, text=True)
    assert r.returncode == 1 and "could not open" in r.stderr


def test_cpp_harness_compiles(tmp_path):
    compile_cpp(str(tmp_path / "harness_cpp"))


@pytest.mark.gpu
def test_harness_sequence_on_gpu(amd, orc, gpu, tmp_path):
    d, nb, nq, k, nprobe, ef = 64, 60_000, 500, 10, 16, 48
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, "IVF256_HNSW32,Flat")
    idx.train(xb[:20_000])
    idx.add(xb)
    fn = str(tmp_path / "hnswivf.faiss")
    amd.write_index(idx, fn)
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    # the Python mirror on a freshly mapped copy of the same file
    ref_idx = amd.read_index(fn, amd.IO_FLAG_MMAP)
    ref_idx.nprobe = nprobe
    ref_idx.quantizer.efSearch = ef
    Dp, Ip, _ = ref_idx.search_stats(xq, k)
    o = orc.IVFOracle.from_index(ref_idx)
    Do, Io, _, _ = o.search(xq, k, nprobe, efSearch=ef, nslices=1)
    assert np.array_equal(Ip, Io) and np.array_equal(Dp, Do)
    for name, comp in (("harness_c", compile_c), ("harness_cpp", compile_cpp)):
        exe = str(tmp_path / name)
        comp(exe)
        out = str(tmp_path / f"{name}.bin")
        r = subprocess.run([exe, fn, str(nq), str(k), str(nprobe), str(ef), "5678", out],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        summ = json.loads(r.stdout.strip().splitlines()[-1])
        assert summ["nq"] == nq and summ["mean_ms"] > 0
        raw = np.fromfile(out, dtype=np.uint8)
        D = raw[:nq * k * 4].view(np.float32).reshape(nq, k)
        I = raw[nq * k * 4:].view(np.int64).reshape(nq, k)
        assert np.array_equal(I, Ip), name
        assert np.array_equal(D, Dp), name
