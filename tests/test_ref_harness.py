"""The C++ drop-in: the reference's own benchmark programs
(tutorial/cpp/benchmark-*/benchmark_*.cpp) compiled in place and unchanged
against include/faiss (this library's classes under namespace faiss) and
linked to libfaiss_amd.so (oracle/ref/Makefile `harness`).

CPU: every <faiss/...> header compiles on its own; the four harnesses compile
and link (needs /root/reference, i.e. this container).
GPU: the compiled benchmark_hnsw_ivf and benchmark_ivf run their whole flow
on a small synthetic SIFT-shaped set — train, write the empty shell, read it
back with flags 0, add in 100k chunks, write, read with IO_FLAG_MMAP, set
nprobe / efSearch, search_stats — and the recall they write to their CSV
equals the recall of the same index built through this library's API and of
the oracle's results on it (data: faiss float_rand streams; ground truth:
exact top-10 by numpy)."""
import csv
import glob
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
HDIR = os.path.join(ROOT, "oracle", "_ref", "harness")
HARNESSES = ["benchmark_hnsw_ivf", "benchmark_ivf", "benchmark_ivf_ondisk", "benchmark_hnsw",
             "example_c", "example_c_refhdr"]
HEADERS = sorted(os.path.relpath(p, os.path.join(ROOT, "include"))
                 for p in glob.glob(os.path.join(ROOT, "include", "faiss", "**", "*.h"),
                                    recursive=True))


@pytest.mark.parametrize("hdr", HEADERS)
def test_faiss_header_compiles_alone(hdr, tmp_path):
    src = tmp_path / "tu.cpp"
    src.write_text(f"#include <{hdr}>\nint main() {{ return 0; }}\n")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{os.path.join(ROOT, 'include')}", str(src)], check=True)


C_HEADERS = sorted(os.path.relpath(p, os.path.join(ROOT, "include", "faiss", "c_api"))
                   for p in glob.glob(os.path.join(ROOT, "include", "faiss", "c_api", "**", "*.h"),
                                      recursive=True))


@pytest.mark.parametrize("hdr", C_HEADERS)
def test_c_api_header_compiles_alone(hdr, tmp_path):
    """Each reference C header name (c_api/*.h) as a plain C99 translation
    unit, both as "X_c.h" from the c_api directory and as <faiss/c_api/X_c.h>."""
    for inc, flag in ((f'"{hdr}"', ["-I-", f"-I{os.path.join(ROOT, 'include', 'faiss', 'c_api')}"]),
                      (f"<faiss/c_api/{hdr}>", [f"-I{os.path.join(ROOT, 'include')}"])):
        src = tmp_path / "tu.c"
        src.write_text(f"#include {inc}\nint main(void) {{ return 0; }}\n")
        r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-pedantic",
                            *flag, str(src)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_faiss_names_are_the_library_types(tmp_path):
    """faiss::X is faiss_amd::X (not a copy): dynamic_cast, catch and
    overload resolution see one type."""
    src = tmp_path / "tu.cpp"
    src.write_text("""
#include <faiss/IndexIVFFlat.h>
#include <faiss/IndexHNSW.h>
#include <faiss/index_io.h>
#include <faiss/impl/FaissAssert.h>
#include <faiss/impl/AuxIndexStructures.h>
#include <type_traits>
static_assert(std::is_same<faiss::IndexIVFFlat, faiss_amd::IndexIVFFlat>::value, "");
static_assert(std::is_same<faiss::Index, faiss_amd::Index>::value, "");
static_assert(std::is_same<faiss::FaissException, faiss_amd::FaissException>::value, "");
static_assert(std::is_base_of<faiss::InterruptCallback, faiss::TimeoutCallback>::value, "");
static_assert(std::is_same<faiss::idx_t, int64_t>::value, "");
static_assert(faiss::METRIC_L2 == 1 && faiss::METRIC_INNER_PRODUCT == 0, "");
namespace faiss { int caller_extension = 1; }  // namespace faiss stays open
int main() { return faiss::caller_extension - 1; }
""")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{os.path.join(ROOT, 'include')}", str(src)], check=True)


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources (build container)")
def test_reference_harnesses_compile_unchanged():
    lib = os.path.join(ROOT, "hnsw-ivf_amd", "lib", "libfaiss_amd.so")
    assert os.path.exists(lib), "build the library first (__graft_entry__.build)"
    subprocess.run(["make", "-B", "harness"], cwd=os.path.join(ROOT, "oracle", "ref"), check=True,
                   capture_output=True)
    for h in HARNESSES:
        exe = os.path.join(HDIR, h)
        assert os.access(exe, os.X_OK), exe
        out = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
        line = [ln for ln in out.splitlines() if "libfaiss_amd.so" in ln]
        assert line and "not found" not in line[0], out
        assert os.path.realpath(line[0].split("=>")[1].split()[0]) == os.path.realpath(lib)


# ------------------------------------------------------------------- GPU runs
def write_fbin(path, x):
    with open(path, "wb") as f:
        np.array(x.shape, dtype=np.int32).tofile(f)
        np.ascontiguousarray(x, dtype=np.float32).tofile(f)


def write_ivecs(path, gt):
    n, k = gt.shape
    a = np.empty((n, k + 1), dtype=np.int32)
    a[:, 0] = k
    a[:, 1:] = gt
    a.tofile(path)


def exact_gt(xb, xq, k):
    xb64 = xb.astype(np.float64)
    bn = (xb64 ** 2).sum(1)
    out = np.empty((xq.shape[0], k), np.int32)
    for q0 in range(0, xq.shape[0], 256):
        xq64 = xq[q0:q0 + 256].astype(np.float64)
        dd = bn[None, :] - 2 * xq64 @ xb64.T
        out[q0:q0 + 256] = np.argsort(dd, axis=1, kind="stable")[:, :k]
    return out


def harness_recall(I, gt, k):
    return sum(len(set(I[i]) & set(gt[i, :k])) for i in range(I.shape[0])) / (I.shape[0] * k)


def run_harness(name, work, config_text):
    exe = os.path.join(HDIR, name)
    assert os.access(exe, os.X_OK), f"{exe} missing: built by __graft_entry__.build()"
    run = work / f"run_{name}"  # (a sibling of ../sift, as the harness expects)
    run.mkdir(exist_ok=True)
    cfg = run / "bench.config"
    cfg.write_text(config_text)
    r = subprocess.run([exe, str(cfg)], cwd=run, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    files = sorted(run.glob("*search_results_*.csv"))
    assert files, r.stdout[-2000:]
    with open(files[-1]) as f:
        return list(csv.DictReader(f)), r.stdout


@pytest.fixture(scope="module")
def sift_small(amd, tmp_path_factory):
    d, nt, nb, nq, k = 64, 20_000, 150_000, 500, 10
    work = tmp_path_factory.mktemp("harness")
    (work / "sift").mkdir()
    xt = amd.float_rand(nt * d, 4321).reshape(nt, d)
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    gt = exact_gt(xb, xq, k)
    write_fbin(work / "sift" / "learn.fbin", xt)
    write_fbin(work / "sift" / "base.fbin", xb)
    write_fbin(work / "sift" / "query.fbin", xq)
    write_ivecs(work / "sift" / "groundtruth.ivecs", gt)
    return dict(work=work, d=d, xt=xt, xb=xb, xq=xq, gt=gt, k=k)


@pytest.mark.gpu
def test_harness_hnsw_ivf_runs_on_the_library(amd, orc, gpu, sift_small):
    """benchmark_hnsw_ivf.cpp:207-427 end to end on the GPU library."""
    s = sift_small
    nlist, efc = 128, 40
    rows, out = run_harness("benchmark_hnsw_ivf", s["work"], f"""build
  param
    nlist:{nlist}
    efconstruction:{efc}
search
  param
    nprobe_ratio:0.0625,0.5
    efsearch_ratio:1.0,3.0
""")
    assert len(rows) == 4, out[-2000:]
    # the same build through this library's API (the harness's call sequence)
    d = s["d"]
    q = amd.IndexHNSWFlat(d, 32)
    q.efConstruction = efc
    q.efSearch = 16
    tr = amd.IndexIVFFlat(q, d, nlist)
    tr.train(s["xt"])
    shell = amd.IndexIVFFlat(q, d, nlist)
    f = str(s["work"] / "shell.index")
    amd.write_index(shell, f)
    idx = amd.read_index(f)
    for c0 in range(0, s["xb"].shape[0], 100_000):
        idx.add(s["xb"][c0:c0 + 100_000])
    ref = orc.IVFOracle.from_index(idx)
    for r in rows:
        nprobe, ef = int(r["nprobe"]), int(r["efsearch"])
        idx.nprobe = nprobe
        amd.ParameterSpace().set_index_parameter(idx, "quantizer_efSearch", ef)
        D, I = idx.search(s["xq"], s["k"])
        Dr, Ir, _, _ = ref.search(s["xq"], s["k"], nprobe, efSearch=ef, nslices=1)
        assert np.array_equal(I, Ir) and np.array_equal(D, Dr), (nprobe, ef)
        rec = harness_recall(I, s["gt"], s["k"])
        assert abs(float(r["recall"]) - rec) < 6e-5, (r, rec)
        assert float(r["qps"]) > 0 and float(r["p99_latency_ms"]) >= float(r["p50_latency_ms"])


@pytest.mark.gpu
def test_harness_ivf_runs_on_the_library(amd, orc, gpu, sift_small):
    """benchmark_ivf.cpp (IVF-Flat with a flat quantizer) end to end."""
    s = sift_small
    nlist = 256
    rows, out = run_harness("benchmark_ivf", s["work"], f"""build
  param
    nlist:{nlist}
search
  param
    nprobe_ratio:0.03125,0.25
""")
    assert len(rows) == 2, out[-2000:]
    d = s["d"]
    q = amd.IndexFlatL2(d)
    idx = amd.IndexIVFFlat(q, d, nlist)
    idx.train(s["xt"])
    idx.add(s["xb"])
    ref = orc.IVFOracle.from_index(idx)
    for r in rows:
        nprobe = int(r["nprobe"])
        idx.nprobe = nprobe
        D, I = idx.search(s["xq"], s["k"])
        Dr, Ir, _, _ = ref.search(s["xq"], s["k"], nprobe, nslices=1)
        assert np.array_equal(I, Ir) and np.array_equal(D, Dr), nprobe
        assert abs(float(r["recall"]) - harness_recall(I, s["gt"], s["k"])) < 6e-5, r


# ------------------------------------------------ the reference's C example
def parse_example_blocks(out):
    """The I= tables example_c.c prints (5 queries x 5 results each), keyed by
    the line announcing the search."""
    import re
    blocks, title, rows = {}, None, []
    for ln in out.splitlines():
        if ln.startswith("Searching"):
            title = ln.strip()
            rows = []
            blocks.setdefault(title, [])
        elif ln.startswith("I="):
            rows = []
            blocks.setdefault(title, []).append(rows)
        else:
            pairs = re.findall(r"(-?\d+) \(d=\s*([-\d.]+)\)", ln)
            if pairs and title is not None:
                rows.append([(int(a), float(b)) for a, b in pairs])
    return blocks


@pytest.mark.gpu
@pytest.mark.parametrize("exe", ["example_c", "example_c_refhdr"])
def test_reference_c_example_runs(amd, gpu, tmp_path, exe):
    """c_api/example_c.c compiled in place and unchanged — against
    include/faiss/c_api (example_c) and against the reference's own C headers
    (example_c_refhdr, the ABI) — runs on the library: IndexFlat through
    faiss_index_factory, add, search, search_with_params with IDSelectorRange /
    Or / And, write_index_fname.  Its data is rand()-seeded by the clock, so
    the checks are the properties its searches must hold: xb[i]'s nearest
    neighbour is i at distance 0, and every label lies in its selector's set."""
    path = os.path.join(HDIR, exe)
    assert os.access(path, os.X_OK), f"{path} missing: built by __graft_entry__.build()"
    r = subprocess.run([path], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ntotal = 100000" in r.stdout and r.stdout.rstrip().endswith("Done.")
    b = parse_example_blocks(r.stdout)
    first, xq = b["Searching..."]
    assert len(first) == 5 and len(xq) == 5
    for i, row in enumerate(first):
        assert row[0] == (i, 0.0), row
    sets = {"Searching w/ IDSelectorRange [50,100]": lambda i: 50 <= i < 100,
            "Searching w/ IDSelectorRange [20,40] OR [45,60]": lambda i: 20 <= i < 40 or 45 <= i < 60,
            "Searching w/ IDSelectorRange [20,40] AND [15,35] = [20,35]": lambda i: 20 <= i < 35}
    for title, member in sets.items():
        (rows,) = b[title]
        assert len(rows) == 5
        for row in rows:
            labels = [i for i, _ in row]
            dists = [dv for _, dv in row]
            assert all(member(i) for i in labels), (title, row)
            assert dists == sorted(dists) and len(set(labels)) == 5, (title, row)
    idx = amd.read_index(str(tmp_path / "example.index"))
    assert idx.ntotal == 100000 and idx.d == 128
