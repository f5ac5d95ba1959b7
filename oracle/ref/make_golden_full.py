#!/usr/bin/env python3
"""Reference-run fixtures: index files written by the reference's own
`faiss::write_index` and the D/I / lims / codes of reference searches over
them.  Writes tests/golden/ref_full/*.faiss and tests/golden/ref_full.npz.

Runs only in the build container: it needs oracle/_ref/libfaissfull.so, the
reference CPU library that `make -C oracle/ref full` compiles in place from
/root/reference (MKL as BLAS).  Every expected array below is produced by the
reference's code (index_factory, train, add, write_index, quantizer->search,
IndexIVF::search / search_preassigned / range_search, encode_vectors,
IndexHNSW::search).  Inputs are faiss float_rand streams; the files are
reference *outputs* (data), no reference text is copied.

Protocol: searches run with one OpenMP thread, so IndexIVF::search treats the
batch as a single slice (the GPU path's slicing); nq >= 20 makes the flat
coarse quantizer take its BLAS form (faiss/utils/distances.cpp:807-823).

    python oracle/ref/make_golden_full.py
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUTD = os.path.join(ROOT, "tests", "golden", "ref_full")
OUT = os.path.join(ROOT, "tests", "golden", "ref_full.npz")

L = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfaissfull.so"), mode=C.RTLD_GLOBAL)
P, I64, F = C.c_void_p, C.c_int64, C.c_float
L.reff_last_error.restype = C.c_char_p
L.reff_index_factory.restype = P
L.reff_index_factory.argtypes = [C.c_int, C.c_char_p, C.c_int]
L.reff_read_index.restype = P
L.reff_read_index.argtypes = [C.c_char_p, C.c_int]
L.reff_write_index.argtypes = [P, C.c_char_p]
L.reff_free.argtypes = [P]
L.reff_train.argtypes = [P, I64, P]
L.reff_add.argtypes = [P, I64, P, P]
L.reff_info.argtypes = [P, P]
L.reff_set_nprobe.argtypes = [P, I64]
L.reff_set_parallel_mode.argtypes = [P, C.c_int]
L.reff_set_quantizer_efsearch.argtypes = [P, C.c_int]
L.reff_ivfpq_set_table.argtypes = [P, C.c_int]
L.reff_search.argtypes = [P, I64, P, I64, P, P]
L.reff_search_params.argtypes = [P, I64, P, I64, I64, I64, P, I64, P, P]
L.reff_quantizer_search.argtypes = [P, I64, P, I64, P, P]
L.reff_search_preassigned.argtypes = [P, I64, P, I64, I64, P, P, C.c_int, P, P]
L.reff_range_search.restype = P
L.reff_range_search.argtypes = [P, I64, P, F, I64]
L.reff_range_total.restype = I64
L.reff_range_total.argtypes = [P]
L.reff_range_copy.argtypes = [P, P, P, P]
L.reff_assign.argtypes = [P, I64, P, P]
L.reff_encode_vectors.argtypes = [P, I64, P, P, P]
L.reff_list_size.restype = I64
L.reff_list_size.argtypes = [P, I64]
L.reff_list_copy.argtypes = [P, I64, P, P]
L.reff_set_threads.argtypes = [C.c_int]
L.reff_set_hnsw_efsearch.argtypes = [P, C.c_int]

REFP = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfaissref.so"))
REFP.ref_float_rand.argtypes = [P, C.c_size_t, C.c_int64]


def p(a):
    return a.ctypes.data_as(P) if a is not None else None


def ok(rc):
    if rc != 0:
        raise RuntimeError(L.reff_last_error().decode())


def float_rand(n, d, seed):
    x = np.empty(n * d, np.float32)
    REFP.ref_float_rand(p(x), n * d, seed)
    return x.reshape(n, d)


def info(h):
    out = np.zeros(10, np.int64)
    ok(L.reff_info(h, p(out)))
    return out


def search(h, x, k):
    D = np.empty((x.shape[0], k), np.float32)
    I = np.empty((x.shape[0], k), np.int64)
    ok(L.reff_search(h, x.shape[0], p(x), k, p(D), p(I)))
    return D, I


def qsearch(h, x, nprobe):
    D = np.empty((x.shape[0], nprobe), np.float32)
    I = np.empty((x.shape[0], nprobe), np.int64)
    ok(L.reff_quantizer_search(h, x.shape[0], p(x), nprobe, p(D), p(I)))
    return D, I


def preassigned(h, x, k, Iq, Dq, store_pairs=0):
    n, nprobe = Iq.shape
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    ok(L.reff_search_preassigned(h, n, p(x), k, nprobe, p(np.ascontiguousarray(Iq)),
                                 p(np.ascontiguousarray(Dq)), store_pairs, p(D), p(I)))
    return D, I


def range_search(h, x, radius, nprobe):
    r = L.reff_range_search(h, x.shape[0], p(x), radius, nprobe)
    if not r:
        raise RuntimeError(L.reff_last_error().decode())
    tot = L.reff_range_total(r)
    lims = np.empty(x.shape[0] + 1, np.int64)
    D = np.empty(max(tot, 1), np.float32)
    I = np.empty(max(tot, 1), np.int64)
    L.reff_range_copy(r, p(lims), p(D), p(I))
    return lims, D[:tot], I[:tot]


def lists_digest(h, nlist, code_size):
    sizes = np.array([L.reff_list_size(h, l) for l in range(nlist)], np.int64)
    sha = hashlib.sha256()
    for l in range(nlist):
        n = int(sizes[l])
        codes = np.empty(max(n * code_size, 1), np.uint8)
        ids = np.empty(max(n, 1), np.int64)
        ok(L.reff_list_copy(h, l, p(codes), p(ids)))
        sha.update(codes[: n * code_size].tobytes())
        sha.update(ids[:n].tobytes())
    return sizes, np.frombuffer(sha.digest(), np.uint8)


def build(desc, d, metric_l2, nt, nb, seed, ids=None):
    h = L.reff_index_factory(d, desc.encode(), metric_l2)
    if not h:
        raise RuntimeError(L.reff_last_error().decode())
    L.reff_set_threads(8)
    xt = float_rand(nt, d, seed)
    ok(L.reff_train(h, nt, p(xt)))
    xb = xt[:nb] if nb <= nt else float_rand(nb, d, seed + 1)
    ok(L.reff_add(h, nb, p(np.ascontiguousarray(xb)), p(ids)))
    L.reff_set_threads(1)
    return h, xb


def save_index(h, name):
    path = os.path.join(OUTD, name + ".faiss")
    ok(L.reff_write_index(h, path.encode()))
    return path


def main():
    os.makedirs(OUTD, exist_ok=True)
    fx = {}
    nq = 64

    # ------------------------------------------------------------ IVF-Flat
    for tag, ml2 in (("flat_l2", 1), ("flat_ip", 0)):
        d, nlist = 32, 64
        ids = (np.arange(3000, dtype=np.int64) * 7 + 11) if tag == "flat_ip" else None
        h, xb = build(f"IVF{nlist},Flat", d, ml2, 3000, 3000, 101 if ml2 else 111, ids)
        save_index(h, tag)
        xq = float_rand(nq, d, 202)
        # duplicated query rows and base rows make exact ties reachable
        xq[-4:] = xb[:4]
        fx[f"{tag}_xq"] = xq
        fx[f"{tag}_info"] = info(h)
        fx[f"{tag}_sizes"], fx[f"{tag}_sha"] = lists_digest(h, nlist, 4 * d)
        for nprobe in (4, 17, nlist):
            Dq, Iq = qsearch(h, xq, nprobe)
            fx[f"{tag}_q{nprobe}_D"], fx[f"{tag}_q{nprobe}_I"] = Dq, Iq
            for k in (1, 10, 100, 300):
                D, I = preassigned(h, xq, k, Iq, Dq)
                fx[f"{tag}_pre_{nprobe}_{k}_D"], fx[f"{tag}_pre_{nprobe}_{k}_I"] = D, I
        Dq, Iq = qsearch(h, xq, 4)
        D, I = preassigned(h, xq, 10, Iq, Dq, store_pairs=1)
        fx[f"{tag}_sp_D"], fx[f"{tag}_sp_I"] = D, I
        for nprobe, k in ((8, 10), (nlist, 100)):
            ok(L.reff_set_nprobe(h, nprobe))
            D, I = search(h, xq, k)
            fx[f"{tag}_full_{nprobe}_{k}_D"], fx[f"{tag}_full_{nprobe}_{k}_I"] = D, I
        ok(L.reff_set_nprobe(h, 8))
        for pm in (1, 2):
            ok(L.reff_set_parallel_mode(h, pm))
            D, I = search(h, xq, 10)
            fx[f"{tag}_pm{pm}_D"], fx[f"{tag}_pm{pm}_I"] = D, I
        ok(L.reff_set_parallel_mode(h, 0))
        # max_codes + IDSelectorBatch (SearchParametersIVF)
        sel = np.unique((np.arange(0, 3000, 3, dtype=np.int64) * 7 + 11) if ids is not None
                        else np.arange(0, 3000, 3, dtype=np.int64))
        D = np.empty((nq, 10), np.float32)
        I = np.empty((nq, 10), np.int64)
        ok(L.reff_search_params(h, nq, p(xq), 10, 8, 300, p(sel), sel.size, p(D), p(I)))
        fx[f"{tag}_params_D"], fx[f"{tag}_params_I"], fx[f"{tag}_params_sel"] = D, I, sel
        radius = float(np.median(fx[f"{tag}_full_8_10_D"][:, 5]))
        lims, D, I = range_search(h, xq, radius, 8)
        fx[f"{tag}_range_radius"] = np.array([radius], np.float32)
        fx[f"{tag}_range_lims"], fx[f"{tag}_range_D"], fx[f"{tag}_range_I"] = lims, D, I
        # add path: assignment of new vectors
        xa = float_rand(500, d, 303)
        la = np.empty(500, np.int64)
        ok(L.reff_assign(h, 500, p(xa), p(la)))
        fx[f"{tag}_xa"], fx[f"{tag}_assign"] = xa, la
        L.reff_free(h)

    # ------------------------------------------------------------ IVF-PQ
    pq_cases = [
        # tag, d, nlist, M, metric_l2, nb
        ("pq_m32d128", 128, 32, 32, 1, 3000),  # c3 geometry: dsub 4, M >= 16
        ("pq_m48d96", 96, 32, 48, 1, 3000),    # c5 geometry: dsub 2
        ("pq_m16d64", 64, 16, 16, 1, 3000),    # dsub 4, one 16-block
        ("pq_m24d96", 96, 16, 24, 1, 2000),    # 16-block + 8 sequential leftovers
        ("pq_m8d64", 64, 16, 8, 1, 2000),      # M = 8 kernel, dsub 8
        ("pq_m4d64", 64, 16, 4, 1, 2000),      # M = 4 kernel, dsub 16 (generic ny)
        ("pq_m12d48", 48, 16, 12, 1, 2000),    # M < 16: sequential sum
        ("pq_ip_m16d64", 64, 16, 16, 0, 3000), # inner product
    ]
    for tag, d, nlist, M, ml2, nb in pq_cases:
        nt = max(nb, 6000)
        h, xb = build(f"IVF{nlist},PQ{M}", d, ml2, nt, nb, 400 + d + M)
        save_index(h, tag)
        inf = info(h)
        fx[f"{tag}_info"] = inf
        fx[f"{tag}_sizes"], fx[f"{tag}_sha"] = lists_digest(h, nlist, int(inf[5]))
        xq = float_rand(nq, d, 500 + M)
        xq[-2:] = xb[:2]
        fx[f"{tag}_xq"] = xq
        tables = (1, 0) if ml2 else (0,)
        for nprobe in (5, nlist):
            Dq, Iq = qsearch(h, xq, nprobe)
            fx[f"{tag}_q{nprobe}_D"], fx[f"{tag}_q{nprobe}_I"] = Dq, Iq
            for t in tables:
                if ml2:
                    ok(L.reff_ivfpq_set_table(h, 1 if t == 1 else -1))
                for k in (10, 100):
                    D, I = preassigned(h, xq, k, Iq, Dq)
                    fx[f"{tag}_t{t}_pre_{nprobe}_{k}_D"] = D
                    fx[f"{tag}_t{t}_pre_{nprobe}_{k}_I"] = I
        if ml2:
            ok(L.reff_ivfpq_set_table(h, 1))
        ok(L.reff_set_nprobe(h, 5))
        D, I = search(h, xq, 10)
        fx[f"{tag}_full_5_10_D"], fx[f"{tag}_full_5_10_I"] = D, I
        radius = float(np.median(D[:, 5]))
        lims, Dr, Ir = range_search(h, xq, radius, 5)
        fx[f"{tag}_range_radius"] = np.array([radius], np.float32)
        fx[f"{tag}_range_lims"], fx[f"{tag}_range_D"], fx[f"{tag}_range_I"] = lims, Dr, Ir
        # add path: coarse assignment + PQ codes of new vectors
        xa = float_rand(400, d, 600 + M)
        la = np.empty(400, np.int64)
        ok(L.reff_assign(h, 400, p(xa), p(la)))
        codes = np.empty((400, int(inf[5])), np.uint8)
        ok(L.reff_encode_vectors(h, 400, p(xa), p(la), p(codes)))
        fx[f"{tag}_xa"], fx[f"{tag}_assign"], fx[f"{tag}_codes"] = xa, la, codes
        L.reff_free(h)

    # ------------------------------------------------------------ HNSW
    d, nlist = 32, 256
    h, xb = build(f"IVF{nlist}_HNSW16,Flat", d, 1, 8000, 3000, 700)
    save_index(h, "hnswivf")
    xq = float_rand(nq, d, 701)
    fx["hnswivf_xq"], fx["hnswivf_info"] = xq, info(h)
    fx["hnswivf_sizes"], fx["hnswivf_sha"] = lists_digest(h, nlist, 4 * d)
    for ef in (16, 64, 200):
        ok(L.reff_set_quantizer_efsearch(h, ef))
        for nprobe in (8, 100):
            Dq, Iq = qsearch(h, xq, nprobe)
            fx[f"hnswivf_ef{ef}_q{nprobe}_D"], fx[f"hnswivf_ef{ef}_q{nprobe}_I"] = Dq, Iq
            ok(L.reff_set_nprobe(h, nprobe))
            D, I = search(h, xq, 10)
            fx[f"hnswivf_ef{ef}_{nprobe}_D"], fx[f"hnswivf_ef{ef}_{nprobe}_I"] = D, I
    L.reff_free(h)

    # standalone IndexHNSWFlat with duplicated vectors (exact distance ties in
    # the candidate and result heaps, tests/test_hnsw.cpp:109-186 territory)
    d = 16
    base = float_rand(600, d, 800)
    xh = np.concatenate([base, base[:150], base[:150], base[300:340]])
    h = L.reff_index_factory(d, b"HNSW8", 1)
    L.reff_set_threads(1)
    ok(L.reff_add(h, xh.shape[0], p(np.ascontiguousarray(xh)), None))
    save_index(h, "hnsw_dup")
    xq = np.concatenate([float_rand(40, d, 801), base[:24]])
    fx["hnsw_dup_xq"] = xq
    for ef in (8, 32, 200):
        ok(L.reff_set_hnsw_efsearch(h, ef))
        for k in (1, 10, 40):
            D, I = search(h, xq, k)
            fx[f"hnsw_dup_ef{ef}_{k}_D"], fx[f"hnsw_dup_ef{ef}_{k}_I"] = D, I
    L.reff_free(h)

    # ------------------------------------------------------------ IxF2
    h = L.reff_index_factory(24, b"Flat", 1)
    xf = float_rand(500, 24, 900)
    ok(L.reff_add(h, 500, p(xf), None))
    save_index(h, "flat")
    xq = float_rand(30, 24, 901)
    fx["flat_xq"] = xq
    fx["flat_10_D"], fx["flat_10_I"] = search(h, xq, 10)
    L.reff_free(h)

    np.savez_compressed(OUT, **fx)
    tot = sum(os.path.getsize(os.path.join(OUTD, f)) for f in os.listdir(OUTD))
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e3:.0f} kB, {len(fx)} arrays) and "
          f"{len(os.listdir(OUTD))} index files ({tot / 1e3:.0f} kB)")


if __name__ == "__main__":
    sys.exit(main())
