"""world_size-2 test of the sharded search exchange (hnsw-ivf_amd/dist.py) on CPU.

gloo stands in for RCCL; the per-shard search and the merge are the CPU
oracle (faiss IndexShardsIVF semantics, faiss/IndexShardsIVF.cpp:158-245).
Each rank holds the vectors with id % world == rank.  Two batch forms:
  weak   — every rank brings its own queries; the merged result must equal
           the unsharded search of those queries;
  strong — one global batch split over the ranks (bench.py c5): each rank
           quantizes its slice in the form the whole batch's size decides
           (BLAS form from 20 queries, faiss/utils/distances.cpp:807-823) and
           the rank outputs, concatenated, equal the unsharded search of the
           whole batch — also when a slice is below 20 queries.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

D_, NB, NLIST, NQ, NPROBE, K = 32, 6000, 32, 64, 6, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_oracle(orc, xb, cent, ids):
    a = orc.knn(xb, cent, 1, blas_form=True, nthreads=1)[1][:, 0]
    order = np.argsort(a, kind="stable")
    off = np.concatenate([[0], np.cumsum(np.bincount(a, minlength=NLIST))]).astype(np.int64)
    codes = np.ascontiguousarray(xb[order]).view(np.uint8).reshape(len(order), -1)
    return orc.IVFOracle(D_, NLIST, 1, off, codes, ids[order], cent)


def _worker(rank, world, port, out_dir, mode="weak", nq_glob=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        orc = ge.load_oracle()
        hdist = ge.load_package_module("dist")
        xb = orc.float_rand(NB * D_, 1234).reshape(NB, D_)
        cent = xb[:NLIST].copy()
        ids = np.arange(NB, dtype=np.int64)
        mine = ids % world == rank
        shard = _shard_oracle(orc, xb[mine], cent, ids[mine])
        if mode == "strong":
            xg = orc.float_rand(nq_glob * D_, 5678).reshape(nq_glob, D_)
            s = nq_glob // world
            xq = np.ascontiguousarray(xg[rank * s:(rank + 1) * s])
            blas = nq_glob >= 20  # the form of the whole batch
        else:
            xq = orc.float_rand(NQ * D_, 5678 + 7919 * rank).reshape(NQ, D_)
            blas = True

        def quantize(x):
            cd, ci = orc.knn(x.numpy(), cent, NPROBE, blas_form=blas, nthreads=1)
            return torch.from_numpy(cd), torch.from_numpy(ci.astype(np.int32))

        def search_pre(xa, ca, cda):
            D, I = shard.search_preassigned(xa.numpy(), K, ca.numpy().astype(np.int64),
                                            cda.numpy(), nthreads=1)
            return torch.from_numpy(D), torch.from_numpy(I)

        def merge(Dr, Ir):
            D, I = orc.merge_knn_results(Dr.numpy(), Ir.numpy(), metric=1)
            return torch.from_numpy(D), torch.from_numpy(I)

        D, I = hdist.sharded_search(torch.from_numpy(xq), K, quantize, search_pre, merge)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), D=D.numpy(), I=I.numpy(), xq=xq)
    finally:
        dist.destroy_process_group()


def test_sharded_search_equals_unsharded(tmp_path, orc):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    xb = orc.float_rand(NB * D_, 1234).reshape(NB, D_)
    full = _shard_oracle(orc, xb, xb[:NLIST].copy(), np.arange(NB, dtype=np.int64))
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        cd, ci = orc.knn(z["xq"], xb[:NLIST], NPROBE, blas_form=True, nthreads=1)
        Dr, Ir = full.search_preassigned(z["xq"], K, ci, cd, nthreads=1)
        assert np.array_equal(z["I"], Ir) and np.array_equal(z["D"], Dr)


@pytest.mark.parametrize("nq_glob", [30, 128])
def test_sharded_search_strong_split(tmp_path, orc, nq_glob):
    """c5's form: one batch of nq_glob queries split over the ranks (15 per
    rank at nq_glob = 30: slices below the BLAS threshold, the batch above)."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "strong", nq_glob),
             nprocs=world, join=True)
    xb = orc.float_rand(NB * D_, 1234).reshape(NB, D_)
    full = _shard_oracle(orc, xb, xb[:NLIST].copy(), np.arange(NB, dtype=np.int64))
    xg = orc.float_rand(nq_glob * D_, 5678).reshape(nq_glob, D_)
    cd, ci = orc.knn(xg, xb[:NLIST], NPROBE, blas_form=True, nthreads=1)
    Dr, Ir = full.search_preassigned(xg, K, ci, cd, nthreads=1)
    z = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert np.array_equal(np.concatenate([t["I"] for t in z]), Ir)
    assert np.array_equal(np.concatenate([t["D"] for t in z]), Dr)
