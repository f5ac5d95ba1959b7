"""world_size-2 sharded search over the library's real device entry points.

hnsw-ivf_amd/dist.py's exchange (all_gather of the batch, per-shard
search_preassigned, all_to_all of the [world][nq][k] tables, merge) driven by
two processes on the box's GPU: quantize_device, search_preassigned_device and
merge_knn_results_device run on device tensors; gloo (CPU tensors) stands in
for RCCL, whose collectives need one GPU per rank.  Each rank holds the
vectors with id % world == rank (faiss shard_type 1) and brings its own
queries; the merged result must equal the unsharded index's search of them
(faiss/IndexShardsIVF.cpp:158-245).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

D_, NB, NLIST, NQ, NPROBE, K = 32, 6000, 32, 64, 6, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _index(amd, xb, cent, ids):
    q = amd.IndexFlatL2(D_)
    q.add(cent)
    idx = amd.IndexIVFFlat(q, D_, NLIST)
    idx._q = q
    idx.add_with_ids(xb, ids)
    idx.nprobe = NPROBE
    return idx


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import __graft_entry__ as ge
        amd = ge.load_package()
        hdist = ge.load_package_module("dist")
        dev = torch.device("cuda:0")
        xb = amd.float_rand(NB * D_, 1234).reshape(NB, D_)
        cent = xb[:NLIST].copy()
        ids = np.arange(NB, dtype=np.int64)
        mine = ids % world == rank
        shard = _index(amd, xb[mine], cent, ids[mine])
        xq = amd.float_rand(NQ * D_, 5678 + 7919 * rank).reshape(NQ, D_)

        def sync():
            torch.cuda.synchronize(dev)

        def quantize(x):
            xd = x.to(dev)
            cd = torch.empty((x.shape[0], NPROBE), dtype=torch.float32, device=dev)
            ci = torch.empty((x.shape[0], NPROBE), dtype=torch.int32, device=dev)
            sync()
            shard.quantize_device(x.shape[0], xd.data_ptr(), NPROBE, cd.data_ptr(), ci.data_ptr())
            sync()
            return cd.cpu(), ci.cpu()

        def search_pre(xa, ca, cda):
            n = xa.shape[0]
            xd, cad, cdd = xa.to(dev), ca.to(dev), cda.to(dev)
            Dd = torch.empty((n, K), dtype=torch.float32, device=dev)
            Id = torch.empty((n, K), dtype=torch.int64, device=dev)
            sync()
            shard.search_preassigned_device(n, xd.data_ptr(), K, NPROBE, cad.data_ptr(),
                                            cdd.data_ptr(), Dd.data_ptr(), Id.data_ptr())
            sync()
            return Dd.cpu(), Id.cpu()

        def merge(Dr, Ir):
            nsh, n, k = Dr.shape
            Dd, Idd = Dr.contiguous().to(dev), Ir.contiguous().to(dev)
            Do = torch.empty((n, k), dtype=torch.float32, device=dev)
            Io = torch.empty((n, k), dtype=torch.int64, device=dev)
            sync()
            amd.merge_knn_results_device(n, k, nsh, Dd.data_ptr(), Idd.data_ptr(), Do.data_ptr(),
                                         Io.data_ptr())
            sync()
            return Do.cpu(), Io.cpu()

        D, I = hdist.sharded_search(torch.from_numpy(xq), K, quantize, search_pre, merge)
        full = _index(amd, xb, cent, ids)
        Dr, Ir = full.search(xq, K)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), D=D.numpy(), I=I.numpy(), Dr=Dr, Ir=Ir)
    finally:
        dist.destroy_process_group()


def test_sharded_device_search_equals_unsharded(tmp_path, gpu):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        np.testing.assert_array_equal(z["I"], z["Ir"])
        np.testing.assert_array_equal(z["D"], z["Dr"])
