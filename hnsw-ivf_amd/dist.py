"""Index shards over one process per GPU (IndexShardsIVF over RCCL / xGMI).

Reference semantics: faiss/IndexShardsIVF.cpp:158-245 — one coarse
quantization, search_preassigned on every shard, merge_knn_results
(faiss/utils/Heap.cpp:159-230; ties -> lower shard).  The reference runs the
shards as host threads (faiss/impl/ThreadedIndex-inl.h:118-147) and merges on
the host; here every rank owns one shard (vectors with id % world == rank, the
faiss GPU default shard_type 1, faiss/gpu/GpuCloner.cpp:298-302) and its own
batch of queries, and the exchange is two collectives on the GPU stream:

  1. coarse-quantize the rank's own queries (centroids replicated),
  2. all_gather(queries, coarse ids, coarse distances)   -> every rank has
     the whole batch (world * nq queries) and its assignments,
  3. search_preassigned of the whole batch on the local shard,
  4. all_to_all of the per-shard top-k so that rank r receives, from every
     shard, the top-k of ITS queries: [world][nq][k] = the layout
     merge_knn_results expects,
  5. merge on the device.

Step 4 moves world*nq*k*12 bytes per rank in total; an all_gather of the
same tables would move world times more (every rank would receive every
query's partial results).  Per-GPU work is constant as the world grows (each
GPU scans nb/world vectors for world*nq queries): weak scaling in queries.

The callables keep this module backend-agnostic: bench.py passes the HIP
entry points (RCCL backend), the CPU tests pass oracle-backed ones (gloo).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def sharded_search(x, k, quantize, search_preassigned, merge, group=None):
    """x: [nq, d] queries of this rank.  Returns (D, I) [nq, k] for them.

    quantize(x) -> (coarse_dis [nq, nprobe] f32, assign [nq, nprobe] i32)
    search_preassigned(x_all, assign_all, coarse_dis_all) -> (D, I) [world*nq, k]
    merge(D_parts, I_parts) with [world, nq, k] inputs -> (D, I) [nq, k]
    """
    world = dist.get_world_size(group)
    nq, d = x.shape
    cd, ci = quantize(x)
    nprobe = ci.shape[1]
    x_all = x.new_empty((world * nq, d))
    ci_all = ci.new_empty((world * nq, nprobe))
    cd_all = cd.new_empty((world * nq, nprobe))
    dist.all_gather_into_tensor(x_all, x.contiguous(), group=group)
    dist.all_gather_into_tensor(ci_all, ci.contiguous(), group=group)
    dist.all_gather_into_tensor(cd_all, cd.contiguous(), group=group)
    Ds, Is = search_preassigned(x_all, ci_all, cd_all)
    Dr = torch.empty_like(Ds)
    Ir = torch.empty_like(Is)
    dist.all_to_all_single(Dr, Ds.contiguous(), group=group)
    dist.all_to_all_single(Ir, Is.contiguous(), group=group)
    return merge(Dr.view(world, nq, k), Ir.view(world, nq, k))


def shard_rows(nb, world, rank):
    """ids of the vectors held by `rank` (faiss shard_type 1: id modulo world)."""
    return torch.arange(rank, nb, world, dtype=torch.int64)
