#!/usr/bin/env python3
"""Benchmark: queries/sec of the batched IVF search hot path on MI355X.

Metric (BASELINE.json): queries/sec @ recall@10, IVF4096 d=128 nq=10k
nprobe=32; 1/2/4/8 GPUs.  One step = one batched search of nq=10k synthetic
uniform queries (faiss float_rand, seed 5678) against IVF4096,Flat over 1M
synthetic vectors (float_rand seed 1234), k=10, inputs resident in HBM.

N=1: the whole path (query prep + bf16x3-MFMA coarse filter + exact re-rank +
list-centric bf16x2-MFMA scan + exact re-rank) through
faiss_amd_Index_search_device.

N>1 (torch.distributed.run, one rank per GPU, torch.distributed over RCCL):
  c1-c4 name one GPU, so `value` is N replicas of the whole index, each rank
  serving its own 10k queries (weak scaling, no data-path collective).  Beside
  it the line carries `rccl_shards`: the same index sharded by id modulo N
  (faiss GPU shard_type 1) with the IndexShardsIVF exchange of
  hnsw-ivf_amd/dist.py (all_gather of queries + coarse results, all_to_all of
  per-shard top-k, device merge), every rank again bringing 10k queries.
  `--shard` makes the sharded form the `value`.
  c5 is the sharded config: the 100M set is split by id modulo N and the
  100k queries of the batch are split over the ranks (nq / N each, strong
  scaling: the total work is fixed); `--weak` instead has every rank bring
  100k queries (global batch N x 100k, labelled weak).

The line names the step's dominant kernel (largest per-step time, HIP events
on the launch stream) and prices it against its roofline; every kernel stage
above 10 % of the step is listed with its own time and fraction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # loaded before libfaiss_amd so both share one HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

CONFIGS = {
    # BASELINE.json configs[0..3]
    "c1": dict(workload="IVF256,Flat", desc="IVF256,Flat", d=64, nb=100_000, nq=1_000,
               nlist=256, nprobe=8, k=10, ntrain=100_000),
    "c2": dict(workload="IVF4096,Flat", desc="IVF4096,Flat", d=128, nb=1_000_000, nq=10_000,
               nlist=4096, nprobe=32, k=10, ntrain=200_000),
    "c3": dict(workload="IVF4096,PQ32x8", desc="IVF4096,PQ32x8", d=128, nb=1_000_000,
               nq=10_000, nlist=4096, nprobe=32, k=10, ntrain=200_000),
    "c4": dict(workload="IVF16384_HNSW32,Flat", desc="IVF16384_HNSW32,Flat", d=128,
               nb=10_000_000, nq=10_000, nlist=16384, nprobe=64, k=10, ntrain=638_976,
               efSearch=64),
    # BASELINE.json configs[4]: IndexShardsIVF, 100M vectors d=96 split over
    # the N ranks (ids == rank mod N, faiss GPU shard_type 1); the 100k
    # queries of a step are split over the ranks (strong scaling).  --shard-of
    # 8 with --gpus 1 builds one rank's share of an 8-GPU run (12.5M vectors)
    # and serves the whole 100k batch on it.
    "c5": dict(workload="IVF65536,PQ48 over 100M", desc="IVF65536,PQ48", d=96,
               nb=100_000_000, sharded=True, nq=100_000, nlist=65536, nprobe=64, k=10,
               ntrain=65536 * 39),
}
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 vector == fp32 MFMA peak
PEAK_HBM_GBS = 8000.0
PEAK_L2_GBS = 34500.0      # MI355X_MICROARCH.md: aggregate L2 (4 MiB per XCD), measured
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
PEAK_LDS_TBS = 150.0       # MI355X_MICROARCH.md: aggregate ds_read_b128 rate, every CU
# kernel stage (library timer name) -> regular expression of the demangled
# symbol of the kernel that stage launches in this round's code, matched in
# this round's committed rocprofv3 PMC summaries (a summary of an older kernel
# or round is never used: traffic is null instead)
ROUND = 6
PMC_SYMBOL = {
    "ivf_flat_scan": r"kern::k_ivf_bf2_stream<true, \d+, \d+, false, true, false>",
    # (rocprofv3 leaves this one mangled: its name holds a __bf16, "DF16b")
    "ivfpq_filter": r"kern::k_ivfpq_filter_w<|k_ivfpq_filter_wILi",
    "coarse_filter": r"kern::k_coarse_stream<",
    "hnsw_search": r"kern::k_hnsw_search<",
    "hnsw_exact": r"kern::k_hnsw_exact(_reg)?[<(]",
    "hnsw_wide": r"kern::k_hnsw_wide<",
    "ivf_rerank": r"kern::k_ivf_rerank<true, \d+, 0>",
    "ivfpq_rerank": r"kern::k_ivf_rerank<true, \d+, [1-9]\d*>",
    "coarse_rerank": r"kern::k_coarse_rerank<",
}


def pmc_traffic(config, stage):
    """HBM bytes per launch of a stage's kernel from this round's committed
    rocprofv3 --pmc summary for the workload (profiles/rNN_<config>_pmc.json,
    written by scripts/pmc_summary.py: FETCH_SIZE x2 per the gfx950 correction
    + WRITE_SIZE, separate passes); (None, None) when there is none."""
    import re
    fn = os.path.join(ROOT, "profiles", f"r{ROUND:02d}_{config}_pmc.json")
    pat = PMC_SYMBOL.get(stage)
    if not pat or not os.path.exists(fn):
        return None, None
    with open(fn) as f:
        summ = json.load(f)
    # several entries can match (the build's launches of the same kernel —
    # k-means assignment, adds through an HNSW quantizer — are kept apart by
    # grid size): the search's is the one that ran last (the timed steps end
    # the profiled run)
    best = None
    for name, ent in summ.items():
        if re.search(pat, name) and "hbm_bytes" in ent:
            if best is None or ent.get("last_dispatch", 0) > best.get("last_dispatch", 0):
                best = ent
    if best is None:
        return None, None
    return best["hbm_bytes"], os.path.relpath(fn, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def timed(fn):
    t = time.perf_counter()
    out = fn()
    return time.perf_counter() - t, out


def cpu_baseline(args, cfg, amd, index, xq, I_gpu, k, nprobe):
    """Best of 3 wall-clock runs of one batched search over a bounded sample
    of the queries (SURVEY 8d protocol), plus a one-thread figure."""
    nq = xq.shape[0]
    ncores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    ef = cfg.get("efSearch")
    ref = None
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import reflib  # noqa: E402  (test infrastructure: the CPU baseline leg)
        if reflib.available():
            import tempfile
            fn = os.path.join(tempfile.gettempdir(), f"bench_ref_{os.getpid()}.faiss")
            amd.write_index(index, fn)
            try:
                ref = reflib.RefIndex(fn)
            finally:
                os.unlink(fn)
            ref.set_nprobe(nprobe)
            if ef:
                ref.set_quantizer_efsearch(ef)
    except Exception as e:  # noqa: BLE001
        log(f"reference CPU library unavailable ({e}); timing the oracle restatement")
        ref = None
    if ref is not None:
        kind = "reference"
        what = ("reference faiss IndexIVF::search (libfaissfull: the reference sources "
                "compiled in place, AVX2 flags, MKL BLAS), same index via write_index / "
                "read_index")

        def search(xs, nt):
            return ref.search(xs, k, nt)
    else:
        kind = "port"
        orc = ge.load_oracle()
        o = orc.IVFOracle.from_index(index)
        what = "IndexIVF::search restated (oracle search, one slice per thread)"

        def search(xs, nt):
            D_, I_, _, _ = o.search(xs, k, nprobe, efSearch=ef or 16, nslices=nt, nthreads=nt)
            return D_, I_
    probe = min(200, nq)
    search(xq[:probe], ncores)  # warm-up
    tp, _ = timed(lambda: search(xq[:probe], ncores))
    # one call ~ cpu_seconds / 4, best of 3
    ns = int(min(nq, max(probe, probe * args.cpu_seconds / 4 / max(tp, 1e-4))))
    best, res = None, None
    for _ in range(3):
        t, r = timed(lambda: search(xq[:ns], ncores))
        if best is None or t < best:
            best, res = t, r
    agree = float(np.mean(res[1] == I_gpu[:ns]))
    n1 = int(max(1, min(ns, ns * (args.cpu_seconds / 5) / max(best * ncores, 1e-4))))
    t1, _ = timed(lambda: search(xq[:n1], 1))
    return {"value": ns / best, "unit": "queries/s", "cores": ncores, "kind": kind,
            "sample": f"best of 3 batched calls over {ns} of the {nq} queries, {what}, "
                      f"{ncores} OpenMP threads on {cpu_model()}",
            "id_agreement_vs_gpu": agree,
            "one_thread": {"value": n1 / t1, "unit": "queries/s", "queries": n1}}


def kernel_breakdown(index, steps):
    """{stage: ms per step} from the library's HIP-event timers."""
    out = {}
    for nm, ms, _ in index.kernel_times():
        out[nm] = out.get(nm, 0.0) + ms
    return {nm: ms / max(steps, 1) for nm, ms in out.items()}


def kernel_roofline(name, ms, work, config):
    """Roofline of one kernel stage from its per-step time and algorithmic
    work (work: dict of the step's quantities, see main)."""
    t = ms * 1e-3
    r = None
    if name == "ivf_flat_scan":
        # one pass over the rows of every distinct probed list: bf16 hi of
        # the dims (padded to 32) + |y|^2 + residual bound = 2 dpad + 8 bytes
        b = work["flat_rows"] * work["flat_row_bytes"]
        r = {"bound": "hbm", "achieved": b / t / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
             "algorithmic_bytes_per_step": b, "bytes_per_row": work["flat_row_bytes"],
             "mfma_dtype": "bf16", "mfma_flops_per_step": work["flat_flops"],
             "mfma_tflops": work["flat_flops"] / t / 1e12,
             "mfma_frac": work["flat_flops"] / t / 1e12 / PEAK_BF16_TFLOPS}
    elif name == "ivfpq_filter" and os.environ.get("FAISS_AMD_PQ_FILTER") == "image":
        # (opt-in) the streamed filter over the decoded residual image: one
        # pass over the rows of every distinct probed list at 2 dpad + 8 bytes
        # per row (the IVF-Flat filter's model); the code bytes beside it
        b = work["flat_rows"] * work["flat_row_bytes"]
        f = work["cands"] * 4.0 * work["dpad32"]
        r = {"bound": "hbm", "achieved": b / t / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
             "algorithmic_bytes_per_step": b, "bytes_per_row": work["flat_row_bytes"],
             "mfma_dtype": "bf16", "mfma_flops_per_step": f, "mfma_tflops": f / t / 1e12,
             "mfma_frac": f / t / 1e12 / PEAK_BF16_TFLOPS,
             "pq_code_bytes_per_step": work["flat_rows"] * work.get("M", 0)}
    elif name == "ivfpq_filter":
        # the default filter streams the code bytes (list x
        # code_size, one pass over the rows of every distinct probed list),
        # priced against HBM; beside it the rate of its LDS decode-table
        # gathers (one ds_read_b128 of 8 bf16 per lane and 16 B of table per
        # (row, 8 dims) of each 32-query task: M / (8 / dsub) gathers of
        # 16 B per row per task) and the bf16 MFMA work it feeds
        b = work["flat_rows"] * work.get("M", 0)
        f = work["cands"] * 4.0 * work["dpad16"]
        lds_b = work["cands"] / 32.0 * work["dpad16"] * 2.0
        r = {"bound": "hbm", "achieved": b / t / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
             "algorithmic_bytes_per_step": b, "bytes_per_row": work.get("M", 0),
             "lds_gather_bytes_per_step": lds_b, "lds_gather_tbs": lds_b / t / 1e12,
             "lds_gather_frac": lds_b / t / 1e12 / PEAK_LDS_TBS,
             "mfma_dtype": "bf16", "mfma_flops_per_step": f, "mfma_tflops": f / t / 1e12,
             "mfma_frac": f / t / 1e12 / PEAK_BF16_TFLOPS}
    elif name == "coarse_filter":
        # bf16x3 x.c of every (query, centroid): 3 products of 2 dpad flops
        f = work["nq_coarse"] * work["nlist"] * 6.0 * work["dpad16"]
        r = {"bound": "mfma", "achieved": f / t / 1e12, "peak": PEAK_BF16_TFLOPS,
             "unit": "TFLOP/s", "mfma_dtype": "bf16", "algorithmic_flops_per_step": f,
             "flops_per_query_centroid": 6 * work["dpad16"]}
    elif name in ("hnsw_search", "hnsw_exact", "hnsw_wide") and work.get("hnsw_ndis"):
        # bytes the traversal must read: per hop the node's level-0 neighbour
        # ids (64 x 4 B); per distance either one fp32 row of the graph's
        # storage or, for the register kernel's prefiltered neighbours, the
        # row's int8 image (128 B + 20 B of scale / bound terms) and the fp32
        # row only when the bound lets it through (counted on the device:
        # cvar.hnsw_row_stats).  The storage (c4: 16384 centroids, 8 MB fp32,
        # 2.4 MB int8) lives in the on-chip caches (4 MiB L2 per XCD, the
        # 256 MiB Infinity Cache), so the bytes are priced against the
        # aggregate L2 bandwidth, not HBM
        f32, q8 = work.get("hnsw_fp32_rows"), work.get("hnsw_q8_rows")
        if f32 is None:
            f32, q8 = work["hnsw_ndis"], 0.0
        b = f32 * 4.0 * work["d"] + q8 * 148.0 + work.get("hnsw_nhops", 0.0) * 256.0
        r = {"bound": "l2", "achieved": b / t / 1e9, "peak": PEAK_L2_GBS, "unit": "GB/s",
             "algorithmic_bytes_per_step": b, "hnsw_ndis_per_step": work["hnsw_ndis"],
             "hnsw_fp32_rows_per_step": f32, "hnsw_q8_rows_per_step": q8,
             "hnsw_nhops_per_step": work.get("hnsw_nhops", 0.0)}
    if r is None:
        return None
    r["frac"] = r["achieved"] / r["peak"]
    traffic, src = pmc_traffic(config, name)
    r["traffic"] = traffic
    if traffic is not None:
        r["traffic_source"] = src
        r["traffic_unit"] = "bytes/launch"
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--recall-queries", type=int, default=1000)
    ap.add_argument("--shard-of", type=int, default=0,
                    help="c5: build one rank's share of a run over this many GPUs")
    ap.add_argument("--shard", action="store_true",
                    help="c1-c4 at N > 1: the IndexShardsIVF exchange over RCCL is the "
                         "value (instead of one replica per GPU)")
    ap.add_argument("--no-shard-figure", action="store_true",
                    help="c1-c4 at N > 1: skip the rccl_shards figure beside the replicas")
    ap.add_argument("--nprobe", type=int, default=0,
                    help="override the config's nprobe (a point of the reference "
                         "harness's grid; not a BASELINE line)")
    ap.add_argument("--efsearch", type=int, default=0,
                    help="override the config's quantizer efSearch (HNSW configs)")
    ap.add_argument("--weak", action="store_true",
                    help="c5: every rank brings nq queries (global batch N x nq)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    sharded = cfg.get("sharded", False)
    replicas = world > 1 and not sharded and not args.shard
    # (local_rank % devices: a rehearsal of N ranks on fewer GPUs)
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        # RCCL; FAISS_AMD_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs
        # (RCCL refuses two ranks on one device)
        be = os.environ.get("FAISS_AMD_BENCH_BACKEND", "nccl")
        if be == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(be)
    amd = ge.load_package()
    amd.set_device(gpu)
    stream = torch.cuda.current_stream().cuda_stream

    if args.nprobe:
        cfg["nprobe"] = args.nprobe
    if args.efsearch and "efSearch" in cfg:
        cfg["efSearch"] = args.efsearch
    d, nb, nq, k, nprobe = cfg["d"], cfg["nb"], cfg["nq"], cfg["k"], cfg["nprobe"]
    # ---- queries: c5 (strong) splits the batch of nq over the ranks; the
    # other forms give every rank its own nq queries
    strong = sharded and not args.weak
    if strong:
        assert nq % world == 0, f"nq={nq} does not split over {world} ranks"
        nq_loc = nq // world
        xq_glob = amd.float_rand(nq * d, 5678).reshape(nq, d)
        xq = np.ascontiguousarray(xq_glob[rank * nq_loc:(rank + 1) * nq_loc])
        nq_glob = nq
    else:
        nq_loc = nq
        xq = amd.float_rand(nq * d, 5678 + 7919 * rank).reshape(nq, d)
        nq_glob = nq * world
    # recall queries: the first of rank 0's (every rank of a sharded run
    # computes its shard's exact top-k for them; rank 0 merges)
    nr = min(args.recall_queries, nq_loc)
    # (float_rand's blocks depend on n: rank 0's rows are re-derived from its
    # whole set, not from a shorter call)
    xr = None
    if nr:
        xr = np.ascontiguousarray((xq_glob if strong else
                                   xq if rank == 0 else
                                   amd.float_rand(nq * d, 5678).reshape(nq, d))[:nr])
    gt_run = None
    t0 = time.time()
    index = amd.index_factory(d, cfg["desc"])
    nshard = max(world, args.shard_of) if sharded else world
    xb = None
    if sharded:
        # rows of the float_rand(nb * d, 1234) set, generated shard-wise and
        # added in chunks (no host image of the whole shard)
        xt = amd.float_rand_rows(nb, d, 1234, 0, 1, cfg["ntrain"])
        log(f"[rank {rank}] data: train {len(xt)} rows in {time.time() - t0:.1f}s")
        index.verbose = True  # k-means progress (keeps long builds visibly alive)
        index.train(xt)
        index.verbose = False
        del xt
        log(f"[rank {rank}] trained in {time.time() - t0:.1f}s")
        ids = np.arange(rank, nb, nshard, dtype=np.int64)
        chunk = 4_000_000
        for c0 in range(0, len(ids), chunk):
            cid = ids[c0:c0 + chunk]
            xc = amd.float_rand_rows(nb, d, 1234, rank + c0 * nshard, nshard, len(cid))
            index.add_with_ids(xc, cid)
            if nr:
                gt = amd.IndexFlatL2(d)
                gt.add(xc)
                Dg, Ig = gt.search(xr, k)
                Ig = np.where(Ig >= 0, cid[np.maximum(Ig, 0)], -1)
                if gt_run is not None:
                    Dg, Ig = amd.merge_knn_results(np.stack([gt_run[0], Dg]),
                                                   np.stack([gt_run[1], Ig]))
                gt_run = (Dg, Ig)
                del gt
            log(f"[rank {rank}] added {c0 + len(cid)} / {len(ids)} in {time.time() - t0:.1f}s")
        del xc
    else:
        xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
        index.train(xb[:cfg["ntrain"]])
        ids = (np.arange(nb, dtype=np.int64) if world == 1 or replicas
               else np.arange(rank, nb, world, dtype=np.int64))
        index.add_with_ids(xb[ids], ids)
    index.nprobe = nprobe
    if "efSearch" in cfg:
        amd.ParameterSpace().set_index_parameter(index, "quantizer_efSearch", cfg["efSearch"])
    index.sync_device()
    log(f"[rank {rank}] index {cfg['desc']} shard {len(ids)} vectors built in "
        f"{time.time() - t0:.1f}s")

    x_t = torch.from_numpy(xq).to(dev)
    D_t = torch.empty((nq_loc, k), dtype=torch.float32, device=dev)
    I_t = torch.empty((nq_loc, k), dtype=torch.int64, device=dev)
    hdist = ge.load_package_module("dist")

    def sharded_step_fn(ix):
        """IndexShardsIVF exchange (dist.py) with `ix` as this rank's shard."""
        cd_t = torch.empty((nq_loc, nprobe), dtype=torch.float32, device=dev)
        ci_t = torch.empty((nq_loc, nprobe), dtype=torch.int32, device=dev)
        Ds_t = torch.empty((world * nq_loc, k), dtype=torch.float32, device=dev)
        Is_t = torch.empty((world * nq_loc, k), dtype=torch.int64, device=dev)

        def quantize(x):
            ix.quantize_device(nq_loc, x.data_ptr(), nprobe, cd_t.data_ptr(), ci_t.data_ptr(),
                               stream)
            return cd_t, ci_t

        def search_pre(xa, ca, cda):
            ix.search_preassigned_device(world * nq_loc, xa.data_ptr(), k, nprobe,
                                         ca.data_ptr(), cda.data_ptr(), Ds_t.data_ptr(),
                                         Is_t.data_ptr(), stream)
            return Ds_t, Is_t

        def merge(Dr, Ir):
            amd.merge_knn_results_device(nq_loc, k, world, Dr.data_ptr(), Ir.data_ptr(),
                                         D_t.data_ptr(), I_t.data_ptr(), amd.METRIC_L2, stream)
            return D_t, I_t

        return lambda: hdist.sharded_search(x_t, k, quantize, search_pre, merge)

    if world == 1 or replicas:
        def step():
            index.search_device(nq_loc, x_t.data_ptr(), k, D_t.data_ptr(), I_t.data_ptr(),
                                stream)
    else:
        step = sharded_step_fn(index)

    def run_timed(step_fn, ix, steps, warmup):
        """warmup steps (the first untimed; the rest with every kernel stage
        timed: the per-step breakdown), then exactly `steps` steps between a
        barrier + synchronize on both sides, with only the dominant stage
        timed.  Returns (max elapsed over ranks, breakdown, dominant stage,
        its ms per step in the timed region)."""
        step_fn()
        torch.cuda.synchronize()
        nb_steps = max(1, warmup - 1)
        amd.set_kernel_timing(True)
        ix.reset_kernel_times()
        for _ in range(nb_steps):
            step_fn()
        torch.cuda.synchronize()
        brk = kernel_breakdown(ix, nb_steps)
        dom = max(brk, key=brk.get) if brk else None
        amd.set_kernel_timing(True, only=dom)
        ix.reset_kernel_times()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps):
            step_fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t1
        amd.set_kernel_timing(False)
        dom_ms = kernel_breakdown(ix, steps).get(dom, float("nan")) if dom else float("nan")
        if dom and not np.isfinite(dom_ms):
            # a stage timer that could not be read (c_api.cpp resolve_times)
            # fails the run instead of printing a NaN roofline
            raise RuntimeError(f"the dominant stage {dom!r} has no readable time "
                               f"({dom_ms}) over the timed steps")
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, brk, dom, dom_ms

    elapsed, brk, dom, dom_ms = run_timed(step, index, args.steps, args.warmup)
    ms_per_step = elapsed / args.steps * 1e3
    qps = nq_glob * args.steps / elapsed

    # ---- the step's algorithmic work (this rank), for the roofline models
    cd_h = torch.empty((nq_loc, nprobe), dtype=torch.float32, device=dev)
    ci_h = torch.empty((nq_loc, nprobe), dtype=torch.int32, device=dev)
    index.quantize_device(nq_loc, x_t.data_ptr(), nprobe, cd_h.data_ptr(), ci_h.data_ptr(),
                          stream)
    torch.cuda.synchronize()
    sizes = np.array([index.get_list_size(l) for l in range(index.nlist)], dtype=np.int64)
    ci_np = ci_h.cpu().numpy().astype(np.int64)
    cand_per_q = float(sizes[ci_np].sum()) / nq_loc
    scan_q = nq_loc if (world == 1 or replicas) else nq_glob  # queries this rank's scan sees
    dpad16 = -(-d // 16) * 16
    dpad32 = -(-d // 32) * 32
    lists = np.unique(ci_np)
    lists = lists[lists >= 0]
    work = {"cands": cand_per_q * scan_q, "dpad16": dpad16, "dpad32": dpad32, "d": d,
            "nlist": cfg["nlist"],
            "nq_coarse": nq_loc,
            # distinct lists of this rank's own batch (the scan of a sharded
            # step sees every rank's: at least these)
            "flat_rows": float(sizes[lists].sum()), "flat_row_bytes": 2 * dpad32 + 8,
            "flat_flops": cand_per_q * scan_q * 2 * 2.0 * dpad32}
    if "PQ" in cfg["desc"]:
        work["M"] = index.pq_info()["M"]
    if "efSearch" in cfg:
        hs = amd.cvar.hnsw_stats
        index.fold_device_stats()
        hs.reset()
        step()
        torch.cuda.synchronize()
        index.fold_device_stats()
        work["hnsw_ndis"] = float(amd.cvar.hnsw_stats.ndis)
        work["hnsw_nhops"] = float(amd.cvar.hnsw_stats.nhops)
        f32, q8 = amd.cvar.hnsw_row_stats
        work["hnsw_fp32_rows"], work["hnsw_q8_rows"] = float(f32), float(q8)
    kernels = []
    # PMC summaries are per workload: a grid point (--nprobe / --efsearch)
    # reads its own (profiles/rNN_<config>_np<P>_ef<E>_pmc.json), never the
    # default point's, whose kernels differ (c4 at efSearch 768 runs the
    # sequential HNSW kernel)
    pmc_key = args.config
    if args.nprobe or args.efsearch:
        pmc_key = f"{args.config}_np{nprobe}_ef{cfg.get('efSearch', 0)}"
    for nm, ms in sorted(brk.items(), key=lambda kv: -kv[1]):
        if ms < 0.1 * ms_per_step and nm != dom:
            continue
        ent = {"name": nm, "ms_per_step": ms, "frac_of_step": ms / ms_per_step}
        rf = kernel_roofline(nm, ms, work, pmc_key)
        if rf is not None:
            ent["roofline_frac"] = rf["frac"]
            ent["bound"] = rf["bound"]
        kernels.append(ent)
    roofline = kernel_roofline(dom, dom_ms, work, pmc_key) if dom else None
    if roofline is None and dom:
        roofline = {"bound": "latency", "achieved": None, "peak": None, "unit": None,
                    "frac": None, "traffic": None}
    if roofline is not None:
        roofline["kernel"] = dom
        roofline["kernel_ms_per_step"] = dom_ms
        roofline["kernel_frac_of_step"] = dom_ms / ms_per_step
        roofline["timing"] = ("HIP events around the stage's launches on its stream, "
                              "every timed step (only this stage timed)")

    # ---- c1-c4 at N > 1: the RCCL shard exchange beside the replicas
    shard_fig = None
    if replicas and not args.no_shard_figure and nb <= 2_000_000:
        shards = amd.index_ivf_to_shards(index, world, 1, devices=[gpu] * world)
        local = shards.shard(rank)
        local.nprobe = nprobe
        local.sync_device()
        sstep = sharded_step_fn(local)
        el2, brk2, dom2, dom2_ms = run_timed(sstep, local, args.steps, args.warmup)
        xbytes = nq_loc * (4 * d + 8 * nprobe)  # queries + coarse (f32 dis, i32 list)
        shard_fig = {
            "value": nq_glob * args.steps / el2, "unit": "queries/s",
            "ms_per_step": el2 / args.steps * 1e3, "global_batch": nq_glob,
            "scaling": "weak", "partition": "id % N (faiss GPU shard_type 1)",
            "vectors_per_gpu": int(local.ntotal),
            "collectives": "all_gather(queries, coarse dis, coarse ids) + "
                           "all_to_all(per-shard top-k) over RCCL",
            "bytes_out_per_rank": world * xbytes, "bytes_back_per_rank": world * nq_loc * k * 12,
            "dominant_kernel": dom2, "dominant_ms_per_step": dom2_ms}
        del local, shards

    # ---- PCIe-inclusive rate (host buffers through faiss_Index_search: query
    # upload + result download); reported beside `value`, never as it
    pcie = None
    if world == 1 and args.steps > 0:
        # three warm calls: a paged host search captures its pages' graphs
        # on the second and replays them from the third
        for _ in range(3):
            index.search(xq, k)
        nh = min(args.steps, 10)
        th = time.perf_counter()
        for _ in range(nh):
            index.search(xq, k)
        th = time.perf_counter() - th
        pcie = {"value": nq_loc * nh / th, "unit": "queries/s", "ms_per_step": th / nh * 1e3,
                "what": "faiss_Index_search on host buffers (H2D queries + search + D2H results)"}

    # ---- recall@10 of rank 0's first queries vs exact search
    recall = None
    if nr:
        step()
        torch.cuda.synchronize()
        I_res = I_t.cpu().numpy()[:nr]
        if sharded:
            # every rank's shard ground truth, merged on rank 0
            Dg = torch.from_numpy(np.ascontiguousarray(gt_run[0])).to(dev)
            Ig = torch.from_numpy(np.ascontiguousarray(gt_run[1])).to(dev)
            if world > 1:
                Dl = [torch.empty_like(Dg) for _ in range(world)]
                Il = [torch.empty_like(Ig) for _ in range(world)]
                dist.all_gather(Dl, Dg)
                dist.all_gather(Il, Ig)
                _, Igt = amd.merge_knn_results(np.stack([t.cpu().numpy() for t in Dl]),
                                               np.stack([t.cpu().numpy() for t in Il]))
            else:
                Igt = gt_run[1]
            gt_note = ("exact top-k over all ranks' shards" if world > 1 or not args.shard_of
                       else f"exact top-k over this rank's 1/{nshard} shard")
        else:
            gt = amd.IndexFlatL2(d)
            gt.add(xb)
            _, Igt = gt.search(xr, k)
            del gt
            gt_note = "exact top-k over the whole set"
        if rank == 0:
            recall = float(np.mean([len(set(a) & set(b)) / k for a, b in zip(I_res, Igt)]))

    # ---- CPU baseline, rank 0, N=1: the reference's own IndexIVF::search
    # (oracle/_ref/libfaissfull.so, compiled from /root/reference here and
    # shipped with the tree) on the same index (written by write_index, read
    # by the reference's read_index) with all host threads; the oracle
    # restatement when that library cannot be loaded.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, amd, index, xq, I_t.cpu().numpy(), k, nprobe)

    if rank == 0:
        par = (f"replicas{world}" if replicas else
               f"shards{world}" if world > 1 else "single")
        out = {
            "metric": "queries/sec @ recall@10, IVF4096 d=128 nq=10k nprobe=32; 1/2/4/8 GPUs"
            if args.config == "c2" else f"queries/sec, {cfg['workload']}",
            "value": qps, "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            # "weak": every GPU brings its own nq queries (replicas / --shard /
            # c5 --weak); "strong": c5's 100M set and 100k-query batch split
            # over the GPUs
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": cfg["workload"], "d": d, "nb": nb,
                       "vectors_per_gpu": len(ids), "nq_per_gpu": nq_loc,
                       "nprobe": nprobe, "k": k, "global_batch": nq_glob,
                       "parallelism": par, "recall_at_10": recall,
                       "recall_ground_truth": gt_note if nr else None,
                       "candidates_per_query": cand_per_q,
                       "efSearch": cfg.get("efSearch"),
                       "grid_point": bool(args.nprobe or args.efsearch)},
            "roofline": roofline,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
        }
        if shard_fig is not None:
            out["rccl_shards"] = shard_fig
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
