#!/usr/bin/env python3
"""Benchmark: queries/sec of the batched IVF search hot path on MI355X.

Metric (BASELINE.json): queries/sec @ recall@10, IVF4096 d=128 nq=10k
nprobe=32; 1/2/4/8 GPUs.  One step = one batched search of nq=10k synthetic
uniform queries (faiss float_rand, seed 5678) against IVF4096,Flat over 1M
synthetic vectors (float_rand seed 1234), k=10, inputs resident in HBM.

N=1: the whole path (query prep + bf16x3-MFMA coarse filter + exact re-rank +
list-centric bf16x2-MFMA scan + exact re-rank) through
faiss_amd_Index_search_device.  N>1 (torch.distributed.run, one rank per GPU):
c1-c4 are one-GPU configs, so every rank serves its own 10k queries from a
replica of the whole index (weak scaling, no collective on the data path;
--shard instead shards the index by id modulo N and runs the IndexShardsIVF
exchange of hnsw-ivf_amd/dist.py over RCCL); c5 is the sharded config: the
100M set is split by id modulo N and the 100k queries are exchanged.
"""
from __future__ import annotations

import argparse
import json
import math
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
    # the N ranks (ids == rank mod N, faiss GPU shard_type 1): every rank
    # holds 100M / N vectors and serves all 100k queries (strong scaling);
    # --shard-of 8 with --gpus 1 builds one rank's share of an 8-GPU run.
    "c5": dict(workload="IVF65536,PQ48 over 100M", desc="IVF65536,PQ48", d=96,
               nb=100_000_000, sharded=True, nq=100_000, nlist=65536, nprobe=64, k=10,
               ntrain=65536 * 39),
}
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 vector == fp32 MFMA peak
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
# dominant kernel per workload (device symbol substring) for the PMC traffic
DOMINANT = {"flat": "k_ivf_bf2_stream", "pq": "k_ivfpq_scan", "pqm": "k_ivfpq_filter"}


def pmc_traffic(config, kernel_sub):
    """HBM bytes per launch of the dominant kernel from the newest committed
    rocprofv3 --pmc summary for this workload (profiles/rNN_<config>_pmc.json,
    written by scripts/pmc_summary.py: FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE, separate passes)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        summ = json.load(f)
    for name, ent in summ.items():
        if kernel_sub in name and "hbm_bytes" in ent:
            return ent["hbm_bytes"], os.path.relpath(files[-1], ROOT)
    return None, None


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
                    help="c1-c4 at N > 1: shard the index by id %% N over RCCL "
                         "(IndexShardsIVF exchange) instead of one replica per GPU")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    # c1-c4 at N > 1 are replicas: their only collectives are the timing
    # barrier and max (gloo, host side); sharded runs exchange device tensors
    # over RCCL.  (local_rank % devices: a rehearsal of N ranks on fewer GPUs)
    replicas = world > 1 and not cfg.get("sharded", False) and not args.shard
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    if world > 1:
        if replicas:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    amd = ge.load_package()
    amd.set_device(gpu)
    dev = torch.device("cuda", gpu)
    stream = torch.cuda.current_stream().cuda_stream

    d, nb, nq, k, nprobe = cfg["d"], cfg["nb"], cfg["nq"], cfg["k"], cfg["nprobe"]
    qseed = 5678 + 7919 * rank
    xq = amd.float_rand(nq * d, qseed).reshape(nq, d)
    nr = min(args.recall_queries, nq) if rank == 0 else 0
    gt_run = None  # sharded: exact top-k of the shard, merged chunk by chunk
    t0 = time.time()
    index = amd.index_factory(d, cfg["desc"])
    sharded = cfg.get("sharded", False)
    nshard = max(world, args.shard_of) if sharded else world
    # c1-c4 name one GPU; at N > 1 each GPU serves its own queries from a
    # replica of the whole index (independent units, no collective) unless
    # --shard asks for the IndexShardsIVF exchange.  c5 is the sharded config.
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
                Dg, Ig = gt.search(xq[:nr], k)
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
    D_t = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I_t = torch.empty((nq, k), dtype=torch.int64, device=dev)

    if world == 1 or replicas:
        def step():
            index.search_device(nq, x_t.data_ptr(), k, D_t.data_ptr(), I_t.data_ptr(), stream)
    else:
        hdist = __import__("hnsw_ivf_amd.dist", fromlist=["sharded_search"])
        cd_t = torch.empty((nq, nprobe), dtype=torch.float32, device=dev)
        ci_t = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
        Ds_t = torch.empty((world * nq, k), dtype=torch.float32, device=dev)
        Is_t = torch.empty((world * nq, k), dtype=torch.int64, device=dev)

        def quantize(x):
            index.quantize_device(nq, x.data_ptr(), nprobe, cd_t.data_ptr(), ci_t.data_ptr(),
                                  stream)
            return cd_t, ci_t

        def search_pre(xa, ca, cda):
            index.search_preassigned_device(world * nq, xa.data_ptr(), k, nprobe, ca.data_ptr(),
                                            cda.data_ptr(), Ds_t.data_ptr(), Is_t.data_ptr(),
                                            stream)
            return Ds_t, Is_t

        def merge(Dr, Ir):
            amd.merge_knn_results_device(nq, k, world, Dr.data_ptr(), Ir.data_ptr(),
                                         D_t.data_ptr(), I_t.data_ptr(), amd.METRIC_L2, stream)
            return D_t, I_t

        def step():
            hdist.sharded_search(x_t, k, quantize, search_pre, merge)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    amd.set_kernel_timing(True)
    index.reset_kernel_times()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t1
    amd.set_kernel_timing(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if replicas else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    qps = world * nq * args.steps / elapsed

    # ---- dominant kernel: HIP events over the timed region (lib-side)
    kt = index.kernel_times()
    scan_name = "ivfpq_scan" if "PQ" in cfg["desc"] else "ivf_flat_scan"
    pq_mfma = any(nm == "ivfpq_filter" for (nm, _, _) in kt)
    if pq_mfma:
        scan_name = "ivfpq_filter"  # list-centric bf16 MFMA filter over decoded codes
    scan = [ms for (nm, ms, _) in kt if nm == scan_name]
    # a step may launch the kernel more than once (query chunks): the per-step
    # kernel time is the sum over the step's launches, priced against the
    # step's whole algorithmic work
    launches_per_step = len(scan) / args.steps if scan else 0.0
    scan_ms = float(np.sum(scan)) / args.steps if scan else float("nan")
    # algorithmic work of one scan launch: sum over (query, probe) of the
    # probed list length x per-candidate cost (Flat: 3*d flops; PQ: M bytes)
    nq_launch = nq if replicas else nq * world
    cd_h = torch.empty((nq, nprobe), dtype=torch.float32, device=dev)
    ci_h = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
    index.quantize_device(nq, x_t.data_ptr(), nprobe, cd_h.data_ptr(), ci_h.data_ptr(), stream)
    torch.cuda.synchronize()
    sizes = np.array([index.get_list_size(l) for l in range(index.nlist)], dtype=np.int64)
    cand_per_q = float(sizes[ci_h.cpu().numpy().astype(np.int64)].sum()) / nq
    cands = cand_per_q * nq_launch
    is_pq = "PQ" in cfg["desc"]
    traffic, traffic_src = pmc_traffic(
        args.config, DOMINANT["pqm" if pq_mfma else "pq" if is_pq else "flat"])
    if is_pq and not pq_mfma:
        M = index.pq_info()["M"]
        work = cands * M  # code bytes streamed (LUT-gather bound)
        achieved = work / (scan_ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                    "kernel": scan_name, "kernel_ms_per_step": scan_ms,
                    "launches_per_step": launches_per_step,
                    "algorithmic_bytes_per_step": work}
    elif is_pq:
        # IVF-PQ on the list-centric filter: codes are decoded to bf16 and
        # multiplied against the queries' bf16 hi + lo split (2 MFMA passes),
        # 2 * 2d bf16 flops per candidate, priced against the dense bf16 peak;
        # the streamed-code model (M bytes per candidate) is reported beside it
        M = index.pq_info()["M"]
        dpad = -(-d // 16) * 16
        work = cands * 2 * 2.0 * dpad
        achieved = work / (scan_ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS, "traffic": traffic,
                    "kernel": scan_name, "kernel_ms_per_step": scan_ms,
                    "launches_per_step": launches_per_step, "mfma_dtype": "bf16",
                    "algorithmic_flops_per_step": work, "flops_per_candidate": 4 * dpad,
                    "streamed_code_bytes_per_step": cands * M,
                    "streamed_code_gbs": cands * M / (scan_ms * 1e-3) / 1e9}
    else:
        # The list-centric filter streams, once per probed list, the bf16 hi
        # image of the rows (2 B/dim, dims padded to 32) plus two fp32 norms
        # per row (|y|^2 and the bf16 residual bound): its algorithmic bytes.
        # Its bf16 MFMA work (codes hi x queries hi+lo = 2 products of 2*dpad
        # flops per candidate) would take less time at the dense bf16 peak
        # than these bytes at the HBM peak, so HBM is the binding roofline;
        # the MFMA fraction is reported beside it.
        nprod = 3 if os.environ.get("FAISS_AMD_IVF_PREC") == "bf16x3" else 2
        dpad = -(-d // 32) * 32
        lists = np.unique(ci_h.cpu().numpy().astype(np.int64))
        lists = lists[lists >= 0]
        work = float(sizes[lists].sum()) * (2.0 * dpad + 8.0) * (1 if replicas else world)
        achieved = work / (scan_ms * 1e-3) / 1e9
        flops = cands * nprod * 2.0 * dpad
        mfma_tf = flops / (scan_ms * 1e-3) / 1e12
        roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                    "kernel": scan_name, "kernel_ms_per_step": scan_ms,
                    "launches_per_step": launches_per_step,
                    "algorithmic_bytes_per_step": work,
                    "bytes_per_row": 2 * dpad + 8,
                    "mfma_dtype": "bf16", "mfma_flops_per_step": flops,
                    "mfma_tflops": mfma_tf, "mfma_frac": mfma_tf / PEAK_BF16_TFLOPS,
                    "fp32_equivalent_tflops": cands * 3.0 * d / (scan_ms * 1e-3) / 1e12}
    if traffic is not None:
        # HBM bytes per launch from rocprofv3 PMC (committed summary), scaled
        # to the step's launches like `achieved`, and the bandwidth they imply
        # at the live kernel time
        roofline["traffic"] = traffic * launches_per_step
        roofline["traffic_source"] = traffic_src
        roofline["traffic_unit"] = "bytes/step"
        roofline["traffic_gbs"] = traffic * launches_per_step / (scan_ms * 1e-3) / 1e9

    # ---- PCIe-inclusive rate (host buffers through faiss_Index_search: query
    # upload + result download); reported beside `value`, never as it
    pcie = None
    if world == 1 and args.steps > 0:
        index.search(xq, k)
        nh = min(args.steps, 5)
        th = time.perf_counter()
        for _ in range(nh):
            index.search(xq, k)
        th = time.perf_counter() - th
        pcie = {"value": nq * nh / th, "unit": "queries/s", "ms_per_step": th / nh * 1e3,
                "what": "faiss_Index_search on host buffers (H2D queries + search + D2H results)"}

    # ---- recall@10 of this rank's queries vs exact search (subset; for
    # sharded configs against the rank's own shard)
    recall = None
    if nr:
        I_t2 = I_t.cpu().numpy()
        if sharded:
            Igt = gt_run[1]
        else:
            gt = amd.IndexFlatL2(d)
            gt.add(xb)
            _, Igt = gt.search(xq[:nr], k)
            del gt
        recall = float(np.mean([len(set(a) & set(b)) / k for a, b in zip(I_t2[:nr], Igt)]))

    # ---- CPU baseline, rank 0, N=1: the reference's own IndexIVF::search
    # (oracle/_ref/libfaissfull.so, compiled from /root/reference here and
    # shipped with the tree) on the same index (written by write_index, read
    # by the reference's read_index) with all host threads; the oracle
    # restatement when that library cannot be loaded.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, amd, index, xq, I_t.cpu().numpy(), k, nprobe)

    if rank == 0:
        out = {
            "metric": "queries/sec @ recall@10, IVF4096 d=128 nq=10k nprobe=32; 1/2/4/8 GPUs"
            if args.config == "c2" else f"queries/sec, {cfg['workload']}",
            "value": qps, "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            # "weak": every GPU brings its own nq queries (replicas / --shard);
            # "strong": c5's 100M set and 100k queries split over the GPUs
            "config": {"workload": cfg["workload"], "d": d, "nb": nb, "vectors_per_gpu": len(ids),
                       "nq_per_gpu": nq,
                       "nprobe": nprobe, "k": k, "global_batch": nq * world,
                       "parallelism": (f"replicas{world}" if replicas else
                                       f"shards{world}" if world > 1 else "single"),
                       "recall_at_10": recall, "candidates_per_query": cand_per_q},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
