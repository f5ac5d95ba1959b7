#!/usr/bin/env python3
"""Experiment: the c2 search step launched directly vs replayed from a HIP
graph captured around faiss_amd_Index_search_device (torch.cuda.graph on a
side stream).  Prints per-step times and checks the results are identical."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
d, nb, nq, nlist, nprobe, k = 128, 1_000_000, 10_000, 4096, 32, 10
xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
index = amd.index_factory(d, f"IVF{nlist},Flat")
index.train(xb[:200_000])
index.add(xb)
index.nprobe = nprobe
index.sync_device()
dev = torch.device("cuda", 0)
x_t = torch.from_numpy(xq).to(dev)
D_t = torch.empty((nq, k), dtype=torch.float32, device=dev)
I_t = torch.empty((nq, k), dtype=torch.int64, device=dev)
side = torch.cuda.Stream()


def step(s):
    index.search_device(nq, x_t.data_ptr(), k, D_t.data_ptr(), I_t.data_ptr(), s)


steps = int(os.environ.get("STEPS", "200"))
with torch.cuda.stream(side):
    for _ in range(5):
        step(side.cuda_stream)
    torch.cuda.synchronize()
    D0, I0 = D_t.clone(), I_t.clone()
    t = time.perf_counter()
    for _ in range(steps):
        step(side.cuda_stream)
    torch.cuda.synchronize()
    direct = (time.perf_counter() - t) / steps * 1e3
print(f"direct: {direct:.4f} ms/step", flush=True)

g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    step(side.cuda_stream)
torch.cuda.synchronize()
D_t.zero_()
I_t.zero_()
g.replay()
torch.cuda.synchronize()
assert torch.equal(D_t, D0) and torch.equal(I_t, I0), "graph replay differs"
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
assert torch.equal(D_t, D0) and torch.equal(I_t, I0), "graph replay differs (repeat)"
t = time.perf_counter()
for _ in range(steps):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t) / steps * 1e3
print(f"graph:  {graph:.4f} ms/step (results identical)", flush=True)
