#!/usr/bin/env python3
"""One c4 quantizer search (the register HNSW kernel over the 10k bench
queries at k = 64, efSearch 64) for rocprofv3 --pmc passes; FAISS_AMD_HNSW_*
environment as set by the caller."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

amd = ge.load_package()
d, nb, nq = 128, 10_000_000, 10_000
idx = amd.index_factory(d, "IVF16384_HNSW32,Flat")
idx.train(amd.float_rand_rows(nb, d, 1234, 0, 1, 638_976))
q = idx.quantizer
q.efSearch = int(os.environ.get("EF", "64"))
xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
q.search(xq, 64)
q.search(xq, 64)
print("done", flush=True)
