"""Debug: IVF256,Flat d=64 nprobe=1 k=1 vs the oracle (fold image on/off by env)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import __graft_entry__ as ge
amd = ge.load_package(); orc = ge.load_oracle()
d, nb = 64, 100_000
xb = orc.float_rand(nb * d, 1234).reshape(nb, d)
xq = orc.float_rand(1000 * d, 5678).reshape(1000, d)[:200]
idx = amd.index_factory(d, "IVF256,Flat"); idx.train(xb); idx.add(xb)
ref = orc.IVFOracle.from_index(idx)
for nprobe, k in [(1, 1), (1, 5), (3, 1), (8, 10)]:
    idx.nprobe = nprobe
    D, I = idx.search(xq, k)
    Dr, Ir, _, _ = ref.search(xq, k, nprobe, nslices=1)
    bad = np.nonzero((I != Ir).any(axis=1))[0]
    print(f"nprobe={nprobe} k={k}: bad {bad.size}", (I[bad[:3]].tolist(), Ir[bad[:3]].tolist()) if bad.size else "", flush=True)
