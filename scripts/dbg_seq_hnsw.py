import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge
amd = ge.load_package(); orc = ge.load_oracle()
for d in (37, 128):
    nb = 5000
    xb = orc.float_rand(nb * d, 61).reshape(nb, d)
    xq = orc.float_rand(50 * d, 63).reshape(50, d)
    h = amd.IndexHNSWFlat(d, 16); h.add(xb)
    g = orc.HNSWGraph.from_index(h)
    for ef, k, env in [(257, 5, None), (100, 10, "1"), (100, 10, None), (768, 10, None)]:
        if env: os.environ["FAISS_AMD_HNSW_EXACT"] = env
        else: os.environ.pop("FAISS_AMD_HNSW_EXACT", None)
        h.efSearch = ef
        D, I = h.search(xq, k)
        Dr, Ir = g.search(xq, k, ef)
        bad = (I != Ir).any(1)
        print(d, ef, k, env, "bad", bad.sum(), "nan", np.isnan(D).sum(), flush=True)
        if bad.any():
            i = np.nonzero(bad)[0][0]
            print("  ", I[i], Ir[i]); print("  ", D[i], Dr[i])
