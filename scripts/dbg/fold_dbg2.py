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
idx.nprobe = 1
os.environ["FAISS_AMD_IVF_DUMP"] = "gpurun_out/dump.bin"
D, I = idx.search(xq, 1)
del os.environ["FAISS_AMD_IVF_DUMP"]
Dr, Ir, _, _ = ref.search(xq, 1, 1, nslices=1)
raw = np.fromfile("gpurun_out/dump.bin", dtype=np.uint8)
n, KE = 200, 8
keys = raw[:4 * n * KE].view(np.uint32).reshape(n, KE)
recs = raw[4 * n * KE:4 * n * KE + 32 * n].view(np.float32).reshape(n, 8)
img = raw[4 * n * KE + 32 * n:].reshape(4, -1)
print("image tails", [r[-16:].view(np.uint16).tolist() for r in img])
fold = os.environ.get("FAISS_AMD_IVF_FOLD") != "0"
for lm in (7, 8, 9):
    pass
lowmask = np.uint32((1 << 7) - 1)
for q in range(6):
    kk = keys[q]
    lo = (kk & ~lowmask).view(np.float32)
    hi = (kk | lowmask).view(np.float32)
    if fold:
        lo, hi = np.maximum(-2 * lo, 0), np.maximum(-2 * hi, 0)
    print(q, "gpu", I[q], D[q], "ref", Ir[q], Dr[q])
    print("   keys", [hex(x) for x in kk])
    print("   lo", lo, "\n   hi", hi)
    print("   pb", recs[q, :4], "mmax", recs[q, 4], "off/len", recs[q, 5:7].view(np.uint32))
