"""IndexIVF::search_device replayed from a captured hipGraph (ivf.cpp): the
second identical call captures, later ones replay.  Every replay must give
the eager result; a change the graph cannot see (new vectors added, nprobe,
k, another output buffer, FAISS_AMD_GRAPH=0) must retire it; kernel timing
must keep one record per replay."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Bufs:
    def __init__(self, xq, k):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.n, self.k = xq.shape[0], k
        self.ptrs = []
        self.px = self._alloc(xq.nbytes)
        self.pd = self._alloc(self.n * k * 4)
        self.pi = self._alloc(self.n * k * 8)
        x = np.ascontiguousarray(xq, dtype=np.float32)
        self.hip.hipMemcpy(self.px, x.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(x.nbytes), 1)

    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 4))) == 0
        self.ptrs.append(p)
        return p

    def search(self, idx, k=None):
        k = k or self.k
        idx.search_device(self.n, self.px.value, k, self.pd.value, self.pi.value)
        assert self.hip.hipDeviceSynchronize() == 0
        D = np.empty((self.n, k), np.float32)
        I = np.empty((self.n, k), np.int64)
        self.hip.hipMemcpy(D.ctypes.data_as(ctypes.c_void_p), self.pd, ctypes.c_size_t(D.nbytes), 2)
        self.hip.hipMemcpy(I.ctypes.data_as(ctypes.c_void_p), self.pi, ctypes.c_size_t(I.nbytes), 2)
        return D, I

    def close(self):
        for p in self.ptrs:
            self.hip.hipFree(p)


@pytest.mark.parametrize("desc", ["IVF256,Flat", "IVF256,PQ16", "IVF2048,PQ16"])
def test_graph_replay_equals_eager(amd, gpu, monkeypatch, desc):
    d, nb, nq, k = 64, 60_000, 3000, 10
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, desc)
    idx.train(xb[:30_000])
    idx.add(xb[:40_000])
    idx.nprobe = 16
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    b = Bufs(xq, k)
    try:
        monkeypatch.setenv("FAISS_AMD_GRAPH", "0")
        ref = b.search(idx)
        monkeypatch.delenv("FAISS_AMD_GRAPH")
        for _ in range(5):  # eager, capture, replays
            D, I = b.search(idx)
            np.testing.assert_array_equal(I, ref[1])
            np.testing.assert_array_equal(D, ref[0])
        # kernel timing: the same records per call as the eager path, the
        # quantizer's stages included (the capture and the replays record
        # fresh events at the timed stages' nodes), every one a completed
        # measurement, and no HIP error left behind by reading them (r05: the
        # captured events read "invalid resource handle", picked up by the
        # caller's next HIP check)
        import collections
        counts = []
        for only in (None, "coarse_filter"):
            amd.set_kernel_timing(True, only=only)
            for genv in ("0", None):
                if genv:
                    monkeypatch.setenv("FAISS_AMD_GRAPH", genv)
                else:
                    monkeypatch.delenv("FAISS_AMD_GRAPH")
                idx.reset_kernel_times()
                for _ in range(4):
                    b.search(idx)
                kt = idx.kernel_times()
                assert b.hip.hipGetLastError() == 0
                assert all(np.isfinite(ms) and ms > 0 for _, ms, _ in kt), kt
                counts.append(collections.Counter(nm for nm, _, _ in kt))
        amd.set_kernel_timing(False)
        assert counts[0] and counts[0] == counts[1], counts
        assert counts[2] == counts[3], counts
        if "coarse_filter" in counts[0]:  # (the quantizer's MFMA path ran)
            assert counts[2] == collections.Counter({"coarse_filter": 4}), counts
        # a change the host sees retires the graph
        idx.nprobe = 8
        monkeypatch.setenv("FAISS_AMD_GRAPH", "0")
        ref8 = b.search(idx)
        monkeypatch.delenv("FAISS_AMD_GRAPH")
        for _ in range(3):
            np.testing.assert_array_equal(b.search(idx)[1], ref8[1])
        idx.add(xb[40_000:])
        monkeypatch.setenv("FAISS_AMD_GRAPH", "0")
        refa = b.search(idx)
        monkeypatch.delenv("FAISS_AMD_GRAPH")
        assert not np.array_equal(refa[1], ref8[1])
        for _ in range(3):
            D, I = b.search(idx)
            np.testing.assert_array_equal(I, refa[1])
            np.testing.assert_array_equal(D, refa[0])
        Dk, Ik = b.search(idx, k=5)
        np.testing.assert_array_equal(Ik, refa[1][:, :5])
    finally:
        b.close()


def test_graph_replay_new_queries_same_buffer(amd, orc, gpu, monkeypatch):
    """The serving loop the graph is for rewrites its input buffer between
    calls: c2's geometry (IVF4096,Flat, 1M vectors, nprobe 32, 10k queries),
    three different query sets written into the same device buffer, each
    searched by a replay of the graph captured on the first set.  Every
    replay equals the eager search of its own queries bit for bit, and a
    subset of each set equals the oracle."""
    d, nb, nq, k = 128, 1_000_000, 10_000, 10
    xb = amd.float_rand(nb * d, 1234).reshape(nb, d)
    idx = amd.index_factory(d, "IVF4096,Flat")
    idx.train(xb[:200_000])
    idx.add(xb)
    idx.nprobe = 32
    sets = [amd.float_rand(nq * d, seed).reshape(nq, d) for seed in (5678, 91, 4242)]
    b = Bufs(sets[0], k)
    ref = orc.IVFOracle.from_index(idx)
    rows = np.arange(0, nq, 25)
    try:
        eager = []
        monkeypatch.setenv("FAISS_AMD_GRAPH", "0")
        for xq in sets:
            b.hip.hipMemcpy(b.px, xq.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(xq.nbytes), 1)
            eager.append(b.search(idx))
        monkeypatch.delenv("FAISS_AMD_GRAPH")
        for rnd in range(2):
            for i, xq in enumerate(sets):
                b.hip.hipMemcpy(b.px, xq.ctypes.data_as(ctypes.c_void_p),
                                ctypes.c_size_t(xq.nbytes), 1)
                D, I = b.search(idx)  # round 0, set 0: eager, set 1: capture, then replays
                np.testing.assert_array_equal(I, eager[i][1])
                np.testing.assert_array_equal(D, eager[i][0])
        for i, xq in enumerate(sets):
            Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), k, 32, nslices=1)
            np.testing.assert_array_equal(eager[i][1][rows], Ir)
            np.testing.assert_array_equal(eager[i][0][rows], Dr)
        assert not np.array_equal(eager[0][1], eager[1][1])
    finally:
        b.close()


def test_graph_retired_by_same_size_content_change(amd, gpu, monkeypatch):
    """A reset + add of the same number of different vectors, synchronised by
    a host search(), leaves ntotal and the buffers unchanged; the next
    search_device must still not replay the graph captured on the old
    content (the upload bumps the index's content version)."""
    d, nb, nq, k = 64, 20_000, 500, 10
    xa = amd.float_rand(nb * d, 11).reshape(nb, d)
    xb = amd.float_rand(nb * d, 12).reshape(nb, d)
    idx = amd.index_factory(d, "IVF64,Flat")
    idx.train(xa)
    idx.add(xa)
    idx.nprobe = 8
    xq = amd.float_rand(nq * d, 13).reshape(nq, d)
    b = Bufs(xq, k)
    try:
        for _ in range(3):  # eager, capture, replay
            old = b.search(idx)
        idx.reset()
        idx.add(xb)
        idx.search(xq[:50], k)  # host entry point: uploads, clears the dirty flag
        monkeypatch.setenv("FAISS_AMD_GRAPH", "0")
        ref = b.search(idx)
        monkeypatch.delenv("FAISS_AMD_GRAPH")
        assert not np.array_equal(ref[1], old[1])
        for _ in range(3):
            D, I = b.search(idx)
            np.testing.assert_array_equal(I, ref[1])
            np.testing.assert_array_equal(D, ref[0])
    finally:
        b.close()
