"""Arenas past the 32-bit work-item count of one dispatch.

An AQL dispatch counts a grid dimension's work-items in 32 bits.  The image
builders launched one work-item per bf16 slot — rows x (DB + 8) of them —
so past 2^32 / (DB + 8) arena rows (31.6M at d = 128) the count wrapped and
the tail of the image was never written (round 5: wrong filter keys on a
100M-row IVF-PQ image).  They are grid-strided now and every launch takes
its grid from a checked helper (csrc/common.h kgrid / stride_grid).

  * IVF-Flat d = 128, 33M vectors (33.1M arena rows): the stream image
    k_ivf_bf2_stream reads (rows x 136 slots = 4.5e9 > 2^32) checked row by
    row against the host formula around the old wrap point and at the end
    of the arena, and a 256-query subset (~90 of its probes land in
    lists past the old wrap row) searched bit-exact against the
    oracle (faiss/IndexIVFFlat.cpp:155-179 scanner, IndexIVF::search).
  * IVF2048,PQ48 d = 96, 42M vectors with the decoded image
    (FAISS_AMD_PQ_FILTER=image: rows x 104 slots = 4.4e9 > 2^32): the last
    rows' decoded residuals and bias fragments against the host decode of
    their codes, and a query subset searched through the image filter
    bit-exact against the oracle.
Data: faiss float_rand streams (xb seed 1234, xq seed 5678).
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

U32 = 2 ** 32


def bf16_bits(x):
    """float32 -> bf16 bit pattern, round to nearest even (as __bf16 casts)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def bf16_val(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def ran_stages(amd, idx, fn):
    amd.set_kernel_timing(True)
    try:
        idx.reset_kernel_times()
        out = fn()
        names = {nm for nm, _, _ in idx.kernel_times()}
    finally:
        amd.set_kernel_timing(False)
    return out, names


def check_tail(tail, real, target):
    """The 16-byte bias fragment {h, m, lo, 1, 1, 1, 0, 0} of a real row
    (h + m + lo = target within the split's 2^-24 relative error) or the
    padding fragment {-inf, 0, 0, 1, 1, 1, 0, 0}."""
    one = 0x3F80
    assert (tail[:, 3:6] == one).all() and (tail[:, 6:8] == 0).all()
    pad = ~real
    assert (tail[pad, 0] == 0xFF80).all() and (tail[pad, 1:3] == 0).all()
    s = (bf16_val(tail[real, 0]).astype(np.float64) + bf16_val(tail[real, 1])
         + bf16_val(tail[real, 2]))
    t = target[real].astype(np.float64)
    assert np.all(np.abs(s - t) <= 1e-6 * np.abs(t) + 1e-30), np.abs(s - t).max()


@pytest.fixture(scope="module")
def flat33m(amd):
    d, nb = 128, 33_000_000
    idx = amd.index_factory(d, "IVF2048,Flat")
    idx.train(amd.float_rand_rows(nb, d, 1234, 0, 1, 262_144))
    for c0 in range(0, nb, 3_000_000):
        idx.add(amd.float_rand_rows(nb, d, 1234, c0, 1, min(3_000_000, nb - c0)))
    idx.nprobe = 8
    return idx


def test_flat_stream_image_past_2_32_work_items(amd, gpu, flat33m):
    idx = flat33m
    rb, rows = idx.debug_rows(2)
    DB = 128
    assert rb == 2 * DB + 16
    assert rows * (DB + 8) > U32, rows  # the launch the old builder wrapped
    wrap_row = U32 // (DB + 8)
    for r0 in (wrap_row - 2048, rows - 4096):
        n = 4096
        img = idx.debug_rows(2, r0, n).view(np.uint16)       # [n][DB + 8] bf16
        code = idx.debug_rows(0, r0, n).view(np.float32)     # [n][128] fp32
        rl = idx.debug_rows(1, r0, n).view(np.uint32)[:, 0]  # row -> list
        real = rl != 0xFFFFFFFF
        assert real.any()
        assert np.array_equal(img[:, :DB], bf16_bits(code)), f"rows from {r0}"
        ynorm = (code.astype(np.float64) ** 2).sum(1).astype(np.float32)
        check_tail(img[:, DB:], real, -0.5 * ynorm)


def test_flat_search_past_32m_rows(amd, orc, gpu, flat33m):
    idx = flat33m
    d, nq = 128, 2048
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    (D, I), names = ran_stages(amd, idx, lambda: idx.search(xq, 10))
    assert "ivf_flat_scan" in names and "ivf_exact_scan" not in names, names
    rows = np.arange(0, nq, 8)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[rows]), 10, 8, nslices=1)
    bad = np.nonzero((I[rows] != Ir).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} queries differ, first {rows[bad[:4]]}"
    assert np.array_equal(D[rows], Dr)


def test_pq_image_past_2_32_work_items(amd, orc, gpu, monkeypatch):
    monkeypatch.setenv("FAISS_AMD_PQ_FILTER", "image")
    d, nb, M = 96, 42_000_000, 48
    idx = amd.index_factory(d, f"IVF2048,PQ{M}")
    idx.train(amd.float_rand_rows(nb, d, 1234, 0, 1, 262_144))
    for c0 in range(0, nb, 3_000_000):
        idx.add(amd.float_rand_rows(nb, d, 1234, c0, 1, min(3_000_000, nb - c0)))
    idx.nprobe = 8
    nq = 1024
    xq = amd.float_rand(nq * d, 5678).reshape(nq, d)
    # (the first search uploads the index and builds the image)
    (D, I), names = ran_stages(amd, idx, lambda: idx.search(xq, 10))
    assert "ivfpq_filter" in names and "ivf_exact_scan" not in names, names
    rb, rows = idx.debug_rows(2)
    DB = 96
    assert rb == 2 * DB + 16 and rows * (DB + 8) > U32, (rb, rows)
    cent = np.asarray(idx.pq_centroids, np.float32).reshape(M, 256, d // M)
    n = 4096
    r0 = rows - n
    img = idx.debug_rows(2, r0, n).view(np.uint16)
    codes = idx.debug_rows(0, r0, n)[:, :M]
    rl = idx.debug_rows(1, r0, n).view(np.uint32)[:, 0]
    real = rl != 0xFFFFFFFF
    assert real.any()
    yr = cent[np.arange(M)[None, :], codes.astype(np.int64)].reshape(n, d)  # decoded y_R
    yr[~real] = 0.0
    assert np.array_equal(img[:, :DB], bf16_bits(yr))
    # bias tail: -term / 2, term = |y_R|^2 + 2 <y_C, y_R> (IndexIVFPQ
    # precomputed-table term; checked through h + m + lo's consistency with
    # the decoded row and its list's centroid)
    q = idx.quantizer
    yc = np.asarray(q.xb, np.float32).reshape(-1, d)[np.where(real, rl, 0)]
    term = ((yr.astype(np.float64) ** 2).sum(1) + 2 * (yc * yr).sum(1)).astype(np.float32)
    tail = img[:, DB:]
    assert (tail[:, 3:6] == 0x3F80).all() and (tail[:, 6:8] == 0).all()
    assert (tail[~real, 0] == 0xFF80).all() and (tail[~real, 1:3] == 0).all()
    s = (bf16_val(tail[real, 0]).astype(np.float64) + bf16_val(tail[real, 1])
         + bf16_val(tail[real, 2]))
    t = -0.5 * term[real].astype(np.float64)
    # (the device evaluates term in fp32 in its own order: relative to the
    # magnitudes summed, not to the possibly cancelling result)
    scale = ((yr.astype(np.float64) ** 2).sum(1) + 2 * np.abs(yc * yr).sum(1))[real]
    assert np.all(np.abs(s - t) <= 1e-5 * scale + 1e-6), np.abs(s - t).max()
    # the image filter's results, bit-exact on a query subset
    sub = np.arange(0, nq, 8)
    ref = orc.IVFOracle.from_index(idx)
    Dr, Ir, _, _ = ref.search(np.ascontiguousarray(xq[sub]), 10, 8, nslices=1)
    bad = np.nonzero((I[sub] != Ir).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} queries differ, first {sub[bad[:4]]}"
    assert np.array_equal(D[sub], Dr)
