"""bench.py's host-side models (no GPU): the PMC summary entry a bench line's
`traffic` is taken from (the search's launch, not the build's — entries are
kept per launch grid and the one that ran last wins), and the HNSW byte model
(fp32 rows, int8-image rows and neighbour-id rows, priced against L2)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_pmc_traffic_takes_the_last_launched_grid(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    name = "void faiss_amd::kern::k_hnsw_exact_reg<true, false, true, false>(...)"
    summ = {
        f"{name} [grid 2097152]": {"launches": 300, "last_dispatch": 600,
                                    "hbm_bytes": 9e9, "hbm_read_bytes": 8e9,
                                    "hbm_write_bytes": 1e9},
        f"{name} [grid 640000]": {"launches": 4, "last_dispatch": 700,
                                   "hbm_bytes": 1.6e9, "hbm_read_bytes": 1.5e9,
                                   "hbm_write_bytes": 1e8},
        f"{name} [grid 368640]": {"launches": 1, "last_dispatch": 601,
                                   "hbm_bytes": 3e8, "hbm_read_bytes": 2e8,
                                   "hbm_write_bytes": 1e8},
    }
    (prof / f"r{bench.ROUND:02d}_c4_pmc.json").write_text(json.dumps(summ))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src = bench.pmc_traffic("c4", "hnsw_exact")
    assert traffic == 1.6e9 and src.endswith("_c4_pmc.json")
    assert bench.pmc_traffic("c4", "ivf_flat_scan") == (None, None)


def test_hnsw_roofline_prices_rows_read():
    work = {"hnsw_ndis": 1000.0, "hnsw_fp32_rows": 150.0, "hnsw_q8_rows": 900.0,
            "hnsw_nhops": 40.0, "d": 128}
    r = bench.kernel_roofline("hnsw_exact", 1e-3, work, "none")
    assert r["bound"] == "l2" and r["unit"] == "GB/s"
    b = 150 * 4 * 128 + 900 * 148 + 40 * 256
    assert r["algorithmic_bytes_per_step"] == b
    assert abs(r["achieved"] - b / 1e-6 / 1e9) < 1e-9
    assert 0 < r["frac"] < 1
