"""bench.py's roofline helpers on the CPU (no GPU calls): the C5 roofline's algorithmic bytes and
the committed kernel-family shares it carries, and the committed PMC summaries the bench line
reads (the newest per pattern)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def test_c5_roofline_bytes_and_families():
    F = 10_333
    samples = 2 * 2_646_000
    r = bench.c5_roofline(1000, 0.5, samples, F)
    per_pair = samples * 8 + bench.DTW_BYTES_PER_CELL * F * F
    assert r["alg_bytes_per_pair"] == pytest.approx(per_pair)
    assert r["achieved"] == pytest.approx(1000 * per_pair / 0.5 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS)
    fam = r["kernel_families"]
    assert fam is not None and fam["source"].startswith("profiles/")
    shares = fam["shares"]
    assert abs(sum(shares.values()) - 1.0) < 1e-3
    assert {"dtw_band", "features"} <= set(shares)


def test_committed_pmc_summaries_load():
    dtw = bench.load_pmc_bytes("*dtw_pmc*.json", "dtw_band_kernel<12, true, false, false")
    assert dtw is not None and dtw["bytes_per_launch"] > 0
