"""Path B parity on the GPU: NCC (CrossCorrelation NormalizedCrossCorrelation /
TimeDomain) and DTW (symmetric2, Euclidean) vs the fp64 oracle.
Peak lag / DTW path are bit-exact; correlations and costs are bit-identical
(same float64 operation order, no FMA)."""
import numpy as np
import pytest

import oracle as O
import sonar

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("na,nb,lag,maxlag", [(5000, 5000, 37, 500), (4000, 5200, -120, 300), (300, 300, 0, 1000),
                                             (1, 1, 0, 5), (2000, 100, 10, 60)])
def test_ncc_matches_oracle(ctx, na, nb, lag, maxlag):
    rng = np.random.default_rng(na + nb)
    base = np.convolve(rng.standard_normal(max(na, nb) + abs(lag) + 10), np.ones(5) / 5, "same")
    a = base[max(lag, 0): max(lag, 0) + na]
    b = base[max(-lag, 0): max(-lag, 0) + nb]
    corr, met = ctx.ncc(a, b, maxlag)
    rc, rm = O.ncc(a, b, maxlag)
    assert np.array_equal(corr, rc)
    for k in ("peak_lag", "peak_index", "overlap_length", "num_lags"):
        assert met[k] == rm[k]
    for k in ("peak_correlation", "snr", "sharpness", "second_peak", "peak_to_sidelobe", "p_value"):
        assert met[k] == pytest.approx(rm[k], rel=1e-12, abs=1e-12)


def test_ncc_errors(ctx):
    with pytest.raises(sonar.SonarError, match="empty signals provided"):
        ctx.ncc(np.zeros(0), np.ones(5), 3)


@pytest.mark.parametrize("nq,nr,dim,band", [(100, 120, 12, -1), (257, 130, 1, -1), (64, 64, 12, -1),
                                           (300, 280, 3, 40), (1, 1, 2, -1), (1, 70, 1, -1), (130, 1, 4, -1),
                                           (500, 499, 12, 5), (2000, 1500, 12, -1), (193, 2500, 12, 300),
                                           (700, 650, 5, -1), (129, 128, 1, 2)])
def test_dtw_matches_oracle(ctx, nq, nr, dim, band):
    rng = np.random.default_rng(nq * 7 + nr)
    q = rng.random((nq, dim))
    r = rng.random((nr, dim))
    got = ctx.dtw(q, r, band=band, want_cost=True)
    ref = O.dtw(q, r, band=band, want_cost=True)
    assert np.array_equal(got["path_q"], ref["path_q"]) and np.array_equal(got["path_r"], ref["path_r"])
    assert np.array_equal(got["cost"], ref["cost"])
    assert np.array_equal(got["path_cost"], ref["path_cost"], equal_nan=True)   # Inf - Inf off the band
    assert got["distance"] == ref["distance"]


def test_dtw_ties_identical_sequences(ctx):
    q = np.repeat(np.arange(5.0), 3)[:, None]     # many equal costs: exercises the tie rule
    got = ctx.dtw(q, q)
    ref = O.dtw(q, q)
    assert np.array_equal(got["path_q"], ref["path_q"]) and np.array_equal(got["path_r"], ref["path_r"])
    assert got["distance"] == 0.0


def test_dtw_errors(ctx):
    with pytest.raises(sonar.SonarError, match="empty sequences provided"):
        ctx.dtw(np.zeros((0, 2)), np.ones((3, 2)))


def test_dtw_nonfinite_inputs(ctx):
    """NaN / Inf inputs take the math.Min path with Go's NaN / -Inf / -0 rules."""
    rng = np.random.default_rng(5)
    q = rng.random((150, 12))
    r = rng.random((140, 12))
    q[20, 3] = np.nan
    r[77, 0] = np.inf
    q[90, 5] = -np.inf
    got = ctx.dtw(q, r, want_cost=True)
    ref = O.dtw(q, r, want_cost=True)
    assert np.array_equal(got["path_q"], ref["path_q"]) and np.array_equal(got["path_r"], ref["path_r"])
    assert np.array_equal(got["cost"], ref["cost"], equal_nan=True)
    assert np.array_equal(got["path_cost"], ref["path_cost"], equal_nan=True)


def test_dtw_large_band_pipeline(ctx):
    """126 bands in flight: the sc1 edge hand-off between bands under full occupancy."""
    rng = np.random.default_rng(11)
    n = 8000
    q = rng.random((n, 12))
    r = np.roll(q, 23, axis=0) + 0.05 * rng.random((n, 12))
    got = ctx.dtw(q, r)
    ref = O.dtw(q, r)
    assert np.array_equal(got["path_q"], ref["path_q"]) and np.array_equal(got["path_r"], ref["path_r"])
    assert np.array_equal(got["path_cost"], ref["path_cost"])
    assert got["distance"] == ref["distance"]
