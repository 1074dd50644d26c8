"""Shared parity checks for the GPU tests (test infrastructure).

* ``assert_rel``: per-element relative error with an explicit floor, so small-valued elements
  are checked too (|got - ref| <= rtol * max(|ref|, floor)).
* ``assert_mfcc``: MFCC rows; every coefficient within ``rtol`` of the row norm, and per
  coefficient relative to itself in tiers (f32: 1e-4 for |c| > 0.1 ||row||, 1e-3 for
  |c| > 0.01 ||row||, 1e-2 for |c| > 1e-3 ||row||; f64: at most 1e-6).  Smaller coefficients are
  rounding noise relative to themselves (SURVEY.md §7 "fp32 vs 1e-4 relative").
* ``rolloff_borderline`` / ``assert_rolloff``: the rolloff bin is an index and must be exact.
  The kernel reproduces Go's sequential chains (spectral_rolloff.go:29-49) on ITS magnitudes;
  those differ from the oracle's by FFT rounding, so a mismatch is allowed only on a frame whose
  oracle cumulative energy sits within ``margin`` * total of the 85 % target at the chosen bin
  (np.cumsum is a sequential running sum, the oracle's and Go's order).
"""
import numpy as np


def assert_rel(got, ref, rtol, floor, name=""):
    g, r = np.asarray(got, float), np.asarray(ref, float)
    if g.size == 0 and r.size == 0:
        return 0.0
    if g.size == 1 and r.size == 1:
        g, r = g.reshape(()), r.reshape(())
    assert g.shape == r.shape, (name, g.shape, r.shape)
    nan = np.isnan(r) | np.isnan(g)
    assert np.array_equal(np.isnan(g), np.isnan(r)), name
    g, r = np.where(nan, 0, g), np.where(nan, 0, r)
    err = np.abs(g - r) / np.maximum(np.abs(r), floor)
    e = float(np.max(err))
    assert e <= rtol, (name, e, int(np.argmax(err)))
    return e


def mfcc_errors(got, ref):
    """(max error relative to the row norm, max per-coefficient relative error over
    |ref| > 1e-3 ||row||, number of frames failing 1e-4 in either measure)."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    norms = np.linalg.norm(ref, axis=1)[:, None]
    norms = np.where(norms == 0, 1.0, norms)
    e_row = np.abs(got - ref) / norms
    big = np.abs(ref) > 1e-3 * norms
    e_coef = np.where(big, np.abs(got - ref) / np.where(big, np.abs(ref), 1.0), 0.0)
    bad = int(np.count_nonzero((e_row.max(axis=1) > 1e-4) | (e_coef.max(axis=1) > 1e-4)))
    return float(e_row.max()), float(e_coef.max()), bad


# per-coefficient tiers of assert_mfcc: (coefficient floor as a fraction of the row norm, bound
# as a multiple of rtol).  f32 (rtol 1e-4, the north star's "float features within 1e-4
# relative"): |c| > 0.1 ||row|| within 1e-4 of itself, |c| > 0.01 ||row|| within 1e-3, |c| > 1e-3
# ||row|| within 1e-2 (measured worst cases over the whole hour: 1.6e-5, ~1.1e-4, 6.7e-4).
MFCC_TIERS_F32 = ((1e-1, 1.0), (1e-2, 10.0), (1e-3, 100.0))


def mfcc_tier_errors(got, ref):
    """{floor: max relative error of the coefficients with |ref| > floor * ||row||}"""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    norms = np.linalg.norm(ref, axis=1)[:, None]
    norms = np.where(norms == 0, 1.0, norms)
    out = {}
    for fl, _ in MFCC_TIERS_F32:
        big = np.abs(ref) > fl * norms
        out[fl] = float(np.max(np.abs(got - ref)[big] / np.abs(ref)[big])) if big.any() else 0.0
    return out


def assert_mfcc(got, ref, rtol):
    """MFCC rows against the oracle: every coefficient within rtol of the row's L2 norm, and per
    coefficient relative to itself by tiers.  rtol >= 1e-5 (f32 kernels): MFCC_TIERS_F32.
    rtol < 1e-5 (f64 kernels): 10 / 100 / 1000 x rtol, capped at 1e-6 for every tier."""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    norms = np.linalg.norm(ref, axis=1)[:, None]
    norms = np.where(norms == 0, 1.0, norms)
    e_row = np.max(np.abs(got - ref) / norms)
    assert e_row < rtol, ("row-norm", e_row)
    errs = mfcc_tier_errors(got, ref)
    for (fl, mult), f64mult in zip(MFCC_TIERS_F32, (10.0, 100.0, 1000.0)):
        bound = rtol * mult if rtol >= 1e-5 else min(rtol * f64mult, 1e-6)
        assert errs[fl] <= bound, (f"per-coefficient (|c| > {fl:g} ||row||)", errs[fl], bound)
    return e_row


def rolloff_margin(mag):
    """Per frame: the oracle's chosen bin and min(cum[i] - target, target - cum[i-1]) / total."""
    mag = np.asarray(mag, np.float64)
    e = mag * mag
    cum = np.cumsum(e, axis=1)
    tot = cum[:, -1]
    target = 0.85 * tot
    reach = cum >= target[:, None]
    idx = np.where(reach.any(axis=1), np.argmax(reach, axis=1), mag.shape[1] - 1)
    rows = np.arange(len(mag))
    hi = cum[rows, idx] - target
    lo = target - np.where(idx > 0, cum[rows, np.maximum(idx - 1, 0)], 0.0)
    with np.errstate(invalid="ignore", divide="ignore"):
        m = np.where(tot > 0, np.minimum(hi, lo) / tot, np.inf)
    return idx, m


def assert_rolloff(got_hz, ref_hz, mag, margin):
    """Exact rolloff frequencies except on frames whose oracle margin is <= ``margin``; on those
    the bin may move by one."""
    g, r = np.asarray(got_hz, np.float64), np.asarray(ref_hz, np.float64)
    assert g.shape == r.shape
    bad = g != r
    if not bad.any():
        return 0
    _, m = rolloff_margin(mag)
    m = m[: len(r)]
    assert np.all(m[bad] <= margin), ("rolloff mismatch on a non-borderline frame",
                                      np.flatnonzero(bad & (m > margin))[:10], m[bad].min())
    return int(bad.sum())
