"""SpectrogramResult.Complex and .Phase (fingerprint/analyzers/spectral.go:490-494) from
sonar_fingerprint (SONAR_FP_COMPLEX / SONAR_FP_PHASE) against the oracle's complex STFT
(`or_stft_complex`: the positive bins of the windowed frame's FFT, atan2(imag, real), skipped
frames all zero).

Tolerances:
  * complex: 1e-11 (f64) / 2e-6 (f32) of the frame's peak |X|, as the magnitude test;
  * phase: atan2 of a perturbed vector moves by at most |dX| / |X|, so bins with
    |X| > 1e-6 (f64) / 1e-3 (f32) of the peak are checked to 4 * tol * peak / |X| + 1e-12 rad
    (wrapped); quieter bins carry no phase information (Go's own rounding flips them);
  * magnitude written by the same call = |complex| of the same call to 1 ulp-scale.
"""
import numpy as np
import pytest

import oracle as O
import sonar

pytestmark = pytest.mark.gpu


def _sig(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 44100.0
    return 0.5 * np.sin(2 * np.pi * 440 * t) + 0.2 * np.sin(2 * np.pi * 3001.3 * t) + 0.1 * rng.standard_normal(n)


def _check(got_c, got_p, ref_c, ref_p, tol, floor):
    cx = got_c[..., 0] + 1j * got_c[..., 1]
    peak = np.maximum(np.abs(ref_c).max(axis=1), 1e-300)[:, None]
    assert np.max(np.abs(cx - ref_c) / peak) < tol
    mag = np.abs(ref_c)
    sel = mag > floor * peak
    dphi = np.abs(np.angle(np.exp(1j * (got_p - ref_p))))
    allowed = 4 * tol * peak / np.maximum(mag, 1e-300) + 1e-12
    assert np.all(dphi[sel] <= allowed[sel])


@pytest.mark.parametrize("W,H", [(1024, 256), (2048, 512), (512, 128), (256, 64), (128, 37)])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_complex_and_phase_match_oracle(ctx, W, H, prec):
    x = _sig(W * 7 + 123)                      # the last partial frame is skipped (zero rows)
    cfg = ctx.config(window_size=W, hop_size=H, precision=prec,
                     flags=sonar.FP_COMPLEX | sonar.FP_PHASE | sonar.FP_MAGNITUDE)
    got = ctx.fingerprint(x, cfg)
    ref_c, ref_p = O.stft_complex(x, W, H)
    assert got["complex"].shape == ref_c.shape + (2,) and got["phase"].shape == ref_p.shape
    tol, floor = (1e-11, 1e-6) if prec == sonar.F64 else (2e-6, 1e-3)
    _check(got["complex"], got["phase"], ref_c, ref_p, tol, floor)
    cx = got["complex"][..., 0] + 1j * got["complex"][..., 1]
    assert np.max(np.abs(np.abs(cx) - got["magnitude"]) / np.maximum(got["magnitude"].max(axis=1), 1e-300)[:, None]) \
        < (1e-14 if prec == sonar.F64 else 1e-6)


def test_complex_with_mfcc_in_one_call(ctx):
    """Requesting the spectrum next to the MFCC leaves the MFCC unchanged (same fused kernel:
    SONAR_FP_GENERIC keeps the MFCC-only reference call on fp_wave_kernel, where the f64 MFCC-only
    configuration would otherwise take mfcc_pair_kernel<double>)."""
    x = _sig(44100 * 3)
    base = dict(window_size=1024, hop_size=256, precision=sonar.F64)
    ref = ctx.fingerprint(x, ctx.config(flags=sonar.FP_MFCC | sonar.FP_GENERIC, **base))["mfcc"]
    got = ctx.fingerprint(x, ctx.config(flags=sonar.FP_MFCC | sonar.FP_COMPLEX | sonar.FP_PHASE, **base))
    assert np.array_equal(got["mfcc"], ref)
    ref_c, ref_p = O.stft_complex(x, 1024, 256)
    _check(got["complex"], got["phase"], ref_c, ref_p, 1e-11, 1e-6)


def test_complex_skipped_and_zero_frames(ctx):
    """Silence gives exact zeros (phase atan2(0, 0) = 0), like Go's untouched rows."""
    x = np.zeros(4096)
    got = ctx.fingerprint(x, ctx.config(window_size=1024, hop_size=512, precision=sonar.F64,
                                        flags=sonar.FP_COMPLEX | sonar.FP_PHASE))
    assert np.all(got["complex"] == 0) and np.all(got["phase"] == 0)


def test_multi_complex_equals_single(ctx):
    x = _sig(44100 * 2, seed=3)
    cfg = dict(window_size=1024, hop_size=256, precision=sonar.F64, flags=sonar.FP_COMPLEX | sonar.FP_PHASE)
    a = ctx.fingerprint(x, ctx.config(**cfg))
    m = sonar.Multi([0])
    try:
        b = m.fingerprint(x, ctx.config(**cfg))
    finally:
        m.close()
    assert np.array_equal(a["complex"], b["complex"]) and np.array_equal(a["phase"], b["phase"])
