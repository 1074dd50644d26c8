"""ComputeSTFTWithWindow and MFCC.ComputeFrames for window lengths the fused kernels do not take
(fingerprint/analyzers/spectral.go:131: go-dsp's FFTReal accepts any W, Bluestein for
non-powers of two): the generic path (stft_dft_kernel, a float64 DFT per frame, then
mfcc_rows_kernel) against the oracle (or_fft: Bluestein for non-powers of two).

Tolerances: magnitude and complex 1e-10 of the frame's peak (direct DFT against Bluestein, both
float64); phase where |X| > 1e-6 of the peak, bounded by |dX| / |X|; MFCC 1e-9 of the row norm.
The spectral descriptors of any W run on spec_rows_kernel over the DFT path's |X| rows (round 6;
rounds 1-5 refused them outside the fused kernels' powers of two); W > 8192 is
SONAR_ERR_UNSUPPORTED."""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc

pytestmark = pytest.mark.gpu
SR = 44100


def _sig(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / SR
    return 0.5 * np.sin(2 * np.pi * 440 * t) + 0.2 * np.sin(2 * np.pi * 2750.5 * t) + 0.1 * rng.standard_normal(n)


@pytest.mark.parametrize("W,H", [(1000, 250), (441, 147), (882, 441), (1536, 512), (3000, 1000), (300, 77),
                                 (4096 + 7, 2048)])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_generic_stft_matches_oracle(ctx, W, H, prec):
    x = _sig(W * 6 + 321, seed=W)                 # the partial last frame is skipped (zero rows)
    cfg = ctx.config(window_size=W, hop_size=H, precision=prec,
                     flags=sonar.FP_MAGNITUDE | sonar.FP_COMPLEX | sonar.FP_PHASE)
    got = ctx.fingerprint(x, cfg)
    assert ctx.last_fp_kernel() == "stft_dft_kernel"
    ref_m = O.stft_mag(x, W, H)
    ref_c, ref_p = O.stft_complex(x, W, H)
    tol = 1e-10 if prec == sonar.F64 else 2e-6    # (f32 mode computes in f64, outputs rounded to f32)
    peak = np.maximum(ref_m.max(axis=1), 1e-300)[:, None]
    assert got["magnitude"].shape == ref_m.shape
    assert np.max(np.abs(got["magnitude"] - ref_m) / peak) < tol
    cx = got["complex"][..., 0] + 1j * got["complex"][..., 1]
    assert np.max(np.abs(cx - ref_c) / peak) < tol
    sel = np.abs(ref_c) > 1e-6 * peak
    dphi = np.abs(np.angle(np.exp(1j * (got["phase"] - ref_p))))
    allowed = 4 * tol * peak / np.maximum(np.abs(ref_c), 1e-300) + 1e-12
    assert np.all(dphi[sel] <= allowed[sel])


@pytest.mark.parametrize("W,H,n_mels", [(1000, 250, 40), (882, 441, 26), (1536, 384, 40)])
def test_generic_mfcc_matches_oracle(ctx, W, H, n_mels):
    x = _sig(SR * 2, seed=W + 1)
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=n_mels, n_mfcc=13,
                     precision=sonar.F64, flags=sonar.FP_MFCC | sonar.FP_MAGNITUDE)
    got = ctx.fingerprint(x, cfg)
    ref = O.mfcc_frames(O.stft_mag(x, W, H), SR, n_coef=13, n_mels=n_mels)
    assert_mfcc(got["mfcc"], ref, 1e-9)


SPEC = ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux", "low_ratio", "high_ratio"]


@pytest.mark.parametrize("W,H,sr", [(1000, 250, 44100), (441, 147, 22050), (3000, 1000, 16000), (4096 + 7, 2048, 0)])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_generic_spectral_descriptors(ctx, W, H, sr, prec):
    """extractSpectralFeatures (speech.go:320-367) on the DFT path's rows: 1e-9 in both modes (the
    DFT path is float64 throughout; f32 rounds the outputs: 1e-6), rolloff bin exact."""
    from parity import assert_rolloff
    x = _sig(SR + 777, seed=W + 3)
    got = ctx.fingerprint(x, ctx.config(window_size=W, hop_size=H, sample_rate=sr, precision=prec,
                                        flags=sonar.FP_SPECTRAL | sonar.FP_MFCC))
    assert ctx.last_fp_kernel() == "stft_dft_kernel"
    mag = O.stft_mag(x, W, H)
    ref = O.spectral_descriptors(mag, sr)
    tol = 1e-9 if prec == sonar.F64 else 1e-6
    for k in SPEC:
        g, r = np.asarray(got[k], np.float64), ref[k]
        assert g.shape == r.shape, k
        if k == "rolloff":
            assert_rolloff(g, r, mag, 1e-12)
            continue
        scale = np.maximum(np.abs(r), np.max(np.abs(r)) * 1e-6 + 1e-30)
        assert np.max(np.abs(g - r) / scale) < (tol * 10 if k == "slope" else tol), k


def test_generic_unsupported_cases(ctx):
    with pytest.raises(sonar.SonarError):
        ctx.fingerprint(np.zeros(20000), ctx.config(window_size=9000, hop_size=1000, flags=sonar.FP_MAGNITUDE))


def test_pow2_window_unchanged(ctx):
    """Power-of-two windows stay on the fused kernel."""
    x = _sig(SR)
    ctx.fingerprint(x, ctx.config(window_size=1024, hop_size=256, precision=sonar.F64, flags=sonar.FP_MAGNITUDE))
    assert ctx.last_fp_kernel() == "fp_wave_kernel"
