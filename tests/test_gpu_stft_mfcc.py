"""Path A parity on the GPU: ComputeSTFTWithWindow magnitude, MFCC.ComputeFrames,
ZCR and ShortTimeEnergy vs the fp64 oracle (oracle/sonar_oracle.c).

Tolerances (north_star: float features within 1e-4 relative):
  * F64 kernels: 1e-9 relative to the frame's peak (magnitude) / MFCC L2 norm.
  * F32 kernels: 1e-4 relative to the frame's MFCC L2 norm on well-conditioned
    input (sweep + noise, every mel band populated); magnitude 2e-6 of frame peak.
  * ZCR crossing counts: bit-exact (integer).
"""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc, assert_rolloff
from sonar import synth

pytestmark = pytest.mark.gpu


def _sig(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 44100.0
    return 0.5 * np.sin(2 * np.pi * 440 * t) + 0.1 * rng.standard_normal(n)


def _rel_rows(a, b, norm):
    return np.max(np.abs(a - b) / np.maximum(norm, 1e-30)[:, None])


@pytest.mark.parametrize("W,H", [(1024, 256), (2048, 512), (512, 128), (256, 64), (1024, 1000), (128, 37)])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_magnitude_matches_oracle(ctx, W, H, prec):
    x = _sig(W * 7 + 123)
    cfg = ctx.config(window_size=W, hop_size=H, flags=sonar.FP_MAGNITUDE, precision=prec)
    got = ctx.fingerprint(x, cfg)["magnitude"]
    ref = O.stft_mag(x, W, H)
    assert got.shape == ref.shape
    tol = 1e-11 if prec == sonar.F64 else 2e-6
    assert _rel_rows(got, ref, ref.max(axis=1)) < tol


@pytest.mark.parametrize("win", ["hann", "hamming", "blackman", "blackman_harris", "kaiser", "tukey",
                                 "rectangular", "bartlett", "welch"])
def test_window_types(ctx, win):
    x = _sig(1024 * 4)
    cfg = ctx.config(window_size=1024, hop_size=256, window_type=win, flags=sonar.FP_MAGNITUDE,
                     precision=sonar.F64)
    got = ctx.fingerprint(x, cfg)["magnitude"]
    ref = O.stft_mag(x, 1024, 256, window_type=win)
    assert _rel_rows(got, ref, ref.max(axis=1)) < 1e-11


def test_frame_count_and_short_signal_rules(ctx):
    # Go truncating division: n in (W-H, W) gives one all-zero frame (spectral.go:409, :524-534)
    assert sonar.stft_frames(1000, 1024, 256) == 1
    assert sonar.stft_frames(768, 1024, 256) == sonar._abi.ERR_TOO_SHORT
    x = _sig(1000)
    got = ctx.fingerprint(x, ctx.config(flags=sonar.FP_MAGNITUDE, precision=sonar.F64))["magnitude"]
    assert got.shape == (1, 513) and np.all(got == 0)
    with pytest.raises(sonar.SonarError, match="signal too short"):
        ctx.fingerprint(_sig(700), ctx.config(flags=sonar.FP_MAGNITUDE))
    with pytest.raises(sonar.SonarError, match="empty signal"):
        ctx.fingerprint(np.zeros(0), ctx.config())
    with pytest.raises(sonar.SonarError, match="hop size must be positive"):
        ctx.fingerprint(_sig(4096), ctx.config(hop_size=0))


@pytest.mark.parametrize("sr,nm,nc,W", [(44100, 40, 13, 1024), (44100, 26, 13, 1024), (16000, 26, 13, 512),
                                       (44100, 26, 13, 2048), (22050, 32, 20, 256)])
def test_mfcc_f64_matches_oracle(ctx, sr, nm, nc, W):
    x = _sig(W * 40)
    H = W // 4
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=sr, n_filters=nm, n_mfcc=nc, precision=sonar.F64)
    got = ctx.fingerprint(x, cfg)["mfcc"]
    ref = O.mfcc_frames(O.stft_mag(x, W, H), sr, n_coef=nc, n_mels=nm)
    assert _rel_rows(got, ref, np.linalg.norm(ref, axis=1)) < 1e-9


def test_mfcc_f32_headline_config(ctx):
    """1 h config's arithmetic: sweep + 0.05 N(0,1), W=1024 H=256, 40 mels -> 13 MFCC, f32."""
    x = synth.c2_hour(seconds=20.0)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    got = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    assert ctx.last_fp_kernel() == "mfcc_pair_kernel"
    ref = O.mfcc_frames(O.stft_mag(x.astype(np.float64), 1024, 256, nthreads=8), 44100, n_coef=13, n_mels=40)
    assert got.shape == ref.shape == (3442, 13)
    e = np.max(np.abs(got - ref), axis=1) / np.linalg.norm(ref, axis=1)
    assert e.max() < 1e-4, (np.nonzero(~(e < 1e-4))[0][:16].tolist(), int((~(e < 1e-4)).sum()))
    assert_mfcc(got, ref, 1e-4)                  # + per-coefficient tiers (parity.MFCC_TIERS_F32)


def test_mfcc_sample_rate_zero_constant(ctx):
    """F1/F2: GenerateFingerprint runs NewMFCC(0, 13) -> all-zero filterbank -> constant MFCC."""
    x = synth.sweep(2.0)
    for prec in (sonar.F64, sonar.F32):
        got = ctx.fingerprint(x, ctx.config(sample_rate=0, precision=prec))["mfcc"]
        tol = 1e-9 if prec == sonar.F64 else 1e-4
        assert np.allclose(got[:, 0], np.sqrt(26) * np.log(1e-10), rtol=0, atol=117.41 * tol)   # -117.409263
        assert np.abs(got[:, 1:]).max() < 117.41 * tol


def test_mfcc_music_power_input_and_bark(ctx):
    x = _sig(1024 * 30)
    mag = O.stft_mag(x, 1024, 256)
    got = ctx.fingerprint(x, ctx.config(mfcc_input_power=1, precision=sonar.F64))["mfcc"]
    ref = O.mfcc_frames(mag ** 2, 44100)          # music.go:311-317 feeds |X|^2 (F5)
    assert _rel_rows(got, ref, np.linalg.norm(ref, axis=1)) < 1e-9
    got = ctx.fingerprint(x, ctx.config(filterbank=1, precision=sonar.F64))["mfcc"]
    ref = O.mfcc_frames(mag, 44100, kind="bark")
    assert _rel_rows(got, ref, np.linalg.norm(ref, axis=1)) < 1e-9


@pytest.mark.parametrize("pcm_dtype", [sonar.F64, sonar.F32])
def test_zcr_bit_exact_and_energy(ctx, pcm_dtype):
    x = _sig(1024 * 50, seed=3)
    if pcm_dtype == sonar.F32:
        x = x.astype(np.float32)
    x64 = x.astype(np.float64)
    cfg = ctx.config(flags=sonar.FP_ZCR | sonar.FP_ENERGY, energy_window=1024, energy_hop=256, sample_rate=16000,
                     pcm_dtype=pcm_dtype)
    got = ctx.fingerprint(x, cfg)
    pre = O.preemphasis(x64, 0.97)
    F = O.stft_frames(len(x), 1024, 256)
    assert np.array_equal(got["zcr"], O.zcr_frames(pre, F, 1024, 256, 16000))
    ref_e = O.short_time_energy(pre, 1024, 256)
    assert np.array_equal(got["energy"], ref_e)   # same sequential float64 order -> bit-identical
    # sr = 0 (F3): ZCR = crossings / (+Inf) = 0
    got0 = ctx.fingerprint(x, ctx.config(flags=sonar.FP_ZCR, sample_rate=0, pcm_dtype=pcm_dtype))
    assert np.all(got0["zcr"] == 0)


SPEC = ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux", "low_ratio", "high_ratio"]


@pytest.mark.parametrize("W,H,sr", [(1024, 256, 44100), (512, 128, 16000), (2048, 512, 44100), (1024, 256, 0),
                                    (256, 100, 22050)])
@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_spectral_descriptors_match_oracle(ctx, W, H, sr, prec):
    """SpeechFeatureExtractor.extractSpectralFeatures per-frame descriptors (speech.go:320-367)
    and the energy-band ratios (speech.go:438-458).  Float features: 1e-9 (F64) / 1e-4 (F32)
    relative; rolloff is a bin index -> frequency, exact: the kernel reproduces Go's sequential
    total and cumulative chains (spectral_rolloff.go:29-49) on its own magnitudes, so it can differ
    from the oracle only on a frame whose cumulative energy sits within magnitude rounding of the
    85 % target (asserted per frame by parity.assert_rolloff)."""
    x = synth.c2_hour(seconds=6.0).astype(np.float64)
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=sr, precision=prec,
                     flags=sonar.FP_SPECTRAL | sonar.FP_MFCC)
    got = ctx.fingerprint(x, cfg)
    mag = O.stft_mag(x, W, H)
    ref = O.spectral_descriptors(mag, sr)
    tol = 1e-9 if prec == sonar.F64 else 1e-4
    for k in SPEC:
        g, r = got[k], ref[k]
        assert g.shape == r.shape, k
        if k == "rolloff":
            # exact bin; a frame may differ only where the oracle's cumulative energy is within
            # 1e-12 (F64) / 1e-5 (F32, f32 magnitudes) of the total from the 85 % target
            assert_rolloff(g, r, mag, 1e-12 if prec == sonar.F64 else 1e-5)
            continue
        scale = np.maximum(np.abs(r), np.max(np.abs(r)) * 1e-6 + 1e-30)
        err = np.max(np.abs(g - r) / scale)
        # slope is a log-log regression over every bin above 1e-10 (f64: 10x the tolerance); in
        # the F32 mode the descriptors take the f64 transform (round 6), so every field, slope
        # included, is held to the north star's 1e-4
        stol = tol * 10 if prec == sonar.F64 else tol
        assert err < (tol if k != "slope" else stol), (k, err)
