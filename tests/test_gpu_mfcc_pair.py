"""Headline kernel (mfcc_pair.hip): float32 STFT(1024) -> mel -> ln -> DCT-II -> lifter,
two frames per 1024-point complex FFT.  Parity against the fp64 oracle (the C restatement
of analyzers/spectral.go:385-545 + spectral/mfcc.go:113-245) on the configurations that
route to it (f32 PCM, f32 output, MFCC only, W = 1024), and against the general fused
kernel (SONAR_FP_GENERIC) on the same input.

Tolerance (north_star: float features within 1e-4 relative): 1e-4 of the frame's MFCC
L2 norm -- the near-zero coefficients c1..c12 carry rounding of the large c0, so a
per-coefficient relative bound is not meaningful in f32."""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc
from sonar import synth

pytestmark = pytest.mark.gpu


def _cfg(ctx, **kw):
    base = dict(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    base.update(kw)
    return ctx.config(**base)


def _ref(x, H=256, sr=44100, nm=40, nc=13, power=False, win="hann"):
    mag = O.stft_mag(x.astype(np.float64), 1024, H, window_type=win, nthreads=8)
    return O.mfcc_frames(mag ** 2 if power else mag, sr, n_coef=nc, n_mels=nm)


_EXPECT = {"kernel": "mfcc_pair_kernel"}


def _fp(ctx, x, cfg, kernel=None):
    out = ctx.fingerprint(x, cfg)["mfcc"]
    assert ctx.last_fp_kernel() == (kernel or _EXPECT["kernel"])
    again = ctx.fingerprint(x, cfg)["mfcc"]
    assert np.array_equal(out, again, equal_nan=True), "nondeterministic: " + str(
        np.nonzero(np.any(out != again, axis=1))[0][:16].tolist())
    return out


class _Err(float):
    """max row-relative error; repr names the worst frames (diagnostics on failure)"""
    def __new__(cls, got, ref):
        e = np.max(np.abs(got.astype(np.float64) - ref), axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        obj = super().__new__(cls, float(np.max(e)) if not np.isnan(e).any() else float("nan"))
        bad = np.nonzero(~(e < 1e-4))[0]
        obj.info = f"{len(bad)} bad of {len(e)} frames: {bad[:16].tolist()} nan={int(np.isnan(got).sum())}"
        return obj

    def __repr__(self):
        return f"{float(self)!r} ({self.info})"


def _err(got, ref):
    """the row-norm error (returned) after the tiered per-coefficient checks of parity.assert_mfcc"""
    e = _Err(got, ref)
    if e < 1e-4:
        assert_mfcc(got.astype(np.float64), ref, 1e-4)
    return e


@pytest.mark.parametrize("seconds", [0.1, 1.0, 7.3])
@pytest.mark.parametrize("H", [256, 100, 1000, 512])
def test_pair_kernel_matches_oracle(ctx, seconds, H):
    x = synth.c2_hour(seconds=seconds)
    got = _fp(ctx, x, _cfg(ctx, hop_size=H))
    ref = _ref(x, H=H)
    assert got.shape == ref.shape
    assert _err(got, ref) < 1e-4


@pytest.mark.parametrize("n_extra", [0, 1, 255, 256, 257, 511])
def test_odd_even_frame_counts(ctx, n_extra):
    """F odd -> the last pair carries one frame; every frame count around a pair boundary."""
    x = synth.c2_hour(seconds=0.5)[: 1024 + 256 * 40 + n_extra]
    got = _fp(ctx, x, _cfg(ctx))
    ref = _ref(x)
    assert got.shape == ref.shape == (sonar.stft_frames(len(x), 1024, 256), 13)
    assert _err(got, ref) < 1e-4


@pytest.mark.parametrize("sr,nm,nc", [(44100, 26, 13), (44100, 40, 13), (22050, 32, 16), (48000, 64, 13),
                                      (16000, 26, 12), (44100, 20, 1)])
def test_filterbank_shapes(ctx, sr, nm, nc):
    x = synth.c2_hour(seconds=2.0)
    # 64 mels at 48 kHz needs > 64 filterbank chunks: served by the general kernel
    got = _fp(ctx, x, _cfg(ctx, sample_rate=sr, n_filters=nm, n_mfcc=nc),
              "fp_wave_kernel" if nm == 64 else None)
    ref = _ref(x, sr=sr, nm=nm, nc=nc)
    assert _err(got, ref) < 1e-4


def test_music_power_input_F5(ctx):
    x = synth.c2_hour(seconds=2.0)
    got = _fp(ctx, x, _cfg(ctx, mfcc_input_power=1))
    assert _err(got, _ref(x, power=True)) < 1e-4


@pytest.mark.parametrize("win", ["hamming", "blackman", "rectangular"])
def test_window_types(ctx, win):
    x = synth.c2_hour(seconds=1.0)
    got = _fp(ctx, x, _cfg(ctx, window_type=win))
    assert _err(got, _ref(x, win=win)) < 1e-4


def test_sample_rate_zero_constant(ctx):
    """F1/F2: all-zero filterbank -> every filter ln(1e-10) -> c0 = sqrt(n_mels) ln(1e-10)."""
    x = synth.sweep(1.0).astype(np.float32)
    got = _fp(ctx, x, _cfg(ctx, sample_rate=0, n_filters=26))
    assert np.allclose(got[:, 0], np.sqrt(26) * np.log(1e-10), rtol=0, atol=117.41e-5)
    assert np.abs(got[:, 1:]).max() < 117.41e-5


def test_single_short_frame(ctx):
    """n in (W-H, W): Go yields one all-zero frame (spectral.go:409, :524-534)."""
    x = synth.c2_hour(seconds=0.1)[:1000]
    got = _fp(ctx, x, _cfg(ctx, n_filters=26))
    assert got.shape == (1, 13)
    assert abs(got[0, 0] - np.sqrt(26) * np.log(1e-10)) < 1e-3 and np.abs(got[0, 1:]).max() < 1e-3


def test_pair_vs_generic_kernel_long(ctx):
    """60 s (10,332 frames): many pairs per wave; the two device kernels agree."""
    x = synth.c2_hour(seconds=60.0)
    a = _fp(ctx, x, _cfg(ctx)).astype(np.float64)
    b = _fp(ctx, x, _cfg(ctx, flags=sonar.FP_MFCC | sonar.FP_GENERIC), "fp_wave_kernel").astype(np.float64)
    assert a.shape == b.shape
    assert _err(a, b) < 1e-4


# ---- float64 (round 6): the same kernel templated on double -- float64 tables, arithmetic and
# output, PCM float32 (widened exactly) or float64 -- at the f64 MFCC tolerance (1e-9 of the row
# norm, tests/parity.py's f64 tiers).  VERDICT r05 item 4: the headline configuration at the
# reference's precision.
def _cfg64(ctx, pcm64=True, **kw):
    return _cfg(ctx, precision=sonar.F64, pcm_dtype=sonar.F64 if pcm64 else sonar.F32, out_dtype=sonar.F64, **kw)


def _x64(x, pcm64):
    return x.astype(np.float64) if pcm64 else x.astype(np.float32)


@pytest.mark.parametrize("pcm64", [True, False])
@pytest.mark.parametrize("H", [256, 100, 1000])
def test_pair_kernel_f64_matches_oracle(ctx, pcm64, H):
    x = _x64(synth.c2_hour(seconds=7.3), pcm64)
    got = _fp(ctx, x, _cfg64(ctx, pcm64, hop_size=H))
    assert got.dtype == np.float64
    ref = _ref(x, H=H)
    assert got.shape == ref.shape
    assert_mfcc(got, ref, 1e-9)


@pytest.mark.parametrize("n_extra", [0, 1, 255, 257])
def test_pair_kernel_f64_odd_even_frames(ctx, n_extra):
    x = synth.c2_hour(seconds=0.5)[: 1024 + 256 * 40 + n_extra].astype(np.float64)
    got = _fp(ctx, x, _cfg64(ctx))
    ref = _ref(x)
    assert got.shape == ref.shape == (sonar.stft_frames(len(x), 1024, 256), 13)
    assert_mfcc(got, ref, 1e-9)


@pytest.mark.parametrize("sr,nm,nc,power,win", [(44100, 26, 13, 0, "hann"), (22050, 32, 16, 0, "hamming"),
                                                (16000, 26, 12, 1, "blackman"), (44100, 20, 1, 0, "rectangular"),
                                                (48000, 64, 13, 0, "hann")])
def test_pair_kernel_f64_banks(ctx, sr, nm, nc, power, win):
    x = synth.c2_hour(seconds=2.0).astype(np.float64)
    got = _fp(ctx, x, _cfg64(ctx, sample_rate=sr, n_filters=nm, n_mfcc=nc, mfcc_input_power=power, window_type=win),
              "fp_wave_kernel" if nm == 64 else None)
    assert_mfcc(got, _ref(x, sr=sr, nm=nm, nc=nc, power=bool(power), win=win), 1e-9)


def test_pair_kernel_f64_sample_rate_zero_and_short(ctx):
    x = synth.sweep(1.0).astype(np.float64)
    got = _fp(ctx, x, _cfg64(ctx, sample_rate=0, n_filters=26))
    assert np.allclose(got[:, 0], np.sqrt(26) * np.log(1e-10), rtol=1e-12, atol=0)
    assert np.abs(got[:, 1:]).max() < 1e-9
    one = _fp(ctx, x[:1000], _cfg64(ctx, n_filters=26))
    assert one.shape == (1, 13)
    assert_mfcc(one, _ref(x[:1000], nm=26), 1e-9)


def test_pair_vs_generic_kernel_f64_long(ctx):
    """60 s: the f64 pair kernel against fp_wave_kernel<double> on the same bytes."""
    x = synth.c2_hour(seconds=60.0).astype(np.float64)
    a = _fp(ctx, x, _cfg64(ctx))
    b = _fp(ctx, x, _cfg64(ctx, flags=sonar.FP_MFCC | sonar.FP_GENERIC), "fp_wave_kernel")
    assert_mfcc(a, b, 1e-9)


@pytest.mark.parametrize("sr,nm", [(8000, 20), (11025, 40), (16000, 48), (22050, 56), (44100, 60), (32000, 64),
                                   (96000, 40), (44100, 8)])
def test_pair_kernel_f64_bank_sweep(ctx, sr, nm):
    """Banks of every shape the pair kernel takes (the widest chunks and largest DCT tables shrink
    the float64 block to fewer waves to fit LDS), or the general kernel where it does not."""
    x = synth.c2_hour(seconds=1.5).astype(np.float64)
    cfg = _cfg64(ctx, sample_rate=sr, n_filters=nm)
    got = ctx.fingerprint(x, cfg)["mfcc"]
    assert ctx.last_fp_kernel() in ("mfcc_pair_kernel", "fp_wave_kernel")
    assert_mfcc(got, _ref(x, sr=sr, nm=nm), 1e-9)
    got32 = ctx.fingerprint(x.astype(np.float32), _cfg(ctx, sample_rate=sr, n_filters=nm))["mfcc"]
    assert _err(got32, _ref(x.astype(np.float32), sr=sr, nm=nm)) < 1e-4
