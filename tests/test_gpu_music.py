"""MusicFeatureExtractor.ExtractFeatures (fingerprint/extractors/music.go:178-583) through
sonar_extract_music_features against the oracle composition (oracle.music_features_reference),
float64 parity mode.

The reference panics in extractTemporalFeatures for every signal of >= 1536 samples
(music.go:403: percentiles 10 / 90 where fractions are expected -> index out of range) and for a
signal without an energy frame (music.go:383: integer divide by zero).  Both are checked: the call
fails with SONAR_ERR_PANIC and Go's runtime message, and the arrays computed before the panic
(spectral group incl. contrast, |X|^4 MFCC, chroma, RMS energy, envelope, amplitudes) match the
oracle.  Below 1536 samples every group is compared (the harmonic block is zero by F7 except for a
1024-sample frame, where DetectPitch runs).

Tolerances: 1e-9 relative (floors at 1e-6 of the array's peak) for the float features, 1e-8 for the
spectral slope (a log-log regression over every bin above 1e-10, as in test_gpu_stft_mfcc), 1e-9
relative or 1e-4 dB for the spectral contrast (a dB ratio whose valley can sit far below the frame's
peak bin), exact for the rolloff bin and counts.  The peak amplitude (max |y| of the preprocessed
signal) is within 1e-9 like the other floats: y carries the DC scan's rounding (DESIGN.md Kernel 4)."""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc, assert_rel
from sonar import synth

pytestmark = pytest.mark.gpu


def _fc(ctx, **kw):
    base = dict(sample_rate=44100, window_size=1024, hop_size=256, stft_window_size=1024, stft_hop_size=256)
    base.update(kw)
    return ctx.feature_config(**base), base


def _close(got, ref, name, rtol=1e-9):
    g, r = np.asarray(got, float), np.asarray(ref, float)
    peak = np.max(np.abs(np.nan_to_num(r))) if r.size else 0.0
    assert_rel(g, r, rtol, max(peak * 1e-6, 1e-30), name)


def _compare(got, ref):
    for k, v in ref.items():
        assert k in got, k
        if k == "mfcc":
            assert_mfcc(got[k], v, 1e-9)
        elif k == "spectral_rolloff":
            assert np.array_equal(np.ravel(np.asarray(got[k], float)), np.ravel(np.asarray(v, float))), k
        elif k == "spectral_slope":
            _close(got[k], v, k, 1e-8)
        elif k == "spectral_contrast":
            # 10 log10(peak / valley) of sorted band powers: a valley far below the frame's peak bin
            # carries the FFT's rounding relative to that PEAK (~1e-16 of it), so in dB the error
            # is absolute: 1e-9 relative or 1e-4 dB, whichever is larger
            g, r = np.asarray(got[k], float), np.asarray(v, float)
            assert g.shape == r.shape, k
            assert np.all(np.abs(g - r) <= np.maximum(1e-9 * np.abs(r), 1e-4)), (k, float(np.max(np.abs(g - r))))
        else:
            _close(got[k], v, k)


def _run(ctx, x, **kw):
    cfg, fc = _fc(ctx, **kw)
    ref, panic = O.music_features_reference(x, 44100, fc)
    try:
        got, err = ctx.extract_music_features(x, 44100, cfg), None
    except sonar.SonarError as e:
        got, err = e.partial, e
    return got, err, ref, panic


@pytest.mark.parametrize("seconds", [2.0, 10.0])
def test_panic_regime_partial_results(ctx, seconds):
    x = synth.sweep(seconds) + 0.01 * np.random.default_rng(3).standard_normal(int(seconds * 44100))
    got, err, ref, panic = _run(ctx, x)
    assert panic is not None and panic.startswith("runtime error: index out of range")
    assert err is not None and err.code == sonar.ERR_PANIC and err.msg == panic, (err, panic)
    assert set(got) == set(ref), sorted(set(got) ^ set(ref))
    _compare(got, ref)
    assert got["spectral_contrast"].shape == (sonar.stft_frames(len(x), 1024, 256), 6)


def test_no_energy_frame_divides_by_zero(ctx):
    """FeatureConfig.WindowSize unset (0, F13): no ShortTimeEnergy frame -> len(pcm) / 0 (:383)."""
    x = synth.sweep(1.0)
    got, err, ref, panic = _run(ctx, x, window_size=0, hop_size=256)
    assert panic == "runtime error: integer divide by zero"
    assert err is not None and err.code == sonar.ERR_PANIC and err.msg == panic
    _compare(got, ref)


@pytest.mark.parametrize("n,W,H,fw,fh", [(1024, 1024, 256, 1024, 256), (1300, 1024, 256, 512, 128),
                                          (1535, 512, 128, 1024, 128), (700, 512, 128, 256, 64),
                                          (1024, 512, 256, 256, 128)])
def test_full_extractor_below_1536_samples(ctx, n, W, H, fw, fh):
    rng = np.random.default_rng(n + W)
    t = np.arange(n) / 44100.0
    x = 0.5 * np.sin(2 * np.pi * 220.0 * t) + 0.05 * rng.standard_normal(n)
    got, err, ref, panic = _run(ctx, x, stft_window_size=W, stft_hop_size=H, window_size=fw, hop_size=fh)
    assert panic is None and err is None, (panic, err)
    assert set(got) == set(ref), sorted(set(got) ^ set(ref))
    _compare(got, ref)
    # n == 1024, W == 1024 is the one frame DetectPitch accepts (F7); the extractor's pre-emphasis
    # (0.95) leaves a low tone below the noise there, so Go (and the oracle) report no pitch either


@pytest.mark.parametrize("n,W,H,fw,fh", [(1300, 256, 64, 256, 512), (88200, 1024, 256, 1024, 512),
                                          (1535, 512, 128, 1024, 256),
                                          (5000, 1024, 256, 1024, 1000)])
def test_chroma_hop_above_spectrogram_hop_panics(ctx, n, W, H, fw, fh):
    """FeatureConfig.HopSize above the spectrogram's: extractChromaFeatures slices
    processedPCM[f hop : min(f hop + n/F, n)] (music.go:348-352), so once (F - 1) hop > n Go panics
    with 'slice bounds out of range [start:n]' at the first frame starting past the end; only the
    spectral group and the MFCC were computed."""
    rng = np.random.default_rng(n)
    x = synth.sweep(n / 44100.0)[:n] + 0.01 * rng.standard_normal(n)
    F = sonar.stft_frames(n, W, H)
    assert (F - 1) * fh > n
    got, err, ref, panic = _run(ctx, x, stft_window_size=W, stft_hop_size=H, window_size=fw, hop_size=fh)
    assert panic == f"runtime error: slice bounds out of range [{(n // fh + 1) * fh}:{n}]"
    assert err is not None and err.code == sonar.ERR_PANIC and err.msg == panic, (err, panic)
    assert "chroma" not in got and "rms_energy" not in got
    assert set(got) == set(ref), sorted(set(got) ^ set(ref))
    _compare(got, ref)


def test_short_signal_temporal_error(ctx):
    """<= 512 samples: the onset STFT (1024 / 512) fails and ExtractFeatures with it (:412-415)."""
    x = synth.sweep(0.011)[:500]
    cfg, fc = _fc(ctx, stft_window_size=256, stft_hop_size=128, window_size=256, hop_size=128)
    with pytest.raises(ValueError):
        O.music_features_reference(x, 44100, fc)
    with pytest.raises(sonar.SonarError) as ei:
        ctx.extract_music_features(x, 44100, cfg)
    assert ei.value.code == sonar.ERR_TOO_SHORT
    assert "temporal feature extraction failed" in ei.value.msg


def test_zero_hop_chroma_error(ctx):
    """FeatureConfig.HopSize unset (0): the chroma STFT rejects it (stft.go:54-56) and
    ExtractFeatures returns the wrapped error (music.go:218-221)."""
    x = synth.sweep(0.5)
    cfg, fc = _fc(ctx, window_size=0, hop_size=0)
    with pytest.raises(ValueError) as oe:
        O.music_features_reference(x, 44100, fc)
    with pytest.raises(sonar.SonarError) as ei:
        ctx.extract_music_features(x, 44100, cfg)
    assert ei.value.code == sonar.ERR_INVALID and ei.value.msg == str(oe.value)


def test_invalid_input(ctx):
    with pytest.raises(sonar.SonarError) as ei:
        ctx.extract_music_features(np.zeros(0), 44100, _fc(ctx)[0])
    assert "invalid input data" in ei.value.msg
