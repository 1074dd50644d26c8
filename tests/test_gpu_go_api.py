"""The C++ mirror of the Go orchestration (GenerateFingerprint -> speech extractor,
AlignmentExtractor) against the oracle composition of the same Go code.
Integer/decision outputs (is_speech, peak lag, DTW path, pitch frames) are exact;
float features use the 1e-4-relative north-star tolerance (F64 kernels: 1e-6, device log/exp are not correctly rounded)."""
import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc, assert_rel, assert_rolloff
from sonar import synth

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, name):
    """Per-element relative error; elements below 1e-6 of the array's peak are checked against
    that floor (explicit, so small values are not hidden behind the peak)."""
    b_ = np.asarray(b, float)
    peak = np.max(np.abs(np.nan_to_num(b_))) if b_.size else 0.0
    assert_rel(a, b, rtol, max(peak * 1e-6, 1e-30), name)


def _cmp(got, ref, rtol, mag=None):
    for k, v in ref.items():
        assert k in got, k
        if k == "spectral_rolloff":
            if mag is None:
                assert np.array_equal(np.asarray(got[k], float), np.asarray(v, float)), k
            else:
                assert_rolloff(got[k], v, mag, 1e-12 if rtol <= 1e-6 else 1e-5)
            continue
        if k == "mfcc" and np.asarray(v).size:
            assert_mfcc(got[k], v, max(rtol, 1e-9))
            continue
        _close(got[k], v, rtol, k)


def test_generate_fingerprint_music_c1(ctx):
    """C1: GenerateFingerprint on the 10 s sweep, ContentType=music, 1024/256 (F1: SampleRate = 0)."""
    x = synth.sweep(10.0)
    cfg = ctx.fingerprint_config(window_size=1024, hop_size=256, feature_window_size=1024, feature_hop_size=256,
                                 precision=sonar.F64)
    got = ctx.generate_fingerprint(x, 44100, "music", cfg)
    ref = O.speech_features_reference(x, 44100, dict(sample_rate=0, window_size=1024, hop_size=256,
                                                     stft_window_size=1024, stft_hop_size=256, enable_mfcc=1,
                                                     enable_speech_features=0, enable_temporal_features=0,
                                                     mfcc_coefficients=13))
    assert got["mfcc"].shape == (1719, 13)
    assert np.allclose(got["mfcc"][:, 0], np.sqrt(26) * np.log(1e-10))    # F2 constant
    assert np.all(got["spectral_centroid"] == 0) and np.all(got["zero_crossing_rate"] == 0)   # F3
    assert np.all(got["pitch_estimate"] == 0)
    _cmp(got, ref, 1e-6)


def test_generate_fingerprint_talk_and_errors(ctx):
    x = synth.c4_speech(seconds=4.0, sr=16000)
    cfg = ctx.fingerprint_config(window_size=512, hop_size=128, feature_window_size=512, feature_hop_size=128,
                                 precision=sonar.F64)
    got = ctx.generate_fingerprint(x, 16000, "talk", cfg)
    ref = O.speech_features_reference(x, 16000, dict(sample_rate=0, window_size=512, hop_size=128,
                                                     stft_window_size=512, stft_hop_size=128, enable_mfcc=1,
                                                     enable_speech_features=1, enable_temporal_features=1,
                                                     mfcc_coefficients=13))
    assert got["is_speech"] == ref["is_speech"]
    _cmp(got, ref, 1e-6)
    # F12: "speech" is not a content type -> ContentDetector.DetectContentType runs (acoustic)
    det = ctx.generate_fingerprint(x, 16000, "speech", cfg)
    want, _ = O.detect_from_audio(x, 16000)
    assert int(det["content_type"].reshape(-1)[0]) == ["music", "news", "sports", "talk", "mixed",
                                                        "unknown"].index(want)
    with pytest.raises(sonar.SonarError, match="signal too short"):
        ctx.generate_fingerprint(x[:300], 16000, "news", cfg)


@pytest.mark.parametrize("prec,rtol", [(sonar.F64, 1e-6), (sonar.F32, 1e-4)])
def test_speech_extractor_real_sample_rate_c4(ctx, prec, rtol):
    """C4 arithmetic: direct speech extractor with FeatureConfig.SampleRate = 16000, W=512 H=128."""
    x = synth.c4_speech(seconds=20.0, sr=16000)
    fc = dict(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
              enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, mfcc_coefficients=13)
    got = ctx.extract_speech_features(x, 16000, ctx.feature_config(is_news=0, precision=prec, **fc))
    ref = O.speech_features_reference(x, 16000, fc)
    for k in ("pitch_estimate", "pitch_confidence", "voicing_strength", "zero_crossing_rate", "short_time_energy"):
        assert np.array_equal(got[k], ref[k]), k            # YIN tau/tracking and ZCR counts are exact
    _cmp(got, ref, rtol, mag=O.stft_mag(x, 512, 128, nthreads=8))    # every field, slope included


def test_generate_fingerprint_music_c1_f32(ctx):
    """C1 in the f32 (throughput) mode: every GenerateFingerprint field within the north star's 1e-4
    of the oracle composition, spectral flatness and slope included (the
    descriptors take the f64 transform in either mode, spectral_flatness.go:31-73)."""
    x = synth.sweep(10.0)
    cfg = ctx.fingerprint_config(window_size=1024, hop_size=256, feature_window_size=1024, feature_hop_size=256,
                                 precision=sonar.F32)
    got = ctx.generate_fingerprint(x, 44100, "music", cfg)
    ref = O.speech_features_reference(x, 44100, dict(sample_rate=0, window_size=1024, hop_size=256,
                                                     stft_window_size=1024, stft_hop_size=256, enable_mfcc=1,
                                                     enable_speech_features=0, enable_temporal_features=0,
                                                     mfcc_coefficients=13))
    assert "spectral_flatness" in ref and "spectral_slope" in ref
    _cmp(got, ref, 1e-4)


def test_align_features_c3_lag(ctx):
    """C3-style: energy NCC + chroma DTW of two streams with an injected lag (60 s, scaled down from 5 min)."""
    q, r = synth.c3_pair(seconds=60.0, lag_s=12.34)
    fq = ctx.extract_speech_features(q, 44100, ctx.feature_config(sample_rate=44100, window_size=1024, hop_size=256))
    fr = ctx.extract_speech_features(r, 44100, ctx.feature_config(sample_rate=44100, window_size=1024, hop_size=256))
    F = sonar.stft_frames(len(q), 1024, 256)
    cq = ctx.chroma_stft(q, F, 256, 44100)
    cr = ctx.chroma_stft(r, F, 256, 44100)
    got = ctx.align_features(fq["short_time_energy"], fr["short_time_energy"], cq, cr, len(q), len(r),
                             sample_rate=44100, feature_sample_rate=44100, hop_size=256, window_size=1024,
                             max_lag_seconds=20.0)
    ref = O.align_features_reference(fq["short_time_energy"], fr["short_time_energy"], cq, cr, len(q), len(r),
                                     44100, 44100, 256, 20.0)
    assert got["peak_lag"] == ref["peak_lag"]
    assert abs(got["peak_lag"] - (-12.34 * 44100 / 256)) <= 1.5 or abs(got["peak_lag"] - 12.34 * 44100 / 256) <= 1.5
    assert np.array_equal(got["correlations"], ref["correlations"])
    assert np.array_equal(got["dtw_path_query"], ref["dtw_path_query"])
    assert got["method"] == ref["method"]
    for k in ("temporal_offset", "offset_confidence", "alignment_similarity", "alignment_quality"):
        assert got[k] == pytest.approx(ref[k], rel=1e-9, abs=1e-12), k


@pytest.mark.parametrize("chunk", [1 << 20, 300_007])
def test_generate_fingerprint_chunked_pcm_equals_one_shot(ctx, chunk, monkeypatch):
    """The host-PCM pipeline (H2D in chunks on a copy stream, every frame computed once its samples
    have landed) gives the same bits as the one-shot schedule: talk content (speech + temporal
    blocks on) at 16 kHz with a real sample rate, and music at 44.1 kHz (F1)."""
    for x, sr, ct in ((synth.c4_speech(seconds=90.0, sr=16000), 16000, "talk"),
                      (synth.c2_hour(seconds=60.0).astype(np.float64), 44100, "music")):
        cfg = ctx.fingerprint_config(window_size=1024, hop_size=256, feature_window_size=1024,
                                     feature_hop_size=256, precision=sonar.F64)
        monkeypatch.delenv("SONAR_PCM_CHUNK", raising=False)
        one = ctx.generate_fingerprint(x, sr, ct, cfg)
        monkeypatch.setenv("SONAR_PCM_CHUNK", str(chunk))
        got = ctx.generate_fingerprint(x, sr, ct, cfg)
        monkeypatch.delenv("SONAR_PCM_CHUNK")
        assert got.keys() == one.keys()
        for k in one:
            assert np.array_equal(np.asarray(got[k]), np.asarray(one[k]), equal_nan=True), (ct, k)


def test_extract_speech_chunked_pcm_real_rate(ctx, monkeypatch):
    """The same at FeatureConfig.SampleRate 16000 (loudness frames, voicing, tilt, formants run)."""
    x = synth.c4_speech(seconds=120.0, sr=16000)
    fc = ctx.feature_config(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
                            enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, is_news=0,
                            precision=sonar.F64)
    monkeypatch.delenv("SONAR_PCM_CHUNK", raising=False)
    one = ctx.extract_speech_features(x, 16000, fc)
    monkeypatch.setenv("SONAR_PCM_CHUNK", "500001")
    got = ctx.extract_speech_features(x, 16000, fc)
    assert got.keys() == one.keys()
    for k in one:
        assert np.array_equal(np.asarray(got[k]), np.asarray(one[k]), equal_nan=True), k


def test_generate_fingerprint_early_tracker_equals_late(ctx, monkeypatch):
    """Music content (no speech block): the harmonic tracker runs per chunk on YIN rows written
    straight into the pinned result block (round 6); SONAR_GF_EARLY=0 runs it after the last chunk.
    Same bits either way, chunked and one-shot."""
    x = synth.c2_hour(seconds=60.0).astype(np.float64)
    cfg = ctx.fingerprint_config(window_size=1024, hop_size=256, feature_window_size=1024, feature_hop_size=256,
                                 precision=sonar.F64)
    monkeypatch.setenv("SONAR_PCM_CHUNK", "400000")
    early = ctx.generate_fingerprint(x, 44100, "music", cfg)
    monkeypatch.setenv("SONAR_GF_EARLY", "0")
    late = ctx.generate_fingerprint(x, 44100, "music", cfg)
    assert early.keys() == late.keys()
    for k in early:
        assert np.array_equal(np.asarray(early[k]), np.asarray(late[k]), equal_nan=True), k
