"""VoiceQualityAnalyzer.AnalyzeVoiceQuality (algorithms/speech/voice_quality.go:56-111) on the GPU
(sonar_voice_quality: YIN scan at hop 256, period RMS and HNR autocorrelation kernels, host period
walk) against the oracle, and its Jitter / Shimmer inside SpeechFeatureExtractor.ExtractFeatures
(speech.go:306-309).  Period counts, lengths and hence jitter are exact (YIN tau and tracking are
bit-exact); the float64 kernels sum in Go's order, so every field matches to 1e-12 relative."""
import os

import numpy as np
import pytest

import oracle as O
import sonar
from sonar import synth

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _same(got, ref):
    for k in O.VOICE_QUALITY_KEYS:
        assert got[k] == pytest.approx(ref[k], rel=1e-12, abs=1e-12), k


@pytest.mark.parametrize("kind", ["voiced", "voiced_f0_220", "tone", "voiced_5h"])
def test_voice_quality_matches_oracle(ctx, kind):
    sr = 16000
    if kind == "tone":
        t = np.arange(2 * sr) / sr
        x = np.sin(2 * np.pi * 200 * t) + 0.3 * np.sin(2 * np.pi * 400 * t)
    elif kind == "voiced_f0_220":
        x = synth.voiced(seconds=3.0, f0=220.0, vibrato=20.0)
    elif kind == "voiced_5h":
        x = synth.voiced(seconds=5.0, harmonics=5)
    else:
        x = synth.voiced(seconds=4.0)
    y = O.preemphasis(x, 0.97)
    ref, st = O.voice_quality(y, sr)
    assert st == 0 and ref["num_periods"] >= 3
    _same(ctx.voice_quality(y, sr), ref)


def test_voice_quality_errors(ctx):
    sr = 16000
    x = synth.voiced(seconds=2.0)
    with pytest.raises(sonar.SonarError, match="need at least 1 second"):
        ctx.voice_quality(x[: sr - 1], sr)
    with pytest.raises(sonar.SonarError, match="insufficient pitch periods"):
        ctx.voice_quality(np.random.default_rng(0).standard_normal(2 * sr), sr)


def test_voice_quality_golden(ctx):
    g = np.load(os.path.join(G, "voice_quality_16k.npz"), allow_pickle=False)
    got = ctx.voice_quality(O.preemphasis(g["pcm"].astype(np.float64), 0.97), 16000)
    _same(got, dict(zip(O.VOICE_QUALITY_KEYS, g["vq"].tolist())))


@pytest.mark.parametrize("prec", [sonar.F64, sonar.F32])
def test_speech_extractor_jitter_shimmer(ctx, prec):
    """A voiced input passes detectSpeech, so AnalyzeSpeech runs voice quality (speech.go:306-309)."""
    x = synth.voiced(seconds=4.0)
    fc = dict(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
              enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, mfcc_coefficients=13)
    got = ctx.extract_speech_features(x, 16000, ctx.feature_config(is_news=0, precision=prec, **fc))
    ref = O.speech_features_reference(x, 16000, fc)
    assert got["is_speech"] == ref["is_speech"] == 1.0
    assert ref["jitter"] > 0 and ref["shimmer"] > 0
    assert got["jitter"] == pytest.approx(ref["jitter"], rel=1e-12)
    assert got["shimmer"] == pytest.approx(ref["shimmer"], rel=1e-12)
