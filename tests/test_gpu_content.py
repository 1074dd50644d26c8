"""ContentDetector (fingerprint/content_detector.go) on the GPU vs the CPU oracle.

DetectFromAudio: zero-crossing rate, energy variance, silence ratio, dynamic range and temporal
stability come from per-frame sums computed in Go's order (bit-identical) and integer counts /
extrema, so they must match the oracle exactly; the spectral centroid, the frequency split and
the harmonic ratio come from the direct DFT, whose sin/cos differ from libm by an ulp: 1e-9
relative.  The metadata rules are checked against a Python restatement of :501-626.
"""
import numpy as np
import pytest

import oracle
from sonar import Context, SonarError, synth

pytestmark = pytest.mark.gpu

EXACT = ["zero_crossing_rate", "energy_variance", "silence_ratio", "dynamic_range", "temporal_stability"]
CLOSE = ["spectral_centroid", "low_freq_energy", "high_freq_energy", "harmonic_ratio",
         "classification_confidence"]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def _signals():
    rng = np.random.default_rng(21)
    sil = np.zeros(44100 * 3)
    sil[::977] = 0.3
    gated = rng.normal(0, 0.2, 44100 * 6) * (np.sin(np.arange(44100 * 6) / 4000.0) > 0)
    return {
        "sweep10s": (synth.sweep(10.0), 44100),
        "noise5s": (rng.normal(0, 0.3, 44100 * 5), 44100),
        "speech30s": (synth.c4_speech(30.0), 16000),
        "sparse": (sil, 44100),
        "gated": (gated, 44100),
        "zeros": (np.zeros(5000), 44100),
        "n1": (np.array([0.5]), 44100),
        "n100": (rng.normal(0, 1, 100), 8000),
        "n2047": (rng.normal(0, 1, 2047), 44100),
        "n2048": (rng.normal(0, 1, 2048), 44100),
        "n3001": (rng.normal(0, 1, 3001), 22050),
        "tone": (0.5 * np.sin(2 * np.pi * 440 * np.arange(44100 * 2) / 44100), 44100),
    }


@pytest.mark.parametrize("name", list(_signals().keys()))
def test_detect_from_audio_vs_oracle(ctx, name):
    x, sr = _signals()[name]
    ct, f = ctx.detect_from_audio(x, sr)
    oct_, of = oracle.detect_from_audio(x, sr)
    for k in EXACT:
        assert f[k] == of[k], (name, k, f[k], of[k])
    for k in CLOSE:
        assert abs(f[k] - of[k]) <= 1e-9 * max(1.0, abs(of[k])), (name, k, f[k], of[k])
    assert ct == oct_, (name, ct, oct_, f)


def test_detect_errors(ctx):
    with pytest.raises(SonarError):
        ctx.detect_from_audio(np.ones(100), 5)          # 100 ms frame loop never ends in Go
    assert ctx.detect_from_audio(np.zeros(0), 44100)[0] == "unknown"


# ---- metadata rules: Python restatement of content_detector.go:501-626 -------------------
MUSIC_G = ["rock", "pop", "jazz", "classical", "hip-hop", "hip hop", "country", "electronic", "blues", "reggae",
           "folk", "metal", "punk", "r&b", "soul", "funk", "dance", "techno", "house", "ambient", "indie",
           "alternative", "grunge", "ska", "latin", "world", "gospel"]
NEWS_G = ["news", "talk", "politics", "current affairs", "public radio", "discussion", "interview", "call-in",
          "spoken word", "commentary", "analysis", "reporting", "journalism", "public affairs"]
SPORTS_G = ["sports", "football", "basketball", "baseball", "soccer", "hockey", "tennis", "golf", "racing",
            "motorsports", "athletics", "cricket", "rugby", "boxing", "mma", "sports talk", "sports news"]
NEWS_S = ["news", "npr", "bbc", "cnn", "cbc", "abc news", "nbc news", "fox news", "public radio", "current affairs",
          "talk radio"]
SPORTS_S = ["sports", "espn", "fox sports", "sports radio", "the fan", "sport", "athletic", "game", "stadium"]
MUSIC_S = ["fm", "music", "hits", "rock", "pop", "jazz", "country", "classic", "radio", "mix", "beat", "sound",
           "groove"]


def py_metadata(md):
    ct, genre, station, url = (md.get(k, "") for k in ("content_type", "genre", "station", "url"))
    if ct:
        v = ct.lower()
        return {"music": "music", "audio/music": "music", "news": "news", "talk": "news", "spoken": "news",
                "sports": "sports"}.get(v, "unknown")
    if genre:
        g = genre.strip().lower()
        for lst, t in ((MUSIC_G, "music"), (NEWS_G, "news"), (SPORTS_G, "sports")):
            if any(w in g for w in lst):
                return t
        return "talk" if "talk" in g and "sports" not in g else "unknown"
    comb = station.strip().lower() + " " + url.lower()
    for lst, t in ((NEWS_S, "news"), (SPORTS_S, "sports"), (MUSIC_S, "music")):
        if any(w in comb for w in lst):
            return t
    return "talk" if "talk" in comb and "sports" not in comb else "unknown"


MD_CASES = [{"content_type": "Music"}, {"content_type": "audio/music"}, {"content_type": "spoken"},
            {"content_type": "TALK"}, {"content_type": "sports"}, {"content_type": "speech"},
            {"genre": "Classic Rock"}, {"genre": " sports talk "}, {"genre": "Baseball"}, {"genre": "talkback"},
            {"genre": "podcast"}, {"station": "ESPN Radio"}, {"station": "", "url": "http://npr.org/live"},
            {"station": "Talk 101"}, {"station": "KXYZ"}, {"station": "The Groove"}, {}]


@pytest.mark.parametrize("md", MD_CASES)
def test_detect_content_type_metadata(ctx, md):
    x = np.zeros(4096)
    got = ctx.detect_content_type(x, 44100, md, acoustic_detection=False, default_content_type="mixed")
    want = py_metadata(md)
    assert got == (want if want != "unknown" else "mixed"), (md, got, want)


def test_detect_content_type_acoustic_and_nil_metadata(ctx):
    x, sr = _signals()["speech30s"]
    want, _ = oracle.detect_from_audio(x, sr)
    assert ctx.detect_content_type(x, sr, None) == (want if want != "unknown" else "unknown")
    assert ctx.detect_content_type(x, sr, {"content_type": "speech"}) == want
    assert ctx.detect_content_type(x, sr, None, acoustic_detection=False, default_content_type="talk") == "talk"


def test_generate_fingerprint_detects_unknown_content(ctx):
    """F12: ContentType "speech" is unknown to ToContentType -> DetectContentType runs; the
    fingerprint then equals the one generated with the detected type given explicitly."""
    x, sr = _signals()["speech30s"]
    want, _ = oracle.detect_from_audio(x, sr)
    cfg = ctx.fingerprint_config(window_size=512, hop_size=128, feature_window_size=512, feature_hop_size=128)
    a = ctx.generate_fingerprint(x, sr, "speech", cfg)
    names = ["music", "news", "sports", "talk", "mixed", "unknown"]
    assert names[int(a["content_type"].reshape(-1)[0])] == want
    b = ctx.generate_fingerprint(x, sr, want, cfg)
    for k in ("mfcc", "spectral_centroid", "short_time_energy"):
        if k in b:
            assert np.array_equal(a[k], b[k]), k
