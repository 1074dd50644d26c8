"""The oracle reproduces the committed fixtures (tests/golden, made by tools/make_golden.py).
Pins the CPU restatement of the Go path against regressions; parity with Go itself is
unpinned."""
import os

import numpy as np
import pytest

import oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


def close(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    if a.dtype.kind in "iub":
        assert np.array_equal(a, b)
    else:
        assert np.allclose(a, b, rtol=1e-12, atol=1e-300, equal_nan=True)


def test_golden_stft_mfcc():
    g = load("stft_mfcc_44k")
    x = g["pcm"].astype(np.float64)
    mag = O.stft_mag(x, 1024, 256)
    close(mag[:4], g["mag_head"])
    close(O.mfcc_frames(mag, 44100, n_coef=13, n_mels=40), g["mfcc40"])
    close(O.mfcc_frames(mag, 44100, n_coef=13, n_mels=26), g["mfcc26"])
    d = O.spectral_descriptors(mag, 44100)
    for k, v in d.items():
        close(v, g["desc_" + k])
    pre = O.preemphasis(x, 0.97)
    close(O.zcr_frames(pre, len(mag), 1024, 256, 44100), g["zcr"])
    close(O.short_time_energy(pre, 1024, 256), g["energy"])


def test_golden_generate_fingerprint():
    g = load("generate_fingerprint_music_c1")
    fc = dict(sample_rate=0, window_size=1024, hop_size=256, stft_window_size=1024, stft_hop_size=256,
              enable_mfcc=1, enable_speech_features=0, enable_temporal_features=0, mfcc_coefficients=13)
    ref = O.speech_features_reference(g["pcm"].astype(np.float64), 44100, fc)
    for k, v in ref.items():
        close(np.asarray(v, dtype=np.float64), g[k])


def test_golden_speech_formants_yin():
    g = load("speech_c4_16k")
    x = g["pcm"].astype(np.float64)
    fc = dict(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
              enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, mfcc_coefficients=13)
    ref = O.speech_features_reference(x, 16000, fc)
    for k, v in ref.items():
        close(np.asarray(v, dtype=np.float64), g["sx_" + k])
    fm = O.formant_frames(x, 16000, want_lpc=True)
    for k, v in fm.items():
        close(v, g["fm_" + k])
    for i, (p, c, t) in enumerate(zip(g["yin_pitch"], g["yin_conf"], g["yin_tau"])):
        pp, cc, tt = O.yin_raw(x[i * 512:i * 512 + 1024], 16000)
        assert (pp, cc, tt) == (p, c, t)


def test_golden_voice_quality():
    g = load("voice_quality_16k")
    x = g["pcm"].astype(np.float64)
    vq, st = O.voice_quality(O.preemphasis(x, 0.97), 16000)
    assert st == int(g["status"])
    close(np.array([vq[k] for k in O.VOICE_QUALITY_KEYS]), g["vq"])
    fc = dict(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
              enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, mfcc_coefficients=13)
    ref = O.speech_features_reference(x, 16000, fc)
    assert ref["is_speech"] == float(g["sx_is_speech"])
    close(np.float64(ref["jitter"]), g["sx_jitter"])
    close(np.float64(ref["shimmer"]), g["sx_shimmer"])


def test_golden_chroma_alignment():
    g = load("chroma_44k")
    close(O.chroma_music(g["pcm"].astype(np.float64), int(g["n_frames"]), 256, 44100), g["chroma"])
    a = load("alignment")
    corr, met = O.ncc(a["ncc_a"], a["ncc_b"], 500)
    close(corr, a["ncc_corr"])
    close(np.array([met[k] for k in O.NCC_KEYS]), a["ncc_metrics"])
    r = O.dtw(a["dtw_q"], a["dtw_r"], want_cost=True)
    close(r["path_q"], a["dtw_path_q"]); close(r["path_r"], a["dtw_path_r"])
    close(r["path_cost"], a["dtw_path_cost"]); close(r["cost"], a["dtw_cost"])
    assert r["distance"] == float(a["dtw_distance"])
