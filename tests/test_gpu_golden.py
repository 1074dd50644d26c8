"""The HIP path against the committed fixtures (tests/golden), at the north-star
tolerances: bit-exact for integer / index / decision outputs, NCC and DTW; float
features 1e-4 relative in f32 mode and 1e-6 in f64 mode."""
import os

import numpy as np
import pytest

import oracle as O
import sonar
from parity import assert_mfcc, assert_rolloff

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


def rel(a, b, floor_frac=1e-6):
    """max per-element relative error; elements below floor_frac of the peak use that floor"""
    a, b = np.asarray(a, float), np.asarray(b, float)
    if a.size == 1 and b.size == 1:
        a, b = a.reshape(()), b.reshape(())
    assert a.shape == b.shape
    if not b.size:
        return 0.0
    floor = max(np.max(np.abs(b)) * floor_frac, 1e-30)
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), floor))


@pytest.mark.parametrize("prec,tol", [(sonar.F64, 1e-6), (sonar.F32, 1e-4)])
def test_gpu_golden_stft_mfcc(ctx, prec, tol):
    g = load("stft_mfcc_44k")
    x = g["pcm"]
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13, precision=prec,
                     pcm_dtype=sonar.F32, out_dtype=sonar.F64,
                     flags=sonar.FP_MFCC | sonar.FP_MAGNITUDE | sonar.FP_SPECTRAL | sonar.FP_ZCR | sonar.FP_ENERGY,
                     energy_window=1024, energy_hop=256, preemph_alpha=0.97)
    got = ctx.fingerprint(x, cfg)
    assert_mfcc(got["mfcc"], g["mfcc40"], tol)
    assert rel(got["magnitude"][:4], g["mag_head"], floor_frac=1e-3 if prec == sonar.F64 else 1e-2) < tol
    for k in ("centroid", "bandwidth", "flatness", "crest", "flux", "low_ratio", "high_ratio"):
        assert rel(got[k], g["desc_" + k]) < tol, k
    mag = O.stft_mag(x.astype(np.float64), 1024, 256, nthreads=8)
    assert_rolloff(got["rolloff"], g["desc_rolloff"], mag, 1e-12 if prec == sonar.F64 else 1e-5)
    assert np.array_equal(got["zcr"], g["zcr"])                              # exact crossing counts
    assert np.array_equal(got["energy"], g["energy"])


def test_gpu_golden_generate_fingerprint(ctx):
    g = load("generate_fingerprint_music_c1")
    cfg = ctx.fingerprint_config(window_size=1024, hop_size=256, feature_window_size=1024, feature_hop_size=256,
                                 precision=sonar.F64)
    got = ctx.generate_fingerprint(g["pcm"].astype(np.float64), 44100, "music", cfg)
    for k in g.files:
        if k == "pcm":
            continue
        if k == "spectral_rolloff":                              # sr = 0 (F3): all zero, exact
            assert np.array_equal(np.asarray(got[k], float), g[k])
            continue
        if k in ("low_energy_ratio", "high_energy_ratio"):       # ratios in [0, 1]; FFT-leakage-level values
            assert np.max(np.abs(np.asarray(got[k]) - g[k])) < 1e-9, k
            continue
        assert rel(got[k], g[k]) < 1e-6, k


def test_gpu_golden_speech_formants_yin(ctx):
    g = load("speech_c4_16k")
    x = g["pcm"].astype(np.float64)
    fc = ctx.feature_config(sample_rate=16000, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
                            enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1,
                            mfcc_coefficients=13, is_news=0, precision=sonar.F64)
    got = ctx.extract_speech_features(x, 16000, fc)
    for k in g.files:
        if not k.startswith("sx_"):
            continue
        name = k[3:]
        v = np.asarray(got[name], float)
        if name in ("pitch_estimate", "pitch_confidence", "voicing_strength", "zero_crossing_rate",
                    "short_time_energy", "is_speech", "formant_frequencies"):
            assert np.array_equal(v.reshape(g[k].shape) if v.size else v, g[k]) or (v.size == g[k].size == 0), name
        elif name == "spectral_rolloff":
            assert_rolloff(v, g[k], O.stft_mag(x, 512, 128, nthreads=8), 1e-12)
        elif g[k].size:
            b = np.nan_to_num(g[k])
            assert rel(np.nan_to_num(v).reshape(b.shape), b) < 1e-6, name
    fm = ctx.formants(x, 16000)
    assert np.array_equal(fm["status"], g["fm_status"])
    assert np.array_equal(fm["frequency"], g["fm_frequency"])
    assert np.allclose(fm["quality"], g["fm_quality"], rtol=1e-6, atol=1e-9)
    p, c, t = ctx.pitch_yin(x, 16000)
    k = len(g["yin_tau"])
    assert np.array_equal(t[:k], g["yin_tau"]) and np.array_equal(p[:k], g["yin_pitch"])
    assert np.array_equal(c[:k], g["yin_conf"])


def test_gpu_golden_chroma_alignment(ctx):
    g = load("chroma_44k")
    got = ctx.chroma_stft(g["pcm"].astype(np.float64), int(g["n_frames"]), 256, 44100)
    assert rel(got, g["chroma"]) < 1e-9
    a = load("alignment")
    corr, met = ctx.ncc(a["ncc_a"], a["ncc_b"], 500)
    assert np.array_equal(corr, a["ncc_corr"])
    assert met["peak_lag"] == a["ncc_metrics"][1]
    r = ctx.dtw(a["dtw_q"], a["dtw_r"], want_cost=True)
    assert np.array_equal(r["path_q"], a["dtw_path_q"]) and np.array_equal(r["path_r"], a["dtw_path_r"])
    assert np.array_equal(r["path_cost"], a["dtw_path_cost"]) and np.array_equal(r["cost"], a["dtw_cost"])
    assert r["distance"] == float(a["dtw_distance"])
