"""ctypes binding for the CPU oracle (oracle/sonar_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.  The oracle is a
float64 restatement of the Go reference (RyanBlaney/sonido-sonar); see
sonar_oracle.h for the parity status ("parity unpinned" w.r.t. Go: no Go
toolchain here, pinned by analytic known-answer tests and numpy instead).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsonar_oracle.so")
_lib = None

WINDOWS = {"hann": 0, "hamming": 1, "blackman": 2, "blackman_harris": 3, "kaiser": 4,
           "tukey": 5, "rectangular": 6, "bartlett": 7, "welch": 8}

_d = C.POINTER(C.c_double)
_i32 = C.POINTER(C.c_int32)
_i64 = C.POINTER(C.c_int64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.or_window.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, _d]
        L.or_fft.argtypes = [_d, _d, C.c_int, _d, _d]
        L.or_stft_frames.argtypes = [C.c_int64, C.c_int, C.c_int]
        L.or_stft_frames.restype = C.c_int64
        L.or_stft_mag.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, _d]
        L.or_stft_mag_window.argtypes = [_d, C.c_int64, C.c_int, C.c_int, _d, C.c_int, _d]
        L.or_stft_complex.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, _d, _d, _d]
        L.or_filterbank.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, _d]
        L.or_mfcc_frames.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                     C.c_double, C.c_int, C.c_double, C.c_int, C.c_int, _d]
        L.or_spectral_descriptors.argtypes = [_d, C.c_int64, C.c_int, C.c_int] + [_d] * 9
        L.or_spectral_contrast.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, _d]
        L.or_preemphasis.argtypes = [_d, C.c_int64, C.c_double, _d]
        L.or_dc_removal.argtypes = [_d, C.c_int64, C.c_double, _d]
        L.or_zcr_frames.argtypes = [_d, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _d]
        L.or_short_time_energy.argtypes = [_d, C.c_int64, C.c_int, C.c_int, _d]
        L.or_short_time_energy.restype = C.c_int64
        L.or_pitch_frames.argtypes = [C.c_int64]
        L.or_pitch_frames.restype = C.c_int64
        L.or_yin_raw.argtypes = [_d, C.c_int, _d, _d, C.POINTER(C.c_int)]
        L.or_pitch_track.argtypes = [_d, C.c_int64, C.c_int, C.c_int, _d, _d, _d]
        L.or_pitch_track.restype = C.c_int64
        L.or_voice_quality.argtypes = [_d, C.c_int64, C.c_int, _d]
        L.or_chroma_music.argtypes = [_d, C.c_int64, C.c_int64, C.c_int, C.c_int, _d]
        L.or_chroma_frames.argtypes = [_d, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _d]
        L.or_ncc.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int, _d, _d]
        L.or_dtw.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int, C.c_int, _d, _i32, _i32, _d, _i64, _d]
        L.or_dtw_stripes.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int, C.c_int, C.c_int, _i32, _i32, _d, _i64,
                                     _d]
        L.or_align_dtw_metrics.argtypes = [_i32, _i32, _d, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_int, _d]
        L.or_align_xcorr_metrics.argtypes = [_d, C.c_int, C.c_int, C.c_int, _d]
        L.or_autocorr_fft.argtypes = [_d, C.c_int, C.c_int, _d]
        L.or_formant_frame.argtypes = [_d, C.c_int64, C.c_int, _d, _d, _d]
        L.or_formant_frames.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, _d, _d, _d]
        L.or_formant_frames.restype = C.c_int64
        L.or_detect_from_audio.argtypes = [_d, C.c_int64, C.c_int, C.c_double, _d, C.POINTER(C.c_int)]
        L.or_fp_compare.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_find_best_matches.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, _i64]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_d)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def window(kind="hann", size=1024, symmetric=True, normalize=True, beta=8.6, alpha=0.5):
    out = np.zeros(size)
    rc = lib().or_window(WINDOWS[kind], size, int(symmetric), int(normalize), beta, alpha, _p(out))
    if rc != 0:
        raise ValueError("invalid window configuration")
    return out


def fft(x):
    x = np.asarray(x)
    re = _f64(x.real)
    im = _f64(x.imag) if np.iscomplexobj(x) else np.zeros(len(x))
    ore, oim = np.zeros(len(x)), np.zeros(len(x))
    lib().or_fft(_p(re), _p(im), len(x), _p(ore), _p(oim))
    return ore + 1j * oim


def stft_frames(n, W, H):
    return int(lib().or_stft_frames(n, W, H))


def stft_mag(pcm, W, H, window_type="hann", nthreads=1):
    pcm = _f64(pcm)
    F = stft_frames(len(pcm), W, H)
    if F < 0:
        raise ValueError("signal too short for given window size and hop size")
    out = np.zeros((F, W // 2 + 1))
    rc = lib().or_stft_mag(_p(pcm), len(pcm), W, H, WINDOWS[window_type], nthreads, _p(out))
    if rc != 0:
        raise ValueError("stft failed")
    return out


def stft_complex(pcm, W, H, window_type="hann"):
    """(complex F x (W/2+1), phase F x (W/2+1)): SpectrogramResult.Complex / .Phase (spectral.go:490-494)"""
    pcm = _f64(pcm)
    F = stft_frames(len(pcm), W, H)
    if F < 0:
        raise ValueError("signal too short for given window size and hop size")
    re, im, ph = np.zeros((F, W // 2 + 1)), np.zeros((F, W // 2 + 1)), np.zeros((F, W // 2 + 1))
    rc = lib().or_stft_complex(_p(pcm), len(pcm), W, H, WINDOWS[window_type], _p(re), _p(im), _p(ph))
    if rc != 0:
        raise ValueError("stft failed")
    return re + 1j * im, ph


def filterbank(n_filters, fft_size, sample_rate, low, high, kind="mel"):
    out = np.zeros((n_filters, fft_size // 2 + 1))
    lib().or_filterbank(1 if kind == "bark" else 0, n_filters, fft_size, sample_rate, low, high, _p(out))
    return out


def mfcc_frames(mag, sample_rate, n_coef=13, n_mels=26, low=0.0, high=0.0, use_lifter=True,
                lifter=22.0, kind="mel"):
    mag = _f64(mag)
    F, K = mag.shape
    nc = n_coef if n_coef > 0 else 13
    out = np.zeros((F, nc))
    rc = lib().or_mfcc_frames(_p(mag), F, K, sample_rate, n_coef, n_mels, low, high, int(use_lifter),
                              lifter, 1 if kind == "bark" else 0, 0, _p(out))
    if rc != 0:
        raise ValueError("failed to create mel filter bank")
    return out


def spectral_descriptors(mag, sample_rate):
    mag = _f64(mag)
    F, K = mag.shape
    names = ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope"]
    outs = {n: np.zeros(F) for n in names}
    outs["flux"] = np.zeros(max(F - 1, 0) + 1)
    outs["low_ratio"] = np.zeros(F)
    outs["high_ratio"] = np.zeros(F)
    lib().or_spectral_descriptors(_p(mag), F, K, sample_rate, *[_p(outs[n]) for n in names],
                                  _p(outs["flux"]), _p(outs["low_ratio"]), _p(outs["high_ratio"]))
    outs["flux"] = outs["flux"][: max(F - 1, 0)]
    return outs


def preemphasis(x, alpha):
    x = _f64(x)
    out = np.zeros_like(x)
    lib().or_preemphasis(_p(x), len(x), alpha, _p(out))
    return out


def dc_removal(x, R=0.995):
    x = _f64(x)
    out = np.zeros_like(x)
    lib().or_dc_removal(_p(x), len(x), R, _p(out))
    return out


def zcr_frames(pcm, F, W, H, sample_rate):
    pcm = _f64(pcm)
    out = np.zeros(F)
    lib().or_zcr_frames(_p(pcm), len(pcm), F, W, H, sample_rate, _p(out))
    return out


def short_time_energy(x, W, H):
    x = _f64(x)
    if W <= 0 or H <= 0 or len(x) < W:
        return np.zeros(0)
    n = (len(x) - W) // H + 1
    out = np.zeros(n)
    m = lib().or_short_time_energy(_p(x), len(x), W, H, _p(out))
    return out[:m]


def yin_raw(frame, sample_rate):
    frame = _f64(frame)
    assert len(frame) == 1024
    p, c, t = C.c_double(), C.c_double(), C.c_int()
    lib().or_yin_raw(_p(frame), sample_rate, C.byref(p), C.byref(c), C.byref(t))
    return p.value, c.value, t.value


def pitch_track(pcm, sample_rate, passes=1):
    pcm = _f64(pcm)
    F = int(lib().or_pitch_frames(len(pcm)))
    p, c, v = np.zeros(F), np.zeros(F), np.zeros(F)
    lib().or_pitch_track(_p(pcm), len(pcm), sample_rate, passes, _p(p), _p(c), _p(v))
    return p, c, v


VOICE_QUALITY_KEYS = ("jitter", "shimmer", "hnr", "noise_measure", "f0_stability", "amplitude_stability",
                      "voicing_strength", "overall_quality", "num_periods", "mean_f0", "f0_range",
                      "analysis_quality")


def voice_quality(signal, sample_rate):
    """VoiceQualityAnalyzer.AnalyzeVoiceQuality (algorithms/speech/voice_quality.go:56-111).
    Returns (dict, status): status 0 ok, -1 shorter than one second, -2 fewer than 3 periods
    (the Go call returns an error and a nil result; the dict is then all zero)."""
    signal = _f64(signal)
    out = np.zeros(12)
    st = lib().or_voice_quality(_p(signal), len(signal), sample_rate, _p(out))
    return dict(zip(VOICE_QUALITY_KEYS, out.tolist())), int(st)


def chroma_music(pcm, F, H, sample_rate):
    pcm = _f64(pcm)
    out = np.zeros((F, 12))
    lib().or_chroma_music(_p(pcm), len(pcm), F, H, sample_rate, _p(out))
    return out


def chroma_frames(y, F, H, fs, sample_rate):
    y = _f64(y)
    out = np.zeros((F, 12))
    lib().or_chroma_frames(_p(y), len(y), F, H, fs, sample_rate, _p(out))
    return out


NCC_KEYS = ["peak_correlation", "peak_lag", "peak_index", "p_value", "snr", "sharpness",
            "second_peak", "peak_to_sidelobe", "overlap_length", "num_lags"]


def ncc(a, b, max_lag):
    a, b = _f64(a), _f64(b)
    if len(a) == 0 or len(b) == 0:
        raise ValueError("empty signals provided")
    L = max(0, min(max_lag, len(a) - 1, len(b) - 1))
    corr = np.zeros(2 * L + 1)
    met = np.zeros(10)
    lib().or_ncc(_p(a), len(a), _p(b), len(b), max_lag, _p(corr), _p(met))
    return corr, dict(zip(NCC_KEYS, met.tolist()))


def dtw(q, r, band=-1, want_cost=False):
    q = _f64(q)
    r = _f64(r)
    if q.ndim == 1:
        q = q[:, None]
    if r.ndim == 1:
        r = r[:, None]
    nq, d = q.shape
    nr = r.shape[0]
    if nq == 0 or nr == 0:
        raise ValueError("empty sequences provided")
    cap = nq + nr + 1
    pq = np.zeros(cap, np.int32)
    pr = np.zeros(cap, np.int32)
    pc = np.zeros(cap)
    plen = C.c_int64()
    dist = C.c_double()
    cost = np.zeros((nq, nr + 1)) if want_cost else None
    rc = lib().or_dtw(_p(q), nq, _p(r), nr, d, band, _p(cost) if want_cost else None,
                      pq.ctypes.data_as(_i32), pr.ctypes.data_as(_i32), _p(pc), C.byref(plen), C.byref(dist))
    if rc != 0:
        raise MemoryError("oracle dtw failed")
    P = plen.value
    return {"distance": dist.value, "path_q": pq[:P], "path_r": pr[:P], "path_cost": pc[:P], "cost": cost}


def dtw_full(q, r, band=-1, nthreads=8):
    """dtw() at any size (dtw_oracle.c): the same values, without the (N+1)(M+1) matrix; the
    fill runs as a stripe wavefront over `nthreads` threads."""
    q = _f64(q)
    r = _f64(r)
    if q.ndim == 1:
        q = q[:, None]
    if r.ndim == 1:
        r = r[:, None]
    nq, d = q.shape
    nr = r.shape[0]
    if nq == 0 or nr == 0:
        raise ValueError("empty sequences provided")
    cap = nq + nr + 1
    pq = np.zeros(cap, np.int32)
    pr = np.zeros(cap, np.int32)
    pc = np.zeros(cap)
    plen = C.c_int64()
    dist = C.c_double()
    rc = lib().or_dtw_stripes(_p(q), nq, _p(r), nr, d, band, nthreads, pq.ctypes.data_as(_i32),
                              pr.ctypes.data_as(_i32), _p(pc), C.byref(plen), C.byref(dist))
    if rc != 0:
        raise MemoryError("oracle dtw_full failed")
    P = plen.value
    return {"distance": dist.value, "path_q": pq[:P], "path_r": pr[:P], "path_cost": pc[:P]}


def align_dtw_metrics(res, nq, nr, sample_rate):
    out = np.zeros(6)
    P = len(res["path_q"])
    lib().or_align_dtw_metrics(np.ascontiguousarray(res["path_q"], np.int32).ctypes.data_as(_i32),
                               np.ascontiguousarray(res["path_r"], np.int32).ctypes.data_as(_i32),
                               _p(_f64(res["path_cost"])), P, nq, nr, res["distance"], sample_rate, _p(out))
    return dict(zip(["similarity", "confidence", "offset", "offset_seconds", "quality", "stability"], out.tolist()))


def align_xcorr_metrics(met, hop, sample_rate, max_lag):
    m = _f64([met[k] for k in NCC_KEYS])
    out = np.zeros(6)
    lib().or_align_xcorr_metrics(_p(m), hop, sample_rate, max_lag, _p(out))
    return dict(zip(["offset", "offset_seconds", "similarity", "confidence", "quality", "noise_level"], out.tolist()))


# ---------------------------------------------------------------------------
# Compositions of the Go orchestration (test infrastructure, pure Python over
# the C primitives; restated from the Go source independently of the product)
# ---------------------------------------------------------------------------

def _median_pos(v):
    f = sorted(x for x in v if x > 0)
    if not f:
        return 0.0
    n = len(f)
    return (f[n // 2 - 1] + f[n // 2]) / 2.0 if n % 2 == 0 else f[n // 2]


class YinTrack:
    """postProcessResult + updateTemporalTracking (pitch_detection.go:767-921)."""

    def __init__(self):
        self.hist, self.prev = [], 0.0

    def step(self, p, c):
        v = c
        if p != 0.0 and self.hist:
            rec = self.hist[-5:]
            if len(rec) >= 3:
                med = _median_pos(rec)
                for r in (0.5, 2.0, 1.0 / 3.0, 3.0):
                    ex = med * r
                    with np.errstate(divide="ignore", invalid="ignore"):
                        if abs(p - ex) / ex < 0.1:
                            if abs(p - med) > abs(ex - med):
                                p = ex
                            break
        if c < 0.5:
            p, c, v = 0.0, 0.0, 0.0
        self.hist.append(p)
        self.hist = self.hist[-20:]
        if len(self.hist) > 1:
            rec = self.hist[-3:]
            p = _median_pos(rec) if len(rec) >= 3 else 0.3 * p + 0.7 * self.prev
        self.prev = p
        return p, c, v


def speech_features_reference(pcm, sample_rate, fc):
    """SpeechFeatureExtractor.ExtractFeatures (fingerprint/extractors/speech.go:135-550), fp64.
    fc: dict(sample_rate, window_size, hop_size, stft_window_size, stft_hop_size, enable_mfcc,
    enable_speech_features, enable_temporal_features, mfcc_coefficients[, nthreads: the STFT's worker
    threads, Go's worker-pool shape, default 8])."""
    pcm = _f64(pcm)
    csr = fc["sample_rate"]
    W, H = fc["stft_window_size"], fc["stft_hop_size"]
    mag = stft_mag(pcm, W, H, nthreads=fc.get("nthreads", 8))
    F = len(mag)
    pre = preemphasis(pcm, 0.97)
    out = {}
    if fc["enable_mfcc"]:
        out["mfcc"] = mfcc_frames(mag, csr, n_coef=fc["mfcc_coefficients"], n_mels=26)
    d = spectral_descriptors(mag, csr)
    for k in ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope"]:
        out["spectral_" + k] = d[k]
    if F > 1:
        out["spectral_flux"] = d["flux"]
    out["zero_crossing_rate"] = zcr_frames(pre, F, W, H, csr)
    ste = short_time_energy(pre, fc["window_size"], fc["hop_size"])
    # YIN raw on the pre-emphasised PCM
    Fp = int(lib().or_pitch_frames(len(pre)))
    raw = []
    for i in range(Fp):
        fr = pre[i * 512: i * 512 + 1024]
        raw.append(yin_raw(fr, csr)[:2] if len(fr) == 1024 else None)
    trk = YinTrack()
    if fc["enable_speech_features"]:
        n = len(pre)
        sp = not (n < int(csr / 4))
        cr = np.sum(((pre[:-1] >= 0) & (pre[1:] < 0)) | ((pre[:-1] < 0) & (pre[1:] >= 0)))
        z = 0.0 if n <= 1 else cr / (n - 1)
        if sp and (z < 0.01 or z > 0.3):
            sp = False
        if sp and np.sqrt(np.sum(pre * pre) / n) < 0.001:
            sp = False
        if sp:
            fr = pre[:1024]
            mc = 0.0
            for lag in range(20, min(400, 512)):
                c = np.sum(fr[:1024 - lag] * fr[lag:]) / (1024 - lag)
                mc = max(mc, c)
            en = np.sum(fr * fr) / 1024
            if en > 0:
                mc /= en
            sp = mc > 0.1 and len(pre) >= 1024
        out["is_speech"] = 1.0 if sp else 0.0
        fq, vtl = np.zeros((0, 0)), 17.5                     # speech.go:279-303
        if sp:
            fm = formant_frame(pre, csr)
            if fm["status"][0] == 0:
                nv = int(fm["n_formants"][0])
                fq = fm["frequency"][0][:nv].reshape(1, nv) if nv else np.zeros((0, 0))
                vtl = float(fm["vocal_tract_length"][0])
        out["formant_frequencies"], out["vocal_tract_length"] = fq, vtl
        jit = shi = 0.0                                      # speech.go:287-288, 306-309
        if sp:
            vq, vst = voice_quality(pre, csr)                # AnalyzeSpeech -> AnalyzeVoiceQuality (:77-80)
            if vst == 0:
                jit, shi = vq["jitter"], vq["shimmer"]
        out["jitter"], out["shimmer"] = jit, shi
        if sp:                                               # estimateSpeechRate (speech.go:779-797)
            with np.errstate(divide="ignore", invalid="ignore"):
                dur = np.float64(len(pre)) / np.float64(csr)     # IEEE like Go: sr 0 -> +Inf
            sil = 0.0
            if len(ste):
                thr = np.sort(ste)[len(ste) // 10]
                sil = np.count_nonzero(ste <= thr) / len(ste)
            with np.errstate(invalid="ignore"):
                st = dur * (1.0 - sil)
                out["speech_rate"] = float(4.0 * st / dur) if st > 0 else 3.0
        else:
            out["speech_rate"] = 0.0
        if sp:
            vo = np.zeros(Fp)
            for i, r in enumerate(raw):
                if r is not None:
                    vo[i] = trk.step(*r)[2]
            out["voicing_probability"] = vo
    pe, pc, vs = np.zeros(Fp), np.zeros(Fp), np.zeros(Fp)
    for i, r in enumerate(raw):
        if r is not None:
            pe[i], pc[i], vs[i] = trk.step(*r)
    out["pitch_estimate"], out["pitch_confidence"], out["voicing_strength"] = pe, pc, vs
    out["harmonic_ratio"], out["inharmonicity_ratio"] = vs * 10.0, 1.0 - vs
    out["tonal_centroid"] = np.where(pe > 0, pe, 0.0)
    out["short_time_energy"] = ste
    out["energy_variance"] = float(np.var(ste, ddof=1)) if len(ste) >= 2 else 0.0
    ent = np.where(ste > 0, -ste * np.log(ste + 1e-10), 0.0)
    lo = np.zeros(len(ste))
    hi = np.zeros(len(ste))
    m = min(len(ste), F)
    lo[:m], hi[:m] = d["low_ratio"][:m], d["high_ratio"][:m]
    out["energy_entropy"], out["low_energy_ratio"], out["high_energy_ratio"] = ent, lo, hi
    return out


def spectral_contrast(mag, sample_rate, num_bands=6):
    """SpectralContrast(sample_rate, num_bands).Compute per magnitude row (spectral_contrast.go:26-185)."""
    mag = _f64(mag)
    F, K = mag.shape
    out = np.zeros((F, num_bands))
    lib().or_spectral_contrast(_p(mag), F, K, sample_rate, num_bands, _p(out))
    return out


def music_features_reference(pcm, sample_rate, fc):
    """MusicFeatureExtractor.ExtractFeatures (fingerprint/extractors/music.go:178-583), fp64, composed
    from the oracle's pieces.  fc: dict(sample_rate, window_size, hop_size, stft_window_size,
    stft_hop_size).  Returns (features, panic): panic is Go's runtime error text where the reference
    panics (music.go:348-352 slice bounds when a chroma frame starts past the signal, (F-1) hop > n;
    music.go:383 integer divide by zero with no energy frame; music.go:403 index out of range
    for >= 2 RMS frames of 1024 / 512, i.e. >= 1536 samples), features then holding what was computed
    before the panic."""
    pcm = _f64(pcm)
    n = len(pcm)
    csr = fc["sample_rate"]
    W, H = fc["stft_window_size"], fc["stft_hop_size"]
    mag = stft_mag(pcm, W, H, nthreads=8)
    F, K = mag.shape
    y = preemphasis(dc_removal(pcm, 0.995), 0.95)                       # preprocessAudio (:245-259)
    out = {}
    d = spectral_descriptors(mag, csr)                                  # extractSpectralFeatures (:261-302)
    for k in ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope"]:
        out["spectral_" + k] = d[k]
    flux = np.zeros(F)
    flux[1:] = d["flux"]
    out["spectral_flux"] = flux
    out["zero_crossing_rate"] = np.zeros(F)
    out["spectral_contrast"] = spectral_contrast(mag, csr, 6)
    out["mfcc"] = mfcc_frames(mag * mag, csr, n_coef=13, n_mels=26)     # Compute(|X|^2) -> |X|^4 (F5)
    if fc["hop_size"] <= 0:                                             # stft.go:54-56 via :358-361
        raise ValueError("chroma feature extraction failed: chroma computation failed at frame 0: "
                         "hop size must be positive")
    if (F - 1) * fc["hop_size"] > n:                                    # pcm[start:end] with start > n (:348-352)
        f = n // fc["hop_size"] + 1
        return out, f"runtime error: slice bounds out of range [{f * fc['hop_size']}:{n}]"
    out["chroma"] = chroma_music(pcm, F, fc["hop_size"], csr)           # (:327-376)
    rms = short_time_energy(y, fc["window_size"], fc["hop_size"])       # extractTemporalFeatures (:378-458)
    out["rms_energy"] = rms
    Fe = len(rms)
    if Fe == 0:
        return out, "runtime error: integer divide by zero"
    fse = n // Fe
    out["envelope_shape"] = short_time_energy(y, fse, fc["hop_size"])
    a = np.abs(y)
    out["peak_amplitude"] = float(a.max())
    out["average_amplitude"] = float(np.cumsum(a)[-1] / n)             # Go's sequential sum
    L = (n - 1024) // 512 + 1 if n >= 1024 else 0
    if L >= 2:
        return out, f"runtime error: index out of range [{int(10.0 * (L - 1))}] with length {L}"
    out["dynamic_range"] = 0.0
    if n <= 512:
        raise ValueError("temporal feature extraction failed: signal too short for given window size and hop size")
    out["onset_density"] = 0.0
    out["attack_time"] = np.zeros(0)
    crest = np.zeros(Fe)
    for i in range(Fe):
        pk = a[i * fse: min(i * fse + fse, n)].max()
        if rms[i] > 0:
            crest[i] = pk / rms[i]
    out["crest_factor"] = crest
    out["silence_ratio"] = 0.0                                          # RMS < -40 never holds
    out["activity_level"] = np.ones(Fe)
    out["short_time_energy"] = rms                                      # extractEnergyFeatures (:460-525)
    out["energy_variance"] = float(np.var(rms, ddof=1)) if Fe >= 2 else 0.0
    out["energy_entropy"] = np.where(rms > 0, -rms * np.log2(np.where(rms > 0, rms, 1.0)), 0.0)
    pos = rms[rms > 0]
    out["loudness_range"] = float(20 * np.log10(rms.max() / pos.min())) if len(pos) else 0.0
    e = mag * mag
    lo, hi = np.zeros(F), np.zeros(F)
    for t in range(F):
        tot = np.cumsum(e[t])[-1]
        l_ = np.cumsum(e[t, : K // 4])[-1] if K // 4 else 0.0
        h_ = np.cumsum(e[t, 3 * K // 4 + 1:])[-1] if K - (3 * K // 4 + 1) > 0 else 0.0
        if tot > 0:
            lo[t], hi[t] = l_ / tot, h_ / tot
    out["low_energy_ratio"], out["high_energy_ratio"] = lo, hi
    pe, pc, vs = np.zeros(F), np.zeros(F), np.zeros(F)                  # extractHarmonicFeatures (:528-583, F7)
    if n // F == 1024:
        pe[0], pc[0], vs[0] = YinTrack().step(*yin_raw(y[:1024], csr)[:2])
    out["pitch_estimate"], out["pitch_confidence"], out["voicing_strength"] = pe, pc, vs
    out["harmonic_ratio"], out["inharmonicity_ratio"] = np.zeros(F), np.zeros(F)
    out["tonal_centroid"] = d["centroid"] * vs
    return out, None


def align_features_reference(qe, re_, qc, rc, q_pcm_len, r_pcm_len, sample_rate, feature_sample_rate, hop,
                             max_lag_seconds):
    """AlignmentExtractor.ExtractAlignmentFeatures (extractors/alignment.go:139-476), corr_energy + dtw_chroma."""
    out = {}
    max_lag_samples = int(max_lag_seconds * feature_sample_rate)
    cands = []
    if qe is not None and re_ is not None and len(qe) and len(re_):
        mlf = min(max_lag_samples // hop if max_lag_samples >= 0 else -((-max_lag_samples) // hop),
                  min(len(qe), len(re_)) - 1)
        corr, met = ncc(qe, re_, mlf)
        s = align_xcorr_metrics(met, hop, sample_rate, mlf)
        out["correlations"], out["peak_lag"] = corr, met["peak_lag"]
        cands.append((1, 1.0, s, None))
    if qc is not None and rc is not None and len(qc) and len(rc):
        r = dtw(qc, rc)
        s = align_dtw_metrics(r, len(qc), len(rc), sample_rate)
        out["dtw_distance"], out["dtw_path_query"], out["dtw_path_reference"] = r["distance"], r["path_q"], r["path_r"]
        cands.append((2, 0.7, s, r))
    best, bs = None, 0.0
    for c in cands:
        sc = c[1] * (0.4 * c[2]["confidence"] + 0.4 * c[2]["similarity"] + 0.2 * c[2]["quality"])
        if sc > bs:
            best, bs = c, sc
    out["method"] = 0 if best is None else best[0]
    if best is not None:
        out["temporal_offset"] = best[2]["offset_seconds"]
        out["offset_confidence"] = best[2]["confidence"]
        out["alignment_similarity"] = best[2]["similarity"]
        out["alignment_quality"] = best[2]["quality"]
    return out


FORMANT_KEYS = ("status", "n_formants", "frequency", "bandwidth", "amplitude", "confidence",
                "vocal_tract_length", "quality", "gain", "residual_energy", "stable")


def _formant_recs(recs):
    recs = np.atleast_2d(recs)
    return {"status": recs[:, 0].astype(np.int32), "n_formants": recs[:, 1].astype(np.int32),
            "frequency": recs[:, 2:6], "bandwidth": recs[:, 6:10], "amplitude": recs[:, 10:14],
            "confidence": recs[:, 14:18], "vocal_tract_length": recs[:, 18], "quality": recs[:, 19],
            "gain": recs[:, 20], "residual_energy": recs[:, 21], "stable": recs[:, 22].astype(np.int32)}


def formant_frames(pcm, sample_rate, frame_size=0, hop_size=0, want_lpc=False):
    """FormantAnalyzer.AnalyzeMultipleFrames (format.go:427-449): one record per attempted frame."""
    pcm = _f64(pcm)
    W = 2048 if sample_rate >= 16000 else 1024
    p = 12 + sample_rate // 1000
    fs = frame_size if frame_size > 0 else W
    hp = hop_size if hop_size > 0 else fs // 2
    F = (len(pcm) - fs - 1) // hp + 1 if len(pcm) > fs else 0
    recs = np.zeros((max(F, 1), 24))
    co = np.zeros((max(F, 1), p + 1))
    rf = np.zeros((max(F, 1), p))
    lib().or_formant_frames(_p(pcm), len(pcm), sample_rate, frame_size, hop_size, _p(recs), _p(co), _p(rf))
    out = _formant_recs(recs[:F])
    if want_lpc:
        out["lpc_coeffs"], out["reflection"] = co[:F], rf[:F]
    return out


def formant_frame(sig, sample_rate):
    """FormantAnalyzer.AnalyzeFormants on one signal (format.go:85-124)."""
    sig = _f64(sig)
    p = 12 + sample_rate // 1000
    rec = np.zeros(24)
    co = np.zeros(p + 1)
    rf = np.zeros(p)
    lib().or_formant_frame(_p(sig), len(sig), sample_rate, _p(rec), _p(co), _p(rf))
    out = _formant_recs(rec)
    out["lpc_coeffs"], out["reflection"] = co, rf
    return out


def autocorr_fft(x, max_lag):
    """AutoCorrelation(maxLag).Compute correlations on the FFT path (lags -L..L)."""
    x = _f64(x)
    L = max(0, min(max_lag, len(x) - 1))
    out = np.zeros(2 * L + 1)
    lib().or_autocorr_fft(_p(x), len(x), max_lag, _p(out))
    return out


# ---- FingerprintComparator (compare_oracle.c) ----------------------------------------
# The structs are the C ABI's layouts (sonar._abi.FpFeatures / CompareCfg / Similarity /
# Match); the oracle reads the full feature arrays on every call, like the Go code.

def fp_compare(fa, fb, cfg):
    """or_fp_compare: Compare(fa, fb) -> Similarity struct (raises on a Go panic case)."""
    from sonar._abi import Similarity
    out = Similarity()
    rc = lib().or_fp_compare(C.addressof(fa), C.addressof(fb), C.addressof(cfg), C.addressof(out))
    if rc:
        raise ValueError(f"oracle compare panics in Go (code {rc})")
    return out


def find_best_matches(fq, fcands, cfg):
    """or_find_best_matches over an array of FpFeatures -> list of Match structs."""
    from sonar._abi import Match
    n = len(fcands)
    out = (Match * max(1, n))()
    k = C.c_int64()
    rc = lib().or_find_best_matches(C.addressof(fq), C.addressof(fcands) if n else None, n,
                                    C.addressof(cfg), C.addressof(out), C.byref(k))
    if rc:
        raise ValueError(f"oracle FindBestMatches panics in Go (code {rc})")
    return [out[i] for i in range(k.value)]


# ---- ContentDetector.DetectFromAudio (content_oracle.c) ---------------------------------
ACOUSTIC_KEYS = ["zero_crossing_rate", "spectral_centroid", "energy_variance", "silence_ratio", "harmonic_ratio",
                 "low_freq_energy", "high_freq_energy", "dynamic_range", "temporal_stability",
                 "classification_confidence"]
CONTENT_NAMES = ["music", "news", "sports", "talk", "mixed", "unknown"]


def detect_from_audio(pcm, sample_rate, thr=2.0):
    x = np.ascontiguousarray(pcm, dtype=np.float64)
    out = np.zeros(10)
    ct = C.c_int()
    rc = lib().or_detect_from_audio(_p(x) if len(x) else None, len(x), sample_rate, thr, _p(out), C.byref(ct))
    if rc:
        raise ValueError("sample rate < 10: the Go loop never ends")
    return CONTENT_NAMES[ct.value], dict(zip(ACOUSTIC_KEYS, out.tolist()))


# ---------------------------------------------------------------------------
# AlignmentAnalyzer.AnalyzeAlignmentConsistency / AlignmentExtractor.TruncateToAlignmentPCM
# (SURVEY.md 8(f) rank 4), composed from the primitives above
# ---------------------------------------------------------------------------

ALIGN_DTW, ALIGN_XCORR, ALIGN_PHASE, ALIGN_HYBRID = 0, 1, 2, 3       # AlignmentMethod (stats/alignment.go:12-17)


def add_noise(features, level=0.01):
    """addNoise (stats/alignment.go:737-749): v + (sin(float64(i*j+i+j)) * level) * v."""
    f = _f64(features)
    i = np.arange(f.shape[0], dtype=np.int64)[:, None]
    j = np.arange(f.shape[1], dtype=np.int64)[None, :]
    return f + (np.sin((i * j + i + j).astype(np.float64)) * level) * f


def align_offset_reference(query, reference, sample_rate, method, max_lag, hop):
    """AlignFeatures (stats/alignment.go:84-106) -> result.Offset, for DTW / xcorr / hybrid."""
    q, r = _f64(query), _f64(reference)
    conf = None
    if method in (ALIGN_XCORR, ALIGN_HYBRID):                         # alignWithCrossCorrelation :151-181
        _, met = ncc(q[:, 0], r[:, 0], max_lag)                       # flatten2DFeatures :363-378
        m = align_xcorr_metrics(met, hop, sample_rate, max_lag)
        off, conf = int(m["offset"]), m["confidence"]
        if method == ALIGN_XCORR or conf > 0.7:                       # alignWithHybrid :315-317
            return off
    res = dtw(q, r)                                                   # alignWithDTW :129-148
    return int(align_dtw_metrics(res, len(q), len(r), sample_rate)["offset"])


class GoPanic(RuntimeError):
    """The Go reference panics on this input (the message is Go's runtime error text)."""


def _go_div(a, b):
    """Go's integer division: truncates toward zero; b == 0 panics."""
    if b == 0:
        raise GoPanic("runtime error: integer divide by zero")
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def analyzer_align_reference(query, reference, sample_rate, method, max_lag, hop, dtw_threads=8):
    """AlignmentAnalyzer.AlignFeatures (stats/alignment.go:84-106) -> every AlignmentResult field.

    alignWithCrossCorrelation (:151-181) on the first component (flatten2DFeatures :363-378), the
    DTW (alignWithDTW :129-148) on the full rows, and alignWithHybrid (:308-337) with Go's result
    aliasing (F8): alignWithCrossCorrelation and alignWithDTW both write into and return the SAME
    *AlignmentResult, so after the DTW the "correlation" confidence and similarity being blended
    are the DTW's own: Confidence = 0.6 c + 0.4 c, Similarity = 0.7 s + 0.3 s (float64, in that
    order); Offset / AlignmentQuality / Stability are the DTW's, NoiseLevel stays the
    correlation's (alignWithDTW never writes it).  The DTW is dtw_full (the same cells and
    operation order as dtw(), stripe wavefront over `dtw_threads` threads)."""
    q, r = _f64(query), _f64(reference)
    if q.ndim == 1:
        q = q[:, None]
    if r.ndim == 1:
        r = r[:, None]
    if len(q) == 0 or len(r) == 0:
        raise ValueError("empty feature sequences provided")
    if method not in (ALIGN_DTW, ALIGN_XCORR, ALIGN_HYBRID):
        raise ValueError(f"unsupported alignment method: {method}")
    res = {"method": method, "query_length": len(q), "reference_length": len(r), "sample_rate": sample_rate,
           "offset": 0, "offset_seconds": 0.0, "confidence": 0.0, "similarity": 0.0, "alignment_quality": 0.0,
           "noise_level": 0.0, "stability": 0.0, "dtw_ran": 0}
    if method in (ALIGN_XCORR, ALIGN_HYBRID):
        corr, met = ncc(np.ascontiguousarray(q[:, 0]), np.ascontiguousarray(r[:, 0]), max_lag)
        m = align_xcorr_metrics(met, hop, sample_rate, max_lag)
        res.update(offset=int(m["offset"]), offset_seconds=m["offset_seconds"], similarity=m["similarity"],
                   confidence=m["confidence"], alignment_quality=m["quality"], noise_level=m["noise_level"])
        res["correlations"] = corr
        res.update(met)
        if method == ALIGN_XCORR or res["confidence"] > 0.7:
            return res
    d = dtw_full(q, r, nthreads=dtw_threads)
    s = align_dtw_metrics(d, len(q), len(r), sample_rate)
    res.update(offset=int(s["offset"]), offset_seconds=s["offset_seconds"], alignment_quality=s["quality"],
               stability=s["stability"], dtw_ran=1, dtw_distance=d["distance"], dtw_path_query=d["path_q"],
               dtw_path_reference=d["path_r"], dtw_path_cost=d["path_cost"])
    if method == ALIGN_DTW:
        res.update(confidence=s["confidence"], similarity=s["similarity"])
    else:
        c, sm = s["confidence"], s["similarity"]
        res.update(confidence=0.6 * c + 0.4 * c, similarity=0.7 * sm + 0.3 * sm)
    return res


def analyzer_energy_features(pcm, window, hop):
    """AlignmentAnalyzer.extractEnergyFeatures (stats/alignment.go:341-361): numFrames = (len - W)
    / H + 1 with Go's truncating division, frame i = pcm[i H : min(i H + W, len)], RMS over its
    own length."""
    x = _f64(pcm)
    nf = _go_div(len(x) - window, hop) + 1
    if nf < 0:
        raise GoPanic("runtime error: makeslice: len out of range")
    if nf == 0:
        return np.zeros(0)
    if len(x) >= window:
        return short_time_energy(x, window, hop)[:nf]
    assert nf == 1 and len(x) > 0
    return short_time_energy(x, len(x), hop)          # one frame over the whole (short) signal


def align_audio_reference(q_pcm, r_pcm, sample_rate, method, max_lag, hop, window):
    """AlignmentAnalyzer.AlignAudio (stats/alignment.go:108-126)."""
    qe, re_ = analyzer_energy_features(q_pcm, window, hop), analyzer_energy_features(r_pcm, window, hop)
    return analyzer_align_reference(qe[:, None], re_[:, None], sample_rate, method, max_lag, hop)


def align_audio_files_reference(q_pcm, r_pcm, sample_rate, feature_sample_rate, hop, window, max_lag_seconds):
    """AlignmentExtractor.AlignAudioFiles (extractors/alignment.go:489-553) with the extractor of
    NewAlignmentExtractorWithMaxLag (:99-136): ShortTimeEnergy of both streams (energy.go:25-50),
    then the Hybrid AlignFeatures at maxLagFrames = int(maxLagSeconds * SampleRate) / HopSize."""
    mlf = _go_div(int(max_lag_seconds * feature_sample_rate), hop)
    qe, re_ = short_time_energy(q_pcm, window, hop), short_time_energy(r_pcm, window, hop)
    try:
        res = analyzer_align_reference(qe[:, None], re_[:, None], sample_rate, ALIGN_HYBRID, mlf, hop)
    except ValueError as e:
        raise ValueError(f"alignment failed: {e}") from None
    res.update(temporal_offset=res["offset_seconds"], offset_confidence=res["confidence"],
               alignment_similarity=res["similarity"], feature_similarity_energy=res["similarity"],
               query_length_seconds=len(q_pcm) / sample_rate, reference_length_seconds=len(r_pcm) / sample_rate,
               time_stretch=0.0, max_lag_frames=mlf)
    return res


def alignment_consistency_reference(query, reference, sample_rate, method, max_lag, hop, num_trials=5):
    """AnalyzeAlignmentConsistency (stats/alignment.go:709-735) + calculateOffsetStats (:751-800).
    Every trial aligns the same deterministic perturbation, run here trial by trial as Go does."""
    if num_trials < 2:
        num_trials = 5
    q, r = _f64(query), _f64(reference)
    if len(q) == 0 or len(r) == 0 or method not in (ALIGN_DTW, ALIGN_XCORR, ALIGN_HYBRID):
        raise ValueError("no successful alignments")
    offs = [float(align_offset_reference(add_noise(q, 0.01), r, sample_rate, method, max_lag, hop))
            for _ in range(num_trials)]
    s = 0.0
    for o in offs:
        s += o
    mean = s / len(offs)
    ssd = 0.0
    for o in offs:
        ssd += (o - mean) * (o - mean)
    sd = float(np.sqrt(ssd / len(offs)))
    srt = sorted(offs)
    n = len(srt)
    median = (srt[n // 2 - 1] + srt[n // 2]) / 2 if n % 2 == 0 else srt[n // 2]
    cons = 1.0 / (1.0 + sd / abs(mean)) if mean != 0 else 1.0
    return {"mean_offset": mean, "stddev_offset": sd, "median_offset": median, "offset_range": srt[-1] - srt[0],
            "consistency": cons, "offset": int(offs[0]), "trials": num_trials}


def truncate_to_alignment_reference(n1, n2, sample_rate, offset_seconds):
    """TruncateToAlignmentPCM (extractors/alignment.go:223-297) -> (start1, start2, length)."""
    import math
    sr = float(sample_rate)
    def off_samples():
        v = abs(offset_seconds) * sr
        return int(math.floor(v + 0.5)) if v >= 0 else 0             # math.Round (half away from zero)
    s1 = s2 = 0
    if offset_seconds > 0:
        s2 = off_samples()
        if s2 >= n2:
            raise ValueError(f"offset too large: need to skip {s2} samples but pcm2 only has {n2}")
        common = min(n1, n2 - s2)
    elif offset_seconds < 0:
        s1 = off_samples()
        if s1 >= n1:
            raise ValueError(f"offset too large: need to skip {s1} samples but pcm1 only has {n1}")
        common = min(n1 - s1, n2)
    else:
        common = min(n1, n2)
    if common <= 0:
        raise ValueError("no overlapping audio after alignment")
    pad = int(0.5 * sr)
    if common > 2 * pad:
        s1, s2, common = s1 + pad, s2 + pad, common - 2 * pad
    return s1, s2, common


def bytes_to_float64(data):
    """Decoder.bytesToFloat64 (transcode/decoder.go:850-871): trim to a multiple of 8 bytes, then
    binary.LittleEndian.Uint64 + math.Float64frombits per sample; None when no sample remains
    (processFFmpegOutput then fails "no audio samples decoded", decoder.go:785-787)."""
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    b = b[: len(b) - len(b) % 8]
    if len(b) == 0:
        return None
    # little-endian assembly of each 8-byte group, written out rather than trusting the host order
    u = np.zeros(len(b) // 8, dtype=np.uint64)
    for k in range(8):
        u |= b[k::8].astype(np.uint64) << np.uint64(8 * k)
    return u.view(np.float64)
