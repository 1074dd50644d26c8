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
        L.or_filterbank.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, _d]
        L.or_mfcc_frames.argtypes = [_d, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                     C.c_double, C.c_int, C.c_double, C.c_int, C.c_int, _d]
        L.or_spectral_descriptors.argtypes = [_d, C.c_int64, C.c_int, C.c_int] + [_d] * 9
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
        L.or_chroma_music.argtypes = [_d, C.c_int64, C.c_int64, C.c_int, C.c_int, _d]
        L.or_chroma_frames.argtypes = [_d, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _d]
        L.or_ncc.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int, _d, _d]
        L.or_dtw.argtypes = [_d, C.c_int64, _d, C.c_int64, C.c_int, C.c_int, _d, _i32, _i32, _d, _i64, _d]
        L.or_align_dtw_metrics.argtypes = [_i32, _i32, _d, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_int, _d]
        L.or_align_xcorr_metrics.argtypes = [_d, C.c_int, C.c_int, C.c_int, _d]
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
