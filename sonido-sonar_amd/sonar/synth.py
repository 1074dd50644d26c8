"""Seeded synthetic inputs of the BASELINE configs.

C1  10 s linear sweep 100 Hz -> 10 kHz, 44.1 kHz            (CPU baseline config)
C2  1 h: the C1 sweep repeated every 10 s + 0.05 N(0,1)      (headline STFT->MFCC)
C3  two 5-min streams, query = reference delayed by 12.34 s  (alignment)
C4  30 min 16 kHz speech-like noise                          (speech config)
C5  1000 x 60 s stream pairs with random lags                (8-GPU config)
All generators are deterministic (NumPy PCG64 seeds as in the survey).
"""
from __future__ import annotations

import numpy as np

SR = 44100


def sweep(seconds=10.0, sr=SR, f0=100.0, f1=10000.0, amp=0.5):
    t = np.arange(int(round(seconds * sr))) / sr
    return amp * np.sin(2 * np.pi * (f0 * t + (f1 - f0) * t ** 2 / (2 * seconds)))


def c2_hour(seconds=3600.0, sr=SR, dtype=np.float32, seed=1234):
    """C1 sweep tiled to `seconds` plus 0.05 N(0,1); built in 10 s blocks to bound memory."""
    n = int(round(seconds * sr))
    base = sweep(10.0, sr)
    out = np.empty(n, dtype=dtype)
    rng = np.random.Generator(np.random.PCG64(seed))
    block = len(base)
    for s in range(0, n, block):
        e = min(n, s + block)
        out[s:e] = base[: e - s] + 0.05 * rng.standard_normal(e - s)
    return out


def _one_pole_noise(n, a, rng):
    x = rng.standard_normal(n)
    # y[n] = a y[n-1] + x[n] via scipy-free recursion in chunks (lfilter equivalent)
    from scipy.signal import lfilter
    return lfilter([1.0], [1.0, -a], x)


def _envelope(n, sr, rng, smooth_s=0.5):
    m = int(np.ceil(n / (smooth_s * sr))) + 2
    pts = rng.uniform(0.2, 1.0, m)
    xp = np.arange(m) * smooth_s * sr
    return np.interp(np.arange(n), xp, pts)


def c3_pair(seconds=300.0, lag_s=12.34, sr=SR, seed=42, env_seed=7):
    """(query, reference): query = base[lag:lag+N], reference = base[0:N]."""
    n = int(round(seconds * sr))
    lag = int(round(lag_s * sr))
    total = n + lag
    rng = np.random.Generator(np.random.PCG64(seed))
    base = _one_pole_noise(total, 0.95, rng)
    base *= _envelope(total, sr, np.random.Generator(np.random.PCG64(env_seed)))
    base /= np.max(np.abs(base))
    return base[lag:lag + n].copy(), base[:n].copy()


def c4_speech(seconds=1800.0, sr=16000, seed=99):
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(round(seconds * sr))
    x = rng.standard_normal(n)
    r, f = 0.95, 500.0
    from scipy.signal import lfilter
    w = 2 * np.pi * f / sr
    y = lfilter([1.0], [1.0, -2 * r * np.cos(w), r * r], x)
    t = np.arange(n) / sr
    syl = 0.5 * (1 + np.sin(2 * np.pi * 4.0 * t))
    gate = (rng.uniform(size=int(np.ceil(seconds / 0.25))) > 0.2).astype(float)
    syl *= np.repeat(gate, int(0.25 * sr))[:n]
    y = y * syl
    return y / np.max(np.abs(y))


def c5_pair(k, seconds=60.0, sr=SR):
    lag = np.random.Generator(np.random.PCG64(2024 + k)).uniform(0, 20.0)
    return c3_pair(seconds, lag, sr, seed=1000 + k, env_seed=5000 + k) + (lag,)


def voiced(seconds=4.0, sr=16000, f0=140.0, vibrato=12.0, seed=5, harmonics=12, noise=3e-4):
    """Voiced speech-like test signal for the voice-quality path: `harmonics` partials (1/h) of a
    glottal rate f0 + vibrato (3 Hz), 5 Hz amplitude tremor, Gaussian noise (seeded).  The YIN of
    DetectPitch runs on twice pre-emphasised samples (extractor + detector), which buries a
    low fundamental under much noise -- keep `noise` small."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(round(seconds * sr))
    t = np.arange(n) / sr
    f = f0 + vibrato * np.sin(2 * np.pi * 3.0 * t)
    ph = 2 * np.pi * np.cumsum(f) / sr
    x = sum(np.sin(h * ph) / h for h in range(1, harmonics + 1))
    return 0.3 * x * (1.0 + 0.2 * np.sin(2 * np.pi * 5.0 * t)) + noise * rng.standard_normal(n)
