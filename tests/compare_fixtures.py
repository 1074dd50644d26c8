"""Seeded synthetic fingerprints for the FingerprintComparator tests (CPU and GPU).

Covers the presence patterns Compare branches on (comparison.go:266-341, 892-1037): nil
Features / nil sub-structs, empty vs non-empty slices, single-frame sequences (gonum
Variance -> NaN), MFCC width mismatches (cosine of unequal lengths -> 0), zero scalars,
content types incl. distinct unknown strings, Metadata feature weights, duplicate IDs.
"""
import numpy as np

from sonar.compare import Features, Fingerprint

CTS = ["music", "news", "talk", "sports", "mixed", "unknown", "podcast"]


def random_fingerprint(rng, k, n_frames=None, full=False, equal_len=None):
    """One fingerprint; `full` forces every feature group; `equal_len` fixes the spectral
    sequence length (detailed metrics need equal lengths)."""
    F = int(n_frames if n_frames is not None else rng.integers(1, 400))
    ct = CTS[int(rng.integers(0, len(CTS)))]
    if not full and rng.random() < 0.05:
        return Fingerprint(id=f"fp{k}", content_type=ct, duration=float(rng.uniform(0, 60)), features=None)
    feat = Features()
    p = (lambda: True) if full else (lambda: rng.random() < 0.8)
    if p():
        C = 13 if full or rng.random() < 0.85 else int(rng.integers(0, 20))
        rows = 0 if (not full and rng.random() < 0.05) else F
        feat.mfcc = rng.normal(0, 3, (rows, C)) + rng.normal(0, 5, C)
    if p():
        rows = 0 if (not full and rng.random() < 0.05) else F
        feat.chroma = np.abs(rng.normal(0.1, 0.05, (rows, 12)))

    def seq(n=None, scale=1.0, off=0.0):
        n = F if n is None else n
        if not full and rng.random() < 0.1:
            n = int(rng.integers(0, 3))       # empty or 1-2 frames
        return np.abs(rng.normal(off, scale, n))

    if p():
        L = equal_len
        feat.spectral = {"centroid": seq(L, 500, 2000) if L is None else np.abs(rng.normal(2000, 500, L)),
                         "rolloff": seq(L, 800, 5000) if L is None else np.abs(rng.normal(5000, 800, L)),
                         "flux": seq(None, 0.5, 1.0)}
    if p():
        feat.temporal = {"dynamic_range": float(rng.choice([0.0, rng.uniform(5, 40)])),
                         "silence_ratio": float(rng.uniform(0, 0.4)),
                         "onset_density": float(rng.choice([0.0, rng.uniform(0.1, 5)])),
                         "rms_energy": seq(None, 0.1, 0.2)}
    if p():
        feat.speech = {"speech_rate": float(rng.choice([0.0, rng.uniform(1, 6)])),
                       "vocal_tract_length": float(rng.choice([0.0, rng.uniform(14, 19)])),
                       "voicing_probability": seq(None, 0.3, 0.5)}
    if p():
        feat.harmonic = {"harmonic_ratio": seq(None, 0.2, 0.5), "pitch_estimate": seq(None, 50, 180)}
    w = None
    if not full and rng.random() < 0.15:
        w = {k: float(rng.uniform(0, 1)) for k in ["mfcc", "spectral", "chroma", "temporal"]}
    fid = f"fp{k}" if rng.random() > 0.05 else "dup"
    return Fingerprint(id=fid, content_type=ct, duration=float(rng.uniform(0, 600)), features=feat,
                       feature_weights=w)


def gallery(seed, n, **kw):
    rng = np.random.default_rng(seed)
    return [random_fingerprint(rng, k, **kw) for k in range(n)]
