import sys, os, numpy as np
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd"), os.path.join(_R, "oracle")]
import sonar, oracle as O
from sonar import synth
ctx = sonar.Context(0)
for secs in (7.3, 20.0, 21.0):
    x = synth.c2_hour(seconds=secs)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    a = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    a2 = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    cfg.flags = sonar.FP_MFCC | sonar.FP_GENERIC
    b = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    e = np.max(np.abs(a - b), axis=1) / np.linalg.norm(b, axis=1)
    bad = np.nonzero(e > 1e-4)[0]
    print(secs, len(a), "bad frames", len(bad), bad[:20], "max", e.max(), "repeat-equal", np.array_equal(a, a2))
    if len(bad):
        f = bad[0]; print(" frame", f, a[f][:6], b[f][:6])
