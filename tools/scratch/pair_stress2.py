"""Failure forensics for the headline kernel: where do bad frames sit and what do they hold."""
import sys, numpy as np
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd")]
import sonar
from sonar import synth
ctx = sonar.Context(0)
rng = np.random.default_rng(int(sys.argv[1]))
base = synth.c2_hour(seconds=12.0)
shown = 0
for it in range(int(sys.argv[2])):
    n = int(rng.integers(1100, len(base)))
    H = int(rng.choice([256, 100, 512]))
    x = np.ascontiguousarray(base[:n])
    cfg = ctx.config(window_size=1024, hop_size=H, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    a = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    cfg.flags = sonar.FP_MFCC | sonar.FP_GENERIC
    b = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    e = np.max(np.abs(a - b), axis=1) / np.linalg.norm(b, axis=1)
    bad = np.nonzero(~(e < 1e-4))[0]
    if len(bad) and shown < 8:
        shown += 1
        F = len(a); NP = (F + 1) // 2; ppw = max(1, -(-NP // (256 * 12)))
        print(f"F={F} H={H} ppw={ppw} bad={bad[:10].tolist()}", flush=True)
        for f in bad[:3]:
            coef_bad = np.nonzero(np.abs(a[f] - b[f]) > 1e-4 * np.linalg.norm(b[f]))[0].tolist()
            # is the bad row a copy of another reference row?
            match = np.nonzero(np.max(np.abs(b - a[f]), axis=1) < 1e-3)[0].tolist()
            print(f"  frame {f} pair {f//2} wave {f//2//ppw} coefs {coef_bad} matches_ref_rows {match[:5]}")
            print("   got", np.round(a[f], 3).tolist())
            print("   ref", np.round(b[f], 3).tolist())
