#!/usr/bin/env python3
"""Median band-kernel / walk / decode ms of sonar_dtw at n x n (12-dim), for library A/Bs (SONAR_LIB)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
import sonar
n = int(sys.argv[1]) if len(sys.argv) > 1 else 51676
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = sonar.Context(0)
rng = np.random.default_rng(7)
q = rng.random((n, 12)); r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
ctx.dtw(q, r)
t = []
for _ in range(reps):
    ctx.dtw(q, r); t.append(ctx.dtw_last_timing())
t = np.array(t)
print(json.dumps({"lib": os.environ.get("SONAR_LIB", "default"), "n": n, "band_ms": float(np.median(t[:, 0])),
                  "band_min": float(t[:, 0].min()), "walk_ms": float(np.median(t[:, 1])), "dec_ms": float(np.median(t[:, 2]))}))
