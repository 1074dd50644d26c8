#!/usr/bin/env python3
"""Isolated sweep step time: one 128-row band (band2) / one 64-row band (band1) against n reference
rows, and the full n x n band kernel, for the kernels selected by SONAR_DTW_BAND2."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
import sonar
n = int(sys.argv[1]) if len(sys.argv) > 1 else 51676
ctx = sonar.Context(0)
rng = np.random.default_rng(7)
q = rng.random((n, 12)); r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
out = {"band2": os.environ.get("SONAR_DTW_BAND2", "0")}
for rows in (64, 128, 256, 1024, 4096):
    ctx.dtw(q[:rows], r)
    t = []
    for _ in range(3):
        ctx.dtw(q[:rows], r); t.append(ctx.dtw_last_timing()[0])
    out[f"rows{rows}_band_ms"] = float(np.median(t))
    out[f"rows{rows}_ns_per_step"] = float(np.median(t)) * 1e6 / (n + rows - 1)
print(json.dumps(out))
