#!/usr/bin/env python3
"""Per-band timing of the 128-row band kernel (dtw_band2_kernel, SONAR_DTW_BAND2=1) at n x n:
start / first-ready / end of every block's sweep and its wait ticks by cause (distances, top edge,
code wave), plus the code wave's and distance wave 0's waits (SONAR_DTW_TRACE)."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
os.environ["SONAR_DTW_BAND2"] = os.environ.get("SONAR_DTW_BAND2", "1")
tp = "/tmp/dtw2_trace.bin"
os.environ["SONAR_DTW_TRACE"] = tp
import sonar
n = int(sys.argv[1]) if len(sys.argv) > 1 else 51676
ctx = sonar.Context(0)
rng = np.random.default_rng(7)
q = rng.random((n, 12)); r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
ctx.dtw(q, r)
res = ctx.dtw(q, r)
ms = ctx.dtw_last_timing()
t = np.fromfile(tp, np.uint64).reshape(-1, 8).astype(np.float64)
band2 = os.environ["SONAR_DTW_BAND2"] == "1"
nb = (n + 127) // 128 if band2 else (n + 63) // 64
t = t[:nb]
t0 = t[:, 0].min()
st, fi, en = (t[:, 0] - t0) / 100, (t[:, 1] - t0) / 100, (t[:, 2] - t0) / 100   # us
S = n + (127 if band2 else 63)
dur = en - fi
out = {"band2": band2, "n": n, "kernel_ms": ms, "blocks": int(nb),
       "span_us": float(en.max()), "first_ready_us_of_last": float(fi[-1]),
       "ns_per_step_band0": float((en[0] - fi[0]) * 1000 / S),
       "ns_per_step_median": float(np.median(dur) * 1000 / S),
       "first_ready_interval_us_median": float(np.median(np.diff(fi))),
       "start_us_of_last": float(st[-1])}
if band2:
    w = t[:, 3:8] / 100
    out["sweep_wait_us_median"] = {"dist": float(np.median(w[:, 0])), "edge": float(np.median(w[:, 1])),
                                   "code": float(np.median(w[:, 2]))}
    out["code_wave_wait_us_median"] = float(np.median(w[:, 3]))
    out["dist0_wait_us_median"] = float(np.median(w[:, 4]))
    out["sweep_wait_us_band0"] = {"dist": float(w[0, 0]), "edge": float(w[0, 1]), "code": float(w[0, 2])}
print(json.dumps(out))
for b in (0, 1, 2, 100, 200, 300, nb - 1):
    if b < nb:
        print(f"  band {b}: start {st[b]:.1f} first {fi[b]:.1f} end {en[b]:.1f} us; ns/step {dur[b]*1000/S:.1f}"
              + (f"; waits dist {t[b,3]/100:.1f} edge {t[b,4]/100:.1f} code {t[b,5]/100:.1f} us; code-wave wait {t[b,6]/100:.1f}, dist0 wait {t[b,7]/100:.1f}" if band2 else ""))
