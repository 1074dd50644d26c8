"""DTW band-pipeline probe (diagnostics, not part of the product or the tests).

Runs sonar_dtw on a C3-size 12-dim input (or DTW_N) with SONAR_DTW_TRACE set, so the band
kernel writes per-band s_memrealtime stamps (100 MHz): start, first edge value seen, end, ticks
spent spinning.  Prints the sweep's wall span, the per-step time of each band (duration / steps),
the band start interval (the hand-off lag), and the per-kernel HIP-event times of the call.

Usage (GPU box): SONAR_DTW_TRACE=/tmp/dtw.bin python3 tools/dtw_probe.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sonido-sonar_amd"))
import sonar  # noqa: E402

n = int(os.environ.get("DTW_N", "51676"))
iters = int(os.environ.get("ITERS", "3"))
rng = np.random.default_rng(7)
q = rng.random((n, 12))
r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
ctx = sonar.Context(0)
ctx.dtw(q[:256], r[:256])
ctx.dtw(q, r)
walls, parts = [], []
for _ in range(iters):
    t0 = time.perf_counter()
    res = ctx.dtw(q, r)
    walls.append(time.perf_counter() - t0)
    parts.append(ctx.dtw_last_timing())
walls = np.array(walls) * 1e3
parts = np.array(parts)
print(f"n={n} wall ms min {walls.min():.2f} med {np.median(walls):.2f}  cells/s {n * n / walls.min() * 1e3:.3e}  "
      f"P={len(res['path_q'])}", flush=True)
print("kernel ms (band, walk, decode) median:", np.round(np.median(parts, axis=0), 3).tolist(), flush=True)

tp = os.environ.get("SONAR_DTW_TRACE")
if tp and os.path.exists(tp):
    t = np.fromfile(tp, dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    base = t[:, 0].min()
    raw3 = np.fromfile(tp, dtype=np.uint64).reshape(-1, 8)[:, 3]
    hw = (raw3 >> np.uint64(32)).astype(np.int64)
    xcc = ((raw3 >> np.uint64(24)) & np.uint64(0xFF)).astype(np.int64)
    sp_raw = (raw3 & np.uint64(0xFFFFFF)).astype(np.float64)
    st, fe, en, sp = (t[:, 0] - base) / 100.0, (t[:, 1] - base) / 100.0, (t[:, 2] - base) / 100.0, sp_raw / 100.0
    S = n + 63
    dur = en - st
    nb = len(t)
    print(f"bands {nb}: sweep span {en.max():.0f} us; last band starts at {st[-1]:.0f} us")
    print("start interval us: median %.2f  p90 %.2f  max %.2f" % tuple(np.percentile(np.diff(st), [50, 90, 100])))
    print("band duration us: min %.0f  median %.0f  max %.0f" % (dur.min(), np.median(dur), dur.max()))
    print("ns per step: band0 %.1f  median %.1f  max %.1f" % (dur[0] / S * 1e3, np.median(dur) / S * 1e3, dur.max() / S * 1e3))
    print("sweep-wave spin us: median %.0f  max %.0f" % (np.median(sp), sp.max()))
    clk = (t[:, 5] - t[:, 4]) / np.maximum(dur, 1e-9) / 1e3
    print("band-0 clock %.2f GHz, %.1f clk/step; median band clock %.2f GHz" % (clk[0], (t[0, 5] - t[0, 4]) / S, np.median(clk)))
    for k in (0, 1, 2, nb // 4, nb // 2, 3 * nb // 4, nb - 1):
        print(f"  band {k:4d}: start {st[k]:8.1f} first-edge {fe[k] - st[k]:7.1f} dur {dur[k]:8.1f} spin {sp[k]:8.1f}"
              f"  dist0 wait {t[k, 6] / 100.0:8.1f} code wait {t[k, 7] / 100.0:8.1f}")
    act = [(np.sum((st <= x) & (en > x))) for x in np.linspace(0, en.max(), 11)]
    print("active bands at 0,10..100% of the span:", act)
    # which sweeps shared a CU / a SIMD: per band, the fraction of its lifetime during which another
    # band's sweep ran on the same CU (same SIMD)
    cu = (xcc << 8) | ((hw >> 8) & 0xFF)
    simd = (hw >> 4) & 3
    print("distinct CUs seen:", len(np.unique(cu)), " sweep SIMD histogram:", np.bincount(simd, minlength=4).tolist())
    ov_cu, ov_simd = np.zeros(nb), np.zeros(nb)
    order = np.argsort(cu, kind="stable")
    for c in np.unique(cu):
        ks = np.nonzero(cu == c)[0]
        for k in ks:
            for m in ks:
                if m == k:
                    continue
                o = max(0.0, min(en[k], en[m]) - max(st[k], st[m]))
                ov_cu[k] += o
                if simd[m] == simd[k]:
                    ov_simd[k] += o
    fcu, fsimd = ov_cu / np.maximum(dur, 1e-9), ov_simd / np.maximum(dur, 1e-9)
    nsps = dur / S * 1e3
    print("co-resident sweep on the CU, fraction of band life: median %.2f; on the same SIMD: median %.2f mean %.2f"
          % (np.median(fcu), np.median(fsimd), fsimd.mean()))
    lo, hi = fsimd < 0.2, fsimd > 0.6
    if lo.any() and hi.any():
        print("ns/step, bands whose sweep shared its SIMD < 20%% of the time: median %.1f (n=%d); > 60%%: %.1f (n=%d)"
              % (np.median(nsps[lo]), lo.sum(), np.median(nsps[hi]), hi.sum()))
    lo, hi = fcu < 0.2, fcu > 0.6
    if lo.any() and hi.any():
        print("ns/step, bands alone on the CU > 80%% of the time: median %.1f (n=%d); shared > 60%%: %.1f (n=%d)"
              % (np.median(nsps[lo]), lo.sum(), np.median(nsps[hi]), hi.sum()))
