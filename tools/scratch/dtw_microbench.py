"""DTW microbenchmark: C3-size chroma DTW through sonar_dtw (host buffers)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sonido-sonar_amd"))
import sonar

n = int(os.environ.get("DTW_N", "51676"))
iters = int(os.environ.get("ITERS", "3"))
rng = np.random.default_rng(7)
q = rng.random((n, 12))
r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
ctx = sonar.Context(0)
ctx.dtw(q[:256], r[:256])
ctx.dtw(q, r)
ctx.enable_kernel_timing(True)
t0 = time.perf_counter()
for _ in range(iters):
    res = ctx.dtw(q, r)
dt = (time.perf_counter() - t0) / iters
ctx.enable_kernel_timing(False)
print(f"n={n} wall {dt*1e3:.2f} ms  kernels(event) {ctx.last_kernel_ms():.2f} ms  cells/s {n*n/dt:.3e}  P={len(res['path_q'])}",
      flush=True)

tp = os.environ.get("SONAR_DTW_TRACE")
if tp and os.path.exists(tp):
    t = np.fromfile(tp, dtype=np.uint64).reshape(-1, 4).astype(np.float64)
    t0 = t[:, 0].min()
    st, fe, en, sp = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0, t[:, 3]
    print("bands", len(t), "end max us", en.max(), "start us [0,1,2,100,400,807]:", st[[0, 1, 2, 100, 400, -1]])
    print("first-edge us:", fe[[1, 2, 100, 400, -1]], "dur us (end-start):", (en - st)[[0, 1, 100, 400, -1]])
    print("sweep wait us:", sp[[0, 1, 2, 100, 400, -1]] / 100.0, "mean", sp.mean() / 100.0)
    d = np.diff(st)
    print("start gaps us: median", np.median(d), "max", d.max())
