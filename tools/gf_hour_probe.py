"""GenerateFingerprint at hour scale: where the time of one
sonar_generate_fingerprint call on 1 h of C2 (host float64 PCM, ContentType "music") goes.

Each call is split into the C call (H2D, kernels, D2H, host epilogue, result build) and the
Python result conversion, with CLOCK_MONOTONIC stamps (time.monotonic_ns, the clock rocprofv3
stamps its records with), so tools/gf_timeline.py can place every kernel and copy of a
rocprofv3 --kernel-trace --memory-copy-trace run inside the call.
Usage: python tools/gf_hour_probe.py [seconds] [reps] > out.json"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
import numpy as np  # noqa: E402

import sonar  # noqa: E402
from sonar import shard  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3600.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
SR, W, H = 44100, 1024, 256
x = np.ascontiguousarray(shard.stream_pcm(0, int(secs * SR)).double().numpy())
ctx = sonar.Context(0)
L = ctx._L
out = {"seconds": secs, "frames": sonar.stft_frames(len(x), W, H), "calls": []}
for name, prec in (("f64", sonar.F64), ("f32", sonar.F32)):
    cfg = ctx.fingerprint_config(window_size=W, hop_size=H, feature_window_size=W, feature_hop_size=H,
                                 precision=prec)
    ctx.generate_fingerprint(x[: SR * 20], SR, "music", cfg)          # tables, buffers
    ctx.generate_fingerprint(x, SR, "music", cfg)                     # buffers at full size
    for r in range(reps):
        time.sleep(0.2)                                               # gaps separate the calls in a trace
        h = C.c_void_p()
        t0 = time.monotonic_ns()
        rc = L.sonar_generate_fingerprint(ctx._h, C.c_void_p(x.ctypes.data), len(x), SR,
                                          b"music", C.byref(cfg), C.byref(h))
        t1 = time.monotonic_ns()
        assert rc == 0, L.sonar_last_error(ctx._h)
        res = ctx._result(h)
        t2 = time.monotonic_ns()
        out["calls"].append({"precision": name, "rep": r, "t0_ns": t0, "t_c_ns": t1, "t_py_ns": t2,
                             "c_call_ms": (t1 - t0) / 1e6, "py_result_ms": (t2 - t1) / 1e6,
                             "total_ms": (t2 - t0) / 1e6,
                             "result_bytes": int(sum(np.asarray(v).nbytes for v in res.values()))})
        del res
        print(json.dumps(out["calls"][-1]), file=sys.stderr, flush=True)
ctx.close()
print(json.dumps(out))
