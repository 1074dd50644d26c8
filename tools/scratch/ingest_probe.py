"""Host-thread sweep of sonar_ingest_f64le (both modes) on 1 h of f64le PCM; one JSON line per setting."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sonido-sonar_amd"))
import sonar  # noqa: E402

n = 158_760_000
x = np.random.default_rng(0).standard_normal(n)
ctx = sonar.Context(0)
buf = torch.empty(n, dtype=torch.float32, device="cuda:0")
for mode in (sonar.INGEST_HOST_CONVERT, sonar.INGEST_DEVICE_CONVERT):
    for T in (4, 8, 16, 24, 32, 48):
        ctx.ingest_f64le(x[: 1 << 22], buf.data_ptr(), sonar.F32, mode, T)
        best = 1e9
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.ingest_f64le(x, buf.data_ptr(), sonar.F32, mode, T)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"mode": mode, "threads": T, "ms": best * 1e3, "f64le_gbs": 8 * n / best / 1e9}), flush=True)
