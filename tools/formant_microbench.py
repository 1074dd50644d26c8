"""Micro-benchmark of formant_kernel: sonar_formants on device-resident float64 PCM (30 min of the
C4 speech signal at 16 kHz by default: W 2048, hop 1024, order 28), one launch per call.  Prints ms
per call (wall clock over ITERS calls) and a checksum of the records (equal across builds =
bit-identical).  Usage: [SONAR_LIB=...] [SECONDS=1800] [ITERS=20] python3 tools/formant_microbench.py"""
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd"), ROOT]
import torch  # noqa: E402
import sonar  # noqa: E402
from sonar import _abi  # noqa: E402

sr = 16000
dev = torch.device("cuda", 0)
n = int(float(os.environ.get("SECONDS", "1800")) * sr)
# the C4 speech signal (sonar.synth.c4_speech: voiced frames with formants), as the bench's c4_formants
from sonar import synth  # noqa: E402
x = torch.from_numpy(np.ascontiguousarray(synth.c4_speech(seconds=n / sr, sr=sr), dtype=np.float64)).to(dev)
ctx = sonar.Context(0)
L = ctx._L
F = int(L.sonar_formant_frame_count(n, sr, 0, 0))
rec = torch.empty(F * C.sizeof(_abi.FormantFrame) // 8 + 1, dtype=torch.float64, device=dev)


def call():
    rc = L.sonar_formants(ctx._h, C.c_void_p(x.data_ptr()), n, sr, 0, 0, C.c_void_p(rec.data_ptr()), None, None, 1)
    assert rc == 0, rc


for _ in range(3):
    call()
ctx.synchronize()
iters = int(os.environ.get("ITERS", "20"))
t0 = time.perf_counter()
for _ in range(iters):
    call()
ctx.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / iters
h = hashlib.sha1(rec.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"kernel": "formant_kernel", "frames": F, "ms": round(ms, 4), "frames_per_s": round(F / ms * 1e3),
                  "rows_sha1": h}), flush=True)
