"""Micro-benchmark of yin_kernel: sonar_pitch_yin on device-resident float64 PCM (1 h of the C2
stream by default, hop 512), one launch per call.  Prints ms per call from torch events over ITERS
calls and a checksum of the pitch / confidence / tau rows (equal across builds = bit-identical).
Usage: [SONAR_LIB=...] [SECONDS=3600] [ITERS=20] python3 tools/yin_microbench.py"""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd"), ROOT]
import torch  # noqa: E402
import sonar  # noqa: E402
from sonar import shard  # noqa: E402

dev = torch.device("cuda", 0)
pcm = shard.stream_pcm(0, int(float(os.environ.get("SECONDS", "3600")) * 44100), device=dev).double()
n = pcm.numel()
F = sonar.pitch_frames(n)
ctx = sonar.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
p = torch.empty(F, dtype=torch.float64, device=dev)
c = torch.empty(F, dtype=torch.float64, device=dev)
t = torch.empty(F, dtype=torch.int32, device=dev)
L = ctx._L


def call():
    rc = L.sonar_pitch_yin(ctx._h, C.c_void_p(pcm.data_ptr()), n, 44100, C.c_void_p(p.data_ptr()),
                           C.c_void_p(c.data_ptr()), C.c_void_p(t.data_ptr()), 1)
    assert rc == 0, rc


for _ in range(3):
    call()
torch.cuda.synchronize()
iters = int(os.environ.get("ITERS", "20"))
# wall clock around ITERS back-to-back calls (one launch each) and a device synchronisation: the
# context's stream is its own, so events on torch's stream would not bracket the launches
import time  # noqa: E402
ctx.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    call()
ctx.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / iters
h = hashlib.sha1()
for x in (p, c, t):
    h.update(x.cpu().numpy().tobytes())
print(json.dumps({"kernel": "yin_kernel", "frames": F, "ms": round(ms, 4), "frames_per_s": round(F / ms * 1e3),
                  "voiced": int((p > 0).sum().item()), "rows_sha1": h.hexdigest()[:16]}), flush=True)
