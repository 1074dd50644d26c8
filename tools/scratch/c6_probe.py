"""Row f1 probe: FindBestMatches / compare / gallery_add timings for rocprofv3 (tools only)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
import numpy as np
import torch
import sonar
from sonar import compare as cmp

dev = torch.device("cuda", 0)
ctx = sonar.Context(0)
buf, st, _ = cmp.device_features(65536, 32, dev, seed=7)
g = cmp.Gallery(ctx)
g.add_raw(st, 65536, keep_sequences=False, device_ptrs=True)
cfg = cmp.make_cfg({"similarity_threshold": 0.5, "max_candidates": 50})
q = np.arange(64)
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = g.find_best_matches(q, None, cfg)
    print("fbm ms", (time.perf_counter() - t0) * 1e3, len(r[0]), flush=True)
big, st2, _ = cmp.device_features(256, 51676, dev, seed=6)
for i in range(3):
    g2 = cmp.Gallery(ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g2.add_raw(st2, 256, keep_sequences=False, device_ptrs=True)
    print("add ms", (time.perf_counter() - t0) * 1e3, flush=True)
    g2.close()
