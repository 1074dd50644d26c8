"""Uncontended energy_kernel launches (ShortTimeEnergy 1024/256 on a 60 s float64 stream), for a
kernel-trace A/B between library variants (SONAR_LIB)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sonido-sonar_amd"))
import sonar  # noqa: E402

n = 44100 * 60
x = torch.from_numpy(np.random.default_rng(1).standard_normal(n)).cuda()
ctx = sonar.Context(0)
cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, precision=sonar.F64, pcm_dtype=sonar.F64,
                 out_dtype=sonar.F64, flags=sonar.FP_ENERGY, energy_window=1024, energy_hop=256,
                 preemph_alpha=0.95)
fe = sonar.energy_frames(n, 1024, 256)
out = torch.empty(fe, dtype=torch.float64, device="cuda")
for _ in range(50):
    ctx.fingerprint_device(x.data_ptr(), n, cfg, energy=out.data_ptr())
ctx.synchronize()
print("ok", fe)
