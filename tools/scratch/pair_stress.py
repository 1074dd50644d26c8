"""Stress check of the headline kernel: random lengths/hops, pair kernel vs the general kernel
and vs itself (determinism).  Prints one summary line."""
import sys, time, numpy as np
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd")]
import sonar
from sonar import synth
ctx = sonar.Context(0)
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
small = len(sys.argv) > 3 and sys.argv[3] == 'small'   # few waves: hazards are not covered by other waves
base = synth.c2_hour(seconds=12.0)
bad_calls = bad_frames = nondet = 0
odd = even = 0
t0 = time.time()
for it in range(iters):
    n = int(rng.integers(1100, int(len(base) * (0.1 if small else 1.0))))
    H = int(rng.choice([256, 100, 512]))
    s0 = int(rng.integers(0, len(base) - n + 1))
    x = np.ascontiguousarray(base[s0:s0 + n])
    cfg = ctx.config(window_size=1024, hop_size=H, sample_rate=44100, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    a = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    a2 = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    cfg.flags = sonar.FP_MFCC | sonar.FP_GENERIC
    b = ctx.fingerprint(x, cfg)["mfcc"].astype(np.float64)
    e = np.max(np.abs(a - b), axis=1) / np.linalg.norm(b, axis=1)
    bad = np.nonzero(~(e < 1e-4))[0]
    nondet += int(not np.array_equal(a, a2))
    if len(bad):
        bad_calls += 1; bad_frames += len(bad); odd += int((bad % 2 == 1).sum()); even += int((bad % 2 == 0).sum())
    if it % 10 == 0 and rng.random() < 0.5:
        time.sleep(0.2)          # idle gaps like a test suite's CPU work
print(f"iters {iters} bad_calls {bad_calls} bad_frames {bad_frames} (odd {odd} even {even}) nondet_calls {nondet} "
      f"in {time.time() - t0:.1f}s", flush=True)
