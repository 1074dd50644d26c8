"""C5 throughput vs concurrency: P pre-generated 60 s pairs, aligned with W worker contexts."""
import os, sys, time, numpy as np, torch
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd")]
from sonar import pairs
P = int(sys.argv[1]); maxlag = 20.0
data = [pairs.c5_pair_device(k, 60.0, device="cuda") for k in range(P)]
torch.cuda.synchronize()
for W in [int(w) for w in sys.argv[2:]]:
    t0 = time.perf_counter()
    R = pairs.align_pairs(range(P), lambda k: data[k], max_lag_seconds=maxlag, workers=W)
    dt = time.perf_counter() - t0
    lag_frames = R[:, -1] * 44100 / 256
    ok = np.minimum(np.abs(R[:, 7] - lag_frames), np.abs(R[:, 7] + lag_frames)) <= 1.5
    print(f"workers {W}: {P} pairs in {dt:.3f} s = {P/dt:.1f} pairs/s, lag_ok {ok.sum()}/{P}", flush=True)
