"""Time the C5 per-pair alignment pipeline on one GPU (device-resident 60 s pairs)."""
import sys, time, numpy as np, torch
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd")]
import sonar
from sonar import pairs
ctx = sonar.Context(0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
maxlag = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
recs = []
t_gen = t_al = 0.0
for k in range(P):
    t0 = time.perf_counter()
    q, r, lag = pairs.c5_pair_device(k, 60.0, device="cuda")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    rec, _ = pairs.align_pair(ctx, q, r, 44100, max_lag_seconds=maxlag, lag_seconds_true=lag)
    t2 = time.perf_counter()
    t_gen += t1 - t0; t_al += t2 - t1
    recs.append(rec)
R = np.array(recs)
lag_frames = R[:, -1] * 44100 / 256
ok = np.minimum(np.abs(R[:, 7] - lag_frames), np.abs(R[:, 7] + lag_frames)) <= 1.5
print(f"pairs {P} gen {t_gen/P*1e3:.2f} ms/pair align {t_al/P*1e3:.2f} ms/pair lag_ok {ok.sum()}/{P}", flush=True)
print("method", R[:, 4].tolist()[:8], "peak_lag", R[:, 7].tolist()[:8], "true", np.round(lag_frames[:8], 1).tolist())
