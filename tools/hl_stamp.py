"""Per-wave start/end times of the headline kernel (an HL_STAMP build: -DHL_STAMP) on 1 h of C2:
how far the slowest wave's end lies past the average wave's, i.e. what a balanced split could gain.

    SONAR_LIB=.../lib_stamp/libsonar_gpu.so python3 tools/hl_stamp.py [reps]"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sonar  # noqa: E402
from sonar import shard  # noqa: E402

dev = torch.device("cuda", 0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
pcm = shard.stream_pcm(0, 3600 * 44100, device=dev)
n = pcm.numel()
ctx = sonar.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13, precision=sonar.F32,
                 pcm_dtype=sonar.F32, out_dtype=sonar.F32, flags=sonar.FP_MFCC)
F = sonar.stft_frames(n, 1024, 256)
out = torch.empty((F, 13), dtype=torch.float32, device=dev)
for _ in range(3):
    ctx.fingerprint_device(pcm.data_ptr(), n, cfg, mfcc=out.data_ptr())
torch.cuda.synchronize()
path = os.path.join(tempfile.mkdtemp(), "stamp.bin")
os.environ["SONAR_HL_STAMP"] = path
for _ in range(reps):
    ctx.fingerprint_device(pcm.data_ptr(), n, cfg, mfcc=out.data_ptr())
torch.cuda.synchronize()
raw = np.fromfile(path, dtype=np.uint64).reshape(reps, -1, 3).astype(np.float64)
raw[:, :, :2] *= 10.0                     # 100 MHz ticks -> ns; word 2 = pairs the wave did
for r in range(reps):
    busy = raw[r, :, 2] > 0
    st, en = raw[r, busy, 0], raw[r, busy, 1]
    t0 = st.min()
    span = en.max() - t0
    print(json.dumps({"rep": r, "waves": int(len(st)), "span_us": round(span / 1e3, 1),
                      "start_spread_us": round((st.max() - t0) / 1e3, 1),
                      "end_us": {q: round((np.percentile(en, q) - t0) / 1e3, 1) for q in (0, 1, 10, 50, 90, 99, 100)},
                      "mean_end_us": round((en.mean() - t0) / 1e3, 1),
                      "dur_us": {q: round(np.percentile(en - st, q) / 1e3, 1) for q in (0, 50, 100)},
                      "balanced_gain": round((en.max() - en.mean()) / span, 4)}), flush=True)
# where the slow waves are: duration by XCD (block % 8 under round-robin dispatch), pairs per wave
busy = raw[-1, :, 2] > 0
dur = (raw[-1, :, 1] - raw[-1, :, 0])[busy]
gw = np.arange(raw.shape[1])[busy]
npairs = raw[-1, busy, 2]
print(json.dumps({"pairs_per_wave": {q: float(np.percentile(npairs, q)) for q in (0, 10, 50, 90, 100)}}))
for name, key in (("xcd", (gw // 12) % 8), ("wave_in_block", gw % 12)):
    print(json.dumps({name: {int(k): round(float(np.median(npairs[key == k])), 1) for k in np.unique(key)}}))
full = dur
hist, edges = np.histogram(full / 1e3, bins=20)
print(json.dumps({"hist_us": [[round(float(edges[i]), 1), int(hist[i])] for i in range(len(hist))]}))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "hl_stamp_raw.npy"), raw)
