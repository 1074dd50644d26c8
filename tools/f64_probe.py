"""Probe: is the whole-hour f64 headline error an input difference or an f64
precision loss?  Device-generated C2 PCM vs the host regeneration (differing samples), then the
f64 kernel on 10 min against the oracle on (a) the identical bytes and (b) the host regeneration.
Usage: python tools/f64_probe.py [seconds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import sonar  # noqa: E402
from sonar import shard  # noqa: E402
from parity import mfcc_tier_errors  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 600.0
SR, W, H = 44100, 1024, 256
n = int(secs * SR)
dev = torch.device("cuda", 0)
t0 = time.time()
pd = shard.stream_pcm(0, n, device=dev)
ph = shard.stream_pcm(0, n)
pdc = pd.cpu()
diff = (pdc != ph)
res = {"seconds": secs, "samples": n, "samples_differ": int(diff.sum()),
       "max_abs_diff": float((pdc.double() - ph.double()).abs().max())}
print(json.dumps(res), flush=True)
ctx = sonar.Context(0)
cfg = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=40, n_mfcc=13,
                 precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=sonar.FP_MFCC)
x_same = pdc.double().numpy()
got = ctx.fingerprint(x_same, cfg)["mfcc"]
res["kernel"] = ctx.last_fp_kernel()
for name, x in (("identical_bytes", x_same), ("host_regenerated", ph.double().numpy())):
    ref = O.mfcc_frames(O.stft_mag(x, W, H, nthreads=16), SR, n_coef=13, n_mels=40)
    norms = np.linalg.norm(ref, axis=1)
    e_row = np.max(np.abs(got - ref), axis=1) / norms
    i = int(np.argmax(e_row))
    res[name] = {"max_rel_err_row_norm": float(e_row.max()), "worst_frame": i,
                 "frames_over_1e-9": int(np.count_nonzero(e_row > 1e-9)),
                 "tiers": {str(k): v for k, v in mfcc_tier_errors(got, ref).items()}}
    if name == "identical_bytes" and e_row.max() > 1e-9:
        res[name]["worst_row_got"] = got[i].tolist()
        res[name]["worst_row_ref"] = ref[i].tolist()
        # power spectrum / mel energies of the worst frame (oracle) to see which band is tiny
        mag = O.stft_mag(x[i * H:i * H + W], W, H)
        res[name]["worst_frame_mag_min"] = float(mag.min())
    print(json.dumps(res[name]), flush=True)
res["wall_s"] = time.time() - t0
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "r05a_f64_probe.json"), "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: v for k, v in res.items() if not isinstance(v, dict)}))
