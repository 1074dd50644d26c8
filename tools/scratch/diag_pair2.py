"""Reproduce the test order: many configurations through one context, then the headline."""
import sys, numpy as np
import os
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_R, "sonido-sonar_amd"), os.path.join(_R, "oracle")]
import sonar, oracle as O
from sonar import synth
ctx = sonar.Context(0)
def cfg(**kw):
    base = dict(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13,
                precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    base.update(kw); return ctx.config(**base)
def check(x, c, tag):
    a = ctx.fingerprint(x, c)["mfcc"].astype(np.float64)
    k = ctx.last_fp_kernel()
    c.flags = sonar.FP_MFCC | sonar.FP_GENERIC
    b = ctx.fingerprint(x, c)["mfcc"].astype(np.float64)
    e = np.max(np.abs(a - b), axis=1) / np.linalg.norm(b, axis=1)
    bad = np.nonzero(~(e < 1e-4))[0]
    print(tag, k, len(a), "bad", len(bad), bad[:12], "max", np.nanmax(e), "nan", np.isnan(a).sum(), flush=True)
    if len(bad):
        f = bad[0]; print("   got", a[f][:5], "\n   ref", b[f][:5])
for it in range(2):
    for H in (256, 100, 1000, 512):
        for secs in (0.1, 1.0, 7.3):
            check(synth.c2_hour(seconds=secs), cfg(hop_size=H), f"H{H} s{secs}")
    check(synth.c2_hour(seconds=2.0), cfg(mfcc_input_power=1), "F5")
    for sr, nm, nc in [(44100, 26, 13), (22050, 32, 16), (16000, 26, 12)]:
        check(synth.c2_hour(seconds=2.0), cfg(sample_rate=sr, n_filters=nm, n_mfcc=nc), f"sr{sr} nm{nm}")
    check(synth.c2_hour(seconds=20.0), cfg(), "headline")
