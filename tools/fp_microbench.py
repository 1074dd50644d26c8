"""Micro-benchmark of the fused path-A kernel variants on 1 h of C2 PCM (device resident).
Prints one line per variant: average kernel ms from HIP events over N launches."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd"), ROOT]
import torch, sonar
from sonar import shard
dev = torch.device("cuda", 0)
pcm = shard.stream_pcm(0, int(float(os.environ.get("SECONDS", "3600")) * 44100), device=dev)
n = pcm.numel()
ctx = sonar.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
variants = {
    "mfcc": dict(flags=sonar.FP_MFCC),
    "mfcc_generic": dict(flags=sonar.FP_MFCC | sonar.FP_GENERIC),
    "fft_only": dict(flags=sonar.FP_MFCC | (1 << 31)),
    "mfcc+spectral": dict(flags=sonar.FP_MFCC | sonar.FP_SPECTRAL),
    "mfcc_w2048": dict(flags=sonar.FP_MFCC, window_size=2048, hop_size=512),
    "mfcc_w512": dict(flags=sonar.FP_MFCC, window_size=512, hop_size=128),
    "mfcc_f64": dict(flags=sonar.FP_MFCC, precision=sonar.F64),
    # float64 arithmetic and output (the pair kernel's double instantiation; _generic: fp_wave_kernel<double>)
    "mfcc_f64o": dict(flags=sonar.FP_MFCC, precision=sonar.F64, out_dtype=sonar.F64),
    "mfcc_f64p": dict(flags=sonar.FP_MFCC, precision=sonar.F64, out_dtype=sonar.F64, pcm_dtype=sonar.F64),
    "mfcc_f64p_generic": dict(flags=sonar.FP_MFCC | sonar.FP_GENERIC, precision=sonar.F64, out_dtype=sonar.F64,
                              pcm_dtype=sonar.F64),
    # the GenerateFingerprint transform: f64 PCM, MFCC + descriptors (two passes: |X| rows + spec_rows_kernel)
    "spec_f64p": dict(flags=sonar.FP_MFCC | sonar.FP_SPECTRAL, precision=sonar.F64, out_dtype=sonar.F64,
                      pcm_dtype=sonar.F64),
}
pcm64 = None
sel = sys.argv[1:] or list(variants)
for name in sel:
    kw = dict(window_size=1024, hop_size=256, sample_rate=44100, n_filters=40, n_mfcc=13, precision=sonar.F32,
              pcm_dtype=sonar.F32, out_dtype=sonar.F32)
    kw.update(variants[name])
    cfg = ctx.config(**kw)
    F = sonar.stft_frames(n, cfg.window_size, cfg.hop_size)
    odt = torch.float64 if cfg.out_dtype == sonar.F64 else torch.float32
    if cfg.pcm_dtype == sonar.F64 and pcm64 is None:
        pcm64 = pcm.double()
    src = pcm64 if cfg.pcm_dtype == sonar.F64 else pcm
    outs = {"mfcc": torch.empty((F, 13), dtype=odt, device=dev)}
    ptrs = {"mfcc": outs["mfcc"].data_ptr()}
    if cfg.flags & sonar.FP_SPECTRAL:
        for k in ["centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux", "low_ratio", "high_ratio"]:
            outs[k] = torch.empty(F, dtype=odt, device=dev)
            ptrs[k] = outs[k].data_ptr()
    for _ in range(3):
        ctx.fingerprint_device(src.data_ptr(), n, cfg, **ptrs)
    torch.cuda.synchronize(); ctx.last_kernel_ms()
    ctx.enable_kernel_timing(True)
    for _ in range(int(os.environ.get("ITERS", "100"))):
        ctx.fingerprint_device(src.data_ptr(), n, cfg, **ptrs)
    torch.cuda.synchronize()
    ctx.enable_kernel_timing(False)
    ms = ctx.last_kernel_ms()
    print(json.dumps({"variant": name, "kernel": ctx.last_fp_kernel(), "frames": F, "kernel_ms": round(ms, 4), "Mframes_per_s": round(F / ms / 1e3, 1)}), flush=True)
