#!/usr/bin/env python3
"""Benchmark of the sonido-sonar hot path on MI355X (see BASELINE.json / DESIGN.md).

Headline: audio frames/sec of the fused STFT -> mel(40) -> MFCC(13) kernel
(W=1024, H=256, 44.1 kHz, float32) on 1 h of synthetic PCM per GPU, PCM
resident in HBM when timing starts.  Multi-GPU (torchrun, one process per
GPU): one stream of N hours is sharded by STFT frames (sonar/shard.py) --
rank g holds its frames' samples plus the 768-sample halo, generated on its
own device by sample index -- with no data-path collective ("scaling":
"weak", 1 h per GPU); the RCCL all-gather that reassembles the feature
timeline runs once after the timed region and is reported separately.  Extra fields: DTW cells/sec (C3 size, float64, cost
matrix in HBM), roofline of the dominant kernel, CPU baseline (the oracle,
a float64 C restatement of the Go path, on a bounded sample).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]

# Path B (C5) runs one HIP stream per worker context (16 by default).  HIP maps a process's streams
# onto GPU_MAX_HW_QUEUES hardware queues (4 by default), so 16 streams would share 4 queues and
# most pairs' kernels would wait behind the others' (measured: 394 -> 669 pairs/s at 16).  Set before HIP initialises.
_HWQ = 16
for _i, _a in enumerate(sys.argv):
    if _a == "--hw-queues" and _i + 1 < len(sys.argv):
        _HWQ = int(sys.argv[_i + 1])
if _HWQ > 0 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < _HWQ:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(_HWQ, 32))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sonar  # noqa: E402
from sonar import pairs, shard  # noqa: E402

W, H, SR, N_MELS, N_MFCC = 1024, 256, 44100, 40, 13
BYTES_PER_FRAME = 4 * H + 4 * N_MFCC            # PCM in (hop, f32) + MFCC out (f32)
FLOPS_PER_FRAME = 31136                          # window + FFT + |X|^2 + mel + ln + DCT + lifter
HBM_PEAK_GBS = 8000.0                            # MI355X_MICROARCH.md: 8 TB/s spec
FP32_PEAK_TFS = 157.3                            # FP32 vector (= f32 MFMA) peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # headline steps are ~0.5 ms launches: 20 untimed warm-up steps let the clocks settle after
    # the process's first GPU work (round 4: 200-step runs timed 0.45 ms per launch, 20-step runs
    # after 3 warm-ups 0.46-0.49 ms on the same build), 50 timed steps are still ~25 ms
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--seconds", type=float, default=3600.0, help="audio seconds per GPU (1 h config)")
    ap.add_argument("--dtw-len", type=int, default=51676, help="DTW sequence length (0 = skip); C3 = 51,676")
    ap.add_argument("--dtw-steps", type=int, default=5, help="C3 DTW repetitions (median reported)")
    ap.add_argument("--c5-pairs", type=int, default=1000, help="C5 stream pairs in total (0 = skip)")
    ap.add_argument("--c5-seconds", type=float, default=60.0)
    ap.add_argument("--c5-max-lag", type=float, default=20.0, help="maxOffsetSeconds (lags are drawn in [0, 20) s)")
    ap.add_argument("--c5-workers", type=int, default=128,
                    help="pairs in flight per rank (sonar_align_pairs: 16 streams x batches of 8)")
    ap.add_argument("--c6-gallery", type=int, default=256, help="C3-sized fingerprints added (0 = skip row f1)")
    ap.add_argument("--c6-frames", type=int, default=51676)
    ap.add_argument("--c6-compare-gallery", type=int, default=65536)
    ap.add_argument("--c6-queries", type=int, default=64)
    ap.add_argument("--c6-reps", type=int, default=3)
    ap.add_argument("--c6-cpu-seconds", type=float, default=5.0)
    ap.add_argument("--c7-seconds", type=float, default=600.0, help="DetectFromAudio input length (0 = skip row f2)")
    ap.add_argument("--c3-seconds", type=float, default=300.0, help="C3 stream length (0 = skip)")
    ap.add_argument("--c4-seconds", type=float, default=1800.0, help="C4 speech length at 16 kHz (0 = skip)")
    ap.add_argument("--ingest-reps", type=int, default=3, help="row f3 PCM-ingest repetitions (0 = skip)")
    ap.add_argument("--batch-signals", type=int, default=1000,
                    help="sonar_fingerprint_batch leg: short streams in one batch (0 = skip)")
    ap.add_argument("--batch-seconds", type=float, default=5.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c1", type=int, default=1, help="C1 GenerateFingerprint leg (0 = skip)")
    ap.add_argument("--c1-hour", type=float, default=3600.0,
                    help="GenerateFingerprint on this many seconds of the C2 stream too (0 = skip)")
    ap.add_argument("--hw-queues", type=int, default=16, help="GPU_MAX_HW_QUEUES for this process (0 = leave as is)")
    ap.add_argument("--cpu-seconds", type=float, default=0.0, help="force CPU-baseline sample length")
    ap.add_argument("--reps", type=int, default=3, help="repetitions of the C3 / C4 / C5 legs (median reported)")
    ap.add_argument("--no-f64", action="store_true", help="skip the float64 headline variant")
    ap.add_argument("--dump-dir", default=None,
                    help="rank 0 saves the gathered MFCC timeline and C5 records there (tests of the N > 1 path)")
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0 over gloo (RCCL
    # refuses two ranks on one device); the driver's multi-GPU runs use neither override
    if os.environ.get("SONAR_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("SONAR_BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def make_shard(seconds, world, rank, device):
    """This rank's frames of the world x `seconds` stream and the samples they read."""
    n_total = world * int(round(seconds * SR))
    F_total = shard.stft_frames(n_total, W, H)
    f0, f1 = shard.frame_range(F_total, world, rank)
    s0, s1 = shard.sample_span(f0, f1, W, H)
    pcm = shard.stream_pcm(s0, s1, device=device)
    counts = [b - a for a, b in (shard.frame_range(F_total, world, g) for g in range(world))]
    return pcm, F_total, f1 - f0, counts


def load_traffic(kernel_name):
    """Per-launch HBM bytes of `kernel_name` from the newest committed rocprofv3 PMC summary
    (profiles/<round>_traffic.json, FETCH_SIZE x2 + WRITE_SIZE; tools/traffic_summary.py).  PMC
    counters need their own rocprofv3 passes, so they cannot be collected inside this run."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if kernel_name and kernel_name in d.get("kernel", ""):
            return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def bench_headline_f64(args, ctx, pcm, F, dev):
    """The headline configuration at the reference's precision: float64 PCM in, every stage in
    float64 (mfcc_pair_kernel<double> since round 6), float64 MFCC out -- what the Go path computes.
    HIP events around 5 launches after 2 warm-ups; the PCM is converted to float64 on the device
    before.  generic_kernel_ms: the general fused kernel (fp_wave_kernel<double>, SONAR_FP_GENERIC)
    on the same bytes, the round-5 path, for comparison."""
    pcm64 = pcm.double()
    n = pcm64.numel()
    out64 = torch.empty((F, N_MFCC), dtype=torch.float64, device=dev)
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=N_MELS, n_mfcc=N_MFCC,
                     precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=sonar.FP_MFCC)
    for _ in range(2):
        ctx.fingerprint_device(pcm64.data_ptr(), n, cfg, mfcc=out64.data_ptr())
    torch.cuda.synchronize()
    ctx.last_kernel_ms()
    ctx.enable_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(5):
        ctx.fingerprint_device(pcm64.data_ptr(), n, cfg, mfcc=out64.data_ptr())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    ctx.enable_kernel_timing(False)
    kms = ctx.last_kernel_ms()
    res = {"frames_per_s": F / dt, "ms_per_step": dt * 1e3, "kernel": ctx.last_fp_kernel(), "kernel_ms": kms,
           "dtype": "f64", "pcm_dtype": "f64",
           "fp64_tflops": F * FLOPS_PER_FRAME / (kms * 1e-3) / 1e12,
           "fp64_frac": F * FLOPS_PER_FRAME / (kms * 1e-3) / 1e12 / FP64_PEAK_TFS,
           "hbm_gbs": F * (8 * H + 8 * N_MFCC) / (kms * 1e-3) / 1e9}
    host = out64.cpu().numpy()
    gen = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=N_MELS, n_mfcc=N_MFCC,
                     precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64,
                     flags=sonar.FP_MFCC | sonar.FP_GENERIC)
    ctx.fingerprint_device(pcm64.data_ptr(), n, gen, mfcc=out64.data_ptr())
    torch.cuda.synchronize()
    ctx.last_kernel_ms()
    ctx.enable_kernel_timing(True)
    for _ in range(3):
        ctx.fingerprint_device(pcm64.data_ptr(), n, gen, mfcc=out64.data_ptr())
    torch.cuda.synchronize()
    ctx.enable_kernel_timing(False)
    res["generic_kernel_ms"] = ctx.last_kernel_ms()
    res["generic_kernel"] = ctx.last_fp_kernel()
    del pcm64, out64
    return res, host


def host_info():
    """The CPU the baselines ran on (BASELINE.md protocol: nproc, model, SMT state, pinning)."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        with open("/proc/cpuinfo") as f:
            info["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        info["cpu_model"] = None
    try:
        with open("/sys/devices/system/cpu/smt/active") as f:
            info["smt_active"] = f.read().strip() == "1"
    except OSError:
        info["smt_active"] = None
    return info


def cpu_threads():
    """Host threads for the CPU baselines: the job's share of the box (OMP_NUM_THREADS, 16 on the
    GPU box; the box's nproc shows the whole machine), capped by the CPUs this process may use."""
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(share, len(os.sched_getaffinity(0))))


class pinned:
    """Pin this process (and the oracle's pthreads, which inherit it) to the first n allowed CPUs."""
    def __init__(self, n):
        self.old = os.sched_getaffinity(0)
        self.cpus = sorted(self.old)[:n]

    def __enter__(self):
        os.sched_setaffinity(0, self.cpus)
        return self.cpus

    def __exit__(self, *a):
        os.sched_setaffinity(0, self.old)


def timed_runs(fn, reps=5, warmup=1):
    """BASELINE.md protocol: warm-up, then the median (and spread) of `reps` timed runs."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(min(ts)), float(max(ts))


def oracle_module():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    return O


def mfcc_parity(got, ref, tol=1e-4):
    """Full-size parity of an MFCC output against the oracle, graded by tests/parity.py::assert_mfcc's
    rule: every coefficient within `tol` of its row's L2 norm, and per coefficient relative to
    itself by tier (|c| above 0.1 / 0.01 / 1e-3 of the row norm).  f32 (tol >= 1e-5): bounds
    1 / 10 / 100 x tol; f64 (tol < 1e-5): 10 / 100 / 1000 x tol, each capped at 1e-6.  Also the
    number of frames over the bound in each measure."""
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    norms = np.linalg.norm(ref, axis=1)[:, None]
    norms = np.where(norms == 0, 1.0, norms)
    e_row = np.abs(got - ref) / norms
    out = {"frames": int(len(ref)), "max_rel_err_row_norm": float(e_row.max()), "tolerance": tol,
           "frames_over_tol_row_norm": int(np.count_nonzero(e_row.max(axis=1) > tol)), "per_coef": {},
           "rule": "tests/parity.py::assert_mfcc (" + ("f32 tiers 1/10/100 x tol" if tol >= 1e-5 else
                                                       "f64 tiers 10/100/1000 x tol, capped at 1e-6") + ")"}
    tiers_ok = True
    for fl, mult, mult64 in ((1e-3, 100.0, 1000.0), (1e-2, 10.0, 100.0), (1e-1, 1.0, 10.0)):
        bound = mult * tol if tol >= 1e-5 else min(mult64 * tol, 1e-6)
        big = np.abs(ref) > fl * norms
        e = np.where(big, np.abs(got - ref) / np.where(big, np.abs(ref), 1.0), 0.0)
        out["per_coef"][f"|c|>{fl:g}*|row|"] = {"max_rel_err": float(e.max()), "bound": bound,
                                                 "frames_over_bound": int(np.count_nonzero(e.max(axis=1) > bound))}
        tiers_ok = tiers_ok and float(e.max()) <= bound
    out["pass"] = bool(e_row.max() < tol) and tiers_ok
    return out


def cpu_baseline(seconds_hint, gpu_mfcc, pcm_host, gpu_mfcc64=None):
    """The oracle (a float64 C restatement of the Go path) on the box's host, pinned: STFT over
    `threads` threads (Go's worker-pool shape), MFCC.ComputeFrames single-threaded, as in Go.  One
    pass over the WHOLE hour doubles as the warm-up and as the parity check of the GPU output --
    on the exact samples the GPU ran (`pcm_host` = the device PCM copied back; a host regeneration
    of the stream differs from the device one in ~1 of 1,500 samples by one f32 ulp, because torch's
    f64 sin / log1p / cos differ between the GPU and the CPU: tools/f64_probe.py, 17,096 of 26.46 M
    samples over 10 min, profiles/r05a_f64_probe.json).  The timed value is the median of 5 runs on
    a bounded sample (~3 s each)."""
    O = oracle_module()
    threads = cpu_threads()
    with pinned(threads) as cpus:
        x = np.asarray(pcm_host, dtype=np.float64)
        ref = O.mfcc_frames(O.stft_mag(x, W, H, nthreads=threads), SR, n_coef=N_MFCC, n_mels=N_MELS)
        parity = mfcc_parity(gpu_mfcc[: len(ref)], ref)
        parity["inputs"] = "identical: the device PCM copied to the host, widened to float64"
        parity64 = None
        if gpu_mfcc64 is not None:                     # the float64 headline variant
            # the f64 kernel against the same oracle rows, graded by tests/parity.py's f64 rule at the
            # 1e-9 row-norm tolerance of test_gpu_stft_mfcc.py / test_gpu_fullsize.py
            parity64 = mfcc_parity(gpu_mfcc64[: len(ref)], ref, tol=1e-9)
            parity64["inputs"] = parity["inputs"]
        del ref
        probe = x[: int(60 * SR)]
        t0 = time.perf_counter()
        O.mfcc_frames(O.stft_mag(probe, W, H, nthreads=threads), SR, n_coef=N_MFCC, n_mels=N_MELS)
        dt = time.perf_counter() - t0
        secs = seconds_hint or min(len(x) / SR, max(60.0, 60.0 * 3.0 / max(dt, 1e-6)))
        xs = x[: int(secs * SR)]
        F = O.stft_frames(len(xs), W, H)
        med, lo, hi = timed_runs(lambda: O.mfcc_frames(O.stft_mag(xs, W, H, nthreads=threads), SR,
                                                       n_coef=N_MFCC, n_mels=N_MELS), reps=5, warmup=0)
    # Go's STFT pool is NumCPU wide (analyzers/spectral.go:215-231): the same sample with the STFT
    # stage over every CPU this process may use, beside the job-share figure
    aff = len(os.sched_getaffinity(0))
    med_aff = None
    if aff > threads:
        with pinned(aff):
            med_aff, _, _ = timed_runs(lambda: O.mfcc_frames(O.stft_mag(xs, W, H, nthreads=aff), SR,
                                                             n_coef=N_MFCC, n_mels=N_MELS), reps=5, warmup=1)
    base = {"value": F / med, "unit": "frames/s", "cores": threads, "kind": "port",
            "stft_threads_at_affinity": aff, "value_at_affinity": (F / med_aff) if med_aff else F / med,
            "sample": f"{secs:.0f} s of the bench stream ({F} frames), float64: STFT over {threads} threads "
                      "(Go worker-pool shape), MFCC.ComputeFrames single-threaded, as in the Go path; "
                      "median of 5 runs after a warm-up pass over the whole hour",
            "runs": 5, "spread_frames_per_s": [F / hi, F / lo], "pinned_cpus": cpus, **host_info()}
    return base, parity, parity64


# Algorithmic HBM bytes per cell of the band kernel in checkpoint mode (the default: the cost matrix
# is not stored unless the caller asks for it): 2-bit direction codes 0.25 B, every 64th column of
# C 8 B / 64 = 0.125 B, the band's bottom edge row 8 B / 64 rows = 0.125 B written and read back
# by the band below 0.125 B.  The inputs (12 doubles per row) are read once: ~0 per cell.
DTW_BYTES_PER_CELL = 0.625
DTW_BYTES_BREAKDOWN = {"direction_codes": 0.25, "checkpoint_columns": 0.125, "edge_store": 0.125, "edge_load": 0.125}
FP64_PEAK_TFS = 78.6          # MI355X FP64 vector (AMD spec)


def load_pmc_bytes(pattern, kernel_prefix):
    """FETCH_SIZE x2 (gfx950 half count) + WRITE_SIZE per launch, bytes, of the first kernel whose
    name starts with `kernel_prefix` in the newest committed profiles/<pattern> PMC summary."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), reverse=True):
        with open(path) as f:
            d = json.load(f)
        for name, k in d.get("kernels", {}).items():
            if name.startswith(kernel_prefix) and "FETCH_SIZE" in k and "WRITE_SIZE" in k:
                return {"bytes_per_launch": (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024.0,
                        "fetch_bytes": 2 * k["FETCH_SIZE"] * 1024.0, "write_bytes": k["WRITE_SIZE"] * 1024.0,
                        "kernel": name, "source": os.path.relpath(path, ROOT)}
    return None


def bench_dtw(ctx, n, steps, parity=False):
    """C3-size DTW (51,676 x 51,676, 12-dim) through the sonar_dtw host entry (H2D of the inputs,
    D2H of the path): cells/s end to end, per-kernel HIP-event times (band sweep, walk, path
    decode) and the band sweep's roofline: bound by the wavefront's dependency chain (chain steps x
    the isolated step time of one band), with the HBM roof beside it at the checkpoint mode's
    0.625 algorithmic B/cell and the PMC bytes of the newest profiles/*dtw_pmc*.json."""
    rng = np.random.default_rng(7)
    q = rng.random((n, 12))
    r = np.roll(q, 37, axis=0) + 0.01 * rng.random((n, 12))
    ctx.dtw(q[:256], r[:256])       # warm-up / allocation of small buffers
    ctx.dtw(q, r)                   # warm-up at full size (codes, checkpoint columns, edges)
    # one band alone (64 query rows against all n reference rows): the isolated step time of the
    # sweep, which prices the wavefront's dependency chain below
    band0 = []
    for _ in range(3):
        ctx.dtw(q[:64], r)
        band0.append(ctx.dtw_last_timing()[0])
    step_ns = float(np.median(band0)) * 1e6 / (n + 63)
    torch.cuda.synchronize()
    walls, parts = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        res = ctx.dtw(q, r)
        walls.append(time.perf_counter() - t0)
        parts.append(ctx.dtw_last_timing())
    dt = float(np.median(walls))
    band_ms, walk_ms, dec_ms = (float(v) for v in np.median(np.array(parts), axis=0))
    cells = n * n
    nb = (n + 63) // 64
    chain_steps = (n + 63) + 64 * (nb - 1)      # band nb-1's last step: every band's 64-step lag, then its sweep
    floor_ms = chain_steps * step_ns * 1e-6
    traffic = load_pmc_bytes("*dtw_pmc*.json", "dtw_band_kernel<12, true, false, false")
    hbm_gbs = cells * DTW_BYTES_PER_CELL / (band_ms * 1e-3) / 1e9
    out = {"dtw_cells_per_s": cells / dt, "dtw_ms": dt * 1e3, "dtw_ms_spread": [min(walls) * 1e3, max(walls) * 1e3],
           "dtw_n": n, "dtw_dim": 12, "dtw_path_len": int(len(res["path_q"])), "dtw_reps": steps,
           "dtw_kernel_ms": {"band_sweep": band_ms, "walk": walk_ms, "path_decode": dec_ms},
           # the binding limit is the wavefront's dependency chain, not a roof: band b starts 64 steps
           # after band b-1, so the last band ends after (n + 63) + 64 (nb - 1) steps at the sweep's
           # isolated step time (one band alone, measured above); frac = that floor / the band kernel
           "dtw_roofline": {"bound": "wavefront", "kernel": "dtw_band_kernel", "achieved": band_ms,
                            "peak": floor_ms, "unit": "ms", "frac": floor_ms / band_ms,
                            "chain_steps": chain_steps, "step_ns_one_band": step_ns,
                            "sweep_cells_per_s": cells / (band_ms * 1e-3),
                            "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": hbm_gbs / HBM_PEAK_GBS,
                                    "algorithmic_bytes_per_cell": DTW_BYTES_PER_CELL,
                                    "algorithmic_bytes_breakdown": DTW_BYTES_BREAKDOWN,
                                    "algorithmic_bytes_per_launch": cells * DTW_BYTES_PER_CELL,
                                    "traffic": traffic["bytes_per_launch"] if traffic else None,
                                    "traffic_detail": traffic},
                            "fp64": {"achieved": cells * 40 / (band_ms * 1e-3) / 1e12, "peak": FP64_PEAK_TFS,
                                     "unit": "TFLOP/s", "frac": cells * 40 / (band_ms * 1e-3) / 1e12 / FP64_PEAK_TFS},
                            "note": "40 flop/cell (12-dim Euclidean + min + add, SURVEY.md 8(d)); 0.625 B/cell "
                                    "algorithmic (checkpoint mode); the sweep is bound by the wavefront's "
                                    "dependency chain, below both the HBM and the FP64 roofs"},
           "dtw_counters": ctx.dtw_counters(reset=True)}
    if parity:
        O = oracle_module()
        threads = cpu_threads()
        with pinned(threads):
            dts = []
            for _ in range(3):
                t0 = time.perf_counter()
                ref = O.dtw_full(q, r, nthreads=threads)
                dts.append(time.perf_counter() - t0)
            dtc = float(np.median(dts))
        out["dtw_parity"] = {"cells": cells, "path_equal": bool(np.array_equal(res["path_q"], ref["path_q"]) and
                                                               np.array_equal(res["path_r"], ref["path_r"])),
                             "path_cost_equal": bool(np.array_equal(res["path_cost"], ref["path_cost"])),
                             "distance_equal": bool(res["distance"] == ref["distance"]),
                             "oracle": "dtw_oracle.c stripe wavefront (same cells and order as or_dtw)"}
        out["dtw_cpu_baseline"] = {"value": cells / dtc, "unit": "cells/s", "cores": threads, "kind": "port",
                                   "sample": f"the same {n} x {n} 12-dim DTW, oracle stripe wavefront over "
                                             f"{threads} threads (the Go reference fills serially), median of 3",
                                   "spread_cells_per_s": [cells / max(dts), cells / min(dts)]}
    return out


def load_c5_families():
    """The newest committed profiles/*_c5_families.json (tools/c5_families.py over a rocprofv3
    kernel trace of a C5 run): each kernel family's share of the summed GPU kernel time."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_c5_families.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        return {"source": os.path.relpath(path, ROOT), "note": d.get("note", ""),
                "shares": {k: round(v["share"], 4) for k, v in d["families"].items()},
                "total_kernel_ms": d["total_kernel_ms"]}
    return None


def c5_roofline(P, dt, samples_per_pair, F):
    """C5's HBM roof (the path is far below it: the bound is the DTW wavefront chains and the
    latency-bound feature kernels).  Algorithmic bytes per pair: both
    streams' f64 PCM read once + the chroma DTW's F x F cells at the checkpoint mode's 0.625 B/cell
    (bench_dtw); achieved = pairs/s x that; the kernel families' GPU-time shares come from the
    newest committed profile."""
    per_pair = samples_per_pair * 8 + DTW_BYTES_PER_CELL * F * F
    achieved = P * per_pair / dt / 1e9
    return {"bound": "wavefront", "unit": "GB/s", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "frac": achieved / HBM_PEAK_GBS, "alg_bytes_per_pair": per_pair,
            "alg_bytes_breakdown": {"pcm_f64": samples_per_pair * 8, "dtw_cells": F * F,
                                    "dtw_bytes_per_cell": DTW_BYTES_PER_CELL},
            "kernel_families": load_c5_families()}


def bench_c5(args, world, rank, dev, ctx):
    """BASELINE config C5 (path B): P stream pairs sharded over the ranks by contiguous pair ranges
    (sonar/pairs.py), each pair through the music-extractor energy + chroma and
    ExtractAlignmentFeatures (NCC + chroma DTW); no data-path collective, the per-pair records
    are all-gathered over RCCL after the timed region.  Pairs are generated on the device
    before timing ("inputs resident in HBM").  The timed call is the product entry
    sonar_align_pairs (worker streams inside the library, no Python threads)."""
    P = args.c5_pairs
    a, b = pairs.pair_range(P, world, rank)
    counts = [pairs.pair_range(P, world, g)[1] - pairs.pair_range(P, world, g)[0] for g in range(world)]
    data = [pairs.c5_pair_device(k, args.c5_seconds, device=dev) for k in range(a, b)]
    torch.cuda.synchronize()
    qp, rp = [q.data_ptr() for q, _, _ in data], [r.data_ptr() for _, r, _ in data]
    nq, nr = [q.numel() for q, _, _ in data], [r.numel() for _, r, _ in data]

    def run(idx):
        return ctx.align_pairs([qp[i] for i in idx], [rp[i] for i in idx], nq=[nq[i] for i in idx],
                               nr=[nr[i] for i in idx], max_lag_seconds=args.c5_max_lag,
                               workers=args.c5_workers, device_ptrs=True)
    # a timed-out band pipeline is a failed call here, never a silent single-pair redo (the
    # library's default retry is off for the whole leg); the warm-up calls' liveness counters are
    # reported before they are reset, so a first-call failure shows in the line
    prev_retry = os.environ.get("SONAR_PAIR_RETRY")
    os.environ["SONAR_PAIR_RETRY"] = "0"
    try:
        return _bench_c5_run(args, world, rank, dev, ctx, P, counts, data, run)
    finally:                                   # the library reads it per call: later legs / callers keep theirs
        if prev_retry is None:
            os.environ.pop("SONAR_PAIR_RETRY", None)
        else:
            os.environ["SONAR_PAIR_RETRY"] = prev_retry


def _bench_c5_run(args, world, rank, dev, ctx, P, counts, data, run):
    nq, nr = [q.numel() for q, _, _ in data], [r.numel() for _, r, _ in data]
    ctx.dtw_counters(reset=True)
    warm_errs, warm_redone = [], 0
    for idx in ([0], list(range(len(data)))):   # warm-up: worker contexts, tables, buffers
        try:                                   # recorded, not raised: the timed repetitions decide
            warm_redone += int(np.count_nonzero(run(idx)["flags"]))
        except sonar.SonarError as e:
            warm_errs.append(str(e))
    torch.cuda.synchronize()
    warm_counters = ctx.dtw_counters(reset=True)
    dts, errs, recd = [], [], None
    for _ in range(args.reps):
        barrier(world)
        t0 = time.perf_counter()
        try:                                   # a failed call must not skip this rank's collectives
            recd = run(list(range(len(data))))
        except sonar.SonarError as e:
            errs.append(str(e))
        torch.cuda.synchronize()
        barrier(world)
        dts.append(max_over_ranks(time.perf_counter() - t0, world))
    counters = ctx.dtw_counters(reset=True)
    if recd is None:
        raise RuntimeError(f"every C5 repetition failed: {errs[0]}")
    dt = float(np.median(dts))
    recs = np.stack([recd[f] for f in sonar.PAIR_FIELDS] + [np.array([lag for _, _, lag in data])], axis=1)
    allrec = pairs.gather_records(torch.tensor(recs, dtype=torch.float64, device=dev), world, counts).cpu().numpy()
    if args.dump_dir and rank == 0:
        np.save(os.path.join(args.dump_dir, "c5_records.npy"), allrec)
    ipl = sonar.PAIR_FIELDS.index("peak_lag")
    lag_frames = allrec[:, -1] * SR / H
    ok = np.minimum(np.abs(allrec[:, ipl] - lag_frames), np.abs(allrec[:, ipl] + lag_frames)) <= 1.5
    F = int((args.c5_seconds * SR - W) // H + 1)
    return {"c5_pairs_per_s": P / dt, "c5_ms": dt * 1e3, "c5_reps": len(dts),
            "c5_roofline": c5_roofline(P, dt, float(np.mean(nq) + np.mean(nr)), F),
            "c5_pairs_per_s_spread": [P / max(dts), P / min(dts)],
            "c5_frames_per_s": 2 * P * F / dt, "c5_frames_note": "both streams' STFT frames of every pair (BASELINE configs[4])",
            "c5_pairs": P, "c5_seconds_per_stream": args.c5_seconds,
            "c5_max_lag_s": args.c5_max_lag, "c5_workers_per_rank": args.c5_workers, "c5_entry": "sonar_align_pairs",
            "c5_lag_recovered": float(ok.mean()), "c5_dtw_cells_per_pair": F * F,
            "c5_dtw_counters_rank0": counters, "c5_failed_reps": len(errs),
            "c5_warmup_dtw_counters": warm_counters, "c5_warmup_failed_calls": len(warm_errs),
            "c5_retry": "off (SONAR_PAIR_RETRY=0)", "c5_redone_pairs_last_rep": int(np.count_nonzero(recd["flags"])),
            "c5_warmup_redone_pairs": warm_redone,
            **({"c5_error": errs[0]} if errs else {}), **({"c5_warmup_error": warm_errs[0]} if warm_errs else {})}


def bench_c3(args, ctx, dev):
    """BASELINE config C3 (path B, one GPU): two 5-min 44.1 kHz streams with an injected 12.34 s lag
    (C3 recipe, generated on the device), the music extractor's energy + chroma for both and
    ExtractAlignmentFeatures with maxOffsetSeconds = 60 (NCC over 20,671 lags, chroma DTW over
    51,676 x 51,676 cells, the scorers).  Timed: the whole align_pair call (feature kernels,
    D2H of the features, the alignment entry with its H2D)."""
    q, r = pairs.c3_pair_device(args.c3_seconds, 12.34, 42, 7, device=dev)
    torch.cuda.synchronize()
    pairs.align_pair(ctx, q[: SR * 20], r[: SR * 20], max_lag_seconds=60.0)       # warm-up (small)
    torch.cuda.synchronize()
    dts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        rec, res = pairs.align_pair(ctx, q, r, max_lag_seconds=60.0, lag_seconds_true=12.34)
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts))
    F = (q.numel() - W) // H + 1
    lag = float(rec[pairs.RECORD_FIELDS.index("peak_lag")])
    want = 12.34 * SR / H
    return {"c3_align": {"seconds_per_stream": args.c3_seconds, "ms": dt * 1e3, "reps": len(dts),
                         "ms_spread": [min(dts) * 1e3, max(dts) * 1e3], "frames_per_stream": F,
                         "dtw_cells": F * F, "dtw_cells_per_s_end_to_end": F * F / dt,
                         "peak_lag_frames": lag, "injected_lag_frames": want,
                         "lag_recovered": bool(min(abs(lag - want), abs(lag + want)) <= 1.5),
                         "temporal_offset_s": float(rec[0]), "method": float(rec[4])}}


def bench_c4(args, ctx):
    """BASELINE config C4: SpeechFeatureExtractor.ExtractFeatures on 30 min of synthetic 16 kHz
    speech-like noise (C4 recipe), FeatureConfig.SampleRate = 16000, W = 512, H = 128 (STFT + MFCC +
    descriptors + ZCR + energy + YIN + temporal features), float64 parity mode.  The C entry takes
    host float64 PCM (as the cgo path hands it over): the H2D copy is inside the timed call.
    The C4 noise has no periodicity, so detectSpeech fails and the extractor skips formants and
    voice quality exactly as the oracle does; the LPC named by configs[3] is therefore timed in two
    more legs: FormantAnalyzer.AnalyzeMultipleFrames (sonar_formants, LPC order 28 on 2048-sample
    frames, hop 1024) over the same 30 min, and the extractor on a voiced 30-min signal
    (synth.voiced: 12 harmonics of 140 Hz + vibrato) that passes detectSpeech, so formants and
    voice quality run inside the call.  Median of --reps runs each.  CPU baselines: the oracle on
    60 s (extractor) and on the same frames' first 60 s (formants), median of 5."""
    from sonar import synth
    sr = 16000
    x = synth.c4_speech(seconds=args.c4_seconds, sr=sr)
    fc = dict(sample_rate=sr, window_size=512, hop_size=128, stft_window_size=512, stft_hop_size=128,
              enable_mfcc=1, enable_speech_features=1, enable_temporal_features=1, mfcc_coefficients=13)
    cfg = ctx.feature_config(is_news=0, **fc)
    ctx.extract_speech_features(x[: sr * 10], sr, cfg)                        # warm-up

    def reps_of(fn):
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            r_ = fn()
            ts.append(time.perf_counter() - t0)
        return r_, float(np.median(ts)), [min(ts) * 1e3, max(ts) * 1e3]

    got, dt, spread = reps_of(lambda: ctx.extract_speech_features(x, sr, cfg))
    F = sonar.stft_frames(len(x), 512, 128)
    out = {"c4_speech": {"seconds": args.c4_seconds, "samples": len(x), "stft_frames": F,
                         "pitch_frames": int(len(got["pitch_estimate"])), "ms": dt * 1e3, "ms_spread": spread,
                         "reps": args.reps, "frames_per_s": F / dt,
                         "is_speech": float(np.ravel(got.get("is_speech", [0]))[0]),
                         "precision": "f64 (parity mode, the extractor's default)"}}
    ctx.formants(x[: sr * 10], sr)                                             # warm-up
    fm, dtf, spf = reps_of(lambda: ctx.formants(x, sr))
    nf = len(fm["status"])
    out["c4_formants"] = {"frames": nf, "lpc_order": 28, "frame": 2048, "hop": 1024, "ms": dtf * 1e3,
                          "ms_spread": spf, "frames_per_s": nf / dtf,
                          "ok_frames": int(np.count_nonzero(np.asarray(fm["status"]) == 0))}
    v = synth.voiced(seconds=args.c4_seconds, sr=sr)
    ctx.extract_speech_features(v[: sr * 10], sr, cfg)
    gv, dtv, spv = reps_of(lambda: ctx.extract_speech_features(v, sr, cfg))
    out["c4_speech_voiced"] = {"seconds": args.c4_seconds, "stft_frames": sonar.stft_frames(len(v), 512, 128),
                               "ms": dtv * 1e3, "ms_spread": spv, "frames_per_s": sonar.stft_frames(len(v), 512, 128) / dtv,
                               "is_speech": float(np.ravel(gv.get("is_speech", [0]))[0]),
                               "jitter": float(np.ravel(gv.get("jitter", [0]))[0]),
                               "vocal_tract_length": float(np.ravel(gv.get("vocal_tract_length", [0]))[0]),
                               "note": "synth.voiced passes detectSpeech: formants (LPC) and voice quality run "
                                       "inside the extractor call"}
    if not args.no_cpu_baseline:
        O = oracle_module()
        threads = cpu_threads()
        n = sr * 60
        Fc = sonar.stft_frames(n, 512, 128)
        with pinned(threads) as cpus:
            med, lo, hi = timed_runs(lambda: O.speech_features_reference(x[:n], sr, fc), reps=5)
            medf, _, _ = timed_runs(lambda: O.formant_frames(x[:n], sr), reps=5)
        nfc = len(O.formant_frames(x[:n], sr)["status"])
        out["c4_cpu_baseline"] = {"value": Fc / med, "unit": "frames/s", "cores": threads, "kind": "port",
                                  "sample": f"60 s of the C4 signal ({Fc} STFT frames): oracle speech-extractor "
                                            f"composition, float64 (STFT over {threads} threads, the rest 1 thread), "
                                            "median of 5", "spread_frames_per_s": [Fc / hi, Fc / lo],
                                  "pinned_cpus": cpus}
        out["c4_formants_cpu_baseline"] = {"value": nfc / medf, "unit": "frames/s", "cores": 1, "kind": "port",
                                           "sample": f"AnalyzeMultipleFrames on 60 s of the C4 signal ({nfc} frames), "
                                                     "oracle, 1 thread, median of 5"}
    return out


# GenerateFingerprint's configuration for C1 (BASELINE configs[0]): FingerprintConfig{W 1024, H 256,
# FeatureConfig{W 1024, H 256}}, Metadata.ContentType "music"; the music generation config runs the
# speech extractor with MFCC on and the speech / temporal blocks off (content_config.go:87-140, F4),
# at FeatureConfig.SampleRate 0 (F1).  The oracle composition of the same Go code:
C1_FC = dict(sample_rate=0, window_size=1024, hop_size=256, stft_window_size=1024, stft_hop_size=256, enable_mfcc=1,
             enable_speech_features=0, enable_temporal_features=0, mfcc_coefficients=13)


def feature_parity(got, ref, rtol):
    """GenerateFingerprint outputs against the oracle composition, tests/test_gpu_go_api.py's rule:
    per element relative error with a floor at 1e-6 of the array's peak (`rtol`); the MFCC by
    tests/parity.py::assert_mfcc; the rolloff bin exact (F3: all zero at sample rate 0)."""
    out, ok = {}, True
    for k, v in ref.items():
        r = np.asarray(v, np.float64)
        if k not in got:
            out[k], ok = "missing", False
            continue
        g = np.asarray(got[k], np.float64).reshape(r.shape) if np.size(got[k]) == r.size else None
        if g is None:
            out[k], ok = f"shape {np.shape(got[k])} vs {r.shape}", False
            continue
        if k == "mfcc":
            p = mfcc_parity(g, r, tol=max(rtol, 1e-9))
            out[k] = {"max_rel_err_row_norm": p["max_rel_err_row_norm"], "pass": p["pass"]}
            ok = ok and p["pass"]
            continue
        if k == "spectral_rolloff":
            e = float(np.max(np.abs(g - r))) if r.size else 0.0
            out[k] = {"max_abs_err": e, "pass": e == 0.0}
            ok = ok and e == 0.0
            continue
        peak = float(np.max(np.abs(np.nan_to_num(r)))) if r.size else 0.0
        e = float(np.max(np.abs(g - r) / np.maximum(np.abs(r), max(peak * 1e-6, 1e-30)))) if r.size else 0.0
        out[k] = {"max_rel_err": e, "pass": e <= rtol}
        ok = ok and e <= rtol
    return {"pass": bool(ok), "rtol": rtol, "fields": out}


def load_gf_kernels(F, n):
    """Per-kernel time of one GenerateFingerprint hour call (f64) from the newest committed
    rocprofv3 timeline (profiles/<round>_gf_timeline.json: tools/gpu_gf_profile.sh, a kernel +
    memory-copy trace of tools/gf_hour_probe.py, placed inside each call by tools/gf_timeline.py),
    and each kernel's roofline: the transform and YIN against the FP64 VALU roof, the descriptor
    pass against HBM, the H2D copy against the PCIe rate of the same run's pageable copy.  A kernel
    trace cannot run inside this process, so these come from the committed profile."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_gf_timeline.json")), reverse=True)
    if not paths:
        return None
    calls = [c for c in json.load(open(paths[0])) if c.get("precision") == "f64"]
    if not calls:
        return None

    def med(pat):
        v = [sum(o["ms"] for k, o in c["ops"].items() if pat in k) for c in calls]
        return float(np.median(v)) if v else None
    K = W // 2 + 1
    yin_frames = (n - 1024) // 512 + 1
    t_fft, t_spec, t_yin, t_h2d = (med("fp_wave_kernel<double"), med("spec_rows_kernel"), med("yin_kernel"),
                                   med("HOST_TO_DEVICE"))
    out = {"source": os.path.relpath(paths[0], ROOT), "calls": len(calls),
           "note": "kernel ms summed over the call's chunked launches, median over the profiled f64 calls"}
    if t_fft:
        out["transform"] = {"kernel": "fp_wave_kernel<double, double, 8, false>", "ms": t_fft, "bound": "fp64_valu",
                            "achieved_tflops": F * FLOPS_PER_FRAME / t_fft / 1e9,
                            "frac": F * FLOPS_PER_FRAME / t_fft / 1e9 / FP64_PEAK_TFS,
                            "flops_per_frame": FLOPS_PER_FRAME}
    if t_spec:
        b = F * K * 8 + F * 9 * 8
        out["descriptors"] = {"kernel": "spec_rows_kernel", "ms": t_spec, "bound": "hbm",
                              "achieved_gbs": b / t_spec / 1e6, "frac": b / t_spec / 1e6 / 8000.0,
                              "bytes_per_frame": K * 8 + 9 * 8}
    if t_yin:
        ops = 512 * 512 * 3
        out["yin"] = {"kernel": "yin_kernel", "ms": t_yin, "frames": yin_frames, "bound": "fp64_valu",
                      "achieved_tflops": yin_frames * ops / t_yin / 1e9,
                      "frac": yin_frames * ops / t_yin / 1e9 / FP64_PEAK_TFS, "ops_per_frame": ops}
    if t_h2d:
        out["h2d"] = {"ms": t_h2d, "gbs": 8 * n / t_h2d / 1e6}
    return out


def bench_c1(args, ctx):
    """BASELINE configs[0] -- the north star's own claim, music fingerprinting in frames/s: the
    product entry sonar_generate_fingerprint (FingerprintGenerator.GenerateFingerprint,
    fingerprint/fingerprint.go:137-236) with ContentType "music" on the C1 10 s 44.1 kHz sweep and on
    1 h of the C2 stream; host float64 PCM in (as the cgo shim hands []float64 over: the H2D copy is
    inside the timed call), every ExtractedFeatures array back on the host.  Work per call: the
    STFT -> 26-mel MFCC at sample rate 0 (F1/F2), the spectral descriptors, ZCR, short-time energy
    and YIN (1024 / 512) with its sequential tracker -- the same stages the oracle composition
    (c1_cpu_baseline) runs.  Both precisions: F64 (parity mode) and F32 (throughput mode).
    Median of --reps (at least 5) after a warm-up; parity on the full 10 s against the oracle."""
    from sonar import synth
    reps = max(args.reps, 5)
    x1 = synth.sweep(10.0)
    F1 = sonar.stft_frames(len(x1), W, H)
    res = {"c1_generate_fingerprint": {"entry": "sonar_generate_fingerprint", "content_type": "music",
                                       "seconds": 10.0, "frames": F1, "reps": reps,
                                       "work": "STFT(1024/256) + MFCC(26 mels, sr 0) + descriptors + ZCR + "
                                               "energy + YIN(1024/512) + tracker, host f64 PCM in, features out"}}
    outs = {}
    for name, prec in (("f64", sonar.F64), ("f32", sonar.F32)):
        cfg = ctx.fingerprint_config(window_size=W, hop_size=H, feature_window_size=W, feature_hop_size=H,
                                     precision=prec)
        ctx.generate_fingerprint(x1, SR, "music", cfg)                     # warm-up: tables, buffers
        med, lo, hi = timed_runs(lambda: ctx.generate_fingerprint(x1, SR, "music", cfg), reps=reps, warmup=0)
        outs[name] = ctx.generate_fingerprint(x1, SR, "music", cfg)
        res["c1_generate_fingerprint"][name] = {"ms": med * 1e3, "ms_spread": [lo * 1e3, hi * 1e3],
                                                "frames_per_s": F1 / med}
    if args.c1_hour > 0:
        x2 = shard.stream_pcm(0, int(args.c1_hour * SR)).double().numpy()
        F2 = sonar.stft_frames(len(x2), W, H)
        r2 = {"seconds": args.c1_hour, "frames": F2, "reps": args.reps}
        for name, prec in (("f64", sonar.F64), ("f32", sonar.F32)):
            cfg = ctx.fingerprint_config(window_size=W, hop_size=H, feature_window_size=W, feature_hop_size=H,
                                         precision=prec)
            ctx.generate_fingerprint(x2[: SR * 20], SR, "music", cfg)
            med, lo, hi = timed_runs(lambda: ctx.generate_fingerprint(x2, SR, "music", cfg), reps=args.reps, warmup=1)
            r2[name] = {"ms": med * 1e3, "ms_spread": [lo * 1e3, hi * 1e3], "frames_per_s": F2 / med}
        # the call is bound by the host -> device copy of the float64 PCM (DESIGN.md Kernel 1b,
        # "GenerateFingerprint pipeline"): its roof is a plain copy of the same pageable bytes
        dev = torch.device("cuda", torch.cuda.current_device())
        xt = torch.from_numpy(x2)
        xt.to(dev)
        torch.cuda.synchronize()
        cmed, _, _ = timed_runs(lambda: (xt.to(dev), torch.cuda.synchronize()), reps=3, warmup=0)
        nbytes = 8 * len(x2)
        r2["roofline"] = {"bound": "pcie", "unit": "GB/s", "achieved": nbytes / r2["f64"]["ms"] / 1e6,
                          "peak": nbytes / cmed / 1e9, "frac": cmed * 1e3 / r2["f64"]["ms"],
                          "traffic": nbytes, "peak_source": "torch pageable H2D copy of the same float64 PCM, "
                                                            "median of 3, same process",
                          "h2d_copy_ms": cmed * 1e3}
        # the call's float64 transform + descriptor pass alone on device-resident PCM (HIP events, one
        # timed region over fp_wave_kernel<double> and spec_rows_kernel): inside the call these
        # kernels share the GPU with YIN and the copies, so the timeline's sums overstate them
        xd = xt.to(dev)
        outs_d = {"mfcc": torch.empty((F2, 13), dtype=torch.float64, device=dev)}
        for k in ("centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux", "low_ratio", "high_ratio"):
            outs_d[k] = torch.empty(F2, dtype=torch.float64, device=dev)
        cfg_t = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=26, n_mfcc=13, precision=sonar.F64,
                           pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=sonar.FP_MFCC | sonar.FP_SPECTRAL)
        ptrs = {k: v.data_ptr() for k, v in outs_d.items()}
        ctx.fingerprint_device(xd.data_ptr(), len(x2), cfg_t, **ptrs)
        torch.cuda.synchronize()
        ctx.last_kernel_ms()
        ctx.enable_kernel_timing(True)
        for _ in range(3):
            ctx.fingerprint_device(xd.data_ptr(), len(x2), cfg_t, **ptrs)
        torch.cuda.synchronize()
        ctx.enable_kernel_timing(False)
        t_iso = ctx.last_kernel_ms()
        r2["transform_isolated"] = {"kernels": "fp_wave_kernel<double, double, 8, false> + spec_rows_kernel",
                                    "ms": t_iso, "bound": "fp64_valu",
                                    "achieved_tflops": F2 * FLOPS_PER_FRAME / t_iso / 1e9,
                                    "frac": F2 * FLOPS_PER_FRAME / t_iso / 1e9 / FP64_PEAK_TFS,
                                    "note": "MFCC + descriptors in float64 on device-resident float64 PCM, mean of 3"}
        del xt, xd, outs_d
        r2["kernels"] = load_gf_kernels(F2, len(x2))
        res["c1_generate_fingerprint"]["c2_hour"] = r2
        del x2
    if not args.no_cpu_baseline:
        O = oracle_module()
        threads = cpu_threads()
        fc = dict(C1_FC, nthreads=threads)
        with pinned(threads) as cpus:
            ref = O.speech_features_reference(x1, SR, fc)
            med, lo, hi = timed_runs(lambda: O.speech_features_reference(x1, SR, fc), reps=5)
        aff = len(os.sched_getaffinity(0))                  # Go's NumCPU STFT pool (spectral.go:215-231)
        med_aff = med
        if aff > threads:
            fca = dict(C1_FC, nthreads=aff)
            with pinned(aff):
                med_aff, _, _ = timed_runs(lambda: O.speech_features_reference(x1, SR, fca), reps=5)
        res["c1_cpu_baseline"] = {
            "value": F1 / med, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"the whole C1 config: 10 s sweep, {F1} frames; oracle composition of GenerateFingerprint "
                      f"(music -> speech extractor, sr 0): STFT over {threads} threads (Go's worker-pool shape), "
                      "MFCC, descriptors, ZCR, energy, YIN + tracker single-threaded, float64; median of 5 "
                      "after a warm-up", "ms": med * 1e3, "spread_frames_per_s": [F1 / hi, F1 / lo],
            "pinned_cpus": cpus, "stft_threads_at_affinity": aff, "value_at_affinity": F1 / med_aff,
            "ms_at_affinity": med_aff * 1e3, **host_info()}
        par = {"f64": feature_parity(outs["f64"], ref, 1e-6), "f32": feature_parity(outs["f32"], ref, 1e-4)}
        par["f32"]["note"] = ("float32 throughput mode: the spectral descriptors take the float64 transform "
                              "(round 6), so every field, flatness and slope included, is held to 1e-4")
        res["c1_generate_fingerprint"]["parity"] = {
            "inputs": "identical (the same float64 host PCM on both sides), full 10 s",
            "f64": par["f64"], "f32": par["f32"]}
        best_cpu = max(res["c1_cpu_baseline"]["value"], res["c1_cpu_baseline"]["value_at_affinity"])
        for name in ("f64", "f32"):
            res["c1_generate_fingerprint"][name]["x_cpu_baseline"] = (
                res["c1_generate_fingerprint"][name]["frames_per_s"] / best_cpu)
        res["c1_generate_fingerprint"]["x_cpu_baseline_against"] = "the faster of the job-share and affinity-wide CPU runs"
    return res


def c5_cpu_baseline(args):
    """The oracle's alignment of one C5 pair (60 s streams): music-extractor energy + chroma of both
    streams, NCC over the lags, chroma DTW, scorers; float64, 1 thread."""
    O = oracle_module()
    q, r, lag = pairs.c5_pair_device(0, args.c5_seconds, device="cpu")
    q, r = q.numpy(), r.numpy()

    def one_pair():
        feats = []
        for x in (q, r):
            y = O.preemphasis(O.dc_removal(x, 0.995), 0.95)
            e = O.short_time_energy(y, W, H)
            F = O.stft_frames(len(x), W, H)
            feats.append((e, O.chroma_music(x, F, H, SR)))
        O.align_features_reference(feats[0][0], feats[1][0], feats[0][1], feats[1][1], len(q), len(r), SR, SR, H,
                                   args.c5_max_lag)
    with pinned(1) as cpus:
        med, lo, hi = timed_runs(one_pair, reps=5)
    F = O.stft_frames(len(q), W, H)
    return {"value": 1.0 / med, "unit": "pairs/s", "cores": 1, "kind": "port", "frames_per_s": 2 * F / med,
            "sample": f"one C5 pair ({args.c5_seconds:.0f} s streams): oracle music features + NCC + chroma DTW "
                      "+ scorers, float64, 1 thread, median of 5", "spread_pairs_per_s": [1.0 / hi, 1.0 / lo],
            "pinned_cpus": cpus}


def bench_c6(args, ctx, dev):
    """Row f1: FingerprintComparator on a device gallery.
    (1) gallery_add of G C3-sized fingerprints (5 min at 44.1 kHz, 51,676 frames, the speech
        extractor's arrays) already in HBM: the per-fingerprint statistics kernels stream every
        feature element once per pass (HBM roofline);
    (2) BatchCompare of Q queries against a gallery of short fingerprints (one compare thread
        per pair, pairs/s) and with EnableDetailedMetrics against the C3-sized gallery (the
        coherence kernel streams both spectral sequences per pair);
    (3) CPU baseline: the oracle's Compare, which rebuilds the statistics from the full arrays
        on every call as comparison.go does, on a bounded sample of C3-sized pairs, 1 thread."""
    from sonar import compare as cmp
    G, F = args.c6_gallery, args.c6_frames
    buf, structs, per_bytes = cmp.device_features(G, F, dev, seed=6)
    torch.cuda.synchronize()
    g = cmp.Gallery(ctx)
    g.add_raw(structs, min(G, 4), keep_sequences=False, device_ptrs=True)     # warm-up
    g.close()
    res = {}
    adds = []
    for rep in range(args.c6_reps):
        g = cmp.Gallery(ctx)
        ctx.last_kernel_ms()
        ctx.enable_kernel_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.add_raw(structs, G, keep_sequences=False, device_ptrs=True)
        dt = time.perf_counter() - t0
        ctx.enable_kernel_timing(False)
        adds.append((dt, ctx.last_kernel_ms()))
        g.close()
    dt, kms = min(adds, key=lambda x: x[0])
    res["c6_gallery_add"] = {"fingerprints": G, "frames_each": F, "feature_bytes_each": per_bytes,
                             "fingerprints_per_s": G / dt, "ms": dt * 1e3, "colstats_kernel_ms": kms,
                             "roofline": {"bound": "hbm", "kernel": "colstats_kernel+colstats_final_kernel",
                                          "achieved": G * per_bytes / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                          "unit": "GB/s", "frac": G * per_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                          "algorithmic_bytes": "every feature element read once (8 B)"}}
    # detailed-metrics compare on the C3-sized gallery (coherence streams the spectral sequences)
    g = cmp.Gallery(ctx)
    g.add_raw(structs, G, keep_sequences=True, device_ptrs=True)
    cfg = cmp.make_cfg({"similarity_threshold": 0.0, "max_candidates": 50, "enable_detailed_metrics": True})
    q = np.arange(min(8, G))
    g.compare(q, None, cfg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.c6_reps):
        g.compare(q, None, cfg)
    dt = (time.perf_counter() - t0) / args.c6_reps
    npair = len(q) * G
    res["c6_compare_detailed"] = {"queries": len(q), "candidates": G, "pairs_per_s": npair / dt, "ms": dt * 1e3,
                                  "coherence_stream_gbs": npair * 2 * F * 8 / dt / 1e9}
    g.close()
    del buf
    # plain BatchCompare throughput on a large gallery of short fingerprints
    G2, Q2 = args.c6_compare_gallery, args.c6_queries
    buf2, st2, _ = cmp.device_features(G2, 32, dev, seed=7)
    g = cmp.Gallery(ctx)
    g.add_raw(st2, G2, keep_sequences=False, device_ptrs=True)
    cfg = cmp.make_cfg({"similarity_threshold": 0.5, "max_candidates": 50})
    q = np.arange(Q2)
    from sonar._abi import Similarity
    import ctypes
    dout = torch.empty(Q2 * G2 * ctypes.sizeof(Similarity), dtype=torch.uint8, device=dev)
    g.compare_device(q, None, cfg, dout.data_ptr())
    torch.cuda.synchronize()
    ctx.last_kernel_ms()
    ctx.enable_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.c6_reps):
        g.compare_device(q, None, cfg, dout.data_ptr())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.c6_reps
    t2 = time.perf_counter()
    g.compare(q, None, cfg)
    dth = time.perf_counter() - t2
    ctx.enable_kernel_timing(False)
    kms = ctx.last_kernel_ms()
    g.find_best_matches(q, None, cfg)        # warm-up: sort scratch allocation
    t1 = time.perf_counter()
    for _ in range(args.c6_reps):
        g.find_best_matches(q, None, cfg)
    dtm = (time.perf_counter() - t1) / args.c6_reps
    res["c6_compare"] = {"queries": Q2, "candidates": G2, "pairs_per_s": Q2 * G2 / dt, "ms": dt * 1e3,
                         "compare_kernel_ms": kms, "kernel_pairs_per_s": Q2 * G2 / (kms * 1e-3),
                         "host_results_ms": dth * 1e3, "find_best_matches_ms": dtm * 1e3,
                         "note": "ms: results left in HBM (device_ptrs); host_results_ms adds the D2H copy of "
                                 "every SimilarityResult into pageable memory"}
    del dout
    g.close()
    del buf2
    return res


def bench_c7(args, ctx):
    """Row f2: ContentDetector.DetectFromAudio on --c7-seconds of the bench stream
    (float64 host PCM, as GenerateFingerprint hands it over).  kernel_ms = the device passes (scan,
    both frame-sum kernels, the 2048-point direct DFT) by HIP events; ms adds the H2D copy and the
    host reductions.  CPU baseline: the oracle (Go's loops), 1 thread, on the same samples."""
    x = shard.stream_pcm(0, int(args.c7_seconds * SR)).double().numpy()
    ctx.detect_from_audio(x[: SR * 5], SR)        # warm-up
    ctx.last_kernel_ms()
    ctx.enable_kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.c6_reps):
        ct, feats = ctx.detect_from_audio(x, SR)
    dt = (time.perf_counter() - t0) / args.c6_reps
    ctx.enable_kernel_timing(False)
    kms = ctx.last_kernel_ms()
    res = {"samples": len(x), "content_type": ct, "ms": dt * 1e3, "kernel_ms": kms,
           "samples_per_s": len(x) / dt, "kernel_samples_per_s": len(x) / (kms * 1e-3),
           "roofline": {"bound": "hbm", "achieved": len(x) * 8 / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": len(x) * 8 / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes": "8 B per PCM sample (read once)"}}
    out = {"c7_detect_from_audio": res}
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        n = min(len(x), int(SR * 60))
        t0 = time.perf_counter()
        oct_, _ = O.detect_from_audio(x[:n], SR)
        dtc = time.perf_counter() - t0
        out["c7_cpu_baseline"] = {"value": n / dtc, "unit": "samples/s", "cores": 1, "kind": "port",
                                  "sample": f"60 s of the bench stream ({n} samples), oracle DetectFromAudio "
                                            "(Go's loops incl. the O(2048^2) direct DFT), float64, 1 thread"}
        out["c7_detect_from_audio"]["agrees_with_oracle_on_60s"] = ctx.detect_from_audio(x[:n], SR)[0] == oct_
    return out


def c6_cpu_baseline(args):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from sonar import compare as cmp
    F = args.c6_frames
    rng = np.random.default_rng(6)
    Fp = F // 2

    def fp(i):
        d = {"mfcc": np.abs(rng.normal(size=(F, 13))), "spectral": {k: np.abs(rng.normal(size=n)) for k, n in
                                                                     (("centroid", F), ("rolloff", F), ("flux", F - 1))},
             "temporal": {"dynamic_range": 20.0, "silence_ratio": 0.1, "onset_density": 1.0,
                          "rms_energy": np.abs(rng.normal(size=F))},
             "speech": {"speech_rate": 3.0, "vocal_tract_length": 17.5, "voicing_probability": np.abs(rng.normal(size=F))},
             "harmonic": {"harmonic_ratio": np.abs(rng.normal(size=Fp)), "pitch_estimate": np.abs(rng.normal(size=Fp))}}
        return cmp.Fingerprint(f"c{i}", "news", F * 256 / 44100.0, cmp.Features(
            mfcc=d["mfcc"], spectral=d["spectral"], temporal=d["temporal"], speech=d["speech"], harmonic=d["harmonic"]))

    fps = [cmp.marshal(fp(i)) for i in range(4)]
    cfg = cmp.make_cfg({"similarity_threshold": 0.0, "max_candidates": 50})
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.c6_cpu_seconds:
        O.fp_compare(fps[n % 4][0], fps[(n + 1) % 4][0], cfg)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{n} Compare calls on C3-sized fingerprints ({F} frames), oracle recomputing the "
                      "statistics per call as comparison.go does, float64, 1 thread"}


def bench_fp_batch(args, ctx, dev, cfg):
    """sonar_fingerprint_batch (SpectralAnalyzer.ComputeSTFTBatch, spectral.go:234-285) over many short
    device-resident streams with the headline configuration: ONE mfcc_pair_kernel launch for the batch,
    against a loop of per-signal sonar_fingerprint calls (the same kernel, one launch per signal).
    Wall time per batch on the ctx stream, median of --reps; rows checked equal between the two."""
    k, secs = args.batch_signals, args.batch_seconds
    rng = np.random.default_rng(11)
    lens = [int(secs * SR) + int(rng.integers(0, 4096)) for _ in range(k)]
    gen = torch.Generator(device=dev).manual_seed(5)
    sigs = [0.3 * torch.randn(L, device=dev, dtype=torch.float32, generator=gen) for L in lens]
    Fs = [sonar.stft_frames(L, cfg.window_size, cfg.hop_size) for L in lens]
    nc = cfg.n_mfcc
    outs_b = [torch.empty((f, nc), device=dev) for f in Fs]
    outs_s = [torch.empty((f, nc), device=dev) for f in Fs]
    ptrs = [x.data_ptr() for x in sigs]
    pb, ps = [o.data_ptr() for o in outs_b], [o.data_ptr() for o in outs_s]

    def batch():
        ctx.fingerprint_batch_device(ptrs, lens, pb, cfg)

    def loop():
        for p_, L, o in zip(ptrs, lens, ps):
            ctx.fingerprint_device(p_, L, cfg, mfcc=o)

    times = {}
    for name, fn in (("batch", batch), ("loop", loop)):
        fn()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(max(args.reps, 1)):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        times[name] = float(np.median(ts))
    ctx.last_kernel_ms()                     # the batched launch alone, HIP events on the ctx stream
    ctx.enable_kernel_timing(True)
    for _ in range(max(args.reps, 1)):
        batch()
    ctx.enable_kernel_timing(False)
    kms = ctx.last_kernel_ms()
    same = all(torch.equal(a, b) for a, b in zip(outs_b, outs_s))
    Ft = int(sum(Fs))
    return {"fp_batch": {"entry": "sonar_fingerprint_batch", "signals": k, "seconds_per_signal": secs,
                         "frames": Ft, "batch_ms": times["batch"] * 1e3, "batch_frames_per_s": Ft / times["batch"],
                         "batch_kernel_ms": kms, "batch_kernel_frames_per_s": Ft / (kms * 1e-3),
                         "batch_kernel_valu_frac": Ft * FLOPS_PER_FRAME / (kms * 1e-3) / 1e12 / FP32_PEAK_TFS,
                         "loop_ms": times["loop"] * 1e3, "loop_frames_per_s": Ft / times["loop"],
                         "speedup_vs_loop": times["loop"] / times["batch"], "rows_equal_single_calls": bool(same),
                         "note": "device-resident f32 streams, wall time incl. host launch overhead"}}


def bench_ingest(args, ctx, pcm, cfg, F):
    """Row f3: the decoder's f64le byte stream of this rank's hour
    (Decoder.bytesToFloat64, transcode/decoder.go:850-871) from pageable host memory into device
    f32 PCM through sonar_ingest_f64le, then the headline MFCC launch: the PCIe-inclusive
    frames/s.  Both conversion modes, plus a plain pageable torch copy of the f64 bytes + a
    device cast as the naive comparison.  Best of --ingest-reps; not the headline `value`."""
    dev = pcm.device
    x = pcm.double().cpu().numpy()                 # the f64le stream as ffmpeg would hand it over
    n = len(x)
    buf = torch.empty(n, dtype=torch.float32, device=dev)
    mf = torch.empty((F, N_MFCC), dtype=torch.float32, device=dev)

    def timed(fn):
        best = 1e30
        for _ in range(args.ingest_reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    res = {"samples": n, "f64le_bytes": 8 * n, "frames": F}
    naive = timed(lambda: buf.copy_(torch.from_numpy(x).to(dev)))
    res["pageable_torch_copy"] = {"ms": naive * 1e3, "gb_per_s": 8 * n / naive / 1e9}
    for name, mode in (("device_convert", sonar.INGEST_DEVICE_CONVERT), ("host_convert", sonar.INGEST_HOST_CONVERT)):
        ctx.ingest_f64le(x[: 1 << 20], buf.data_ptr(), sonar.F32, mode)       # pinned ring + pool warm-up
        t_in = timed(lambda: ctx.ingest_f64le(x, buf.data_ptr(), sonar.F32, mode))
        exact = bool(torch.equal(buf, pcm))

        def e2e():
            ctx.ingest_f64le(x, buf.data_ptr(), sonar.F32, mode)
            ctx.fingerprint_device(buf.data_ptr(), n, cfg, mfcc=mf.data_ptr())
        t_e2e = timed(e2e)
        res[name] = {"ingest_ms": t_in * 1e3, "f64le_gb_per_s": 8 * n / t_in / 1e9,
                     "pcie_bytes_per_sample": 8 if mode == sonar.INGEST_DEVICE_CONVERT else 4,
                     "end_to_end_ms": t_e2e * 1e3, "end_to_end_frames_per_s": F / t_e2e,
                     "bit_exact_vs_resident_pcm": exact}
    return {"ingest_f64le": res}


def main():
    args = parse()
    world, rank, local = dist_setup()
    dev = torch.device("cuda", local)
    pcm, F_total, F, counts = make_shard(args.seconds, world, rank, dev)
    n = pcm.numel()
    assert sonar.stft_frames(n, W, H) == F
    out = torch.empty((F, N_MFCC), dtype=torch.float32, device=dev)
    ctx = sonar.Context(local)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    cfg = ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=N_MELS, n_mfcc=N_MFCC,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32, flags=sonar.FP_MFCC)

    def step():
        ctx.fingerprint_device(pcm.data_ptr(), n, cfg, mfcc=out.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # then untimed steps until the device has been busy for >= 0.3 s: the first ~0.2 s of GPU work
    # in a fresh process runs at ramping clocks (round 4: 20 steps after 5 warm-ups timed 0.46 ms
    # per launch, 200 after 20 timed 0.43 ms on the same build), and the timed K steps are ~10 ms
    warm_extra, tw = 0, time.perf_counter()
    while time.perf_counter() - tw < 0.3:
        for _ in range(16):
            step()
        warm_extra += 16
        torch.cuda.synchronize()
    ctx.last_kernel_ms()              # drop warm-up event pairs
    ctx.enable_kernel_timing(True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    ctx.enable_kernel_timing(False)
    kernel_ms = ctx.last_kernel_ms()
    kernel_name = ctx.last_fp_kernel()
    elapsed = max_over_ranks(elapsed, world)
    ms_per_step = elapsed / args.steps * 1e3
    value = F_total / (elapsed / args.steps)

    # RCCL all-gather of the MFCC timeline (reassembly of the frame-sharded stream
    # over xGMI), once, outside the timed region
    gather_ms = None
    if world > 1:
        torch.cuda.synchronize()
        barrier(world)
        tg = time.perf_counter()
        timeline = shard.gather_rows(out, world, counts)
        torch.cuda.synchronize()
        gather_ms = max_over_ranks((time.perf_counter() - tg) * 1e3, world)
        assert timeline.shape == (F_total, N_MFCC)
        f0 = sum(counts[:rank])
        assert torch.equal(timeline[f0:f0 + F], out)
        if args.dump_dir and rank == 0:
            np.save(os.path.join(args.dump_dir, "mfcc_timeline.npy"), timeline.cpu().numpy())

    # every leg after the headline is wrapped: its exception is recorded as "<leg>_error" in the
    # line (which is still printed) and the process exits non-zero.  Legs with collectives (C5)
    # catch their own errors inside, so the ranks' collective sequences stay aligned.
    extra, errors = {}, {}

    def leg(name, fn):
        try:
            r_ = fn()
            if r_:
                extra.update(r_)
        except Exception as e:  # noqa: BLE001 -- recorded in the line, exit status non-zero
            errors[f"{name}_error"] = f"{type(e).__name__}: {e}"
            traceback.print_exc(file=sys.stderr)

    out64 = None
    if not args.no_f64:
        def f64_leg():
            nonlocal out64
            res, out64 = bench_headline_f64(args, ctx, pcm, F, dev)
            return {"headline_f64": res}
        leg("headline_f64", f64_leg)
    cpu, parity = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        def cpu_leg():
            nonlocal cpu, parity
            cpu, parity, parity64 = cpu_baseline(args.cpu_seconds, out.cpu().numpy(), pcm.cpu().numpy(), out64)
            if parity64 is not None and "headline_f64" in extra:
                extra["headline_f64"]["parity"] = parity64
        leg("cpu_baseline", cpu_leg)
    if args.c1:
        leg("c1", lambda: bench_c1(args, ctx))
    if args.dtw_len > 0:
        leg("dtw", lambda: bench_dtw(ctx, args.dtw_len, args.dtw_steps,
                                     parity=rank == 0 and world == 1 and not args.no_cpu_baseline))
    if args.ingest_reps > 0:
        leg("ingest", lambda: bench_ingest(args, ctx, pcm, cfg, F))
    if args.batch_signals > 0:
        leg("fp_batch", lambda: bench_fp_batch(args, ctx, dev, cfg))
    if args.c5_pairs > 0:
        # the earlier legs' device buffers (the hour's |X| scratch, the C3 DTW's codes and
        # checkpoints: several GB) are released first, so C5 runs in the memory state it has alone
        ctx.trim()
        torch.cuda.empty_cache()
        leg("c5", lambda: bench_c5(args, world, rank, dev, ctx))
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            leg("c5_cpu_baseline", lambda: {"c5_cpu_baseline": c5_cpu_baseline(args)})
    if args.c3_seconds > 0:
        leg("c3", lambda: bench_c3(args, ctx, dev))
    if args.c4_seconds > 0:
        leg("c4", lambda: bench_c4(args, ctx))
    if args.c6_gallery > 0:
        leg("c6", lambda: bench_c6(args, ctx, dev))
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            leg("c6_cpu_baseline", lambda: {"c6_cpu_baseline": c6_cpu_baseline(args)})
    if args.c7_seconds > 0:
        leg("c7", lambda: bench_c7(args, ctx))
    if "c5_error" in extra:
        errors["c5_error"] = extra["c5_error"]

    achieved_gbs = F * BYTES_PER_FRAME / (kernel_ms * 1e-3) / 1e9
    achieved_tfs = F * FLOPS_PER_FRAME / (kernel_ms * 1e-3) / 1e12
    traffic, traffic_src = load_traffic(kernel_name)
    line = {
        "metric": "audio frames/sec (STFT->MFCC, 1024/256)",
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_extra_steps": warm_extra,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic C2-shaped stream (10 s 100 Hz-10 kHz sweep repeated + 0.05 N(0,1) from a "
                "counter hash), N x 1 h, frame-sharded with halo",
        "config": {"workload": "STFT(W=1024,H=256,Hann)->mel(40)->ln->DCT-II(13)->lifter(22) on 1 h of "
                               "44.1 kHz float32 PCM per GPU", "frames_total": F_total, "frames_rank0": F,
                   "samples_rank0": n, "parallelism": f"frame-shard x{world}"},
        # 31,136 flop/frame against 1,076 B/frame is above the FP32 ridge, so the
        # binding roof is the FP32 VALU (157.3 TF); the north star's HBM figure is kept beside it
        "roofline": {"bound": "valu", "achieved": achieved_tfs, "peak": FP32_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": achieved_tfs / FP32_PEAK_TFS,
                     "traffic": traffic, "traffic_source": traffic_src, "kernel": kernel_name, "kernel_ms": kernel_ms,
                     "algorithmic_flops_per_frame": FLOPS_PER_FRAME, "algorithmic_bytes_per_frame": BYTES_PER_FRAME,
                     "hbm_achieved_gbs": achieved_gbs, "hbm_peak_gbs": HBM_PEAK_GBS,
                     "hbm_frac": achieved_gbs / HBM_PEAK_GBS},
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if gather_ms is not None:
        line["allgather_ms"] = gather_ms
        line["allgather_bytes"] = F_total * N_MFCC * 4
    line.update(extra)
    line.update(errors)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    if errors:
        sys.exit(1)


if __name__ == "__main__":
    main()
