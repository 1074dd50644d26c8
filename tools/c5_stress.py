#!/usr/bin/env python3
"""Repeat the bench's C5 leg (sonar_align_pairs over 1000 device-resident 60 s pairs, 128 in
flight = 16 streams x batches of 8) --reps times and report, per repetition, the wall time, the
band pipeline's liveness counters (sonar_dtw_counters: edge refresh fences, fences followed by new
edge values, timed-out DTWs / waves) and the failure text of any pair whose pipeline timed out
(its diagnostic record, see DtwArgs::diag).  One JSON line per call (the warm-up included), then a
summary line, on stdout and APPENDED to --out (every call's record is kept across runs and variants:
a timeout's role, band and ticket survive the next run).  The library's single-pair redo of a
timed-out band pipeline is off unless --retry 1 (SONAR_PAIR_RETRY), so a timeout fails the call.

Usage: python tools/c5_stress.py [--reps 40] [--pairs 1000] [--seconds 60] [--out gpurun_out/c5_stress.jsonl]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import torch  # noqa: E402

import sonar  # noqa: E402
from sonar import pairs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--pairs", type=int, default=1000)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--workers", type=int, default=128)
    ap.add_argument("--retry", default="0", help="SONAR_PAIR_RETRY for the run (0: a timeout fails the call)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c5_stress.jsonl"),
                    help="JSON lines appended here too ('' = stdout only)")
    ap.add_argument("--tag", default="", help="label stored in every line (variant name)")
    a = ap.parse_args()
    os.environ["SONAR_PAIR_RETRY"] = a.retry
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)

    def emit(d):
        d = {"tag": a.tag, "pid": os.getpid(), "time": time.time(), **d}
        line = json.dumps(d)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
    ctx = sonar.Context(0)
    data = [pairs.c5_pair_device(k, a.seconds, device="cuda") for k in range(a.pairs)]
    torch.cuda.synchronize()
    qp, rp = [q.data_ptr() for q, _, _ in data], [r.data_ptr() for _, r, _ in data]
    nq, nr = [q.numel() for q, _, _ in data], [r.numel() for _, r, _ in data]

    def run():
        return ctx.align_pairs(qp, rp, nq=nq, nr=nr, max_lag_seconds=20.0, workers=a.workers, device_ptrs=True)

    def counters():
        try:
            return ctx.dtw_counters(reset=True)
        except AttributeError:               # an A/B build of an earlier round
            return {}

    t0 = time.perf_counter()
    werr = None
    try:
        run()
    except sonar.SonarError as e:
        werr = str(e)
    emit({"warmup": True, "s": round(time.perf_counter() - t0, 4), **counters(), "error": werr})
    fails, tot = 0, {}
    for i in range(a.reps):
        t0 = time.perf_counter()
        err = None
        try:
            run()
        except sonar.SonarError as e:
            err = str(e)
            fails += 1
        dt = time.perf_counter() - t0
        c = counters()
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        emit({"rep": i, "s": round(dt, 4), "pairs_per_s": round(a.pairs / dt, 1), **c, "error": err})
    emit({"summary": True, "reps": a.reps, "failed_reps": fails, "warmup_failed": werr is not None, **tot})
    ctx.close()


if __name__ == "__main__":
    main()
