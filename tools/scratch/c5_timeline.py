#!/usr/bin/env python3
"""Per-queue timeline summary of a C5 run's rocprofv3 kernel trace (diagnostics only).
Usage: python tools/scratch/c5_timeline.py <kernel_trace.csv>
For each queue: time in DTW sweep kernels, in the feature / NCC kernels, in walk / path kernels,
in runtime copy/fill kernels, and the gaps between one kernel's end and the next one's start on that
queue (host submission, synchronisation, scorers); plus the chip-wide DTW concurrency."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
k0 = rows[0].keys()
qkey = next(k for k in ("Queue_Id", "Stream_Id", "Queue_ID") if k in k0)


def cat(name):
    if "dtw_wave_kernel" in name or "dtw_band_kernel" in name or "dtw_band2_kernel" in name:
        return "dtw"
    if any(x in name for x in ("dc_pass", "dc_carry", "energy", "chroma", "ncc_")):
        return "feat"
    if "dtw_" in name or "nonfinite" in name:
        return "walk"
    if "rocclr" in name or "Fill" in name or "fill" in name:
        return "copy"
    return "other"


# the C5 window: dispatches of queues that ran DTW kernels (the worker streams)
wq = {r[qkey] for r in rows if cat(r["Kernel_Name"]) == "dtw"}
rows = [r for r in rows if r[qkey] in wq]
byname = defaultdict(list)
for r in rows:
    byname[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
byq = defaultdict(list)
for r in rows:
    byq[r[qkey]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cat(r["Kernel_Name"]), r["Kernel_Name"]))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
print(f"span {(t1 - t0) / 1e6:.1f} ms, {len(rows)} dispatches, {len(byq)} queues")
tot = defaultdict(float)
for q, ev in sorted(byq.items()):
    ev.sort()
    acc = defaultdict(float)
    gap = 0.0
    for k, (s, e, c, n) in enumerate(ev):
        acc[c] += e - s
        if k:
            gap += max(0, s - ev[k - 1][1])
    span = ev[-1][1] - ev[0][0]
    for c in acc:
        tot[c] += acc[c]
    tot["gap"] += gap
    tot["span"] += span
    if len(ev) > 50:
        print(f"q{q}: n={len(ev)} span {span / 1e6:.1f} ms  " + "  ".join(f"{c} {acc[c] / span:.2f}" for c in sorted(acc)) + f"  gaps {gap / span:.2f}")
print("all queues (fraction of summed queue spans): " + "  ".join(f"{c} {tot[c] / tot['span']:.3f}" for c in sorted(tot) if c != "span"))
# chip-wide number of DTW kernels in flight over time
ev = sorted([(s, 1) for q in byq for (s, e, c, n) in byq[q] if c == "dtw"] + [(e, -1) for q in byq for (s, e, c, n) in byq[q] if c == "dtw"])
cur, last, hist = 0, t0, defaultdict(float)
for t, d in ev:
    hist[cur] += t - last
    cur += d
    last = t
hist[cur] += t1 - last
print("DTW kernels in flight (share of span): " + "  ".join(f"{k}:{v / (t1 - t0):.3f}" for k, v in sorted(hist.items())))
print("kernels by total time (worker queues):")
for nm, d in sorted(byname.items(), key=lambda kv: -sum(kv[1]))[:16]:
    print(f"  {sum(d) / 1e6:9.1f} ms  n={len(d):6d}  mean {sum(d) / len(d) / 1e3:8.1f} us  {cat(nm):5s} {nm[:90]}")
