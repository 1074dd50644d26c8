"""Attribute every millisecond of the GenerateFingerprint calls of tools/gf_hour_probe.py:
reads the probe's JSON (call stamps) and a rocprofv3 --kernel-trace --memory-copy-trace output
directory (CSV), and prints per call: each kernel / copy (start, duration, relative to the call),
the union of device-busy time, and the host-only remainder.
Usage: python tools/gf_timeline.py probe.json trace_dir > timeline.json"""
import csv
import glob
import json
import os
import sys


def rows(d, suffix):
    out = []
    for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("sonar::", "")[:60]


probe = json.load(open(sys.argv[1]))
d = sys.argv[2]
ops = []
for r in rows(d, "kernel_trace.csv"):
    ops.append(("kernel", short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for r in rows(d, "memory_copy_trace.csv"):
    ops.append(("copy", r.get("Direction", "copy"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
ops.sort(key=lambda o: o[2])
report = []
for c in probe["calls"]:
    t0, t1, t2 = c["t0_ns"], c["t_c_ns"], c["t_py_ns"]
    inside = [o for o in ops if o[3] > t0 and o[2] < t1]
    # union of device-busy intervals
    busy, cur = 0, None
    for o in sorted(inside, key=lambda o: o[2]):
        s, e = max(o[2], t0), min(o[3], t1)
        if cur is None or s > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        busy += cur[1] - cur[0]
    agg = {}
    for o in inside:
        k = f"{o[0]}:{o[1]}"
        a = agg.setdefault(k, {"n": 0, "ms": 0.0, "first_start_ms": (o[2] - t0) / 1e6})
        a["n"] += 1
        a["ms"] += (o[3] - o[2]) / 1e6
        a["last_end_ms"] = (o[3] - t0) / 1e6
    last_dev = max((o[3] for o in inside), default=t0)
    report.append({"precision": c["precision"], "rep": c["rep"], "c_call_ms": c["c_call_ms"],
                   "py_result_ms": c["py_result_ms"], "device_busy_union_ms": busy / 1e6,
                   "host_only_ms": c["c_call_ms"] - busy / 1e6,
                   "after_last_device_op_ms": (t1 - last_dev) / 1e6,
                   "ops": dict(sorted(agg.items(), key=lambda kv: kv[1]["first_start_ms"]))})
print(json.dumps(report, indent=1))
