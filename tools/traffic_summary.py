"""Turn a tools/profile_round.sh output directory into the committed profiles/<tag>_*.

profiles/<tag>_kernel_stats.csv : rocprofv3 --kernel-trace --stats summary of `python3 bench.py`
profiles/<tag>_traffic.json     : per-launch HBM bytes of the fused kernel from FETCH_SIZE/WRITE_SIZE
Units/corrections per MI355X_MICROARCH.md "HBM": counters are KiB; on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced streaming reads, so it is doubled."""
import csv, glob, json, os, shutil, sys, collections

src, tag = sys.argv[1], sys.argv[2]
pat = sys.argv[3] if len(sys.argv) > 3 else "mfcc_pair_kernel"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)

stats = glob.glob(f"{src}/trace/**/*kernel_stats.csv", recursive=True)
shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
trace = glob.glob(f"{src}/trace/**/*kernel_trace.csv", recursive=True)
durs = collections.defaultdict(list)
if trace:
    for r in csv.DictReader(open(trace[0])):
        durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
else:   # the per-dispatch CSV is dropped on the box (size): average and count from the stats summary
    for r in csv.DictReader(open(stats[0])):
        n = int(r["Calls"])
        durs[r["Name"]] = [float(r["AverageNs"]) / 1e6] * n

per = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(float)
    name = None
    for f in glob.glob(f"{src}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] == c:
                acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
                name = r["Kernel_Name"]
    v = sorted(acc.values())
    per[c] = {"kernel": name, "dispatches": len(v), "kib_per_dispatch_mean": sum(v) / len(v),
              "kib_per_dispatch_min": v[0], "kib_per_dispatch_max": v[-1]}
fetch = per["FETCH_SIZE"]["kib_per_dispatch_mean"] * 1024 * 2      # gfx950 half-count correction
write = per["WRITE_SIZE"]["kib_per_dispatch_mean"] * 1024
kname = next(k for k in durs if pat in k)
out = {"tag": tag, "kernel": kname,
       "kernel_trace_avg_ms": sum(durs[kname]) / len(durs[kname]), "kernel_trace_launches": len(durs[kname]),
       "fetch_bytes_per_launch_corrected": fetch, "write_bytes_per_launch": write,
       "hbm_bytes_per_launch": fetch + write,
       "raw": per,
       "note": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB -> bytes; separate --pmc passes"}
json.dump(out, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
