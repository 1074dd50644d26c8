"""Summarise rocprofv3 --pmc CSVs: per-dispatch average of every counter for kernels matching a pattern."""
import csv, glob, json, sys, collections
root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "fp_wave_kernel")
acc = collections.defaultdict(list)
dur = []
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES" or r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "GRBM_GUI_ACTIVE"):
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for (d, c), v in per.items():
        acc[c].append(v)
out = {c: sum(v) / len(v) for c, v in acc.items()}
out["_dispatches_per_pass"] = {c: len(v) for c, v in acc.items()}
print(json.dumps(out, indent=1))
