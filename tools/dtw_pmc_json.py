"""Summarise tools/pmc_run.sh passes over tools/dtw_probe.py into profiles/<tag>_dtw_pmc.json.

For every kernel whose name contains one of the patterns, the counters of its LAST dispatch in
each pass (dtw_probe.py's final call: the full-size C3 DTW) and that dispatch's duration.  Units
per MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE in KiB; FETCH_SIZE counts wide coalesced
reads at half their bytes on gfx950, so bench.py's load_pmc_bytes doubles it.

Usage: python tools/dtw_pmc_json.py gpurun_out/pmc_<tag> <tag> [pattern ...]
"""
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
pats = sys.argv[3:] or ["dtw_band_kernel", "dtw_band2_kernel", "dtw_walk", "dtw_exit_map", "dtw_path"]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
kern = {}
for p in sorted(glob.glob(f"{src}/p*/")):
    rows = {}
    for f in glob.glob(f"{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(s in name for s in pats):
                continue
            d = rows.setdefault(name, {}).setdefault(int(r["Dispatch_Id"]), {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tag_p = os.path.basename(os.path.normpath(p))
    for name, disp in rows.items():
        last = disp[max(disp)]
        k = kern.setdefault(name.split("(")[0].replace("sonar::", "").replace("void ", ""), {})
        for c, v in last.items():
            k[f"ms_{tag_p}" if c == "_ms" else c] = v
out = {"source": f"rocprofv3 --pmc passes (tools/pmc_run.sh) over tools/dtw_probe.py, last dispatch of each "
                 f"kernel per pass (the full-size call); FETCH_SIZE / WRITE_SIZE in KiB (FETCH_SIZE x2 for the "
                 f"gfx950 half count)", "tag": tag, "kernels": kern}
json.dump(out, open(os.path.join(root, "profiles", f"{tag}_dtw_pmc.json"), "w"), indent=1)
for name, k in kern.items():
    if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        print(name, "HBM bytes/launch", (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024)
