#!/usr/bin/env python3
"""Group a rocprofv3 kernel-stats CSV of a C5 run (bench.py with only the C5 leg, or
tools/c5_stress.py) into kernel families and write their GPU-time shares as JSON.

    python3 tools/c5_families.py <kernel_stats.csv> <out.json> [--note TEXT]

The shares are of summed kernel durations (kernels of the 16 worker streams overlap, so the sum
exceeds the wall time): what fraction of the GPU's kernel time each family holds.  bench.py puts
the newest profiles/*_c5_families.json into the line's c5_roofline."""
import csv
import json
import re
import sys

FAMILIES = [                       # first match wins
    ("features", r"dc_block_kernel|dc_carry_kernel|dc_pass_kernel|energy_|chroma_wave_kernel|chroma_kernel"),
    ("ncc", r"ncc_"),
    ("dtw_band", r"dtw_band_kernel"),
    ("dtw_walk", r"dtw_exit_map_kernel|dtw_walk_"),
    ("dtw_path", r"dtw_path_|dtw_tile"),
    ("probe_and_fill", r"nonfinite_"),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def main():
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    src, dst = sys.argv[1], sys.argv[2]
    note = sys.argv[sys.argv.index("--note") + 1] if "--note" in sys.argv else ""
    tot = {}
    calls = {}
    kernels = {}
    with open(src) as f:
        for row in csv.DictReader(f):
            fam = family(row["Name"])
            ns = float(row["TotalDurationNs"])
            tot[fam] = tot.get(fam, 0.0) + ns
            calls[fam] = calls.get(fam, 0) + int(row["Calls"])
            short = re.sub(r"\(.*", "", row["Name"]).replace("void ", "")
            kernels.setdefault(fam, []).append({"kernel": short, "calls": int(row["Calls"]), "total_ms": ns / 1e6})
    all_ns = sum(tot.values())
    out = {"source": src, "note": note, "total_kernel_ms": all_ns / 1e6,
           "families": {k: {"total_ms": v / 1e6, "share": v / all_ns, "calls": calls[k],
                            "kernels": sorted(kernels[k], key=lambda r: -r["total_ms"])}
                        for k, v in sorted(tot.items(), key=lambda kv: -kv[1])}}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in out["families"].items():
        print(f"{k:16s} {v['total_ms']:10.1f} ms  {100 * v['share']:5.1f} %  ({v['calls']} calls)")


if __name__ == "__main__":
    main()
