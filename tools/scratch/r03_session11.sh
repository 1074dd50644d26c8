#!/bin/bash
# C5 (1 rep after a warm-up) under rocprofv3 --kernel-trace; per-queue timeline summary on the box
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
OUT="$R/gpurun_out/r03s11"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/c5_stress.py" --reps 1 > "$OUT/c5.jsonl" 2> "$OUT/c5.err" || { echo "trace failed"; tail -5 "$OUT/c5.err"; exit 1; }
F=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/scratch/c5_timeline.py" "$F" > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
rm -f "$F"
