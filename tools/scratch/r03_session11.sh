#!/bin/bash
# C5 (1 rep after a warm-up) under rocprofv3 --kernel-trace; per-queue timeline summary on the box
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
OUT="$R/gpurun_out/r03s11"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SONAR_DTW_BATCH_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/c5_stress.py" --reps 1 > "$OUT/c5.jsonl" 2> "$OUT/c5.err" || { echo "trace failed"; tail -5 "$OUT/c5.err"; exit 1; }
F=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/scratch/c5_timeline.py" "$F" > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
rm -f "$F"
python3 - "$OUT/c5.err" <<'PY'
import json, sys
L=[json.loads(l)["dtw_batch_trace"] for l in open(sys.argv[1]) if l.startswith('{"dtw_batch_trace"')]
half=L[len(L)//2:]   # the timed repetition (the warm-up run's batches come first)
b=sum(x["band_us"] for x in half); f=sum(x["first_wait_us"] for x in half); sp=sum(x["spin_us"] for x in half)
print("batches", len(half), "band-time s", round(b/1e6,3), "compute share", round(1-(f+sp)/b,3), "ns/step compute", round((b-f-sp)*1e3/sum(x["steps"] for x in half),1))
PY
tail -1 "$OUT/c5.jsonl" | cut -c1-120
