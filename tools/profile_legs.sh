#!/bin/bash
# Kernel-trace summaries of the bench's legs in isolation (so one kernel's average is not mixed with
# another leg's launches): the C3-size DTW alone, the C5 pairs alone.  Usage: bash tools/profile_legs.sh <tag>
set -o pipefail
TAG=${1:-r02}
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
OUT="$R/gpurun_out/legs_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
NOLEGS="--no-cpu-baseline --no-f64 --ingest-reps 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dtw" -o run -- \
    python3 "$R/bench.py" $NOLEGS --c5-pairs 0 --dtw-steps 3 > "$OUT/dtw.json" 2> "$OUT/dtw.err" || { echo "dtw trace failed"; exit 1; }
rm -f "$OUT"/dtw/*_kernel_trace.csv
echo "dtw trace done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o run -- \
    python3 "$R/bench.py" $NOLEGS --dtw-len 0 --reps 1 > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo "c5 trace failed"; exit 1; }
rm -f "$OUT"/c5/*_kernel_trace.csv
echo "c5 trace done"
