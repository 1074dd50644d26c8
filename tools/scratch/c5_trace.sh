#!/bin/bash
# rocprofv3 kernel-trace stats of the C5 bench leg alone (path B kernels), then two plain C5 lines.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
TAG=${1:-c5}; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
C5="--steps 2 --warmup 1 --dtw-len 0 --c6-gallery 0 --c7-seconds 0 --c3-seconds 0 --c4-seconds 0 --ingest-reps 0 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" $C5 > "$OUT/traced.json" 2> "$OUT/traced.err" || { echo "trace failed"; exit 1; }
for i in 1 2 3; do
  timeout -k 10 200 python3 "$R/bench.py" $C5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['c5_pairs_per_s'],1))" || exit 1
done
