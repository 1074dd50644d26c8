#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the default bench command,
# separate FETCH_SIZE / WRITE_SIZE PMC passes (never combined with trace domains),
# then the plain bench line.  Usage: bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" > "$OUT/bench_traced.log" 2>&1 || { echo "trace pass failed"; exit 1; }
rm -f "$OUT"/trace/*_kernel_trace.csv   # per-dispatch rows: tens of MB, the stats CSV is the summary
echo "trace done"
# the headline alone under the tracer, 200 timed steps after 20 warm-up steps: the stats average is
# then steady-state launches only, and the same traced run's own JSON line (its HIP-event
# kernel_ms and ms_per_step) is the like-for-like comparison
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/hl_trace" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 --steps 200 --warmup 20 > "$OUT/hl_traced.json" 2> "$OUT/hl_traced.err" || { echo "headline trace failed"; exit 1; }
rm -f "$OUT"/hl_trace/*_kernel_trace.csv
f=$(find "$OUT/hl_trace" -name '*kernel_stats.csv' | head -1)
cp "$f" "$R/gpurun_out/${TAG}_headline_kernel_stats.csv"; cp "$OUT/hl_traced.json" "$R/gpurun_out/${TAG}_headline_traced.json"
echo "headline trace done"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o run -- \
      python3 "$R/bench.py" --no-cpu-baseline --dtw-len 0 --c5-pairs 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 --no-f64 --c3-seconds 0 --c4-seconds 0 --steps 5 --warmup 1 > "$OUT/$c.log" 2>&1 \
      || { echo "pmc $c failed"; exit 1; }
  echo "$c done"
done
# per-launch HBM bytes -> profiles/<tag>_traffic.json (read by bench.py's roofline.traffic); the
# PMC and headline-trace runs skip the fp_batch leg, whose 1000 per-signal launches share the kernel's name
(cd "$R" && python3 tools/traffic_summary.py "$OUT" "$TAG" mfcc_pair > "$OUT/traffic_summary.log") \
    || { echo "traffic summary failed"; exit 1; }
timeout -k 10 600 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; exit 1; }
cat "$OUT/bench.json"
cp "$OUT/bench.json" "$R/profiles/${TAG}_bench.json"
