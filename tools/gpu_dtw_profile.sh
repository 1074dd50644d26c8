# DTW / C5 profile at HEAD: the band-pipeline PMC passes over one C3-size DTW (tools/pmc_run.sh over
# tools/dtw_probe.py, summarised locally by tools/dtw_pmc_json.py) and a kernel-trace of one C5 call
# (tools/c5_stress.py --reps 1, summarised by tools/c5_families.py).
# Usage (GPU box): bash tools/gpu_dtw_profile.sh <tag>
set -o pipefail
TAG=${1:-r05}
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R" || exit 1
mkdir -p gpurun_out
ITERS=1 bash tools/pmc_run.sh "${TAG}_dtw" tools/dtw_probe.py || exit 1
OUT="$R/gpurun_out/c5trace_$TAG"; mkdir -p "$OUT"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/tools/c5_stress.py" --reps 1 --out "$OUT/c5.jsonl" > "$OUT/c5.log" 2>&1) || { echo "c5 trace failed"; exit 1; }
rm -f "$OUT"/*/*_kernel_trace.csv "$OUT"/*_kernel_trace.csv
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
cp "$f" "gpurun_out/${TAG}_c5_kernel_stats.csv"
echo "c5 trace done"
