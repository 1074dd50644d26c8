# GenerateFingerprint at hour scale: the changed GPU tests, the plain probe,
# the probe under a kernel + memory-copy trace (timeline), and SQ / traffic PMC passes over a
# 10-minute probe (the float64 transform, spec_rows_kernel and yin_kernel).  Summaries go to gpurun_out/<tag>_*.
# Usage (GPU box): bash tools/gpu_gf_profile.sh <tag> [tests...]
set -o pipefail
TAG=${1:-r06a}; shift
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R" || exit 1
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit 1; }
fi
timeout -k 10 300 python3 tools/gf_hour_probe.py 3600 3 > gpurun_out/${TAG}_gf_probe.json 2> gpurun_out/${TAG}_gf_probe.err \
  || { echo "probe failed"; tail -5 gpurun_out/${TAG}_gf_probe.err; exit 1; }
cat gpurun_out/${TAG}_gf_probe.err
OUT="$R/gpurun_out/gf_$TAG"; mkdir -p "$OUT"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$OUT/trace" -o run -- python3 "$R/tools/gf_hour_probe.py" 3600 2 > "$OUT/probe_traced.json" 2> "$OUT/probe_traced.err") \
  || { echo "trace failed"; tail -5 "$OUT/probe_traced.err"; exit 1; }
python3 tools/gf_timeline.py "$OUT/probe_traced.json" "$OUT/trace" > gpurun_out/${TAG}_gf_timeline.json || exit 1
f=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${TAG}_gf_kernel_stats.csv
rm -f "$OUT"/trace/*/*_kernel_trace.csv "$OUT"/trace/*_kernel_trace.csv
echo "timeline done"
ITERS=1 timeout -k 10 900 bash tools/pmc_run.sh "${TAG}_gf" tools/gf_hour_probe.py 600 1 || exit 1
for k in "fp_wave_kernel<double, double, 8, false" spec_rows_kernel yin_kernel; do
  python3 tools/pmc_summary.py "gpurun_out/pmc_${TAG}_gf" "$k"
done > gpurun_out/${TAG}_gf_pmc.txt
echo "pmc done"
