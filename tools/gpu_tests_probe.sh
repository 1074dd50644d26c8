# The named GPU tests, then the plain GenerateFingerprint hour probe (tools/gf_hour_probe.py) and,
# with PROF=1, its kernel + memory-copy timeline (tools/gf_timeline.py).
# Usage (GPU box): [PROF=1] bash tools/gpu_tests_probe.sh <tag> [tests...]
set -o pipefail
TAG=${1:-r06}; shift
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R" || exit 1
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -40; exit 1; }
fi
timeout -k 10 300 python3 tools/gf_hour_probe.py 3600 3 > gpurun_out/${TAG}_gf_probe.json 2> gpurun_out/${TAG}_gf_probe.err \
  || { echo "probe failed"; tail -5 gpurun_out/${TAG}_gf_probe.err; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_gf_probe.err
if [ "$PROF" = 1 ]; then
  OUT="$R/gpurun_out/gf_$TAG"; mkdir -p "$OUT"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
      -d "$OUT/trace" -o run -- python3 "$R/tools/gf_hour_probe.py" 3600 2 > "$OUT/probe_traced.json" 2> "$OUT/probe_traced.err") \
    || { echo "trace failed"; tail -5 "$OUT/probe_traced.err"; exit 1; }
  python3 tools/gf_timeline.py "$OUT/probe_traced.json" "$OUT/trace" > gpurun_out/${TAG}_gf_timeline.json || exit 1
  f=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${TAG}_gf_kernel_stats.csv
  rm -f "$OUT"/trace/*/*_kernel_trace.csv "$OUT"/trace/*_kernel_trace.csv
  echo "timeline done"
fi
