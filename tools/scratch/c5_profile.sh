set -o pipefail
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pitch_chroma.py tests/test_gpu_pairs.py tests/test_gpu_golden.py > gpurun_out/c_tests.log 2>&1 || exit 1
for w in 8 16; do
  timeout -k 10 300 python -u bench.py --steps 3 --dtw-len 0 --c6-gallery 0 --c7-seconds 0 --c3-seconds 0 --c4-seconds 0 --no-cpu-baseline --c5-workers $w > gpurun_out/bench_c5w$w.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c5trace" -o run -- python3 "$R/bench.py" --steps 3 --dtw-len 0 --c6-gallery 0 --c7-seconds 0 --c3-seconds 0 --c4-seconds 0 --no-cpu-baseline --c5-pairs 200 > "$R/gpurun_out/c5trace.log" 2>&1
