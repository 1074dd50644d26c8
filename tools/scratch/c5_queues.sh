# C5 throughput vs hardware queues per process (GPU_MAX_HW_QUEUES) and worker streams
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_alignment.py tests/test_gpu_pairs.py tests/test_gpu_pitch_chroma.py tests/test_gpu_golden.py tests/test_gpu_go_api.py > gpurun_out/q_tests.log 2>&1 || exit 1
for qw in "16 16" "32 32" "32 24" "16 24"; do
  set -- $qw
  echo -n "queues $1 workers $2: "
  timeout -k 10 300 python -u bench.py --steps 3 --dtw-len 0 --c6-gallery 0 --c7-seconds 0 --c3-seconds 0 --c4-seconds 0 --no-cpu-baseline --hw-queues $1 --c5-workers $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['c5_pairs_per_s'], d['c5_lag_recovered'])" || exit 1
done
