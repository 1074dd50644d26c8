set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_dtw_walk.py > gpurun_out/r04j_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/r04j_tests.log)"; [ $rc -le 1 ] || exit 1
rm -f gpurun_out/r04j_trace.bin
SONAR_DTW_TRACE=$PWD/gpurun_out/r04j_trace.bin SONAR_PAIR_RETRY=0 timeout -k 10 150 python3 tools/c5_stress.py --reps 1 > gpurun_out/r04j_c5_traced.jsonl 2>/dev/null || { echo "c5 trace fail"; exit 1; }
python3 tools/dtw_batch_trace.py gpurun_out/r04j_trace.bin 10396 | tee gpurun_out/r04j_trace_summary.txt
rm -f gpurun_out/r04j_trace.bin
