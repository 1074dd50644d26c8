set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for t in claim1024 prio; do
  SONAR_LIB=$PWD/sonido-sonar_amd/lib_$t/libsonar_gpu.so timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py > gpurun_out/r04i_tests_$t.log 2>&1
  rc=$?
  echo "tests $t: $(tail -1 gpurun_out/r04i_tests_$t.log)"
  [ $rc -le 1 ] || { echo "test run ended with rc=$rc"; tail -20 gpurun_out/r04i_tests_$t.log; exit 1; }
done
for t in default claim256 claim1024 prio default claim1024 claim256 prio; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04i_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; tail -3 gpurun_out/r04i_c5_$t.jsonl; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*\|"dtw_timeouts": [0-9]*' gpurun_out/r04i_c5_$t.jsonl | tr '\n' ' ')"
done
rm -f gpurun_out/r04i_trace.bin
SONAR_DTW_TRACE=$PWD/gpurun_out/r04i_trace.bin SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/sonido-sonar_amd/lib_claim1024/libsonar_gpu.so timeout -k 10 150 python3 tools/c5_stress.py --reps 1 > gpurun_out/r04i_c5_traced.jsonl 2>/dev/null || { echo "c5 trace fail"; exit 1; }
python3 tools/dtw_batch_trace.py gpurun_out/r04i_trace.bin 10396 | tee gpurun_out/r04i_trace_summary.txt
rm -f gpurun_out/r04i_trace.bin
