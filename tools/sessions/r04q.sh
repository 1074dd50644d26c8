set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_dtw_walk.py tests/test_gpu_dtw_checkpoint.py tests/test_gpu_pairs.py tests/test_gpu_alignment.py tests/test_gpu_dist.py > gpurun_out/r04q_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/r04q_tests.log)"; [ $rc -le 1 ] || exit 1
for t in prev default prev default prev default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04q_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*\|"dtw_timeouts": [1-9][0-9]*' gpurun_out/r04q_c5_$t.jsonl | tr '\n' ' ')"
done
