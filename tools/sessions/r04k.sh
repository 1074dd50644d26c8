set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for t in cprio_oq64; do
  SONAR_LIB=$PWD/sonido-sonar_amd/lib_$t/libsonar_gpu.so timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_dtw_walk.py tests/test_gpu_dtw_checkpoint.py > gpurun_out/r04k_tests_$t.log 2>&1
  rc=$?; echo "tests $t: $(tail -1 gpurun_out/r04k_tests_$t.log)"; [ $rc -le 1 ] || exit 1
done
for t in default cprio oq64 cprio_oq64 default cprio oq64 cprio_oq64; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04k_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*\|"dtw_timeouts": [1-9][0-9]*' gpurun_out/r04k_c5_$t.jsonl | tr '\n' ' ')"
done
for t in default cprio_oq64 default cprio_oq64; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f64 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --steps 3 > gpurun_out/r04k_dtw_$t.json 2>/dev/null || { echo "dtw fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04k_dtw_$t.json')); print('c3dtw $t', round(d['dtw_ms'],2), 'ms', d['dtw_kernel_ms'], d.get('dtw_parity'))"
done
