set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --maxfail=10 --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/r04f_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r04f_tests.log
# a failed test goes on to the A/B; a crash or a time limit ends the call
[ $rc -le 1 ] || { echo "test run ended with rc=$rc"; exit 1; }
for t in noslp16 noslp16nopf; do
SONAR_LIB=$PWD/sonido-sonar_amd/lib_$t/libsonar_gpu.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_mfcc_pair.py > gpurun_out/r04f_tests_$t.log 2>&1 || { echo "tests $t failed"; tail -30 gpurun_out/r04f_tests_$t.log; exit 1; }
echo "$t: $(tail -1 gpurun_out/r04f_tests_$t.log)"
done
for round in 1 2 3; do
for t in base tl4 noslp noslp16 noslp16nopf wpb16 wpb16nopf; do
  L=sonido-sonar_amd/lib_$t/libsonar_gpu.so
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --steps 20 > gpurun_out/r04f_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04f_ab_$t.json')); print('$t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
for t in tl4 default nofeat nodtw default tl4; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04f_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*' gpurun_out/r04f_c5_$t.jsonl | tr '\n' ' ')"
done
