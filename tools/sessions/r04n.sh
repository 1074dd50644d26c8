set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --maxfail=10 --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/r04n_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04n_tests.log; [ $rc -le 1 ] || { echo "test run rc=$rc"; exit 1; }
for t in prev default prev default prev default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04n_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*\|"dtw_timeouts": [1-9][0-9]*' gpurun_out/r04n_c5_$t.jsonl | tr '\n' ' ')"
done
for t in hp1 hp2; do
  SONAR_LIB=$PWD/sonido-sonar_amd/lib_$t/libsonar_gpu.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_mfcc_pair.py > gpurun_out/r04n_tests_$t.log 2>&1 || { echo "tests $t failed"; tail -20 gpurun_out/r04n_tests_$t.log; exit 1; }
done
for round in 1 2 3; do
for t in default hp1 hp2; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --steps 20 > gpurun_out/r04n_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04n_ab_$t.json')); print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
( cd /tmp && export TMPDIR=/tmp && SONAR_PAIR_RETRY=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04n_c5prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/c5_stress.py" --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/r04n_c5prof.log" 2>&1 ) || { echo "c5 profile failed"; exit 1; }
f=$(find gpurun_out/r04n_c5prof -name '*kernel_stats.csv' | head -1)
python3 tools/c5_families.py "$f" gpurun_out/r04n_c5_families.json --note "tools/c5_stress.py --reps 1 (warm-up + 1 timed call, 1000 x 60 s pairs) under rocprofv3 --kernel-trace --stats; feature / path kernels sized to co-reside with the band kernel"
rm -f gpurun_out/r04n_c5prof/*kernel_trace.csv 2>/dev/null; true
