set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_music.py tests/test_gpu_mfcc_pair.py tests/test_gpu_stft_mfcc.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py > gpurun_out/r04e_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
for round in 1 2 3; do
for t in base default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --steps 20 > gpurun_out/r04e_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04e_ab_$t.json')); print('$t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
for t in default nofeat nodtw default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_PAIR_RETRY=0 SONAR_LIB=$PWD/$L timeout -k 10 150 python3 tools/c5_stress.py --reps 2 > gpurun_out/r04e_c5_$t.jsonl 2>/dev/null || { echo "c5 fail $t"; exit 1; }
  echo "c5 $t: $(grep -o '"pairs_per_s": [0-9.]*' gpurun_out/r04e_c5_$t.jsonl | tr '\n' ' ')"
done
