# Headline without the lgkmcnt(0) drain at each wave-private LDS phase boundary (SONAR_NO_LGKM_SYNC:
# a wave's LDS operations execute in order, the fence + wave barrier keep the compiler's order):
# headline/batch/golden tests on that build, its 1 h MFCC timeline bit-compared with the default
# build's, then three alternating A/B rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04x3_def gpurun_out/r04x3_nol
NL=$PWD/sonido-sonar_amd/lib_nolgkm/libsonar_gpu.so
SONAR_LIB=$NL timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py tests/test_gpu_golden.py > gpurun_out/r04x3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04x3_tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; tail -30 gpurun_out/r04x3_tests.log; exit 1; }
NOLEGS="--no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0"
timeout -k 10 120 python3 bench.py $NOLEGS --dump-dir gpurun_out/r04x3_def > /dev/null 2>&1 || { echo "dump def failed"; exit 1; }
SONAR_LIB=$NL timeout -k 10 120 python3 bench.py $NOLEGS --dump-dir gpurun_out/r04x3_nol > /dev/null 2>&1 || { echo "dump nol failed"; exit 1; }
python3 -c "
import numpy as np
a=np.load('gpurun_out/r04x3_def/mfcc_timeline.npy'); b=np.load('gpurun_out/r04x3_nol/mfcc_timeline.npy')
print('timeline', a.shape, 'bit-identical', bool(np.array_equal(a, b)), 'max abs diff', float(np.max(np.abs(a-b))))"
rm -f gpurun_out/r04x3_def/*.npy gpurun_out/r04x3_nol/*.npy
for round in 1 2 3; do
for t in default nolgkm; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py $NOLEGS > gpurun_out/r04x3_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04x3_ab_$t.json')); print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
