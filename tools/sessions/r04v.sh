# Headline with the window in LDS (read per pair; build-time HL_WLDS, a define in mfcc_pair.hip at the time, not kept) and the ln phase's source offsets in the freed
# registers (HL_WLDS=1: one dependent LDS round trip less per pair; 80 LDS instructions per pair
# against 84): tests on that build, then three alternating A/B rounds against the shipped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
WL=$PWD/sonido-sonar_amd/lib_wlds/libsonar_gpu.so
SONAR_LIB=$WL timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py tests/test_gpu_golden.py > gpurun_out/r04v_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04v_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04v_tests.log; exit 1; }
NOLEGS="--no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0"
for round in 1 2 3 4; do
for t in default wlds; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py $NOLEGS > gpurun_out/r04v_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04v_ab_$t.json')); print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
