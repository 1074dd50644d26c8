# Headline / batch kernel with 32-bit pair indices and a per-signal "frames inside the signal"
# count (wave-uniform compares stay scalar): headline, batch, golden, edge and full-size tests, then
# three alternating A/B rounds against the previous HEAD (lib_head), headline and fp_batch legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_multi.py tests/test_gpu_c_abi.py > gpurun_out/r04w_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04w_tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; tail -40 gpurun_out/r04w_tests.log; exit 1; }
NOLEGS="--no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0"
for round in 1 2 3; do
for t in default head; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py $NOLEGS > gpurun_out/r04w_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04w_ab_$t.json')); b=d['fp_batch']; print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4), 'batch kernel', round(b['batch_kernel_ms'],4), 'call', round(b['batch_ms'],4), b['rows_equal_single_calls'])"
done
done
