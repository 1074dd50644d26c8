# DTW A/B: the band-kernel tests on the default build, then alternating C3-DTW + C5 bench legs of
# the default build and the lib_<tag> variants named on the command line.
# Usage: bash tools/gpu_ab_dtw.sh <out-tag> <variant> [<variant> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dtw_walk.py tests/test_gpu_dtw_liveness.py tests/test_gpu_c5_batch.py tests/test_gpu_pair_batch.py tests/test_gpu_fullsize.py::test_c3_dtw_20000_slice_bit_exact > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
LEGS="--no-cpu-baseline --no-f64 --c1 0 --seconds 60 --steps 5 --warmup 2 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 --dtw-len 51676 --dtw-steps 3 --c5-pairs 1000 --reps 2"
for round in 1 2 3; do
for t in default "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 300 python3 bench.py $LEGS > gpurun_out/${TAG}_ab_$t.json 2>gpurun_out/${TAG}_ab_$t.err || { echo "fail $t"; tail -5 gpurun_out/${TAG}_ab_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_ab_$t.json'))
print('dtw $t', 'band', round(d['dtw_kernel_ms']['band_sweep'],3), 'ms  dtw', round(d['dtw_ms'],2), 'ms  c5', round(d['c5_pairs_per_s'],1), 'pairs/s  timeouts', d['c5_dtw_counters_rank0'].get('dtw_timeouts'), d['c5_warmup_dtw_counters'].get('dtw_timeouts'))" | tee -a gpurun_out/${TAG}_ab.log
done
done
