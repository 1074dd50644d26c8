# Headline A/B: correctness subset on the default build, then alternating bench headline runs of the
# default build and the lib_<tag> variants named on the command line.
# Usage: bash tools/gpu_ab_headline.sh <out-tag> <variant> [<variant> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py::test_c2_full_hour_mfcc tests/test_gpu_features_edges.py tests/test_gpu_multi.py tests/test_gpu_stream.py tests/test_gpu_stft_mfcc.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
NOLEGS="--no-cpu-baseline --no-f64 --c1 0 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0"
for round in 1 2 3; do
for t in default "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py $NOLEGS > gpurun_out/${TAG}_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_ab_$t.json')); print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))" | tee -a gpurun_out/${TAG}_ab.log
done
done
