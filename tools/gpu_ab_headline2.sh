# Headline kernel A/B: the pair-kernel tests on the default build, then the fused-kernel microbench
# (f32 headline + f64 pair) of the default build and the lib_<tag> variants, three alternating rounds.
# Usage (GPU box): bash tools/gpu_ab_headline2.sh <out-tag> [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mfcc_pair.py tests/test_gpu_fingerprint_batch.py tests/test_gpu_fullsize.py::test_c2_full_hour_mfcc > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit 1; }
for round in 1 2 3; do
for t in default "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L ITERS=50 timeout -k 10 200 python3 tools/fp_microbench.py ${MB:-mfcc mfcc_f64p} > gpurun_out/${TAG}_mb_$t.jsonl 2>gpurun_out/${TAG}_mb_$t.err || { echo "fail $t"; tail -3 gpurun_out/${TAG}_mb_$t.err; exit 1; }
  sed "s/^/$t /" gpurun_out/${TAG}_mb_$t.jsonl | tee -a gpurun_out/${TAG}_mb.log
done
done
