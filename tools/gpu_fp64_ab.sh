# f64 transform A/B: the f64 / SPEC correctness subset on the default build, then the fused-kernel
# microbench (tools/fp_microbench.py) of the default build and of the lib_<tag> variants named.
# Usage (GPU box): bash tools/gpu_fp64_ab.sh <out-tag> [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stft_mfcc.py tests/test_gpu_golden.py tests/test_gpu_stft_complex.py "tests/test_gpu_fullsize.py::test_c2_f64_headline_10min" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit 1; }
for round in 1 2; do
for t in default "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L ITERS=30 timeout -k 10 200 python3 tools/fp_microbench.py mfcc_f64 mfcc+spectral mfcc_generic > gpurun_out/${TAG}_ab_$t.jsonl 2>gpurun_out/${TAG}_ab_$t.err || { echo "fail $t"; tail -3 gpurun_out/${TAG}_ab_$t.err; exit 1; }
  sed "s/^/$t /" gpurun_out/${TAG}_ab_$t.jsonl | tee -a gpurun_out/${TAG}_ab.log
done
done
