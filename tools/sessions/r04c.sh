set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dist.py tests/test_gpu_mfcc_pair.py tests/test_gpu_stft_mfcc.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_go_api.py tests/test_gpu_stft_generic.py tests/test_gpu_multi.py tests/test_gpu_pair_batch.py tests/test_gpu_dtw_liveness.py > gpurun_out/r04c_tests.log 2>&1
rc=$?
grep -E 'PASS|FAIL|ERROR|passed|failed' gpurun_out/r04c_tests.log | tail -60
exit $rc
