#!/bin/bash
# LEAN one-wave DTW kernel (no cross-chunk pipelining, 155 VGPRs, 2-3 waves/SIMD): bit-exactness
# on the batch tests, then a C5 A/B against the default pipelined kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py -k "agree" > gpurun_out/r03s6_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03s6_tests.log; exit 1; }
tail -3 gpurun_out/r03s6_tests.log
SONAR_DTW_LEAN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_c5_batch.py > gpurun_out/r03s6_c5test.log 2>&1 || { echo "c5 test failed"; tail -30 gpurun_out/r03s6_c5test.log; exit 1; }
tail -3 gpurun_out/r03s6_c5test.log
SONAR_LIB=$PWD/sonido-sonar_amd/lib_r96/libsonar_gpu.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py -k "agree" > gpurun_out/r03s6_tests96.log 2>&1 || { echo "r96 tests failed"; tail -30 gpurun_out/r03s6_tests96.log; exit 1; }
tail -2 gpurun_out/r03s6_tests96.log
timeout -k 10 700 bash tools/scratch/ab_stress.sh 3 default lean lean96 default lean lean96 > gpurun_out/r03s6_ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r03s6_ab.log; exit 1; }
grep c5 gpurun_out/r03s6_ab.log | cut -c1-70
