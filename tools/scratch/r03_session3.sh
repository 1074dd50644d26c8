#!/bin/bash
# DTW tests with grouped bands per wave, then C5 A/B over the group size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_pairs.py tests/test_gpu_multi.py > gpurun_out/r03s3_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03s3_tests.log; exit 1; }
tail -1 gpurun_out/r03s3_tests.log
SONAR_DTW_GROUP=21 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5_batch.py tests/test_gpu_pair_batch.py > gpurun_out/r03s3_tests_g21.log 2>&1 || { echo "g21 tests failed"; tail -30 gpurun_out/r03s3_tests_g21.log; exit 1; }
tail -1 gpurun_out/r03s3_tests_g21.log
timeout -k 10 600 bash tools/scratch/ab_stress.sh 4 default g1 g4 g8 band default g1 g4 g8 band > gpurun_out/r03s3_ab.log 2>&1 || { echo "ab failed"; exit 1; }
grep c5 gpurun_out/r03s3_ab.log | cut -c1-70
