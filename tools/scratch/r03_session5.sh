#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py > gpurun_out/r03s5_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03s5_tests.log; exit 1; }
tail -1 gpurun_out/r03s5_tests.log
timeout -k 10 800 bash tools/scratch/ab_stress.sh 4 default n0 n32 n128 p64 p160 band default n0 n32 n128 p64 p160 band > gpurun_out/r03s5_ab.log 2>&1 || { echo "ab failed"; exit 1; }
grep c5 gpurun_out/r03s5_ab.log | cut -c1-60
