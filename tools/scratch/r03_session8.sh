#!/bin/bash
# interleaved (fenced) one-wave DTW kernel, now the batch default: bit-exactness, C5 test, C5 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py > gpurun_out/r03s8_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03s8_tests.log; exit 1; }
tail -2 gpurun_out/r03s8_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_c5_batch.py > gpurun_out/r03s8_c5test.log 2>&1 || { echo "c5 test failed"; tail -30 gpurun_out/r03s8_c5test.log; exit 1; }
tail -2 gpurun_out/r03s8_c5test.log
timeout -k 10 700 bash tools/scratch/ab_stress.sh 3 default il0 default il0 > gpurun_out/r03s8_ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r03s8_ab.log; exit 1; }
grep c5 gpurun_out/r03s8_ab.log | cut -c1-70
