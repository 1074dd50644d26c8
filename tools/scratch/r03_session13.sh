#!/bin/bash
# batched music features + NCC per pair batch: bit-exactness, C5 test, C5 A/B against per-pair launches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_pairs.py tests/test_gpu_alignment.py > gpurun_out/r03s13_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03s13_tests.log; exit 1; }
tail -2 gpurun_out/r03s13_tests.log
timeout -k 10 800 bash tools/scratch/ab_c5env.sh 3 "pipe|lib||128" "nopipe|lib|SONAR_PAIR_PIPELINE=0|128" "pipe|lib||128" "nopipe|lib|SONAR_PAIR_PIPELINE=0|128" "pipe8|lib|SONAR_PAIR_STREAMS=8 GPU_MAX_HW_QUEUES=8|128" "pipe12|lib|SONAR_PAIR_STREAMS=12 GPU_MAX_HW_QUEUES=12|192" > gpurun_out/r03s13_ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r03s13_ab.log; exit 1; }
cat gpurun_out/r03s13_ab.log
