#!/bin/bash
# C5 concurrency: feature kernels at issue priority 3, more streams / pairs in flight
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pair_batch.py tests/test_gpu_dtw_walk.py > gpurun_out/r03s10_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03s10_tests.log; exit 1; }
tail -2 gpurun_out/r03s10_tests.log
timeout -k 10 1000 bash tools/scratch/ab_c5env.sh 3 \
  "base|lib|SONAR_SCAN_THREADS=1024|128" "scan256|lib||128" "prio|lib_prio||128" "s24|lib|SONAR_PAIR_STREAMS=24 GPU_MAX_HW_QUEUES=24|192" "s32|lib|SONAR_PAIR_STREAMS=32 GPU_MAX_HW_QUEUES=32|256" \
  "base|lib|SONAR_SCAN_THREADS=1024|128" "scan256|lib||128" "prio|lib_prio||128" "s24|lib|SONAR_PAIR_STREAMS=24 GPU_MAX_HW_QUEUES=24|192" "s32|lib|SONAR_PAIR_STREAMS=32 GPU_MAX_HW_QUEUES=32|256" \
  > gpurun_out/r03s10_ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r03s10_ab.log; exit 1; }
cat gpurun_out/r03s10_ab.log
