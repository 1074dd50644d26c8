#!/bin/bash
# round-3 GPU session: DTW tests with the one-wave batch kernel, C5 A/B, headline SQ/traffic
# counters for both headline kernels, DTW band-kernel PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dtw_checkpoint.py tests/test_gpu_dtw_walk.py tests/test_gpu_alignment.py tests/test_gpu_pairs.py tests/test_gpu_pair_batch.py tests/test_gpu_golden.py tests/test_gpu_go_api.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_multi.py > gpurun_out/r03s2_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r03s2_tests.log; exit 1; }
tail -1 gpurun_out/r03s2_tests.log
timeout -k 10 300 bash tools/scratch/ab_stress.sh 4 default band default band > gpurun_out/r03s2_ab.log 2>&1 || { echo "ab failed"; exit 1; }
grep c5 gpurun_out/r03s2_ab.log | cut -c1-60
SONAR_MFCC_PAIR2=1 ITERS=5 bash tools/pmc_run.sh r03hl2 tools/scratch/fp_microbench.py mfcc || exit 1
SONAR_MFCC_PAIR2=0 ITERS=5 bash tools/pmc_run.sh r03hl1 tools/scratch/fp_microbench.py mfcc || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_r03hl2 mfcc_pair > gpurun_out/r03hl2_pmc.json
python3 tools/pmc_summary.py gpurun_out/pmc_r03hl1 mfcc_pair > gpurun_out/r03hl1_pmc.json
ITERS=1 bash tools/pmc_run.sh r03b tools/dtw_probe.py > gpurun_out/r03b_pmc.log 2>&1 || { echo "dtw pmc failed"; exit 1; }
python3 tools/dtw_pmc_json.py gpurun_out/pmc_r03b r03b > gpurun_out/r03b_pmc_json.log 2>&1 && cp profiles/r03b_dtw_pmc.json gpurun_out/
echo session done
