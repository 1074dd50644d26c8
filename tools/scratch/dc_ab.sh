#!/bin/bash
# A/B of library variants on path B (DC chunk, energy batch): parity tests + the C5 bench leg.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R" && mkdir -p gpurun_out
C5="--steps 2 --warmup 1 --dtw-len 0 --c6-gallery 0 --c7-seconds 0 --c3-seconds 0 --c4-seconds 0 --ingest-reps 0 --no-cpu-baseline"
for tag in "$@"; do
  lib="$R/sonido-sonar_amd/lib_$tag/libsonar_gpu.so"; [ "$tag" = base ] && lib="$R/sonido-sonar_amd/lib/libsonar_gpu.so"
  SONAR_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_pitch_chroma.py tests/test_gpu_stft_mfcc.py tests/test_gpu_go_api.py -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/dc_$tag.log 2>&1 || { echo "$tag tests failed"; tail -20 gpurun_out/dc_$tag.log; exit 1; }
  echo "$tag tests: $(tail -1 gpurun_out/dc_$tag.log)"
done
for rep in 1 2; do
  for tag in "$@"; do
    lib="$R/sonido-sonar_amd/lib_$tag/libsonar_gpu.so"; [ "$tag" = base ] && lib="$R/sonido-sonar_amd/lib/libsonar_gpu.so"
    SONAR_LIB=$lib timeout -k 10 200 python bench.py $C5 > gpurun_out/dc_b_$tag.json 2>/dev/null || { echo "$tag bench failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/dc_b_$tag.json')); print('$tag', round(d['c5_pairs_per_s'],1), d['c5_lag_recovered'])"
  done
done
