#!/bin/bash
# Rebuild libsonar_gpu.so with each DTW scheduling-group size and time the C3-size DTW.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R/sonido-sonar_amd"
for G in "$@"; do
  make -s clean >/dev/null 2>&1
  make -s -j16 EXTRA_DEFS="-DDTW_G=$G" > /dev/null 2>&1 || { echo "build G=$G failed"; exit 1; }
  echo "G=$G"
  SONAR_DTW_TRACE=/tmp/dtwtrace.bin ITERS=2 timeout -k 10 120 python3 "$R/tools/dtw_microbench.py" || exit 1
done
