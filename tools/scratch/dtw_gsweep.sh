#!/bin/bash
# Rebuild libsonar_gpu.so with each (distance waves, scheduling group) pair and time the C3-size DTW.
# Usage: bash tools/dtw_gsweep.sh "NDW:G:RROWS:DQ" ...
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R/sonido-sonar_amd"
for cfg in "$@"; do
  IFS=: read -r N G RR DQ <<< "$cfg"
  make -s clean >/dev/null 2>&1
  make -s -j16 EXTRA_DEFS="-DDTW_NDW=$N -DDTW_G=$G -DDTW_RROWS_CFG=$RR -DDTW_DQ_CFG=$DQ" > /dev/null 2>&1 \
      || { echo "build $cfg failed"; exit 1; }
  echo "NDW=$N G=$G RROWS=$RR DQ=$DQ"
  SONAR_DTW_TRACE=/tmp/dtwtrace.bin ITERS=2 timeout -k 10 120 python3 "$R/tools/dtw_microbench.py" || exit 1
done
make -s clean >/dev/null 2>&1; make -s -j16 >/dev/null 2>&1
