#!/bin/bash
# Alternate the headline microbench between the default library and lib_<tag> variants (N rounds).
# Usage: bash tools/ab_run3.sh N tagA tagB ...
N=$1; shift
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
for i in $(seq $N); do
  echo -n "base "; timeout -k 10 100 python "$R/tools/fp_microbench.py" mfcc || exit 1
  for t in "$@"; do
    echo -n "$t "; SONAR_LIB="$R/sonido-sonar_amd/lib_$t/libsonar_gpu.so" timeout -k 10 100 python "$R/tools/fp_microbench.py" mfcc || exit 1
  done
done
