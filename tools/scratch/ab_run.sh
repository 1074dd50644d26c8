#!/bin/bash
# Alternate the headline microbench between the default library and lib_<tag> (N rounds).
TAG=$1; N=${2:-3}
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
for i in $(seq $N); do
  echo -n "A "; timeout -k 10 100 python "$R/tools/fp_microbench.py" mfcc || exit 1
  echo -n "B "; SONAR_LIB="$R/sonido-sonar_amd/lib_$TAG/libsonar_gpu.so" timeout -k 10 100 python "$R/tools/fp_microbench.py" mfcc || exit 1
done
