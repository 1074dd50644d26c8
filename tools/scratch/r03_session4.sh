#!/bin/bash
# one-wave DTW kernel register variants: C5 A/B and the single-band step time
set -o pipefail
mkdir -p gpurun_out
for t in default pipe; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L SONAR_DTW_WAVE=1 SONAR_DTW_BAND2=0 timeout -k 10 100 python tools/scratch/dtw2_probe.py 51676 > gpurun_out/r03s4_probe_$t.txt 2>&1 || { echo "probe $t failed"; tail -5 gpurun_out/r03s4_probe_$t.txt; exit 1; }
  head -c 400 gpurun_out/r03s4_probe_$t.txt; echo
done
timeout -k 10 700 bash tools/scratch/ab_stress.sh 4 default pipe w2 band default pipe w2 band > gpurun_out/r03s4_ab.log 2>&1 || { echo "ab failed"; exit 1; }
grep c5 gpurun_out/r03s4_ab.log | cut -c1-60
