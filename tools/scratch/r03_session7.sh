#!/bin/bash
# f64 issue rate vs waves/SIMD; then C5 A/B: default vs the LEAN kernel with capped persistent waves
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/scratch/f64_rate > gpurun_out/r03s7_f64_rate.txt 2>&1 || { echo "f64_rate failed"; exit 1; }
cat gpurun_out/r03s7_f64_rate.txt
timeout -k 10 900 bash tools/scratch/ab_stress.sh 3 default l128 l160 l96 default l128 l160 l96 > gpurun_out/r03s7_ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r03s7_ab.log; exit 1; }
grep c5 gpurun_out/r03s7_ab.log | cut -c1-70
