#!/bin/bash
# C5 A/B of library builds: bash tools/scratch/ab_c5.sh default <tag>...  (lib_<tag> from tools/ab_build.sh)
set -o pipefail
mkdir -p gpurun_out
for t in "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 2 --warmup 1 --dtw-len 0 --no-cpu-baseline \
      --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 > gpurun_out/c5ab_$t.json 2>gpurun_out/c5ab_$t.err || { echo "fail $t"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5ab_$t.json').read().strip().splitlines()[-1]);print('$t', round(d['c5_pairs_per_s'],1), [round(x,1) for x in d['c5_pairs_per_s_spread']], d['c5_lag_recovered'])"
done
