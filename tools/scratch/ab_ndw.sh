#!/bin/bash
# A/B of the number of distance waves per DTW band block (lib_ndw<n> from tools/ab_build.sh):
# C3-size DTW probe and the C5 leg of bench.py per build
set -o pipefail
TAGS=${TAGS:-default ndw4}
mkdir -p gpurun_out
bash tools/scratch/ab_dtw.sh $TAGS || exit $?
for t in $TAGS; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 2 --warmup 1 --dtw-len 0 --c3-seconds 0 --c4-seconds 0 \
    --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 > gpurun_out/abn_$t.json 2> gpurun_out/abn_$t.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/abn_$t.json').read().strip().splitlines()[-1])
print('$t C5', round(d['c5_pairs_per_s'],1), [round(x,1) for x in d['c5_pairs_per_s_spread']])"
done
