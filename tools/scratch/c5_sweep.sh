#!/bin/bash
# C5 throughput vs pair streams and DTW variant (diagnostics): one bench C5 leg per setting
set -o pipefail
mkdir -p gpurun_out
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --dtw-len 0 \
      --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 \
      > gpurun_out/sw_$name.json 2> gpurun_out/sw_$name.err || return $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/sw_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['c5_pairs_per_s'],1), [round(x,1) for x in d['c5_pairs_per_s_spread']], d['c5_lag_recovered'])" | tee -a gpurun_out/c5_sweep.log
}
for pre in 1 0; do
  run nobatch_pre$pre SONAR_DTW_PRE=$pre SONAR_PAIR_BATCH=0 || exit $?
  for st in 4 8 16; do
    run pre${pre}_st$st SONAR_DTW_PRE=$pre SONAR_PAIR_STREAMS=$st || exit $?
  done
done
