#!/bin/bash
# C5 throughput vs pairs per batch: worker streams x pairs in flight (diagnostics)
set -o pipefail
mkdir -p gpurun_out
run() {   # name, streams, workers
  local name=$1 st=$2 wk=$3
  SONAR_PAIR_STREAMS=$st timeout -k 10 200 python bench.py --steps 2 --warmup 1 --dtw-len 0 --no-cpu-baseline \
      --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 --c5-workers $wk \
      > gpurun_out/bs_$name.json 2> gpurun_out/bs_$name.err || return $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/bs_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['c5_pairs_per_s'],1), [round(x,1) for x in d['c5_pairs_per_s_spread']], d['c5_lag_recovered'])" | tee -a gpurun_out/c5_batch_sweep.log
}
for cfg in "st16_w128 16 128" "st4_w128 4 128" "st2_w128 2 128" "st4_w256 4 256" "st8_w256 8 256" "st2_w256 2 256" "st16_w128b 16 128"; do
  run $cfg || exit $?
done
