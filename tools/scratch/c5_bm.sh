#!/bin/bash
# C5 A/B: DTW-major vs band-major batch tickets at several (streams, in-flight) shapes
set -o pipefail
mkdir -p gpurun_out
run() {   # name workers env...
  local name=$1 wk=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --dtw-len 0 --c3-seconds 0 --c4-seconds 0 \
      --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 --c5-workers $wk > gpurun_out/bm_$name.json 2> gpurun_out/bm_$name.err || return $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/bm_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['c5_pairs_per_s'],1), [round(x,1) for x in d['c5_pairs_per_s_spread']])"
}
run dm_s8_w16 16 SONAR_DTW_BAND_MAJOR=0 SONAR_PAIR_STREAMS=8 || exit $?
run bm_s8_w16 16 SONAR_PAIR_STREAMS=8 || exit $?
run bm_s4_w16 16 SONAR_PAIR_STREAMS=4 || exit $?
run bm_s4_w32 32 SONAR_PAIR_STREAMS=4 || exit $?
run bm_s8_w32 32 SONAR_PAIR_STREAMS=8 || exit $?
run bm_s8_w64 64 SONAR_PAIR_STREAMS=8 || exit $?
