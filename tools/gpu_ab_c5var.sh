# C5 A/B over run-time variants of one build: alternating C5 bench legs, each variant given as
# name:'VAR=VALUE ...':'--bench-args ...' (either part may be empty).
# Usage: bash tools/gpu_ab_c5var.sh <out-tag> <variant> [<variant> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
LEGS="--no-cpu-baseline --no-f64 --c1 0 --seconds 60 --steps 5 --warmup 2 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 --dtw-len 0 --c5-pairs 1000 --reps 3"
for round in 1 2 3; do
for v in "$@"; do
  name=${v%%:*}; rest=${v#*:}; ENVS=${rest%%:*}; ARGS=${rest#*:}
  env $ENVS timeout -k 10 300 python3 bench.py $LEGS $ARGS > gpurun_out/${TAG}_ab_$name.json 2>gpurun_out/${TAG}_ab_$name.err || { echo "fail $name"; tail -5 gpurun_out/${TAG}_ab_$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_ab_$name.json'))
print('c5 $name', round(d['c5_pairs_per_s'],1), 'pairs/s', [round(x,1) for x in d['c5_pairs_per_s_spread']], 'timeouts', d['c5_dtw_counters_rank0'].get('dtw_timeouts'), d['c5_warmup_dtw_counters'].get('dtw_timeouts'))" | tee -a gpurun_out/${TAG}_ab.log
done
done
