# C5 A/B over an environment switch of one build: the pair-path tests, then alternating C5 bench
# legs with and without the given VAR=VALUE.
# Usage: bash tools/gpu_ab_c5env.sh <out-tag> VAR=VALUE
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; KV=$2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pair_batch.py tests/test_gpu_c5_batch.py tests/test_gpu_dtw_liveness.py tests/test_gpu_alignment.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
LEGS="--no-cpu-baseline --no-f64 --c1 0 --seconds 60 --steps 5 --warmup 2 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 --dtw-len 0 --c5-pairs 1000 --reps 3"
for round in 1 2 3; do
for t in default env; do
  if [ $t = env ]; then E="env $KV"; else E="env"; fi
  $E timeout -k 10 300 python3 bench.py $LEGS > gpurun_out/${TAG}_ab_$t.json 2>gpurun_out/${TAG}_ab_$t.err || { echo "fail $t"; tail -5 gpurun_out/${TAG}_ab_$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_ab_$t.json'))
print('c5 $t', round(d['c5_pairs_per_s'],1), 'pairs/s', [round(x,1) for x in d['c5_pairs_per_s_spread']], 'timeouts', d['c5_dtw_counters_rank0'].get('dtw_timeouts'), d['c5_warmup_dtw_counters'].get('dtw_timeouts'))" | tee -a gpurun_out/${TAG}_ab.log
done
done
