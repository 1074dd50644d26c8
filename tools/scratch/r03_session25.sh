#!/bin/bash
# the batch default back on the 8-wave band kernel: fresh-process C5 (no redo), GPU tests, smoke, bench line
# failure rate of the C5 DTW pipeline in fresh processes (the two timeouts so far were in the first
# C5 call of a process): batched features (default) against per-pair feature launches, alternating
set -o pipefail
mkdir -p gpurun_out/r03s25
for i in $(seq 1 4); do
  for t in default; do
    EV="SONAR_PAIR_RETRY=0"; L=lib
    env $EV SONAR_LIB=$PWD/sonido-sonar_amd/$L/libsonar_gpu.so timeout -k 10 200 python tools/c5_stress.py --reps 2 > gpurun_out/r03s25/${t}_$i.jsonl 2>/dev/null || { echo "run $t $i failed rc=$?"; exit 1; }
    python3 -c "
import json; L=[json.loads(l) for l in open('gpurun_out/r03s25/${t}_$i.jsonl')]
e=[x.get('warmup_error') or x.get('error') for x in L if (x.get('warmup_error') or x.get('error'))]
v=[round(x['pairs_per_s']) for x in L if 'rep' in x]
w=[x for x in L if x.get('warmup')][0]; r=[x for x in L if 'rep' in x]
print('$t', $i, v, 'warmup', w['s'], 'fences', w.get('edge_refresh_fences'), 'hits', w.get('edge_refresh_hits'), 'timeouts', w.get('dtw_timeouts'), 'rep fences', [x.get('edge_refresh_fences') for x in r], ('ERR ' + e[0][:160]) if e else 'ok', flush=True)"
  done
done

timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r03f_tests.log; exit 1; }
tail -2 gpurun_out/r03f_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03f_smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/r03f_smoke.log; exit 1; }
cat gpurun_out/r03f_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03f_bench.json')); print({k: d.get(k) for k in ('value','c5_pairs_per_s','c5_pairs_per_s_spread','c5_warmup_failed_calls','c5_failed_reps','dtw_ms','c3_align')}); print(d['roofline']['frac'], d['c5_dtw_counters_rank0'])"
