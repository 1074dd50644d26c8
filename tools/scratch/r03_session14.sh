#!/bin/bash
# liveness stress of the default C5 path (batched features, 16 streams x 8): 12 repetitions, then the
# pipelined option at 8 streams (12 repetitions) for its failure rate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/c5_stress.py --reps 12 > gpurun_out/r03s14_default.jsonl 2> gpurun_out/r03s14_default.err || { echo "default c5 stress failed"; tail -3 gpurun_out/r03s14_default.err; exit 1; }
tail -1 gpurun_out/r03s14_default.jsonl | cut -c1-200
python3 -c "
import json; L=[json.loads(l) for l in open('gpurun_out/r03s14_default.jsonl')]; v=sorted(x['pairs_per_s'] for x in L if 'rep' in x); print('default', len(v), 'median', v[len(v)//2], 'min', v[0], 'max', v[-1], [x.get('warmup_error') for x in L if 'warmup_error' in x][:1])"
SONAR_PAIR_PIPELINE=1 SONAR_PAIR_STREAMS=8 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/c5_stress.py --reps 12 > gpurun_out/r03s14_pipe8.jsonl 2> gpurun_out/r03s14_pipe8.err || { echo "pipe8 c5 stress failed"; tail -3 gpurun_out/r03s14_pipe8.err; exit 1; }
tail -1 gpurun_out/r03s14_pipe8.jsonl | cut -c1-200
python3 -c "
import json; L=[json.loads(l) for l in open('gpurun_out/r03s14_pipe8.jsonl')]; v=sorted(x['pairs_per_s'] for x in L if 'rep' in x); print('pipe8', len(v), 'median', v[len(v)//2], 'min', v[0], 'max', v[-1], [x.get('warmup_error','')[:300] for x in L if 'warmup_error' in x][:1], [x['error'][:300] for x in L if x.get('error')][:2])"
