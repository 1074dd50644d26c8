#!/bin/bash
# C5 A/B over library builds, environments and pairs in flight (tools/c5_stress.py), alternating.
# Usage: bash tools/scratch/ab_c5env.sh <reps> "<tag>|<lib dir>|<env>|<workers>" ...
set -o pipefail
mkdir -p gpurun_out
REPS=$1; shift
for spec in "$@"; do
  IFS='|' read -r t L EV W <<< "$spec"
  env $EV SONAR_LIB=$PWD/sonido-sonar_amd/$L/libsonar_gpu.so timeout -k 10 200 python tools/c5_stress.py --reps $REPS --workers $W > gpurun_out/abe_$t.jsonl 2>gpurun_out/abe_$t.err || { echo "c5 fail $t"; tail -3 gpurun_out/abe_$t.err; exit 1; }
  python3 -c "
import json, numpy as np
L=[json.loads(l) for l in open('gpurun_out/abe_$t.jsonl')]
v=np.array([x['pairs_per_s'] for x in L if 'rep' in x]); s=L[-1]
print('$t', 'c5 median', np.median(v), 'min', v.min(), 'max', v.max(), 'failed', s['failed_reps'])"
done
