#!/bin/bash
# Alternating A/B of library builds on C5 (tools/c5_stress.py) and the C3-size DTW band kernel.
# Usage: bash tools/scratch/ab_stress.sh <reps per C5 run> <tag>...  (default = sonido-sonar_amd/lib)
set -o pipefail
mkdir -p gpurun_out
REPS=$1; shift
for t in "$@"; do
  EV=""
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so;
  elif [ $t = b2 ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; EV="SONAR_DTW_BAND2=1";   # 128-row band kernel
  elif [ ${t:0:1} = n ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; EV="SONAR_DTW_WAVES=${t:1}";   # persistent waves per batch
  elif [ ${t:0:1} = p ]; then L=sonido-sonar_amd/lib_pipe/libsonar_gpu.so; EV="SONAR_DTW_WAVES=${t:1}";   # DTWW_PIPE build
  elif [ $t = lean ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; EV="SONAR_DTW_LEAN=1";   # LEAN one-wave kernel
  elif [ $t = lean96 ]; then L=sonido-sonar_amd/lib_r96/libsonar_gpu.so; EV="SONAR_DTW_LEAN=1";   # LEAN + 96-row ring
  elif [ ${t:0:1} = l ] && [ $t != lean ] && [ $t != lean96 ]; then L=sonido-sonar_amd/lib_r96/libsonar_gpu.so; EV="SONAR_DTW_LEAN=1 SONAR_DTW_WAVES=${t:1}";   # LEAN + r96 + persistent waves per batch
  elif [ $t = il ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; EV="SONAR_DTW_IL=1";   # fenced interleaved wave kernel
  elif [ $t = band ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; EV="SONAR_DTW_WAVE=0";   # 8-wave band kernel
  else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  env $EV SONAR_LIB=$PWD/$L timeout -k 10 120 python tools/scratch/dtw_band_ms.py 51676 5 || { echo "dtw fail $t"; exit 1; }
  env $EV SONAR_LIB=$PWD/$L timeout -k 10 200 python tools/c5_stress.py --reps $REPS > gpurun_out/abs_$t.jsonl 2>gpurun_out/abs_$t.err || { echo "c5 fail $t"; exit 1; }
  python3 -c "
import json, numpy as np
L=[json.loads(l) for l in open('gpurun_out/abs_$t.jsonl')]
v=np.array([x['pairs_per_s'] for x in L if 'rep' in x]); s=L[-1]
print('$t', 'c5 median', np.median(v), 'min', v.min(), 'max', v.max(), 'failed', s['failed_reps'], {k: s[k] for k in s if k not in ('summary','reps','failed_reps')})"
done
