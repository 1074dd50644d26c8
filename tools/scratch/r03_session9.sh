#!/bin/bash
# where the batched DTW's wave-time goes under C5: per-batch band trace (SONAR_DTW_BATCH_TRACE=1)
set -o pipefail
mkdir -p gpurun_out
SONAR_DTW_BATCH_TRACE=1 timeout -k 10 200 python tools/c5_stress.py --reps 2 > gpurun_out/r03s9_c5.jsonl 2> gpurun_out/r03s9_trace.txt || { echo "c5 trace failed"; tail -5 gpurun_out/r03s9_trace.txt; exit 1; }
python3 - <<'PY'
import json
L=[json.loads(l)["dtw_batch_trace"] for l in open("gpurun_out/r03s9_trace.txt") if l.startswith('{"dtw_batch_trace"')]
tot={k: sum(x[k] for x in L) for k in ("band_us","first_wait_us","spin_us","steps")}
print("batches", len(L))
print("band-time share: first-edge wait %.3f, later edge waits %.3f, compute %.3f" % (tot["first_wait_us"]/tot["band_us"], tot["spin_us"]/tot["band_us"], 1-(tot["first_wait_us"]+tot["spin_us"])/tot["band_us"]))
print("ns/step over band-time %.1f, over compute %.1f" % (tot["band_us"]*1e3/tot["steps"], (tot["band_us"]-tot["first_wait_us"]-tot["spin_us"])*1e3/tot["steps"]))
span=sorted(x["span_us"] for x in L); print("batch DTW span us median", span[len(span)//2])
PY
tail -2 gpurun_out/r03s9_c5.jsonl | cut -c1-200
