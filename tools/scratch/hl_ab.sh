NOLEGS="--no-cpu-baseline --dtw-len 0 --c5-pairs 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --no-f64 --c3-seconds 0 --c4-seconds 0"
for k in 1 0 1 0; do
  SONAR_MFCC_PAIR2=$k timeout -k 10 200 python bench.py $NOLEGS > gpurun_out/hl_$k.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/hl_$k.json')); r=d['roofline']
print('pair2=$k', d['value'], r['kernel'], r['kernel_ms'], r['frac'])"
done
