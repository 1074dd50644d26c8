# Headline work split: one full residency of waves (shipped) against 2 and 4 rounds of shorter pair runs (HL_WAVE_ROUNDS, a build-time define in sonar_api.cpp at the time, not kept)

set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
NOLEGS="--no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0"
for round in 1 2 3; do
for t in default wr2 wr4; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py $NOLEGS > gpurun_out/r04x5_ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04x5_ab_$t.json')); print('hl $t', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4))"
done
done
