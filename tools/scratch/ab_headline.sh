# Headline-kernel A/B: bash tools/scratch/ab_headline.sh default <tag>...  (lib_<tag> from tools/ab_build.sh)
set -o pipefail
for round in 1 2; do
for t in "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --steps 20 > /tmp/ab_$t.json 2>/dev/null || { echo "fail $t"; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ab_$t.json')); print('$t', round(d['roofline']['kernel_ms'],4), 'ms', '%.3e' % d['value'])"
done
done
