# A/B of DTW builds: bash tools/scratch/ab_dtw.sh default <tag>...  (lib_<tag> from tools/ab_build.sh)
set -o pipefail
mkdir -p gpurun_out
for t in "$@"; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  echo "== $t"
  SONAR_LIB=$PWD/$L ITERS=2 SONAR_DTW_TRACE=/tmp/dtw_$t.bin timeout -k 10 120 python3 tools/dtw_probe.py > gpurun_out/ab_$t.log 2>&1 || { echo "fail $t"; tail -5 gpurun_out/ab_$t.log; exit 1; }
  grep -E "kernel ms|band0|clock|band    0|active" gpurun_out/ab_$t.log
done
