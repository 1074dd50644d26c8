# formant_kernel A/B: tools/formant_microbench.py on lib_<tag> variants and the default build.
# Usage (GPU box): bash tools/gpu_ab_formant.sh <out-tag> [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2; do
for t in "$@" default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 200 python3 tools/formant_microbench.py > gpurun_out/${TAG}_fmt.json 2> gpurun_out/${TAG}_fmt.err || { echo "fail $t"; tail -3 gpurun_out/${TAG}_fmt.err; exit 1; }
  sed "s/^/$t /" gpurun_out/${TAG}_fmt.json | tee -a gpurun_out/${TAG}_fmt_ab.log
done
done
