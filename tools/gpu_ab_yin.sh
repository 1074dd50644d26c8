# yin_kernel A/B: tools/yin_microbench.py on the default build and lib_<tag> variants, alternating.
# Usage (GPU box): bash tools/gpu_ab_yin.sh <out-tag> [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
for round in 1 2 3; do
for t in "$@" default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L timeout -k 10 200 python3 tools/yin_microbench.py > gpurun_out/${TAG}_yin.json 2> gpurun_out/${TAG}_yin.err || { echo "fail $t"; tail -3 gpurun_out/${TAG}_yin.err; exit 1; }
  sed "s/^/$t /" gpurun_out/${TAG}_yin.json | tee -a gpurun_out/${TAG}_yin_ab.log
done
done
