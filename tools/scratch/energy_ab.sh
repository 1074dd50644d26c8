#!/bin/bash
# kernel-trace A/B of energy_kernel: default library vs lib_<tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
TAG=$1; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/eab/base" -o run -- python3 "$R/tools/energy_micro.py" || exit 1
SONAR_LIB="$R/sonido-sonar_amd/lib_$TAG/libsonar_gpu.so" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/eab/$TAG" -o run -- python3 "$R/tools/energy_micro.py" || exit 1
grep energy_kernel "$R"/gpurun_out/eab/*/run_kernel_stats.csv | cut -d, -f1-7
