#!/bin/bash
# Build an A/B variant of libsonar_gpu.so into sonido-sonar_amd/lib_<tag>/ with extra defines.
# Usage: bash tools/ab_build.sh <tag> "-DFOO -DBAR"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; DEFS=$2
make -s -C "$R/sonido-sonar_amd" OBJDIR=build_$TAG LIB=lib_$TAG/libsonar_gpu.so EXTRA_DEFS="$DEFS" -j8
echo "$R/sonido-sonar_amd/lib_$TAG/libsonar_gpu.so"
