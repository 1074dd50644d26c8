#!/bin/bash
# One GPU session: gpu tests, smoke, then the round profile (trace + PMC + bench line).
# Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"; [ -z "$R" ] && R=/root/repo
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/${TAG}_smoke.log; exit 1; }
cat gpurun_out/${TAG}_smoke.log
bash tools/profile_round.sh "$TAG"
