#!/bin/bash
# one GPU session: tests, smoke, bench, kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/s1_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/s1_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/s1_bench.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o s1 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --dtw-len 10332 > "$GRAFT_REPO_ROOT/gpurun_out/s1_prof.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/s1_prof.log"
