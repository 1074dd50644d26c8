# Round-4 final evidence, part 2 (after part 1's summaries are committed under profiles/):
# GPU tests, smoke, full-bench kernel trace, steady-state headline trace, FETCH/WRITE PMC, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh r04z || exit 1
cp profiles/r04z_bench.json profiles/r04z_traffic.json profiles/r04z_kernel_stats.csv gpurun_out/ 2>/dev/null; true
