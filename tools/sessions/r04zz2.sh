# Round profile again with the fp_batch leg kept out of the PMC and headline-trace runs (r04zz's
# traffic averaged the leg's 1000 small per-signal launches of the same kernel name).  Product code
# unchanged since r04zz (whose GPU tests, smoke and SQ counters stand).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f profiles/r04zz_traffic.json
bash tools/profile_round.sh r04zz || exit 1
cp profiles/r04zz_bench.json profiles/r04zz_traffic.json gpurun_out/ 2>/dev/null; true
