# Round-4 final evidence at the final HEAD (after the 32-bit index change): headline SQ
# counters, then the round profile (all GPU tests, smoke, full-bench and steady-state headline
# traces, FETCH/WRITE PMC -> traffic, bench line).  DTW and C5 code are unchanged since r04z, so
# r04z_dtw_pmc.json and r04z_c5_families.json stand.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/pmc_headline.sh r04zf_hl || exit 1
bash tools/gpu_round.sh r04zf || exit 1
cp profiles/r04zf_bench.json profiles/r04zf_traffic.json gpurun_out/ 2>/dev/null; true
