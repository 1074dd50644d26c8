# Round-4 final evidence, part 1: PMC passes (separate runs, no trace domains) on the final HEAD:
# the DTW band kernel (C3 size, tools/dtw_probe.py) and the headline kernel (tools/pmc_headline.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ITERS=2 bash tools/pmc_run.sh r04z_dtw tools/dtw_probe.py || exit 1
python3 tools/dtw_pmc_json.py gpurun_out/pmc_r04z_dtw r04z dtw_band_kernel dtw_walk dtw_exit_map dtw_path && cp profiles/r04z_dtw_pmc.json gpurun_out/ || exit 1
bash tools/pmc_headline.sh r04z_hl || exit 1
