# Round-4 final evidence, part 1 (tools/sessions/r04z2.sh is part 2): PMC passes on the final HEAD (DTW band
# kernel at C3 size, headline kernel) and the C5 kernel families; the summaries the bench line
# reads (profiles/*dtw_pmc*, *_c5_families) are committed before part 2 runs the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ITERS=2 bash tools/pmc_run.sh r04z_dtw tools/dtw_probe.py || exit 1
python3 tools/dtw_pmc_json.py gpurun_out/pmc_r04z_dtw r04z dtw_band_kernel dtw_walk dtw_exit_map dtw_path && cp profiles/r04z_dtw_pmc.json gpurun_out/ || exit 1
bash tools/pmc_headline.sh r04z_hl || exit 1
( cd /tmp && export TMPDIR=/tmp && SONAR_PAIR_RETRY=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04z_c5prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/c5_stress.py" --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/r04z_c5prof.log" 2>&1 ) || { echo "c5 profile failed"; exit 1; }
f=$(find gpurun_out/r04z_c5prof -name '*kernel_stats.csv' | head -1)
python3 tools/c5_families.py "$f" gpurun_out/r04z_c5_families.json --note "final HEAD: tools/c5_stress.py --reps 1 (warm-up + 1 timed call, 1000 x 60 s pairs) under rocprofv3 --kernel-trace --stats" && cp gpurun_out/r04z_c5_families.json profiles/ || exit 1
rm -f gpurun_out/r04z_c5prof/*kernel_trace.csv 2>/dev/null
