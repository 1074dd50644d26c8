set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/r04m_trace.bin
SONAR_DTW_TRACE=$PWD/gpurun_out/r04m_trace.bin SONAR_PAIR_RETRY=0 timeout -k 10 150 python3 tools/c5_stress.py --reps 1 > gpurun_out/r04m_c5_traced.jsonl 2>/dev/null || { echo "c5 trace fail"; exit 1; }
python3 tools/dtw_batch_trace.py gpurun_out/r04m_trace.bin 10396 | tee gpurun_out/r04m_trace_summary.txt
rm -f gpurun_out/r04m_trace.bin
( cd /tmp && export TMPDIR=/tmp && SONAR_PAIR_RETRY=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04m_c5prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/c5_stress.py" --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/r04m_c5prof.log" 2>&1 ) || { echo "c5 profile failed"; exit 1; }
f=$(find gpurun_out/r04m_c5prof -name '*kernel_stats.csv' | head -1)
python3 tools/c5_families.py "$f" gpurun_out/r04m_c5_families.json --note "tools/c5_stress.py --reps 1 (warm-up + 1 timed call, 1000 x 60 s pairs) under rocprofv3 --kernel-trace --stats, code wave at s_setprio 2"
rm -f gpurun_out/r04m_c5prof/*/*kernel_trace.csv gpurun_out/r04m_c5prof/*kernel_trace.csv 2>/dev/null; true
