# C5 kernel traces: serial (one worker stream, 64 pairs: every kernel uncontended) and the default
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r04b"; mkdir -p "$O"
SONAR_PAIR_RETRY=0 SONAR_PAIR_STREAMS=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/serial" -o run -- \
  python3 "$R/tools/c5_stress.py" --reps 1 --pairs 64 --workers 8 > "$O/serial.log" 2>&1 || { echo serial failed; tail "$O/serial.log"; exit 1; }
SONAR_PAIR_RETRY=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/full" -o run -- \
  python3 "$R/tools/c5_stress.py" --reps 1 > "$O/full.log" 2>&1 || { echo full failed; tail "$O/full.log"; exit 1; }
find "$O" -name '*.csv' | xargs ls -la
