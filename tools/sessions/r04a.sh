set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/r04a_smoke.log; exit 1; }
for i in 1 2 3; do
  SONAR_PAIR_RETRY=0 timeout -k 10 120 python -u tools/c5_stress.py --reps 2 > gpurun_out/r04a_c5fresh_$i.jsonl 2>&1 || { echo "c5 stress $i failed"; tail -5 gpurun_out/r04a_c5fresh_$i.jsonl; exit 1; }
done
cat gpurun_out/r04a_c5fresh_*.jsonl | cut -c1-400
