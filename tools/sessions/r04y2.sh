# sonar_fingerprint_batch with pinned table staging: its GPU tests and the bench leg (wall and kernel time)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py > gpurun_out/r04y2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04y2_tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; tail -40 gpurun_out/r04y2_tests.log; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 1000 --reps 5 > gpurun_out/r04y2_batch.json 2>gpurun_out/r04y2_batch.err || { echo "batch bench failed"; tail gpurun_out/r04y2_batch.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04y2_batch.json')); print(json.dumps(d.get('fp_batch'), indent=1)); print(d.get('errors'), d['roofline']['kernel_ms'])"
