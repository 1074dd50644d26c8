# sonar_fingerprint_batch (one mfcc_pair_kernel launch over many signals): its GPU tests, the
# headline kernel's tests (the single-signal instance is unchanged), and a headline bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py > gpurun_out/r04y_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04y_tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 > gpurun_out/r04y_hl.json 2>gpurun_out/r04y_hl.err || { echo "bench failed"; tail gpurun_out/r04y_hl.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04y_hl.json')); print('hl', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4), d['steps'], d['warmup'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 1000 > gpurun_out/r04y_batch.json 2>gpurun_out/r04y_batch.err || { echo "batch bench failed"; tail gpurun_out/r04y_batch.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04y_batch.json')); print(json.dumps(d.get('fp_batch'), indent=1)); print(d.get('errors'))"
