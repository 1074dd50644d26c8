# Sanity after removing the replaced headline forms from the source (identical ISA): headline and
# batch tests, smoke, one headline bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fingerprint_batch.py tests/test_gpu_mfcc_pair.py tests/test_gpu_golden.py > gpurun_out/r04zg_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04zg_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04zg_tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-f64 --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 > gpurun_out/r04zg_hl.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04zg_hl.json')); print('hl', round(d['roofline']['kernel_ms'],4), 'ms', '%.4e' % d['value'], round(d['roofline']['frac'],4), d['roofline']['traffic_source'])"
