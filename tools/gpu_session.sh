# round 5 session c: full GPU suite, bench (headline + C1 + f64 legs), C5 stress with the spin-priority change
set -o pipefail
TAG=${1:-r05c}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
timeout -k 10 400 python -u bench.py --dtw-len 0 --c5-pairs 0 --c3-seconds 0 --c4-seconds 0 --c6-gallery 0 --c7-seconds 0 --ingest-reps 0 --batch-signals 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 python -u tools/c5_stress.py --reps 5 --tag spin0_${TAG} --out gpurun_out/${TAG}_c5_stress.jsonl > /dev/null 2> gpurun_out/${TAG}_c5.err || { tail -5 gpurun_out/${TAG}_c5.err; exit 1; }
tail -1 gpurun_out/${TAG}_c5_stress.jsonl
