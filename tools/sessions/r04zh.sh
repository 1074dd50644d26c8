# Final HEAD: the whole -m gpu suite and smoke once more (after the source-only prune and the
# reverted LDS-window experiment).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04zh_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04zh_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04zh_tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
