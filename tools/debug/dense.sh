set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/dense_tests.log 2>&1 || { tail -40 gpurun_out/dense_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/dense_tests.log | tail -3
bash tools/debug/distover.sh
