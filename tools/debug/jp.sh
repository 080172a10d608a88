set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_join_predicates.py tests/test_executor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/jp.log 2>&1; rc=$?
tail -40 gpurun_out/jp.log; exit $rc
