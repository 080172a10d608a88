set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_window_msd.py -m gpu -x -q -k "big_and_clustered or counting or clustered" --timeout 120 --timeout-method thread > gpurun_out/wt2.log 2>&1 || { tail -30 gpurun_out/wt2.log; exit 1; }
tail -1 gpurun_out/wt2.log
