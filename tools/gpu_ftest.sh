set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_window_msd.py tests/test_pipeline.py -m gpu -x -q -k "full_size" --timeout 240 --timeout-method thread > gpurun_out/ftest.log 2>&1 || { tail -30 gpurun_out/ftest.log; exit 1; }
tail -1 gpurun_out/ftest.log
