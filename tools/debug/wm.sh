set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_window_msd.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wm.log 2>&1; rc=$?
tail -30 gpurun_out/wm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_configs.py --only cfg5,window > gpurun_out/wm_bench.log 2>&1; rc=$?
tail -5 gpurun_out/wm_bench.log | cut -c1-900; exit $rc
