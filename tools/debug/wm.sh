set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_window_msd.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wm.log 2>&1; rc=$?
tail -30 gpurun_out/wm.log
[ $rc -eq 0 ] || exit $rc
TAG=base timeout -k 10 120 python tools/debug/wm_time.py && TAG=skipsort QEH_WM_SKIP_SORT=1 timeout -k 10 120 python tools/debug/wm_time.py
