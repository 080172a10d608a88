set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=base timeout -k 10 120 python tools/debug/wm_time.py && TAG=skipsort QEH_WM_SKIP_SORT=1 timeout -k 10 120 python tools/debug/wm_time.py
