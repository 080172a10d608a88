set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest7.log 2>&1; rc=$?
tail -40 gpurun_out/pytest7.log
exit $rc
