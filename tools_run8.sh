set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest8.log 2>&1; rc=$?
tail -30 gpurun_out/pytest8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench8.log 2>&1 || { tail gpurun_out/bench8.log; exit 1; }
cat gpurun_out/bench8.log | tail -1
