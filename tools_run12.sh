set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest12.log 2>&1; rc=$?
tail -5 gpurun_out/pytest12.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest12.log; exit $rc; }
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs12.log 2>&1 || { tail -20 gpurun_out/configs12.log; exit 1; }
cat gpurun_out/configs12.log
bash tools_run11.sh
