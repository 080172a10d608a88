set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest13.log 2>&1; rc=$?
tail -5 gpurun_out/pytest13.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest13.log; exit $rc; }
bash tools/prof_configs.sh b --only cfg5,cfg3,filter,cfg2 --scale 0.25
