set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -x > gpurun_out/pytest14.log 2>&1; rc=$?
tail -3 gpurun_out/pytest14.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest14.log; exit $rc; }
bash tools/prof_configs.sh c --only cfg5,cfg3 --scale 0.25 || exit 1
bash tools/pmc_cmd.sh sort "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" -- python3 tools/bench_configs.py --only cfg5 --scale 0.25
