set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wmprof -o wm -- python tools/bench_configs.py --only cfg5 > gpurun_out/wm_prof.log 2>&1; rc=$?
tail -2 gpurun_out/wm_prof.log | cut -c1-600
f=$(find gpurun_out/wmprof -name "*kernel_stats.csv" | head -1); head -20 "$f" | cut -d, -f1-8
exit $rc
