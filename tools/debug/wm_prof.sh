set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wmprof -o wm -- python tools/debug/wm_time.py > gpurun_out/wm_prof.log 2>&1; rc=$?
f=$(find gpurun_out/wmprof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -24
exit $rc
