#!/bin/bash
# config 5 per-kernel times and HBM bytes (one ROW_NUMBER query at 1e9 rows): kernel trace + FETCH/WRITE passes
set -e
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_wm/${1:-run}
mkdir -p $out
QEH_AB_CHILD=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/exp/wm_parts.py kt 1000000000 1048576 > $out/kt.log 2>&1
QEH_AB_CHILD=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 tools/exp/wm_parts.py fetch 1000000000 1048576 > $out/fetch.log 2>&1
QEH_AB_CHILD=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 tools/exp/wm_parts.py write 1000000000 1048576 > $out/write.log 2>&1
python3 tools/pmc_traffic.py $out > $out/summary.txt
echo done
