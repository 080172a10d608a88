#!/bin/bash
# Round-4 GPU session g: box calibration + phase B / shard A/B of the fused pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 3 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
head -12 $O/floor.txt
timeout -k 10 500 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_SHARDS=1 libqeh.so:QEH_FUSED_PV=1 \
    libqeh.so:QEH_NO_FUSED=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 tools/probes/host_overhead.py > $O/host.txt 2>&1 && QEH_NO_FUSED=1 timeout -k 10 120 python3 tools/probes/host_overhead.py >> $O/host.txt 2>&1
cat $O/host.txt
