#!/bin/bash
# Round-4 GPU session j: phase A as two 512-thread workgroups per CU (QEH_FUSED_2WG=1) -- parity, then
# A/B against the one-workgroup default on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4j; mkdir -p $O
QEH_FUSED_2WG=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py -k "fused or slice_partitioned or metric_shape" > $O/tests_2wg.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests_2wg.txt; exit 1; }
tail -2 $O/tests_2wg.txt
timeout -k 10 600 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh.so:QEH_FUSED_2WG=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
