#!/bin/bash
# Round-4 GPU session k: phase A without staging (ring kernel, default) -- parity, then A/B against the
# staged kernel (QEH_FUSED_RING=0) and the ring kernel with 8192-row tiles (libqeh_r4.so) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
QEH_LIB_PATH=$PWD/query-engine_amd/libqeh_r4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py -k "fused or metric_shape" > $O/tests_r4.txt 2>&1 || { echo "tests r4 failed"; tail -30 $O/tests_r4.txt; exit 1; }
tail -2 $O/tests_r4.txt
timeout -k 10 600 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh.so:QEH_FUSED_RING=0 libqeh_r4.so > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc = 0 ] || exit $rc
