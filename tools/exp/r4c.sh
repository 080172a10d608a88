#!/bin/bash
# Round-4 GPU session c: phase A with / without the build beside it, early-issue variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 500 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_OVERLAP=1 libqeh_exp1.so \
    libqeh_exp1.so:QEH_NO_OVERLAP=1 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
