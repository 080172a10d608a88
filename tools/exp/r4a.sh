#!/bin/bash
# Round-4 first GPU session: phase-A traffic floor, early-issue A/B, the new parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 120 tools/ubench/floor_ubench 1000000000 5 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
cat $O/floor.txt
timeout -k 10 400 python3 tools/exp_slice.py --rounds 3 libqeh.so libqeh_exp1.so > $O/early.txt 2>&1 || { echo ab failed; cat $O/early.txt; exit 1; }
cat $O/early.txt
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lds_rank.py \
    tests/test_merge.py "tests/test_pipeline.py::test_config2_full_size_vs_oracle" \
    "tests/test_pipeline.py::test_metric_full_size_vs_oracle" > $O/tests.txt 2>&1
rc=$?; tail -30 $O/tests.txt; exit $rc
