#!/bin/bash
# Round-4 GPU session b: write-layout floor (interleaved slots) + the payload-sort fix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 180 tools/ubench/floor_ubench 1000000000 5 > $O/floor.txt 2>&1 || { echo floor failed; cat $O/floor.txt; exit 1; }
cat $O/floor.txt
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lds_rank.py \
    tests/test_merge.py "tests/test_pipeline.py::test_config2_full_size_vs_oracle" \
    "tests/test_pipeline.py::test_metric_full_size_vs_oracle" > $O/tests.txt 2>&1
rc=$?; tail -30 $O/tests.txt; exit $rc
