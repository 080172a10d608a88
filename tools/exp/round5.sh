#!/bin/bash
# Round-5 GPU sessions, one function each (the runs the profiles/r05 records and DESIGN.md quote).
# usage (on the GPU box, from the repo root): bash tools/exp/round5.sh <session>, e.g. r5a
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"

run_tests() {  # $1 = output file, rest = pytest targets
    local out=$1; shift
    timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu "$@" > "$out" 2>&1
    local rc=$?; tail -25 "$out"; return $rc
}

r5a() {
# phase A: flush after rank (no store round trip in front of the loop head's vmcnt wait) and the
# branch-free predicate, A/B against the round-4 library; then the new parity tests
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 500 python3 tools/exp_slice.py --rounds 3 libqeh_base.so libqeh_late0.so libqeh.so > $O/ab.txt 2>&1 \
    || { echo ab failed; cat $O/ab.txt; exit 1; }
cat $O/ab.txt
run_tests $O/tests.txt tests/test_employees_departments.py tests/test_config4.py \
    "tests/test_distributed.py::test_device_tensor_collectives_several_ranks_on_one_gpu" tests/test_pipeline.py
}

"$@"
