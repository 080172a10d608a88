#!/bin/bash
# Round-4 GPU session d: the fused pipeline -- parity tests, then A/B against the prelaunch path, then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pipeline.py \
    > $O/tests.txt 2>&1 || { echo tests failed; tail -40 $O/tests.txt; exit 1; }
tail -5 $O/tests.txt
timeout -k 10 400 python3 tools/exp_slice.py --rounds 2 libqeh.so libqeh.so:QEH_NO_FUSED=1 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
