#!/bin/bash
# Round-4 GPU session i: the new fused defaults (64-item chunks, paired phase-B loads, one state copy),
# the bench line, and the N = 8 per-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipeline.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), d["roofline"]["kernel_split_ms"])' $O/bench.json
QEH_BENCH_RANK_OF=0/8 PYTHONFAULTHANDLER=1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.json 2>$O/rank08.err
echo "rank08 rc=$?"; cat $O/rank08.json; tail -5 $O/rank08.err
timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg5leg,cfg5 > $O/cfg5.jsonl 2>$O/cfg5.err || { tail $O/cfg5.err; exit 1; }
cat $O/cfg5.jsonl
