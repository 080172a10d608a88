#!/bin/bash
# Round-4 GPU session m: the MSD payload sort (parity, then Merge::sorted A/B against the LSD passes) and
# the N = 8 rank rehearsal with the stats copy queued ahead of phase A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_merge.py tests/test_executor.py \
    > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_NO_MSD_SORT=1"; do
  env $m timeout -k 10 300 python3 -u tools/bench_configs.py --only merge > $O/merge.jsonl 2>$O/merge.err || { tail $O/merge.err; exit 1; }
  echo "[$m] $(cut -c1-400 $O/merge.jsonl)"
done
QEH_BENCH_RANK_OF=0/8 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/rank08.json 2>$O/rank08.err || { tail $O/rank08.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("rank08", round(d["ms_per_step"],3), d["roofline"]["kernel_split_ms"])' $O/rank08.json
