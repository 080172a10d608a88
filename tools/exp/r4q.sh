#!/bin/bash
# Round-4 GPU session q: window pass-1 histogram folded into the key min/max read -- parity, then
# config 5 A/B against the separate histogram (QEH_WM_NO_FOLD=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_join_sort_window.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in "" "QEH_WM_NO_FOLD=1" "" "QEH_WM_NO_FOLD=1"; do
  env $m timeout -k 10 300 python3 -u tools/bench_configs.py --only cfg5 > $O/cfg5.jsonl 2>$O/cfg5.err || { tail $O/cfg5.err; exit 1; }
  echo "[$m] $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(round(d["ms_per_run"],2), round(d["kernel_ms"],2), round(d["window_partition"],2), round(d["window_sort"],2), round(d["window_place"],2))' $O/cfg5.jsonl)"
done
