#!/bin/bash
# Round-4 GPU session s: window groups of 2^sb keys (key ranges up to 2^24) -- parity, then the wide-key shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_lds_rank.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python3 -u tools/bench_configs.py --only window_lsd,cfg5 > $O/window.jsonl 2>$O/window.err || { tail $O/window.err; exit 1; }
python3 - $O/window.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d['config'], round(d['ms_per_run'],2), round(d['kernel_ms'],2), round(d['frac_of_8TBs'],4), d.get('kernel_split_ms'))
PY
