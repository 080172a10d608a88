#!/bin/bash
# Window path: GPU window tests, then config 5 under several env settings (MODES, ';'-separated),
# alternating, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-win}; O=gpurun_out/r3/$TAG; mkdir -p $O
T="timeout -k 10"
if [ -z "$NOTEST" ]; then
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_msd.py tests/test_window.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
IFS=';' read -ra MS <<< "${MODES:-QEH_X=0;QEH_WM_INV2C=0}"
for r in 1 2; do
  for mode in "${MS[@]}"; do
    env $mode $T 300 python tools/bench_configs.py --only ${CFGS:-cfg5} > $O/cfg.jsonl 2> $O/cfg.err || { tail -5 $O/cfg.err; exit 1; }
    python3 -c "
import json
for l in open('$O/cfg.jsonl'):
    d=json.loads(l); print('[$mode]', d['config'][:28], round(d['kernel_ms'],2), 'ms', round(d['frac_of_8TBs'],4))" | tee -a $O/ab.txt
  done
done
