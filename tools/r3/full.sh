#!/bin/bash
# Whole GPU suite, smoke, metric bench, widened metric shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-full}; O=gpurun_out/r3/$TAG; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$T 300 python bench.py --cpu-sample 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('metric', round(d['ms_per_step'],3), round(d['value']/1e9,1), 'G rows/s frac', round(d['roofline']['frac'],4), d['roofline']['kernel_split_ms'])"
$T 300 python tools/bench_configs.py --only ${CFGS:-shapes} > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'][:44], round(d['kernel_ms'],2), 'ms', round(d['frac_of_8TBs'],4), d['dominant_kernel'][:50])"
