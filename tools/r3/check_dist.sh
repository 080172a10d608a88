#!/bin/bash
# After a change to the distributed plan / bench: its GPU tests, smoke, the default bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r3/${1:-checkdist}; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py tests/test_pipeline.py tests/test_abi.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$T 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(round(d['value']/1e9,1),'G rows/s', round(d['ms_per_step'],3),'ms', 'frac', round(d['roofline']['frac'],3), d['roofline']['kernel_split_ms'])"
