#!/bin/bash
# Round-4 GPU session p: the secondary configs on the current tree + the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), d["roofline"]["kernel_split_ms"])' $O/bench.json
timeout -k 10 900 python3 -u tools/bench_configs.py --only cfg2,cfg3,filter,limit,left,full,shapes,partition,merge,window,cfg4leg,cfg5leg,cfg5 > $O/configs.jsonl 2>$O/configs.err || { tail $O/configs.err; exit 1; }
python3 - $O/configs.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    f=d.get("frac_of_8TBs")
    print(f'{d["config"][:70]:70s} {d["ms_per_run"]:8.2f} ms  kernel {d.get("kernel_ms") or 0:8.2f}  frac {f if f is None else round(f,3)}')
PY
