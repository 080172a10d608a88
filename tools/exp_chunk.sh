#!/bin/bash
# A/B of slice-pipeline variants on the metric bench, alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/v_$name.log 2>&1 || { tail -5 gpurun_out/v_$name.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/v_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel ms', {k: round(v,3) for k,v in r['kernel_split_ms'].items()})"
}
for rep in 1 2; do
  run base X=1
  run cached QEH_SLICE_CACHED_STORE=1
  run chunk16k QEH_SLICE_CHUNK_TILES=16384
  run chunk32k QEH_SLICE_CHUNK_TILES=32768
  run noprelaunch QEH_NO_OVERLAP=1
done
