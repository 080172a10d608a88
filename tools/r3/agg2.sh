mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_aggregate.py > gpurun_out/r3/pyt_agg2.log 2>&1; rc=$?
tail -3 gpurun_out/r3/pyt_agg2.log
[ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/bench_configs.py --only shapes > gpurun_out/r3/shapes.jsonl 2> gpurun_out/r3/shapes.err || { tail -5 gpurun_out/r3/shapes.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3/shapes.jsonl'):
    d=json.loads(l); print(d['config'][:40], round(d['kernel_ms'],2), round(d['frac_of_8TBs'],4), d['dominant_kernel'])"
