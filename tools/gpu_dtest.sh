set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dtest.log 2>&1 || { tail -30 gpurun_out/dtest.log; exit 1; }
tail -1 gpurun_out/dtest.log
for w in cfg4 metric cfg4; do
timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_$w.log 2>&1 || { tail -5 gpurun_out/b_$w.log; exit 1; }
tail -1 gpurun_out/b_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d.get('result_check','')[:60])"
done
