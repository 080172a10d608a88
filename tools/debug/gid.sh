set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline.py -m gpu > gpurun_out/gid_tests.log 2>&1 || { tail -30 gpurun_out/gid_tests.log; exit 1; }
tail -3 gpurun_out/gid_tests.log
timeout -k 10 400 python tools/bench_configs.py --only shapes > gpurun_out/shapes_gid.jsonl 2> gpurun_out/shapes_gid.err || { tail -5 gpurun_out/shapes_gid.err; exit 1; }
cut -c1-300 gpurun_out/shapes_gid.jsonl
grep -h -o '"kernel_split_ms": {[^}]*}' gpurun_out/shapes_gid.jsonl
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/bench_gid.log 2>&1 || { tail -5 gpurun_out/bench_gid.log; exit 1; }
tail -1 gpurun_out/bench_gid.log | grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"kernel_split_ms": {[^}]*}'
