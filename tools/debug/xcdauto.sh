set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_pipeline.py -m gpu -k "full_size or metric_shape" > gpurun_out/xa_tests.log 2>&1 || { tail -30 gpurun_out/xa_tests.log; exit 1; }
tail -1 gpurun_out/xa_tests.log
for rows in 125000000 1000000000 125000000 1000000000; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --rows $rows > gpurun_out/xa.log 2>&1 || { tail -5 gpurun_out/xa.log; exit 1; }
  echo "rows $rows $(tail -1 gpurun_out/xa.log | grep -o '"ms_per_step": [0-9.]*\|"build_ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
