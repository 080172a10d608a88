set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_pipeline.py -m gpu -x -q > gpurun_out/pytest1.log 2>&1 || { echo "pytest failed rc=$?"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke1.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-sample 20000000 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; exit 1; }
cat gpurun_out/bench1.log
