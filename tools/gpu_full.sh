set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/bench_configs.py --only window > gpurun_out/window.jsonl 2>&1 || { tail -5 gpurun_out/window.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*' gpurun_out/window.jsonl
