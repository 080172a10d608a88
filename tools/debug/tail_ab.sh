set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_pipeline.py tests/test_executor.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { tail -20 gpurun_out/tail_tests.log; exit 1; }
tail -1 gpurun_out/tail_tests.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/t_$name.log 2>&1 || { tail -5 gpurun_out/t_$name.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/t_$name.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],3), 'ms/step', round(r['kernel_ms'],3), 'kernel', {k: round(v,3) for k,v in r['kernel_split_ms'].items()})"
}
for rep in 1 2 3; do run after X=1; run beside QEH_TAIL_BESIDE=1; done
