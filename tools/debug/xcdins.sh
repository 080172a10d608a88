set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rows in 125000000 1000000000; do for x in 0 1 0 1; do
  QEH_INSERT_XCD=$x timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --rows $rows > gpurun_out/xi_$x.log 2>&1 || { tail -5 gpurun_out/xi_$x.log; exit 1; }
  echo "rows $rows xcd $x $(tail -1 gpurun_out/xi_$x.log | grep -o '"ms_per_step": [0-9.]*\|"build_ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done; done
