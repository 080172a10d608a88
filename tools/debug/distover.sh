# fixed per-step overhead of the N > 1 metric plan, measured at N = 1 on the per-rank share of N = 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rows in 125000000 1000000000; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --rows $rows > gpurun_out/do_local_$rows.log 2>&1 || { tail -5 gpurun_out/do_local_$rows.log; exit 1; }
  echo "local $rows $(tail -1 gpurun_out/do_local_$rows.log | grep -o '"ms_per_step": [0-9.]*')"
  QEH_BENCH_FORCE_DIST=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 --rows $rows > gpurun_out/do_dist_$rows.log 2>&1 || { tail -5 gpurun_out/do_dist_$rows.log; exit 1; }
  echo "dist  $rows $(tail -1 gpurun_out/do_dist_$rows.log | grep -o '"ms_per_step": [0-9.]*')"
done
