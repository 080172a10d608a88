set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for th in 1000 49 -1; do
  for nt in 0 1; do
  QEH_NT_LOADS=$nt timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --threshold $th > gpurun_out/bench3_th${th}_nt$nt.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "th=$th nt=$nt $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench3_th${th}_nt$nt.log)"
  done
done
