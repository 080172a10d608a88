set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for R in 16777216 33554432 67108864 268435456 1000000000; do
  for P in fused part; do
    if [ $P = part ]; then export QEH_PART_MIN_BYTES=0; else unset QEH_PART_MIN_BYTES; fi
    timeout -k 10 300 python bench.py --rows $R --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/b11_${P}_${R}.log 2>&1 || { tail gpurun_out/b11_${P}_${R}.log; exit 1; }
    python - "$R" "$P" gpurun_out/b11_${P}_${R}.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r=d["roofline"]; n=int(sys.argv[1])
print(sys.argv[2], n, "kernel_ms=%.3f ns_per_row=%.4f step_ms=%.3f frac=%.3f" % (r["kernel_ms"], r["kernel_ms"]*1e6/n, d["ms_per_step"], r["frac"]))
PY
  done
done
