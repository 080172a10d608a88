set -o pipefail
for S in 0 3 6 0 2; do
  QEH_SLICE_SPLITS=$S timeout -k 10 200 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/b_$S.log 2>&1 || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/b_$S.log').read().strip().splitlines()[-1]); print('splits=$S', round(d['ms_per_step'],3), d['roofline']['kernel_split_ms'])"
done
