#!/bin/bash
# Local chain (C2, C5): ms/step over the lane / wave walker split (SG_SHORT_MAX), one box.
mkdir -p gpurun_out
for w in ${WORKLOADS:-c2 c5}; do
  for sm in ${SPLITS:-256 128 64 32}; do
    SG_SHORT_MAX=$sm timeout -k 10 300 python -u bench_configs.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/split_${w}_$sm.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/split_${w}_$sm.log').read().strip().splitlines()[-1]); print('$w', $sm, round(d['ms_per_step'], 4))"
  done
done
