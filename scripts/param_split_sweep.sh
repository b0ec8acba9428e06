#!/bin/bash
# C4 (hot-parameter token bucket): ms/step over the lane / wave walker split (SG_PARAM_SHORT_MAX), one box.
mkdir -p gpurun_out
for sm in ${SPLITS:-16 4 8 32 64}; do
  SG_PARAM_SHORT_MAX=$sm timeout -k 10 300 python -u bench_configs.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/psplit_$sm.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/psplit_$sm.log').read().strip().splitlines()[-1]); print('c4', $sm, round(d['ms_per_step'], 4))"
done
