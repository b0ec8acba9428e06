#!/bin/bash
# ms/step of one bench_configs workload over its lane / wave walker split: WL=pace VAR=SG_PACE_SHORT_MAX SPLITS="..."
mkdir -p gpurun_out
for sm in $SPLITS; do
  env $VAR=$sm timeout -k 10 300 python -u bench_configs.py --workload $WL --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/split_${WL}_$sm.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/split_${WL}_$sm.log').read().strip().splitlines()[-1]); print('$WL', $sm, round(d['ms_per_step'], 4))"
done
