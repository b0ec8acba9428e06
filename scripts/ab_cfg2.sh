#!/bin/bash
# A/B of library builds on one bench_configs workload with short runs: WL=c5 STEPS=3 WARMUP=1 SPECS="a:ENV=V,.. b:.."
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $SPECS; do
    label=${spec%%:*}; envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 400 python -u bench_configs.py --workload $WL --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline > gpurun_out/abc_${WL}_$label$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abc_${WL}_$label$r.log').read().strip().splitlines()[-1]); print('$WL', '$label', $r, round(d['ms_per_step'],4), d.get('fixed_point_rounds'))"
  done
done
