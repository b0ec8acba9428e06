#!/bin/bash
# A/B of two library builds on one bench_configs workload: WL=c4 SPECS="old:SG_LIB_PATH=... new:SG_LIB_PATH=..."
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $SPECS; do
    label=${spec%%:*}; envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python -u bench_configs.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abc_$label$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abc_$label$r.log').read().strip().splitlines()[-1]); print('$WL', '$label', $r, round(d['ms_per_step'],4))"
  done
done
