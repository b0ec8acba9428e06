# A/B runs on one box: bench (pipelined C3) for each "label:ENV=V,ENV=V" spec in $SPECS, $ROUNDS rounds each.
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $SPECS; do
    label=${spec%%:*}; envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/ab_$label$r.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab_$label$r.log').read().strip().splitlines()[-1]); print('$label', $r, round(d['ms_per_step'],4), round(d['phases_ms']['device_total_one_batch_unpipelined'],4))"
  done
done
