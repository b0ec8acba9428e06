# A/B of the pipelined local path on one box: C2 and C5 (bench_configs) for each "label:ENV=V,ENV=V" in $SPECS.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/abl
for r in $(seq 1 ${ROUNDS:-1}); do
  for w in ${WORKLOADS:-c2 c5}; do
    st="--steps 10 --warmup 3"; [ $w = c5 ] && st="--steps 4 --warmup 1"; [ $w = cparam ] && st="--steps 4 --warmup 2"
    for spec in $SPECS; do
      label=${spec%%:*}; envs=${spec#*:}
      env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python -u bench_configs.py --workload $w $st --no-cpu-baseline > gpurun_out/abl/${w}_$label$r.log 2>&1 || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/abl/${w}_$label$r.log').read().strip().splitlines()[-1]); print('$w', '$label', $r, round(d['ms_per_step'],4))"
    done
  done
done
