#!/bin/bash
# Cluster param lane / wave walker split re-checked (SG_CPARAM_SHORT_MAX), same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for r in 1 2; do
  for sm in 64 32 128; do
    SG_CPARAM_SHORT_MAX=$sm timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/cpsm_${sm}_$r.json 2>/dev/null || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/cpsm_*.json
