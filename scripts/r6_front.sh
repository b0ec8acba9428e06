#!/bin/bash
# C3 front/back CU split re-checked after the k_prep histogram change (SG_FRONT_EIGHTHS), same box, 2 rounds each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for r in 1 2; do
  for k in 4 3 2 5; do
    SG_FRONT_EIGHTHS=$k timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/front_${k}_$r.json 2>/dev/null || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/front_*.json
