#!/bin/bash
# C3 lane / wave walker split re-checked on the final build (SG_SHORT_MAX), same box, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for r in 1 2; do
  for sm in 256 192 320; do
    SG_SHORT_MAX=$sm timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/c3sm_${sm}_$r.json 2>/dev/null || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/c3sm_*.json
