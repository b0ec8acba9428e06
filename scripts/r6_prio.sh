#!/bin/bash
# The auxiliary (wave walker) stream at the highest priority (SG_AUX_PRIO=1) against the default, same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for r in 1 2; do
  for p in 0 1; do
    SG_AUX_PRIO=$p timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/prio_pace_${p}_$r.json 2>/dev/null || exit 1
    SG_AUX_PRIO=$p timeout -k 10 200 python -u bench_configs.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/prio_c4_${p}_$r.json 2>/dev/null || exit 1
    SG_AUX_PRIO=$p timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r6/prio_cp_${p}_$r.json 2>/dev/null || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/prio_*.json
