#!/bin/bash
# Secondary benchmark lines (C2, C4, C5, pace, codec, cparam) into gpurun_out/bc_*.log.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for w in c2 c4; do
  timeout -k 10 300 python -u bench_configs.py --workload $w > gpurun_out/bc_$w.log 2>&1 || exit $?
  echo "$w: $(tail -1 gpurun_out/bc_$w.log | cut -c1-200)"
done
timeout -k 10 600 python -u bench_configs.py --workload c5 --steps 3 --warmup 1 > gpurun_out/bc_c5.log 2>&1 || exit $?
echo "c5: $(tail -1 gpurun_out/bc_c5.log | cut -c1-200)"
for w in pace codec cparam; do
  timeout -k 10 400 python -u bench_configs.py --workload $w --steps 3 --warmup 1 > gpurun_out/bc_$w.log 2>&1 || exit $?
  echo "$w: $(tail -1 gpurun_out/bc_$w.log | cut -c1-200)"
done
