#!/bin/bash
# Kernel statistics of the slot workload (the cx walkers after the LDS changes).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/slotprof -o run --output-format csv -- \
  python -u bench_configs.py --workload slot --steps 2 --warmup 1 > gpurun_out/r6/slotprof.log 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/slotprof/*kernel_stats.csv | head -1) > gpurun_out/r6/slot_kstats.txt
rm -f gpurun_out/r6/slotprof/*kernel_trace.csv
