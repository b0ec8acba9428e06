#!/bin/bash
# C5 lane walker: timing with and without the exits' event gathers (noev: a timing build, wrong results).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
P="python -u bench_configs.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline"
for v in lbase noev; do
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/c5x_$v -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
  echo "$v $(python scripts/kstats.py $(ls gpurun_out/r6/c5x_$v/*kernel_stats.csv | head -1) | grep -E 'k_lwalk_(long|short)' | tr -s ' ' | tr '\n' ' ')"
  rm -f gpurun_out/r6/c5x_$v/*kernel_trace.csv
done
