#!/bin/bash
# k_local_prep with and without its first-digit LDS histogram (lpnohist: a timing build, wrong sort; the
# SG_LP_NO_HIST macro lived in a temporary build of local.hip).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for w in c2 c5; do
  P="python -u bench_configs.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline"
  for v in lpbase lpnohist; do
    SG_LIB_PATH=build/ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/lpx_${w}_$v -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
    echo "$w $v $(python scripts/kstats.py $(ls gpurun_out/r6/lpx_${w}_$v/*kernel_stats.csv | head -1) | grep -E 'k_local_prep' | tr -s ' ')"
    rm -f gpurun_out/r6/lpx_${w}_$v/*kernel_trace.csv
  done
done
