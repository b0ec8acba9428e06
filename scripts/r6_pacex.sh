#!/bin/bash
# Pace walker timing experiments (variants built with scripts/build_variant.sh; the skip ones give wrong results).
# (The SG_PACE_SKIP_* / SG_PACE_LONG_GRID macros lived in a temporary build of pace.hip for these runs only.)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
P="python -u bench_configs.py --workload pace --steps 3 --warmup 1 --no-cpu-baseline"
for v in cur skipshort skiplong; do
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/px_$v -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
  echo "$v $(python scripts/kstats.py $(ls gpurun_out/r6/px_$v/*kernel_stats.csv | head -1) | grep -E 'k_pace_(long|short)' | tr -s ' ' | tr '\n' ' ')"
  rm -f gpurun_out/r6/px_$v/*kernel_trace.csv
done
for v in cur skipshort skiplong; do
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/px_$v.json 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/px_$v.json | sed "s/^/$v /"
done
