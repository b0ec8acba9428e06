#!/bin/bash
# Cluster param round-0 walkers alone and together (cpskips / cpskipl: timing builds that skip one walker in round 0,
# wrong results; the SG_CP_SKIP_* macros lived in a temporary build of cparam.hip).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
P="python -u bench_configs.py --workload cparam --steps 3 --warmup 1 --no-cpu-baseline"
for v in cpcur cpskips cpskipl; do
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/cpx_$v.json 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/cpx_$v.json | sed "s/^/$v /"
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/cpx_$v -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
  python scripts/kstats.py $(ls gpurun_out/r6/cpx_$v/*kernel_stats.csv | head -1) > gpurun_out/r6/cpx_$v.txt 2>&1 || true
  rm -f gpurun_out/r6/cpx_$v/*kernel_trace.csv
  echo "$v"; grep -E "k_cp_walk2" gpurun_out/r6/cpx_$v.txt
done
