#!/bin/bash
# Kernel traces of the node bench at G = 1 and 4 same-device shards (the G=4 regression), timelines of the last
# steps, and of the C5 leg at N=1 (where the per-step metric rollup's time goes).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for g in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/nprof_g$g -o run --output-format csv -- \
    python -u bench_configs.py --workload node --shards $g --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r6/nprof_g$g.log 2>&1 || exit 1
  python scripts/node_tl.py $(ls gpurun_out/r6/nprof_g$g/*kernel_trace.csv | head -1) 10 > gpurun_out/r6/ntl_g$g.txt || exit 1
  python scripts/kstats.py $(ls gpurun_out/r6/nprof_g$g/*kernel_stats.csv | head -1) > gpurun_out/r6/nkstats_g$g.txt || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/c5prof -o run --output-format csv -- \
  python -u bench.py --workload c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r6/c5prof.log 2>&1 || exit 1
python scripts/node_tl.py $(ls gpurun_out/r6/c5prof/*kernel_trace.csv | head -1) 12 > gpurun_out/r6/c5tl.txt
python scripts/kstats.py $(ls gpurun_out/r6/c5prof/*kernel_stats.csv | head -1) > gpurun_out/r6/c5kstats.txt
