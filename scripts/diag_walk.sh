#!/bin/bash
# Walker diagnostics: serialised-walker kernel times (SG_DEBUG=2), short-class and long-length timers.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
SG_DEBUG=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ser -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ser.log 2>&1 || exit $?
python scripts/kstats.py $(find gpurun_out/ser -name '*kernel_stats.csv' | head -1)
timeout -k 10 120 python -u scripts/walk_counters.py > gpurun_out/wc.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wc.log
timeout -k 10 120 python -u scripts/walk_counters_long.py > gpurun_out/wcl.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wcl.log
