#!/bin/bash
# Hot-param walkers with the bucketed millisecond lookup: parity, same-box A/B against the previous build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_param_gpu.py > gpurun_out/r6/param_tests.txt 2>&1 || { tail -20 gpurun_out/r6/param_tests.txt; exit 1; }
tail -1 gpurun_out/r6/param_tests.txt
for r in 1 2; do
  timeout -k 10 200 python -u bench_configs.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/c4_new_$r.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/parambase.so timeout -k 10 200 python -u bench_configs.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/c4_base_$r.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/c4_new_*.json gpurun_out/r6/c4_base_*.json
P="python -u bench_configs.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/c4_prof -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/c4_prof/*kernel_stats.csv | head -1) > gpurun_out/r6/c4_kstats.txt
rm -f gpurun_out/r6/c4_prof/*kernel_trace.csv
head -8 gpurun_out/r6/c4_kstats.txt
