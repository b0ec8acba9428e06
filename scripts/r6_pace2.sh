#!/bin/bash
# Pace long walker with index-domain guessed searches: parity, same-box A/B against the previous build, kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pace_gpu.py > gpurun_out/r6/pace2_tests.txt 2>&1 || { tail -20 gpurun_out/r6/pace2_tests.txt; exit 1; }
tail -1 gpurun_out/r6/pace2_tests.txt
for r in 1 2; do
  timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace2_new_$r.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/pacebase.so timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace2_base_$r.json 2>/dev/null || exit 1
done
for sm in; do
  SG_PACE_SHORT_MAX=$sm timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace2_sm$sm.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/pace2_new_*.json gpurun_out/r6/pace2_base_*.json gpurun_out/r6/pace2_sm*.json
P="python -u bench_configs.py --workload pace --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/pace2_prof -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/pace2_prof/*kernel_stats.csv | head -1) > gpurun_out/r6/pace2_kstats.txt
rm -f gpurun_out/r6/pace2_prof/*kernel_trace.csv
cat gpurun_out/r6/pace2_kstats.txt | head -12
for v in; do
  [ -f build/ab/$v.so ] || continue
  SG_LIB_PATH=build/ab/$v.so timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace2_$v.json 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/pace2_$v.json | sed "s/^/$v /"
done
