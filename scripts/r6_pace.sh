#!/bin/bash
# Pace with records carrying acquire and the millisecond table: parity, same-box A/B against the previous build, the
# PMC traffic of the new kernels (three passes) and their kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pace_gpu.py tests/test_local_rules_gpu.py > gpurun_out/r6/pace_tests.txt 2>&1 || { tail -20 gpurun_out/r6/pace_tests.txt; exit 1; }
tail -1 gpurun_out/r6/pace_tests.txt
for r in 1 2; do
  timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace_new_$r.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/pacebase.so timeout -k 10 200 python -u bench_configs.py --workload pace --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/pace_base_$r.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/pace_new_*.json gpurun_out/r6/pace_base_*.json
P="python -u bench_configs.py --workload pace --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6/pace_fetch -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6/pace_write -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d gpurun_out/r6/pace_size -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/r6/pace_fetch gpurun_out/r6/pace_write gpurun_out/r6/pace_pmc_summary.json gpurun_out/r6/pace_size || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/pace_prof -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/pace_prof/*kernel_stats.csv | head -1) > gpurun_out/r6/pace_kstats.txt
rm -f gpurun_out/r6/pace_prof/*kernel_trace.csv
find gpurun_out/r6/pace_fetch gpurun_out/r6/pace_write gpurun_out/r6/pace_size -name "*.csv" -size +20M -delete
