#!/bin/bash
# cparam parity tests, then the bench line and a kernel trace (one GPU call)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cparam_gpu.py tests/test_golden_gpu.py tests/test_lim_exchange_gpu.py tests/test_metrics_gpu.py tests/test_host_mirror_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_cp.log 2>&1
rc=$?; tail -3 gpurun_out/pt_cp.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cp_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/cp_bench.log').read().strip().splitlines()[-1]);print('cparam', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms/step rounds', d.get('fixed_point_rounds'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cp_prof -o cp --output-format csv -- python3 bench_configs.py --workload cparam --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cp_prof.log 2>&1 || exit $?
python scripts/kstats.py gpurun_out/cp_prof/cp_kernel_stats.csv > gpurun_out/cp_kstats.txt 2>&1
head -16 gpurun_out/cp_kstats.txt
python scripts/cp_rounds.py gpurun_out/cp_prof/cp_kernel_trace.csv > gpurun_out/cp_rounds.txt
