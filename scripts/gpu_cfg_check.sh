#!/bin/bash
# gpu_cfg_check.sh <workload> <test files...>: parity tests, then the bench_configs line and a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
w=$1; shift
timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$w.log 2>&1
rc=$?; tail -3 gpurun_out/pt_$w.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench_configs.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${w}_bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/${w}_bench.log').read().strip().splitlines()[-1]);print('$w', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms/step frac', round(d['roofline']['frac'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${w}_prof -o run --output-format csv -- python3 bench_configs.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${w}_prof.log 2>&1 || exit $?
python scripts/kstats.py gpurun_out/${w}_prof/run_kernel_stats.csv > gpurun_out/${w}_kstats.txt 2>&1
grep "k_\|sg::" gpurun_out/${w}_kstats.txt | head -14
