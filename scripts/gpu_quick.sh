#!/bin/bash
# Quick GPU check: cluster-flow parity tests, then the C3 bench and a kernel-trace profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_flow_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/q_bench.log 2>&1 || { tail -20 gpurun_out/q_bench.log; exit 1; }
tail -1 gpurun_out/q_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value']/1e9, 'G/s ms', d['ms_per_step'], d['phases_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/q_prof.log 2>&1 || exit 1
python scripts/kstats.py $(find gpurun_out/qprof -name '*kernel_stats.csv' | head -1)
