#!/bin/bash
# Cluster param lane walker changes: parity (single handle and node), same-box A/B against the previous build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cparam_gpu.py tests/test_node_tokens_gpu.py > gpurun_out/r6/cp_tests.txt 2>&1 || { tail -20 gpurun_out/r6/cp_tests.txt; exit 1; }
tail -1 gpurun_out/r6/cp_tests.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/cp_new_$r.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/cpbase.so timeout -k 10 300 python -u bench_configs.py --workload cparam --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/cp_base_$r.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/cp_new_*.json gpurun_out/r6/cp_base_*.json
