#!/bin/bash
# Round 6 node handle: node GPU tests, then the node bench lines at G = 1, 2, 4 same-device shards (per-shard walker
# CU shares) and one C3 single-handle line on the same box for the ratio.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/node6
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_node_gpu.py \
  > gpurun_out/node6/tests.log 2>&1 || { tail -30 gpurun_out/node6/tests.log; exit 1; }
tail -2 gpurun_out/node6/tests.log
for g in 1 2 4; do
  timeout -k 10 300 python -u bench_configs.py --workload node --shards $g --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/node6/g$g.log 2>&1 || exit $?
  echo "node g$g: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/node6/g$g.log)"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/node6/c3.log 2>&1 || exit $?
echo "single handle: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/node6/c3.log)"
