#!/bin/bash
# Node param / concurrent token parity, then the cparam workload through one handle and the node handle (G = 1, 2, 3).
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_node_tokens_gpu.py tests/test_node_gpu.py > gpurun_out/r6/node_tokens.txt 2>&1 || exit 1
for G in 0 1 2 3; do
  timeout -k 10 240 python -u bench_configs.py --workload cparam --shards $G --no-cpu-baseline --steps 5 --warmup 2 >> gpurun_out/r6/cparam_node.jsonl 2>> gpurun_out/r6/cparam_node.err || exit 1
done
