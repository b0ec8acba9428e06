#!/bin/bash
# Node handle with the shards enqueued from parallel host threads: node tests, node bench lines at G = 1, 2, 4, and
# the C5 node leg at N = 1 after the metric-pass host changes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6 && rm -f gpurun_out/r6/node2.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_node_gpu.py tests/test_node_tokens_gpu.py tests/test_metrics_gpu.py tests/test_local_shard_gpu.py > gpurun_out/r6/node2_tests.txt 2>&1 || exit 1
for g in 1 2 4; do
  timeout -k 10 240 python -u bench_configs.py --workload node --shards $g --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r6/node2.jsonl 2>> gpurun_out/r6/node2.err || exit 1
done
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/c5_n1b.json 2> gpurun_out/r6/c5_n1b.err || exit 1
