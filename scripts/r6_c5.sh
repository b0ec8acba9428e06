#!/bin/bash
# Node param / concurrent tokens and the device metric rows (parity), the C5 multi-GPU leg rehearsed on one GPU
# (2 ranks, gloo, parity on), the C5 leg at N=1 full size, and the cparam workload through one handle and the node.
set -o pipefail
mkdir -p gpurun_out/r6 && rm -f gpurun_out/r6/cparam_node.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_node_tokens_gpu.py tests/test_node_gpu.py tests/test_local_shard_gpu.py tests/test_metrics_gpu.py > gpurun_out/r6/c5_tests.txt 2>&1 || exit 1
SG_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --workload c5 --gpus 2 --resources 200000 --requests 2000000 --steps 4 --warmup 2 > gpurun_out/r6/c5_rehearsal.json 2> gpurun_out/r6/c5_rehearsal.err || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/r6/c5_n1.json 2> gpurun_out/r6/c5_n1.err || exit 1
for G in 0 1 2 3; do
  timeout -k 10 240 python -u bench_configs.py --workload cparam --shards $G --no-cpu-baseline --steps 5 --warmup 2 >> gpurun_out/r6/cparam_node.jsonl 2>> gpurun_out/r6/cparam_node.err || exit 1
done
rm -f gpurun_out/r6/node_hwq.jsonl
for G in 2 4; do
  timeout -k 10 240 python -u bench_configs.py --workload node --shards $G --no-cpu-baseline --steps 10 --warmup 3 >> gpurun_out/r6/node_hwq.jsonl 2>> gpurun_out/r6/node_hwq.err || exit 1
  GPU_MAX_HW_QUEUES=16 timeout -k 10 240 python -u bench_configs.py --workload node --shards $G --no-cpu-baseline --steps 10 --warmup 3 >> gpurun_out/r6/node_hwq.jsonl 2>> gpurun_out/r6/node_hwq.err || exit 1
done
