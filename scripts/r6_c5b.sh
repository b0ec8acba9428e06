#!/bin/bash
# The C5 node leg with the metric pass enqueued behind the batch (no pipeline drain): device-row parity tests, the
# two-rank rehearsal with parity, the N=1 line; then the C3 env-knob A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_local_shard_gpu.py tests/test_metrics_gpu.py tests/test_local_gpu.py > gpurun_out/r6/c5b_tests.txt 2>&1 || { tail -20 gpurun_out/r6/c5b_tests.txt; exit 1; }
tail -1 gpurun_out/r6/c5b_tests.txt
SG_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c5 --gpus 2 --resources 200000 --requests 2000000 --steps 4 --warmup 2 > gpurun_out/r6/c5b_rehearsal.json 2> gpurun_out/r6/c5b_rehearsal.err || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/r6/c5b_n1.json 2> gpurun_out/r6/c5b_n1.err || exit 1
bash scripts/r6_ab2.sh
