#!/bin/bash
# Rehearsal of the driver's multi-rank launch on the one-GPU box (gloo on CPU tensors, every rank on device 0), C3
# and the C5 leg, plus the node line at N=1: the N>1 code paths run end to end.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
SG_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --requests 4000000 > gpurun_out/r6/multi_c3.json 2> gpurun_out/r6/multi_c3.err || exit 1
timeout -k 10 300 python -u bench.py --node --gpus 1 --steps 10 --warmup 3 > gpurun_out/r6/node1.json 2> gpurun_out/r6/node1.err || exit 1
grep -o '"ms_per_step": [0-9.]*\|"n_gpus": [0-9]*' gpurun_out/r6/multi_c3.json gpurun_out/r6/node1.json
