#!/bin/bash
# cparam workload: bench line + per-kernel stats (run from the repo root on the GPU box)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench_configs.py --workload cparam --steps 3 --warmup 1 --cpu-events 1000000 > gpurun_out/cparam_bench.json 2> gpurun_out/cparam_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cparam_prof -o cp --output-format csv -- python3 bench_configs.py --workload cparam --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cparam_prof.log 2>&1
