#!/bin/bash
# Parity tests, the C3 bench, and a kernel-trace profile with the walkers serialised (SG_DEBUG=2), so each
# kernel's duration is its standalone time. Usage: scripts/gpu_prof.sh [tag] [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-p}; shift
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_$TAG.log | cut -c1-300
grep -o '"phases_ms": {[^}]*}' gpurun_out/bench_$TAG.log
SG_DEBUG=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/rocprof_$TAG.log 2>&1 || exit $?
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -n 1)
grep -E '"k_|Name' "$f" | cut -d, -f1-4
