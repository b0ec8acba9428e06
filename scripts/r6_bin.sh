#!/bin/bash
# Round 6: binned front half — its GPU tests, the C3 tests, then the bench. Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bin_gpu.py tests/test_flow_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/bin_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/r6/bin_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_timed_path_gpu.py tests/test_fullsize_gpu.py tests/test_async_gpu.py tests/test_codec_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/c3_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r6/c3_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r6/bench_bin.log 2>&1
rc=$?; tail -n 2 gpurun_out/r6/bench_bin.log; [ $rc -ne 0 ] && exit $rc
SG_BIN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r6/bench_nobin.log 2>&1
rc=$?; tail -n 2 gpurun_out/r6/bench_nobin.log; exit $rc
