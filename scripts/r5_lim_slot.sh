# Round-5: limiter batches pipelined (tests, bench lines with and without SG_LIM_PIPE=0, kernel stats) and the slot
# workload (bench line + kernel stats).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/ls; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_async_gpu.py \
  tests/test_lim_exchange_gpu.py tests/test_flow_gpu.py tests/test_node_gpu.py > gpurun_out/ls/tests.log 2>&1 || { tail -30 gpurun_out/ls/tests.log; exit 1; }
tail -2 gpurun_out/ls/tests.log
for v in 1 0; do
  SG_LIM_PIPE=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 --limiter-qps 1e12 > gpurun_out/ls/lim_pipe$v.log 2>&1 || exit $?
  echo "limiter 1e12 SG_LIM_PIPE=$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ls/lim_pipe$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ls/prof_lim -o run --output-format csv -- \
  python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 --limiter-qps 1e12 > gpurun_out/ls/prof_lim.log 2>&1 || exit $?
timeout -k 10 900 python -u bench_configs.py --workload slot --steps 2 --warmup 1 > gpurun_out/ls/slot.log 2>&1 || { tail -5 gpurun_out/ls/slot.log; exit 1; }
echo "slot: $(tail -1 gpurun_out/ls/slot.log | cut -c1-300)"
echo done
