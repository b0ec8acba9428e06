# Round-5: pipelined node batches (tests + bench lines), bench.py --node, and the C3 limiter-on lines with kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/node2; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_node_gpu.py \
  > gpurun_out/node2/tests.log 2>&1 || { tail -30 gpurun_out/node2/tests.log; exit 1; }
tail -2 gpurun_out/node2/tests.log
for g in 1 2 4; do
  timeout -k 10 300 python -u bench_configs.py --workload node --shards $g --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/node2/g$g.log 2>&1 || exit $?
  echo "node g$g: $(tail -1 gpurun_out/node2/g$g.log | python -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_per_step"],3), d["extra"])')"
done
timeout -k 10 300 python -u bench_configs.py --workload node --shards 1 --steps 10 --warmup 3 --no-cpu-baseline --local-sync > gpurun_out/node2/g1_sync.log 2>&1 || exit $?
echo "node g1 sync: $(tail -1 gpurun_out/node2/g1_sync.log | cut -c1-200)"
timeout -k 10 300 python -u bench.py --node --gpus 1 --steps 10 --warmup 3 > gpurun_out/node2/bench_node1.log 2>&1 || exit $?
echo "bench --node: $(tail -1 gpurun_out/node2/bench_node1.log | cut -c1-300)"
for q in 1e12 30000; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 --limiter-qps $q > gpurun_out/node2/lim_$q.log 2>&1 || exit $?
  echo "limiter $q: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/node2/lim_$q.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/node2/prof_lim -o run --output-format csv -- \
  python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 --limiter-qps 1e12 > gpurun_out/node2/prof_lim.log 2>&1 || exit $?
echo done
