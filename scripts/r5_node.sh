# Round-5 node handle: the node / host-mirror / RLS / pslot-cluster GPU tests, then node bench lines (records path,
# and the legacy sub-request path for comparison).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/node
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_node_gpu.py \
  tests/test_host_mirror_gpu.py tests/test_rls_gpu.py tests/test_pslot_cluster_gpu.py > gpurun_out/node/tests.log 2>&1 \
  || { tail -30 gpurun_out/node/tests.log; exit 1; }
tail -2 gpurun_out/node/tests.log
for g in 1 2 4; do
  timeout -k 10 300 python -u bench_configs.py --workload node --shards $g --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/node/g$g.log 2>&1 || exit $?
  echo "node g$g: $(tail -1 gpurun_out/node/g$g.log | cut -c1-400)"
done
SG_NODE_LEGACY=1 timeout -k 10 300 python -u bench_configs.py --workload node --shards 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/node/g2_legacy.log 2>&1 || exit $?
echo "node g2 legacy: $(tail -1 gpurun_out/node/g2_legacy.log | cut -c1-400)"
