cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/shard
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_local_shard_gpu.py \
  tests/test_metrics_gpu.py tests/test_slot_chain_gpu.py > gpurun_out/shard/tests.log 2>&1 || { tail -30 gpurun_out/shard/tests.log; exit 1; }
tail -2 gpurun_out/shard/tests.log
