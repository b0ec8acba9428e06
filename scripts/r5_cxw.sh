# Round-5: the cx wave walker — parity (slot chain, local chain, pslot-cluster, embedded server) and the slot line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/cxw
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_slot_chain_gpu.py \
  tests/test_local_gpu.py tests/test_local_rules_gpu.py tests/test_pslot_cluster_gpu.py tests/test_embedded_server_gpu.py \
  tests/test_local_shard_gpu.py tests/test_local_pipeline_gpu.py tests/test_pslot_gpu.py \
  > gpurun_out/cxw/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/cxw/tests.log | head -20; tail -5 gpurun_out/cxw/tests.log; exit 1; }
tail -2 gpurun_out/cxw/tests.log
SG_DEBUG=64 timeout -k 10 900 python -u bench_configs.py --workload slot --steps 2 --warmup 1 > gpurun_out/cxw/slot.log 2>&1 || { tail -5 gpurun_out/cxw/slot.log; exit 1; }
grep "cxw " gpurun_out/cxw/slot.log; echo "slot: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cxw/slot.log)"
if [ -n "$CXW_MIN_ALT" ]; then
  SG_CXW_MIN=$CXW_MIN_ALT timeout -k 10 900 python -u bench_configs.py --workload slot --steps 2 --warmup 1 > gpurun_out/cxw/slot_alt.log 2>&1 || { tail -5 gpurun_out/cxw/slot_alt.log; exit 1; }
  echo "slot SG_CXW_MIN=$CXW_MIN_ALT: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cxw/slot_alt.log)"
fi
