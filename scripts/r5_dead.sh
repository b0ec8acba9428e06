# Round-5: the dead-period parity test of the slot chain (every walker mode).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/dead
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_slot_chain_gpu.py::test_dead_periods" \
  > gpurun_out/dead/tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/dead/tests.log | head -20; tail -5 gpurun_out/dead/tests.log; exit 1; }
tail -2 gpurun_out/dead/tests.log
