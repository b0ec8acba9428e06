# Round-5: C3 walker broadcasts A/B (same box) after the full GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_final.log | head; tail -3 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
ROUNDS=3 SPECS="pre:SG_LIB_PATH=build/ab/pre.so cur:SG_LIB_PATH=build/ab/cur.so" bash scripts/ab.sh
