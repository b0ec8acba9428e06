cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T="tests/test_flow_gpu.py::test_cluster_flow_checker_occupy_pass_gpu"
for d in 34; do
  echo "== SG_DEBUG=$d"
  SG_DEBUG=$d timeout -k 5 40 python -u -m pytest "$T" -x -q -m gpu --timeout 25 --timeout-method thread > gpurun_out/dbg_$d.log 2>&1
  rc=$?; echo rc=$rc; grep -v "^  \|^    " gpurun_out/dbg_$d.log | head -30
  [ $rc -le 1 ] || exit $rc
done
