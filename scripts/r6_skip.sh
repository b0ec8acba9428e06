#!/bin/bash
# k_skip_apply on the wave walker's stream (beside the short walker): flow / node / bin parity, then the C3 step
# against the previous build on the same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6 && rm -f gpurun_out/r6/ab.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flow_gpu.py tests/test_bin_gpu.py tests/test_node_gpu.py tests/test_golden_gpu.py tests/test_timed_path_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r6/skip_tests.txt 2>&1 || { tail -20 gpurun_out/r6/skip_tests.txt; exit 1; }
tail -1 gpurun_out/r6/skip_tests.txt
bash scripts/r6_ab.sh 3 "new=SG_X=0" "base=SG_LIB_PATH=build/ab/c3base.so"
