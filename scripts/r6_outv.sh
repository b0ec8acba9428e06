#!/bin/bash
# k_prep's default results as whole 16-B stores per tile (SG_PREP_OUTV): parity tests of the flow paths, then a
# same-box A/B of the C3 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6 && rm -f gpurun_out/r6/ab.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flow_gpu.py tests/test_bin_gpu.py tests/test_node_gpu.py tests/test_golden_gpu.py tests/test_async_gpu.py tests/test_codec_gpu.py > gpurun_out/r6/outv_tests.txt 2>&1 || { tail -20 gpurun_out/r6/outv_tests.txt; exit 1; }
tail -1 gpurun_out/r6/outv_tests.txt
bash scripts/r6_ab.sh 3 "outv1=SG_PREP_OUTV=1" "outv0=SG_PREP_OUTV=0"
