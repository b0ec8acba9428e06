#!/bin/bash
# Round 5: parity of the walker variants (C3 GPU tests through SG_LIB_PATH), then same-box A/B of the pipelined C3 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
T="tests/test_flow_gpu.py tests/test_timed_path_gpu.py tests/test_golden_gpu.py tests/test_fullsize_gpu.py::test_c3_full_size_two_batches"
for v in lpg:0 rs2:1024; do
  lib=${v%%:*} dbg=${v#*:}
  SG_LIB_PATH=build/ab/$lib.so SG_DEBUG=$dbg timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > gpurun_out/r5_par_$lib.txt 2>&1
  rc=$?; echo "parity $lib rc=$rc"; tail -2 gpurun_out/r5_par_$lib.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
SPECS="base:SG_LIB_PATH=build/ab/base.so lp:SG_LIB_PATH=build/ab/lp.so lpg:SG_LIB_PATH=build/ab/lpg.so rs2:SG_LIB_PATH=build/ab/rs2.so,SG_DEBUG=1024" ROUNDS=2 bash scripts/ab.sh || exit $?
SG_LIB_PATH=build/ab/lpg.so timeout -k 10 300 python -u scripts/walk_diag.py --steps 3 --splits 256 > gpurun_out/r5_walkdiag_lpg.txt 2>&1 || exit $?
SG_LIB_PATH=build/ab/lpg.so bash scripts/exp_timeline.sh lpg=0 || exit $?
echo done
