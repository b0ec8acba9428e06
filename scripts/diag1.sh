#!/bin/bash
# Round-5 first session: the new parity tests, then C3 walker diagnostics (per length class), a bench line and a
# kernel timeline of the pipelined step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pslot_cluster_gpu.py tests/test_rls_gpu.py tests/test_pslot_gpu.py > gpurun_out/r5_newtests.txt 2>&1
rc=$?; echo "newtests rc=$rc"; tail -3 gpurun_out/r5_newtests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/walk_diag.py --steps 5 > gpurun_out/r5_walkdiag.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r5_base_bench.txt 2>&1 || exit $?
bash scripts/exp_timeline.sh base=0 || exit $?
echo done
