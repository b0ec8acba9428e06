#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile. Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>; continue only on exit 0/1 (test failures), stop on faults
  local name=$1 tmo=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 400 python -u bench.py --steps 10 --warmup 3
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batches 0
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
  # HBM traffic: one counter per pass (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2)
  step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-batches 0
  step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-batches 0
  step pmc_size 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_size -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-batches 0
  step pmc_summary 60 python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_summary.json gpurun_out/pmc_size
fi
if [ "$MODE" = sq ]; then
  # two passes of 8 SQ counters (one block's limit per pass)
  step sq1 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/sq1 -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-batches 0
  step sq2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT -d gpurun_out/sq2 -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-batches 0
  step sq_summary 60 python scripts/sq_summary.py gpurun_out/sq_summary.json 0 gpurun_out/sq1 gpurun_out/sq2
fi
echo done
