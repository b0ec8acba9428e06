#!/bin/bash
# HBM bytes per kernel of the C3 pipeline (serialized walkers): FETCH_SIZE and WRITE_SIZE in separate passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp SG_DEBUG=${SG_DEBUG:-2}
rm -rf gpurun_out/pmcb; mkdir -p gpurun_out/pmcb
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcb/f -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcb/f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcb/w -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcb/w.log 2>&1 || exit 1
python scripts/pmc_table.py gpurun_out/pmcb
