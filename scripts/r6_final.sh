#!/bin/bash
# Round 6 final checkpoint: the whole -m gpu suite, smoke, the C3 bench line, the pace and C4 lines, and the pace
# kernels' PMC traffic after the search change.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6z
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6z/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r6z/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r6z/pytest_gpu.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6z/bench.json 2> gpurun_out/r6z/bench.err || exit 1
cat gpurun_out/r6z/bench.json
timeout -k 10 300 python -u bench_configs.py --workload pace --steps 10 --warmup 3 > gpurun_out/r6z/pace.json 2> gpurun_out/r6z/pace.err || exit 1
timeout -k 10 300 python -u bench_configs.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6z/c4.json 2> gpurun_out/r6z/c4.err || exit 1
timeout -k 10 400 python -u bench_configs.py --workload cparam --steps 5 --warmup 2 > gpurun_out/r6z/cparam.json 2> gpurun_out/r6z/cparam.err || exit 1
P="python -u bench_configs.py --workload pace --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6z/pace_fetch -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6z/pace_write -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d gpurun_out/r6z/pace_size -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/r6z/pace_fetch gpurun_out/r6z/pace_write gpurun_out/r6z/pace_pmc_summary.json gpurun_out/r6z/pace_size || exit 1
find gpurun_out/r6z/pace_fetch gpurun_out/r6z/pace_write gpurun_out/r6z/pace_size -name "*.csv" -size +20M -delete
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6z/pace.json gpurun_out/r6z/c4.json gpurun_out/r6z/cparam.json
