#!/bin/bash
# Round 6 checkpoint: the whole -m gpu suite and smoke, the C3 bench, the pace line, and a kernel-trace proof that the
# LDS poison kernel runs before the library's kernels under SG_LDS_POISON=1 (one small test file).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6f
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6f/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r6f/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r6f/pytest_gpu.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6f/bench.json 2> gpurun_out/r6f/bench.err || exit 1
timeout -k 10 300 python -u bench_configs.py --workload pace --steps 5 --warmup 2 > gpurun_out/r6f/pace.json 2> gpurun_out/r6f/pace.err || exit 1
SG_LDS_POISON=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6f/poison -o run --output-format csv -- \
  python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flow_gpu.py tests/test_node_gpu.py > gpurun_out/r6f/poison.txt 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6f/poison/*kernel_stats.csv | head -1) > gpurun_out/r6f/poison_kstats.txt
grep -i "poison" $(ls gpurun_out/r6f/poison/*kernel_stats.csv | head -1) > gpurun_out/r6f/poison_stats_row.txt
rm -f gpurun_out/r6f/poison/*kernel_trace.csv  # (hundreds of MB: gpurun copies back at most 64 MiB)
