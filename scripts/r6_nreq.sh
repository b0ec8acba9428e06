#!/bin/bash
# Node token routing (k_nreq_keys) with wave-aggregated shard counts: node token tests, same-box A/B on the node
# cparam line (G = 1, 2) against the previous build, and the routing kernel's time.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_node_tokens_gpu.py tests/test_node_tokens_fullsize_gpu.py > gpurun_out/r6/nreq_tests.txt 2>&1 || { tail -20 gpurun_out/r6/nreq_tests.txt; exit 1; }
tail -1 gpurun_out/r6/nreq_tests.txt
for G in 1 2; do
  timeout -k 10 300 python -u bench_configs.py --workload cparam --shards $G --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r6/nreq_new_$G.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/nbase.so timeout -k 10 300 python -u bench_configs.py --workload cparam --shards $G --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r6/nreq_base_$G.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/nreq_*.json
for v in cur nbase; do
  L=""; [ $v = nbase ] && L=build/ab/nbase.so
  SG_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/nreq_$v -o run --output-format csv -- python -u bench_configs.py --workload cparam --shards 1 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  echo "$v $(python scripts/kstats.py $(ls gpurun_out/r6/nreq_$v/*kernel_stats.csv | head -1) | grep k_nreq_keys | tr -s ' ')"
  rm -f gpurun_out/r6/nreq_$v/*kernel_trace.csv
done
