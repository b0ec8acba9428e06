#!/bin/bash
# cx walkers with LArgs staged in LDS (no per-lane scratch copy): local / slot-chain parity, then the slot workload
# against the previous build on the same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_slot_chain_gpu.py tests/test_local_rules_gpu.py tests/test_local_gpu.py tests/test_pslot_gpu.py tests/test_embedded_server_gpu.py tests/test_local_shard_gpu.py tests/test_local_pipeline_gpu.py tests/test_pslot_cluster_gpu.py tests/test_slot_fullsize_gpu.py > gpurun_out/r6/cx_tests.txt 2>&1 || { tail -20 gpurun_out/r6/cx_tests.txt; exit 1; }
tail -1 gpurun_out/r6/cx_tests.txt
timeout -k 10 400 python -u bench_configs.py --workload slot --steps 3 --warmup 1 > gpurun_out/r6/cx_new.json 2> gpurun_out/r6/cx_new.err || exit 1
SG_LIB_PATH=build/ab/cxbase.so timeout -k 10 400 python -u bench_configs.py --workload slot --steps 3 --warmup 1 > gpurun_out/r6/cx_base.json 2> gpurun_out/r6/cx_base.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/cx_new.json gpurun_out/r6/cx_base.json
