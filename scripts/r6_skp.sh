#!/bin/bash
# Skip-apply kernels with 8 record rows loaded together (k_skip_apply, k_lskip_apply): the whole -m gpu suite, then a
# same-box A/B against the previous build on C3 (bench.py), C2 and C5.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/skp_pytest.txt 2>&1 || { tail -30 gpurun_out/r6/skp_pytest.txt; exit 1; }
tail -1 gpurun_out/r6/skp_pytest.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/skp_c3_new_$r.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/hbase.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/skp_c3_base_$r.json 2>/dev/null || exit 1
done
for w in c2 c5; do
  timeout -k 10 300 python -u bench_configs.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/skp_${w}_new.json 2>/dev/null || exit 1
  SG_LIB_PATH=build/ab/hbase.so timeout -k 10 300 python -u bench_configs.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6/skp_${w}_base.json 2>/dev/null || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/skp_*.json
P="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/skp_prof -o run --output-format csv -- $P > /dev/null 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/skp_prof/*kernel_stats.csv | head -1) > gpurun_out/r6/skp_kstats.txt
rm -f gpurun_out/r6/skp_prof/*kernel_trace.csv
head -8 gpurun_out/r6/skp_kstats.txt
