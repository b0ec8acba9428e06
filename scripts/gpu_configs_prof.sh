#!/bin/bash
# Secondary configs (C2, C4, C5) with evidence: a kernel trace (--stats) and separate FETCH_SIZE / WRITE_SIZE
# passes (+ the read-request sizes) per workload, summarised by pmc_summary.py, then the bench line with that traffic.
# Outputs under gpurun_out/cfg_<w>/; stops at the first step that fails.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c4 c5}; do
  d=gpurun_out/cfg_$w
  mkdir -p $d
  short="--workload $w --steps 3 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python -u bench_configs.py $short > $d/trace.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $d/pmc_fetch -o run --output-format csv -- python -u bench_configs.py $short > $d/fetch.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $d/pmc_write -o run --output-format csv -- python -u bench_configs.py $short > $d/write.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d $d/pmc_size -o run --output-format csv -- python -u bench_configs.py $short > $d/size.log 2>&1 || exit $?
  python scripts/pmc_summary.py $d/pmc_fetch $d/pmc_write $d/pmc_summary.json $d/pmc_size || exit $?
  timeout -k 10 600 python -u bench_configs.py --workload $w --pmc-summary $d/pmc_summary.json > $d/bench.log 2>&1 || exit $?
  echo "$w: $(tail -1 $d/bench.log | cut -c1-240)"
done
echo done
