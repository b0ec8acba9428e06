# Round-5: HBM traffic of the slot workload (FETCH_SIZE / WRITE_SIZE / request sizes, separate passes) and its bench
# line with that traffic.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
d=gpurun_out/cfg_slot
mkdir -p $d
short="--workload slot --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $d/pmc_fetch -o run --output-format csv -- python -u bench_configs.py $short > $d/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $d/pmc_write -o run --output-format csv -- python -u bench_configs.py $short > $d/write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -d $d/pmc_size -o run --output-format csv -- python -u bench_configs.py $short > $d/size.log 2>&1 || exit $?
python scripts/pmc_summary.py $d/pmc_fetch $d/pmc_write $d/pmc_summary.json $d/pmc_size || exit $?
timeout -k 10 600 python -u bench_configs.py --workload slot --steps 2 --warmup 1 --pmc-summary $d/pmc_summary.json > $d/bench.log 2>&1 || exit $?
echo "slot: $(tail -1 $d/bench.log | cut -c1-200)"
