# Round-5: the slot workload (bench line, then its kernel trace).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/slot; export TMPDIR=/tmp
timeout -k 10 900 python -u bench_configs.py --workload slot --steps 2 --warmup 1 > gpurun_out/slot/slot.log 2>&1 || { tail -5 gpurun_out/slot/slot.log; exit 1; }
echo "slot: $(tail -1 gpurun_out/slot/slot.log | cut -c1-400)"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/slot/prof -o run --output-format csv -- \
  python -u bench_configs.py --workload slot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/slot/prof.log 2>&1 || exit $?
echo done
