cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/slotp; export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/slotp/prof -o run --output-format csv -- \
  python -u bench_configs.py --workload slot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/slotp/prof.log 2>&1 || exit $?
echo "slot: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/slotp/prof.log)"
