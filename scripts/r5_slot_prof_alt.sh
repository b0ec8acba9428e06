# Round-5: kernel trace of the slot workload with the wave walker taking the 65-256-record cx class too.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/slotp2; export TMPDIR=/tmp
export SG_CXW_MIN=65
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/slotp2/prof -o run --output-format csv -- \
  python -u bench_configs.py --workload slot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/slotp2/prof.log 2>&1 || exit $?
echo "slot: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/slotp2/prof.log)"
