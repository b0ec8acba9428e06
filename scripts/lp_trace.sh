# Kernel traces of the pipelined local path (C5, C2) for scripts/timeline.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for w in ${WORKLOADS:-c5 c2}; do
  st="--steps 6 --warmup 2"; [ $w = c5 ] && st="--steps 4 --warmup 1"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lpt_$w -o run --output-format csv -- python -u bench_configs.py --workload $w $st --no-cpu-baseline > gpurun_out/lpt_$w.log 2>&1 || exit $?
  echo "$w: $(tail -1 gpurun_out/lpt_$w.log | cut -c1-120)"
done
