cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/lp
timeout -k 10 400 python -u -m pytest tests/test_local_pipeline_gpu.py tests/test_local_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lp/tests.log 2>&1; rc=$?; tail -3 gpurun_out/lp/tests.log; [ $rc -eq 0 ] || exit $rc
for m in pipe sync; do
  f=""; [ $m = sync ] && f="--local-sync"
  timeout -k 10 300 python -u bench_configs.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline $f > gpurun_out/lp/c2_$m.log 2>&1 || exit $?
  echo "c2 $m: $(tail -1 gpurun_out/lp/c2_$m.log | cut -c1-200)"
done
for m in pipe sync; do
  f=""; [ $m = sync ] && f="--local-sync"
  timeout -k 10 400 python -u bench_configs.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline $f > gpurun_out/lp/c5_$m.log 2>&1 || exit $?
  echo "c5 $m: $(tail -1 gpurun_out/lp/c5_$m.log | cut -c1-200)"
done
