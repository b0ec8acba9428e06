#!/bin/bash
# Round-4 secondary configs: kernel traces + bench lines for C4, C5 and cparam (and the adversarial cparam chain).
# Outputs under gpurun_out/r4cfg_<w>/; stops at the first step that fails.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for w in ${WORKLOADS:-c4 c5 cparam}; do
  d=gpurun_out/r4cfg_$w
  mkdir -p $d
  st="--steps 3 --warmup 1"
  [ $w = c4 ] && st="--steps 5 --warmup 2"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python -u bench_configs.py --workload $w $st --no-cpu-baseline > $d/trace.log 2>&1 || exit $?
  timeout -k 10 600 python -u bench_configs.py --workload $w $st > $d/bench.log 2>&1 || exit $?
  echo "$w: $(tail -1 $d/bench.log | cut -c1-260)"
done
if [ -n "${CHAIN:-}" ]; then
  d=gpurun_out/r4cfg_chain
  mkdir -p $d
  timeout -k 10 600 python -u bench_configs.py --workload cparam --steps 3 --warmup 1 --no-cpu-baseline --chain $CHAIN > $d/bench.log 2>&1 || exit $?
  echo "chain $CHAIN: $(tail -1 $d/bench.log | cut -c1-260)"
fi
echo done
