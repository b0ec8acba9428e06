#!/bin/bash
# Kernel-trace profile of the C2 / C5 local-chain benches (serialised walkers: SG_DEBUG=2).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
for w in ${WLS:-c2 c5}; do
  extra=""; [ $w = c5 ] && extra="--steps 2 --warmup 1"
  rm -rf gpurun_out/pc_$w
  SG_DEBUG=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pc_$w -o run --output-format csv -- python -u bench_configs.py --workload $w --no-cpu-baseline $extra > gpurun_out/pc_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/pc_$w.log | cut -c1-200
  python - "$w" <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/pc_{sys.argv[1]}/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name'].split('(')[0].replace('void ','').replace('sg::','')
    if n.startswith('k_'): print(f"  {n.split('<')[0]:20s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
