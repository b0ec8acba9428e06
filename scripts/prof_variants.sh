#!/bin/bash
# k_walk_short / k_walk_long device time under SG_DEBUG variants (serialised stream), kernel-trace only.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
for d in ${VARIANTS:-0}; do
  rm -rf gpurun_out/pv_$d
  SG_DEBUG=$((d | 2)) SG_SHORT_MAX=${SM:-64} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$d -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pv_$d.log 2>&1 || exit $?
  python - "$d" <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/pv_{sys.argv[1]}/**/run_kernel_stats.csv',recursive=True)[0]
out=[]
for r in csv.DictReader(open(f)):
    n=r['Name'].split('(')[0].replace('void ','').replace('sg::','')
    if n.startswith(('k_walk','k_seg','k_skip','k_prep','k_radix')): out.append(f"{n.split('<')[0]}={float(r['AverageNs'])/1e3:.0f}us")
print('dbg', sys.argv[1], ' '.join(out))
PY
done
