#!/bin/bash
# Kernel statistics of the cparam workload (1000 rules x 16M requests) on the round's kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/cpprof -o run --output-format csv -- \
  python -u bench_configs.py --workload cparam --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/r6/cpprof.log 2>&1 || exit 1
python scripts/kstats.py $(ls gpurun_out/r6/cpprof/*kernel_stats.csv | head -1) > gpurun_out/r6/cp_kstats.txt
python - <<'PY' > gpurun_out/r6/cp_tl.txt
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/r6/cpprof/*kernel_trace.csv')[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_cp_prep2' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]['Start_Timestamp'])
for r in rows[a:b]:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sg::', '')[:40]
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    print(f"{n:40s} {s:8.1f} {e:8.1f} ({e - s:6.1f}) q{r.get('Queue_Id')}")
PY
rm -f gpurun_out/r6/cpprof/*kernel_trace.csv
