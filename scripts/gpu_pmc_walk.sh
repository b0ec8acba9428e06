#!/bin/bash
# Memory-pipeline counters of the sg:: kernels (walkers serialised), one rocprofv3 pass per counter group.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
export SG_DEBUG=2
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmcw$i -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcw$i.log; exit 1; }
done
python - <<'PY'
import csv,glob,collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcw*/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        n=r['Kernel_Name'].split('(')[0].replace('void ', '')
        if not n.startswith('sg::'): continue
        agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n,d in agg.items():
    print(n, {c: round(sum(v)/len(v)) for c,v in sorted(d.items())})
PY
