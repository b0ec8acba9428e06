#!/bin/bash
# SQ counters of the sg:: kernels (walkers serialised on one stream), one rocprofv3 pass, plus the
# short-walker cycle counters (SG_DEBUG & 64).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
export SG_DEBUG=2
[ -n "$PROF_SM" ] && export SG_SHORT_MAX=$PROF_SM
timeout -k 10 200 python -u scripts/walk_counters.py > gpurun_out/walk_counters.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/walk_counters.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d gpurun_out/pmc_sq -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq.log 2>&1 || exit $?
python - <<'PY'
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_sq/**/*counter_collection.csv',recursive=True)[0]
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n=r['Kernel_Name'].split('(')[0].replace('void ', '')
    if not n.startswith('sg::'): continue
    agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n,d in agg.items():
    print(n, {c: round(sum(v)/len(v)) for c,v in d.items()})
PY
