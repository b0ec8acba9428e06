#!/bin/bash
# Parity tests of the flow path, then a short bench per walker split (SG_SHORT_MAX) and a kernel-trace profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_flow_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tune_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/tune_pytest.log; [ $rc -eq 0 ] || exit $rc
for sm in ${SMS:-16 64 256}; do
  SG_SHORT_MAX=$sm timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tune_bench_$sm.log 2>&1 || exit $?
  echo "short_max=$sm"; python -c "import json,sys; d=json.loads(open('gpurun_out/tune_bench_$sm.log').read().strip().splitlines()[-1]); print(d['value']/1e9, d['phases_ms'], d['roofline']['frac'])"
done
SG_DEBUG=2 SG_SHORT_MAX=${PROF_SM:-64} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tune_prof.log 2>&1 || exit $?
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/tprof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name'].split('(')[0][:60]
    if not n.startswith('sg::'): continue
    print(f"{n:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
