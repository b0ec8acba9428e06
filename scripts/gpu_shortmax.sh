#!/bin/bash
# C3 bench under different short/long walker splits (env SG_SHORT_MAX).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
for m in ${SPLITS:-256 64 16}; do
  SG_SHORT_MAX=$m timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sm$m.log 2>&1 || { tail -5 gpurun_out/sm$m.log; exit 1; }
  echo "short_max=$m: $(tail -1 gpurun_out/sm$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', d['phases_ms'])")"
done
