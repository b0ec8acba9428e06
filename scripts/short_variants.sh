#!/bin/bash
# Short walker kernel time (serialised walkers) under debug variants: 0 full, 1024 prologue only (no walk),
# 512 no bucket stores, 256 no result stores.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-2 1026 514 258}; do
  SG_DEBUG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sv$v -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sv$v.log 2>&1 || exit $?
  echo "== SG_DEBUG=$v"; python scripts/kstats.py $(find gpurun_out/sv$v -name '*kernel_stats.csv' | head -1) | grep walk
done
