#!/bin/bash
# Kernel-trace timelines of the pipelined C3 bench under several SG_DEBUG settings:
#   exp_timeline.sh <tag>=<SG_DEBUG value> ...   → gpurun_out/tl_<tag>.txt (last 3 pipelined batches) + bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "$@"; do
  tag=${kv%%=*} val=${kv#*=}
  echo "== $tag (SG_DEBUG=$val)"
  SG_DEBUG=$val timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$tag -o run --output-format csv -- \
    python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batches 0 > gpurun_out/tl_$tag.log 2>&1 || exit $?
  python scripts/timeline.py $(ls gpurun_out/tl_$tag/*kernel_trace.csv | head -1) 3 > gpurun_out/tl_$tag.txt
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/tl_$tag.log
done
