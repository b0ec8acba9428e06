#!/bin/bash
# Round 6: kernel trace + stats of the C3 bench (binned front half unless SG_BIN=0 is passed through), and the
# pipelined timeline. Usage: r6_prof.sh <tag>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
tag=${1:-bin}
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_$tag -o run --output-format csv -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r6/prof_$tag.log 2>&1 || exit $?
python scripts/kstats.py $(ls gpurun_out/r6/prof_$tag/*kernel_stats.csv | head -1) > gpurun_out/r6/kstats_$tag.txt
python scripts/timeline.py $(ls gpurun_out/r6/prof_$tag/*kernel_trace.csv | head -1) 3 > gpurun_out/r6/tl_$tag.txt
cat gpurun_out/r6/kstats_$tag.txt
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/prof_$tag.log
