#!/bin/bash
# Round 6 A/B on one box: bench.py ms/step for env variants, interleaved rounds.
# Usage: r6_ab.sh <rounds> "<tag>=<ENV=V ENV2=V>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 "$R"); do
  for kv in "$@"; do
    tag=${kv%%=*} envs=${kv#*=}
    env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r6/ab_${tag}_$r.log 2>&1 || { echo "fail $tag"; exit 1; }
    echo "$tag r$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6/ab_${tag}_$r.log)" | tee -a gpurun_out/r6/ab.txt
  done
done
