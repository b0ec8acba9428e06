#!/bin/bash
# Short-walker class timers under debug variants (SG_DEBUG bits: 256 no result stores, 512 no bucket stores).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
for v in 0 256 512 768; do
  echo "== SG_DEBUG=$v"
  SG_DEBUG=$v timeout -k 10 200 python -u scripts/walk_counters.py 2>&1 | grep -v amdgpu.ids || exit $?
done
