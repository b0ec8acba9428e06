#!/bin/bash
# Runs GPU steps in order: gpu_steps.sh <name> <timeout_s> <command> [<name> <timeout_s> <command> ...].
# Each step's output goes to gpurun_out/<name>.log; a test failure (rc 1) goes on to the next step, any other
# non-zero status (fault, abort, timeout) ends the call there.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -ge 3 ]; do
  name=$1 tmo=$2 cmd=$3
  shift 3
  echo "== $name"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
