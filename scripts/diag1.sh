cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/walk_diag.py --steps 5 > gpurun_out/r5_walkdiag.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/r5_base_bench.txt 2>&1 || exit $?
bash scripts/exp_timeline.sh base=0 || exit $?
echo done
