cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/cxw
SG_DEBUG=64 timeout -k 10 900 python -u bench_configs.py --workload slot --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/cxw/diag.log 2>&1 || { tail -5 gpurun_out/cxw/diag.log; exit 1; }
grep "cxw per batch" gpurun_out/cxw/diag.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/cxw/diag.log
