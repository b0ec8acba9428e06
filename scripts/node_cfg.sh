# Node handle lines (G same-device shards, routing inside) and the codec profile set, on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/node
for g in 1 2 4; do
  timeout -k 10 300 python -u bench_configs.py --workload node --shards $g --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/node/g$g.log 2>&1 || exit $?
  echo "node g$g: $(tail -1 gpurun_out/node/g$g.log | cut -c1-160)"
done
WORKLOADS=codec bash scripts/gpu_configs_prof.sh
