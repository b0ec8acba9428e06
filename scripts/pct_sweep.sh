# Pipelined C3 bench over CU partitions between the front half and the walkers (SG_FRONT_EIGHTHS).
mkdir -p gpurun_out
for k in ${SWEEP:-0 2 3 4}; do
  SG_FRONT_EIGHTHS=$k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-batches 0 > gpurun_out/front_$k.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/front_$k.log').read().strip().splitlines()[-1]); print($k, round(d['ms_per_step'],4), d['phases_ms'])"
done
