"""Binned front half diagnostics (SG_DEBUG=65536): per-phase wall clock of k_bin_sort's regular bins on the C3
bench workload, averaged per block, plus the unpipelined sort / walk phases.

    python scripts/bin_diag.py [--requests N] [--flows K]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SG_DEBUG"] = "65536"

from bench import ShardWorkload  # noqa: E402
from sentinel_amd import abi  # noqa: E402
from sentinel_amd.engine import FlowEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--requests", type=int, default=16_000_000)
ap.add_argument("--flows", type=int, default=1_000_000)
ap.add_argument("--steps", type=int, default=4)
args = ap.parse_args()
dev = torch.device("cuda", 0)
wl = ShardWorkload(args.flows, args.requests, 0, 1, dev)
eng = FlowEngine(device=0, max_batch=args.requests)
ns = np.zeros(1, abi.NS_DTYPE)
ns["connected_count"] = 1
ns["max_allowed_qps"] = 30000
eng.set_namespaces(ns)
eng.load_rules(wl.rules)
out = torch.empty(args.requests * 12, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
batches = [wl.batch(b) for b in range(args.steps + 2)]
for b in range(2):
    eng.decide_device(batches[b].data_ptr(), args.requests, out.data_ptr(), st)
torch.cuda.synchronize()
d0 = eng.debug_copy(5, np.uint64, 64).astype(np.int64)
eng.enable_stats(True)
acc = {"sort_ms": 0.0, "walk_ms": 0.0, "total_ms": 0.0}
for b in range(2, args.steps + 2):
    eng.decide_device(batches[b].data_ptr(), args.requests, out.data_ptr(), st)
    s = eng.stats()
    for k in acc:
        acc[k] += s[k] / args.steps
d = eng.debug_copy(5, np.uint64, 64).astype(np.int64) - d0
blocks = max(int(d[44]), 1)
us = lambda x: round(x * 0.01 / blocks, 2)  # s_memrealtime ticks at 100 MHz
print(json.dumps({"phases_ms": {k: round(v, 4) for k, v in acc.items()},
                  "bin_blocks_per_batch": blocks / args.steps, "avg_us_per_block": {
                      "load+zero": us(d[40]), "count": us(d[41]), "scan+lists": us(d[42]), "place": us(d[43]),
                      "place:positions": us(d[48]), "place:windows": us(d[49]), "place:atomic_wait": us(d[50]),
                      "place:emit": us(d[51])},
                  "blocks_reloading": int(d[45]) / args.steps, "max_bin_len": int(d[46]),
                  "avg_bin_len": int(d[47]) / blocks}))
