"""Walker diagnostics on the C3 bench workload: per-step device phases for a few walker splits
(SG_SHORT_MAX), then one run with SG_DEBUG=64 (per length class: groups, gather and walk wave-time of the
short walker; per length bucket: segments, summed and max wave-time of the wave walker).

    python scripts/walk_diag.py [--requests N] [--splits 256,128,64]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import ShardWorkload  # noqa: E402
from sentinel_amd import abi  # noqa: E402
from sentinel_amd.engine import FlowEngine  # noqa: E402


def run(wl, n, steps, env):
    for k in ("SG_SHORT_MAX", "SG_DEBUG"):
        os.environ.pop(k, None)
    os.environ.update(env)
    eng = FlowEngine(device=0, max_batch=n)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules)
    out = torch.empty(n * 12, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    batches = [wl.batch(b) for b in range(steps + 2)]
    for b in range(2):
        eng.decide_device(batches[b].data_ptr(), n, out.data_ptr(), st)
    eng.enable_stats(True)
    acc = {"sort_ms": 0.0, "walk_ms": 0.0, "total_ms": 0.0}
    for b in range(2, steps + 2):
        eng.decide_device(batches[b].data_ptr(), n, out.data_ptr(), st)
        s = eng.stats()
        for k in acc:
            acc[k] += s[k] / steps
    res = dict(env=env, **{k: round(v, 4) for k, v in acc.items()}, long_segments=eng.stats()["long_segments"])
    if int(env.get("SG_DEBUG", "0")) & 64:
        d = eng.debug_copy(5, np.uint64, 32).astype(np.int64)
        tick_us = 0.01  # s_memrealtime: 100 MHz
        per = steps + 2
        res["short_total_wave_ms"] = d[0] * tick_us / 1000 / per
        res["short_classes"] = [
            {"class": c, "groups_per_step": int(d[1 + c]) / per,
             "gather_us_per_group": (d[7 + c] & 0xFFFFFFFF) * tick_us / max(1, d[1 + c]),
             "walk_us_per_group": (d[7 + c] >> 32) * tick_us / max(1, d[1 + c])} for c in range(6)]
        res["long_buckets"] = [
            {"bucket": ["<=64", "<=256", "<=1024", ">1024"][b], "segs_per_step": int(d[16 + 2 * b]) / per,
             "us_per_seg": d[17 + 2 * b] * tick_us / max(1, d[16 + 2 * b]), "max_us": d[24 + b] * tick_us}
            for b in range(4)]
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=16_000_000)
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--splits", default="256")
    ap.add_argument("--envs", default="", help="extra runs: 'K=V,K=V;K=V' (e.g. SG_DEBUG=4 for the register walker)")
    args = ap.parse_args()
    wl = ShardWorkload(args.flows, args.requests, 0, 1, torch.device("cuda", 0))
    for sm in args.splits.split(","):
        print(json.dumps(run(wl, args.requests, args.steps, {"SG_SHORT_MAX": sm})), flush=True)
    for spec in filter(None, args.envs.split(";")):
        env = dict(kv.split("=", 1) for kv in spec.split(","))
        print(json.dumps(run(wl, args.requests, args.steps, env)), flush=True)
    print(json.dumps(run(wl, args.requests, args.steps, {"SG_DEBUG": "64"})), flush=True)


if __name__ == "__main__":
    main()
