"""Full-size parity of the exact code path bench.py times: sg_flow_enqueue with batches back to back (two
alternating workspaces, the front half of batch i+1 on its CU partition beside the walkers of batch i, the
cross-batch time check in the back half), over bench.ShardWorkload's own GPU-generated C3 trace — 1M flowIds,
16M requests per 1000 ms batch, Zipf(1.0), 1 % prioritized, 10 % acquire U{2..4} — four batches in flight at once,
as bench.run_steps enqueues them. Every result of every batch and, at the end, every flowId's window and occupy
counters are compared bit-exactly with the oracle's replay (ClusterFlowChecker.java:55-112 through
oracle.binding.ShardedClusterTokenService: flowIds share no state without a namespace limiter, so the per-shard
sequential replay equals the global one).

A second test pins the bench trace itself: one ShardWorkload batch copied to the host and replayed through the
single-threaded oracle over its first 2M requests (all flowIds' state starting empty) equals the device's
synchronous decision of the same prefix.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle.binding import ClusterTokenService, ShardedClusterTokenService
from sentinel_amd import abi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_FLOWS = 1_000_000
N_REQ = 16_000_000


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def _ns():
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    return ns


def _same(want, got, what):
    if not np.array_equal(want, got):
        bad = np.nonzero(want != got)[0]
        raise AssertionError(f"{what}: {len(bad)} of {len(want)} differ; first at {bad[0]}: oracle={want[bad[0]]} "
                             f"gpu={got[bad[0]]}")


def test_bench_pipeline_full_size_four_batches_in_flight():
    from bench import ShardWorkload
    from sentinel_amd.engine import FlowEngine
    from tests.test_fullsize_gpu import _compare_flow_state
    dev = torch.device("cuda:0")
    wl = ShardWorkload(N_FLOWS, N_REQ, 0, 1, dev)
    eng = FlowEngine(device=0, max_batch=N_REQ)
    eng.set_namespaces(_ns())
    eng.load_rules(wl.rules)
    n_batches = 4
    batches = [wl.batch(b) for b in range(n_batches)]
    outs = [torch.empty(N_REQ * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(n_batches)]
    torch.cuda.synchronize()
    tickets = [eng.enqueue_device(batches[b].data_ptr(), N_REQ, outs[b].data_ptr()) for b in range(n_batches)]
    for t in tickets:
        eng.wait(t)
    ora = ShardedClusterTokenService(wl.rules, _ns(), _threads())
    try:
        seen = set()
        for b in range(n_batches):
            req = batches[b].cpu().numpy().view(abi.REQ_DTYPE)
            want = ora.decide(req)
            got = outs[b].cpu().numpy().view(abi.RES_DTYPE)
            _same(want, got, f"pipelined batch {b}")
            seen |= set(np.unique(want["status"]).tolist())
        assert {abi.OK, abi.BLOCKED, abi.SHOULD_WAIT} <= seen
        ring, occ = ora.export_state(eng.state_stride())
        _compare_flow_state(eng, ring, occ, len(wl.rules))
    finally:
        ora.close()


def test_bench_trace_prefix_single_thread_oracle():
    from bench import ShardWorkload
    from sentinel_amd.engine import FlowEngine
    dev = torch.device("cuda:0")
    wl = ShardWorkload(N_FLOWS, N_REQ, 0, 1, dev)
    req = wl.batch(0).cpu().numpy().view(abi.REQ_DTYPE)[:2_000_000].copy()
    eng = FlowEngine(device=0, max_batch=len(req))
    eng.set_namespaces(_ns())
    eng.load_rules(wl.rules)
    ora = ClusterTokenService()
    ora.set_namespaces(_ns())
    ora.load_rules(wl.rules)
    _same(ora.decide(req), eng.decide_host(req), "bench trace prefix")
