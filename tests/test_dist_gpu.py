"""Two ranks, each with its own HIP engine handle (both on device 0 of the one-GPU box), deciding the flowIds
the hash sharding gives them (sentinel_amd/cluster.py), with the gloo metric rollup: the node-level results,
windows and rolled-up snapshot must equal one sequential oracle replay of the whole node trace (SURVEY §8(e):
flows are independent, so sharding by flow changes nothing). Also: a shard refuses the node-wide namespace
QPS limiter (GlobalRequestLimiter.java:46-55), in either call order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sentinel_amd import abi
from sentinel_amd.cluster import MetricRollup, route_requests, shard_flows

pytestmark = pytest.mark.gpu

N_FLOWS, N_REQ, BATCHES = 5000, 200_000, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _node_workload():
    from sentinel_amd.workload import ClusterWorkload
    wl = ClusterWorkload(n_flows=N_FLOWS, n_requests=N_REQ, seed=11, prio_frac=0.05)
    return wl.rules(), [wl.requests(b) for b in range(BATCHES)]


def _ns(limiter=False):
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    ns["limiter_enabled"] = 1 if limiter else 0
    return ns


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sentinel_amd.engine import FlowEngine
        rules, batches = _node_workload()
        shard = shard_flows(N_FLOWS, rank, world)
        local = np.full(N_FLOWS, -1, np.int64)
        local[shard] = np.arange(len(shard))
        eng = FlowEngine(device=0, max_batch=N_REQ)
        eng.set_shard(rank, world)
        eng.set_namespaces(_ns())
        eng.load_rules(rules[shard])
        outs = []
        for req in batches:
            keys = (req["key"] & abi.KEY_INDEX).astype(np.int64)
            order, counts = route_requests(keys, world)
            start = int(counts[:rank].sum())
            mine = np.sort(order[start:start + counts[rank]])  # arrival order within the shard
            sub = req[mine].copy()
            sub["key"] = local[keys[mine]].astype(np.uint32) | (sub["key"] & np.uint32(abi.KEY_PRIO))
            outs.append((mine, eng.decide_host(sub)))
        now = int(batches[-1]["ts_ms"][-1]) + 1
        snap = torch.from_numpy(eng.snapshot(now, len(shard)).copy())
        roll = MetricRollup(len(shard), "cpu")
        totals = roll.run(snap)
        node = roll.node_snapshot([shard_flows(N_FLOWS, r, world) for r in range(world)])
        ring, occ = eng.export_state(len(shard))
        q.put((rank, outs, totals.numpy().copy(), node.numpy().copy(), shard, ring, occ))
    except BaseException as e:  # surface the failure in the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_engine_ranks_equal_node_replay():
    from oracle.binding import ClusterTokenService
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
    for r in res:
        assert len(r) > 2, f"rank {r[0]} failed: {r[1]}"
    assert all(p.exitcode == 0 for p in procs)
    rules, batches = _node_workload()
    ora = ClusterTokenService()
    ora.set_namespaces(_ns())
    ora.load_rules(rules)
    wants = [ora.decide(req) for req in batches]
    stride = int(rules["sample_count"].max())
    ring_all, occ_all = ora.export_state(N_FLOWS, stride)  # before avg(): its currentWindow may reset a bucket
    now = int(batches[-1]["ts_ms"][-1]) + 1
    node = np.array([[ora.avg(k, now, abi.EV_PASS), ora.avg(k, now, abi.EV_BLOCK)] for k in range(N_FLOWS)])
    for b, want in enumerate(wants):
        got = np.zeros_like(want)
        for rank, outs, *_ in res:
            mine, out = outs[b]
            got[mine] = out
        assert np.array_equal(got, want), f"batch {b}: {(got != want).sum()} results differ"
    for rank, outs, totals, node_snap, shard, ring, occ in res:
        assert np.array_equal(node_snap, node)
        assert np.allclose(totals, node.sum(0), rtol=1e-12)
        s = min(ring.shape[1], ring_all.shape[1])
        assert np.array_equal(ring[:, :s], ring_all[shard][:, :s])
        assert np.array_equal(occ, occ_all[shard])


def test_shard_refuses_namespace_limiter():
    from sentinel_amd.engine import EngineError, FlowEngine
    eng = FlowEngine(device=0, max_batch=1024)
    eng.set_shard(1, 2)
    with pytest.raises(EngineError) as ei:
        eng.set_namespaces(_ns(limiter=True))
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    eng2 = FlowEngine(device=0, max_batch=1024)
    eng2.set_namespaces(_ns(limiter=True))
    with pytest.raises(EngineError) as ei:
        eng2.set_shard(0, 2)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    eng2.set_shard(0, 1)  # a single shard is the whole node
