"""Two ranks, each with its own HIP engine handle (both on device 0 of the one-GPU box), deciding the flowIds
the hash sharding gives them (sentinel_amd/cluster.py), with the gloo metric rollup: the node-level results,
windows and rolled-up snapshot must equal one sequential oracle replay of the whole node trace (SURVEY §8(e):
flows are independent, so sharding by flow changes nothing). With a namespace QPS limiter
(GlobalRequestLimiter.java:46-55) the ranks run the §8(e) exchange (cluster.LimiterExchange over gloo) and must
equal the oracle replay of the node batch in the node's arrival order (ts, rank, position)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sentinel_amd import abi
from sentinel_amd.cluster import LimiterExchange, MetricRollup, node_order, route_requests, shard_flows

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


def _shard_batch(req, rank, world, local):
    keys = (req["key"] & abi.KEY_INDEX).astype(np.int64)
    order, counts = route_requests(keys, world)
    start = int(counts[:rank].sum())
    mine = np.sort(order[start:start + counts[rank]])  # arrival order within the shard
    sub = req[mine].copy()
    sub["key"] = local[keys[mine]].astype(np.uint32) | (sub["key"] & np.uint32(abi.KEY_PRIO))
    return mine, sub


def _worker(rank, world, port, q, limiter=False):
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
        eng.set_namespaces(_ns(limiter))
        eng.load_rules(rules[shard])
        xch = LimiterExchange(eng, "cuda:0", coll_device="cpu") if limiter else None
        outs = []
        for req in batches:
            mine, sub = _shard_batch(req, rank, world, local)
            if xch is None:
                outs.append((mine, eng.decide_host(sub)))
                continue
            dev_req = torch.from_numpy(sub.view(np.uint8).copy()).to("cuda:0")
            n = len(sub)
            xch.arm(dev_req.data_ptr(), n, int(sub["ts_ms"][0]) if n else None, int(sub["ts_ms"][-1]) if n else None)
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


@pytest.mark.parametrize("limiter", [False, True])
def test_two_engine_ranks_equal_node_replay(limiter):
    from oracle.binding import ClusterTokenService
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, limiter)) for r in range(world)]
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
    ora.set_namespaces(_ns(limiter))
    ora.load_rules(rules)
    res.sort(key=lambda r: r[0])
    for b, req in enumerate(batches):
        # node order: (ts, rank, position in the rank's batch) — the original order when there is no limiter
        cat_idx = np.concatenate([outs[b][0] for _, outs, *_ in res])
        perm = node_order([req["ts_ms"][outs[b][0]] for _, outs, *_ in res]) if limiter else np.argsort(cat_idx)
        want_node = ora.decide(req[cat_idx[perm]])
        want = np.empty_like(want_node)
        want[perm] = want_node
        got = np.concatenate([outs[b][1] for _, outs, *_ in res])
        assert np.array_equal(got, want), f"batch {b}: {(got != want).sum()} results differ"
        if limiter:
            assert (want["status"] == abi.TOO_MANY_REQUEST).any()
    stride = int(rules["sample_count"].max())
    ring_all, occ_all = ora.export_state(N_FLOWS, stride)  # before avg(): its currentWindow may reset a bucket
    now = int(batches[-1]["ts_ms"][-1]) + 1
    node = np.array([[ora.avg(k, now, abi.EV_PASS), ora.avg(k, now, abi.EV_BLOCK)] for k in range(N_FLOWS)])
    for rank, outs, totals, node_snap, shard, ring, occ in res:
        assert np.array_equal(node_snap, node)
        assert np.allclose(totals, node.sum(0), rtol=1e-12)
        s = min(ring.shape[1], ring_all.shape[1])
        assert np.array_equal(ring[:, :s], ring_all[shard][:, :s])
        assert np.array_equal(occ, occ_all[shard])
