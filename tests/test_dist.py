"""Multi-rank path on CPU (gloo, world_size 2 and 4): hash sharding of flowIds, request routing, and the
metric rollup collective (sentinel_amd/cluster.py). Each rank decides its shard with the oracle (no GPU
here); the node-level result must equal one sequential replay of the whole node trace: flows are
independent, so sharding by flow changes nothing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sentinel_amd import abi
from sentinel_amd.cluster import MetricRollup, owner_of, route_requests, shard_flows, splitmix64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _node_workload(n_flows, n_req, seed=5):
    from sentinel_amd.workload import ClusterWorkload
    wl = ClusterWorkload(n_flows=n_flows, n_requests=n_req, seed=seed, prio_frac=0.05)
    return wl.rules(), wl.requests(0)


def _ns():
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    return ns


def _worker(rank, world, port, n_flows, n_req, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.binding import ClusterTokenService
        rules, req = _node_workload(n_flows, n_req)
        shard = shard_flows(n_flows, rank, world)
        local = np.full(n_flows, -1, np.int64)
        local[shard] = np.arange(len(shard))
        keys = (req["key"] & abi.KEY_INDEX).astype(np.int64)
        order, counts = route_requests(keys, world)
        start = int(counts[:rank].sum())
        mine = np.sort(order[start:start + counts[rank]])   # arrival order within the shard
        sub = req[mine].copy()
        sub["key"] = (local[keys[mine]].astype(np.uint32)) | (sub["key"] & np.uint32(abi.KEY_PRIO))
        ora = ClusterTokenService()
        ora.set_namespaces(_ns())
        ora.load_rules(rules[shard])
        out = ora.decide(sub)
        now = int(req["ts_ms"][-1]) + 1
        snap = torch.tensor([[ora.avg(k, now, abi.EV_PASS), ora.avg(k, now, abi.EV_BLOCK)]
                             for k in range(len(shard))], dtype=torch.float64).reshape(-1, 2)
        roll = MetricRollup(len(shard), "cpu")
        totals = roll.run(snap)
        node = roll.node_snapshot([shard_flows(n_flows, r, world) for r in range(world)])
        q.put((rank, mine, out, totals.numpy().copy(), node.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_splitmix64_and_owner_are_stable():
    x = np.array([0, 1, 2, 12345678901234], dtype=np.uint64)
    assert list(splitmix64(x)) == [0xE220A8397B1DCDAF, 0x910A2DEC89025CC1, 0x975835DE1C9756CE, splitmix64(x)[3]]
    own = owner_of(np.arange(100_000, dtype=np.uint64), 8)
    counts = np.bincount(own, minlength=8)
    assert counts.min() > 11_000 and counts.max() < 14_000


def test_shards_partition_the_flows():
    for world in (1, 2, 4, 8):
        parts = [shard_flows(10_000, r, world) for r in range(world)]
        allf = np.sort(np.concatenate(parts))
        assert np.array_equal(allf, np.arange(10_000))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_decisions_and_rollup_equal_node_replay(world):
    from oracle.binding import ClusterTokenService
    n_flows, n_req = 3000, 60_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_flows, n_req, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # node-level sequential replay
    rules, req = _node_workload(n_flows, n_req)
    ora = ClusterTokenService()
    ora.set_namespaces(_ns())
    ora.load_rules(rules)
    want = ora.decide(req)
    now = int(req["ts_ms"][-1]) + 1
    node = np.array([[ora.avg(k, now, abi.EV_PASS), ora.avg(k, now, abi.EV_BLOCK)] for k in range(n_flows)])
    got = np.zeros_like(want)
    for rank, mine, out, totals, node_snap in res:
        got[mine] = out
        assert np.array_equal(node_snap, node)
        assert np.allclose(totals, node.sum(0), rtol=1e-12)
    assert np.array_equal(got, want)
