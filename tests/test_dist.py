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


class _CountingEngine:
    """Stands in for the engine's two exchange entry points (no GPU here): records what LimiterExchange asks for."""

    def __init__(self):
        self.calls = []

    def lim_slots(self):
        return 2

    def lim_arrivals(self, req_ptr, n, t_base, n_ms, counts_ptr, stream_ptr=0, counts_words=None):
        assert counts_words == 2 * n_ms
        self.calls.append(("arrivals", n, t_base, n_ms))

    def lim_exchange(self, gathered_ptr, t_base, n_ms, gathered_words=None):
        self.calls.append(("exchange", t_base, n_ms, gathered_words))


def _xch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sentinel_amd.cluster import LimiterExchange
        eng = _CountingEngine()
        x = LimiterExchange(eng, "cpu")
        # rank r's batch spans [100 + 10 r, 150 + 20 r]; the last rank has no requests in the second batch
        t_first, t_last = 100 + 10 * rank, 150 + 20 * rank
        r1 = x.arm(0, 5, t_first, t_last)
        empty = rank == world - 1
        r2 = x.arm(0, 0 if empty else 3, None if empty else 500 + rank, None if empty else 600 - rank)
        q.put((rank, r1, r2, eng.calls, tuple(x._gathered.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_limiter_exchange_time_range_and_gather(world):
    """cluster.LimiterExchange (SURVEY §8(e) limiter exchange) over gloo: every rank derives the same node-wide
    millisecond range (empty batches are neutral), counts with it, gathers world x n_lim x n_ms counts and arms."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
    lo1, hi1 = 100, 150 + 20 * (world - 1)
    lo2, hi2 = 500, 600
    for rank, r1, r2, calls, shape in res:
        assert r1 == (lo1, hi1 - lo1 + 1)
        assert r2 == (lo2, hi2 - lo2 + 1)
        assert calls[0] == ("arrivals", 5, lo1, hi1 - lo1 + 1)
        assert calls[1] == ("exchange", lo1, hi1 - lo1 + 1, world * 2 * (hi1 - lo1 + 1))
        assert calls[3] == ("exchange", lo2, hi2 - lo2 + 1, world * 2 * (hi2 - lo2 + 1))
        assert shape == (world * 2 * (hi2 - lo2 + 1),)


def test_node_order_is_ts_then_rank_then_position():
    from sentinel_amd.cluster import node_order
    ts = [np.array([5, 5, 7]), np.array([4, 5, 7, 7])]
    perm = node_order(ts)
    # concatenation: r0 = [5, 5, 7] at 0..2, r1 = [4, 5, 7, 7] at 3..6
    assert perm.tolist() == [3, 0, 1, 4, 2, 5, 6]
