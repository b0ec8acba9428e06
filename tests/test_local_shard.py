"""The local slot chain sharded over a node's GPUs (sentinel_amd/cluster.py: local_owners, split_local_events,
LocalMetricRollup; the C ABI's sg_local_owners / sg_local_metrics_raw): every rank loads the same rules and decides
the entries and exits of the resources it owns — key groups (RELATE references) on one owner — and the node's
metric rows, Constants.ENTRY_NODE included, are merged over the ranks. On CPU with gloo (world size 2 and 3): each
rank decides its share with the oracle (no GPU here); every result and every metrics.log row must equal one
sequential replay of the whole node trace (resources of different groups share no decision state)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sentinel_amd import abi
from sentinel_amd.cluster import (ENTRY_NODE_RESOURCE, DeviceLocalMetricRollup, LocalMetricRollup, local_group_keys,
                                  local_owners, merge_metric_rows, split_local_events)

N_RES, N_ORIGINS = 48, 2
T0 = 1_700_000_000_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def node_setup(seed=3):
    """Rules of the node (plain, origin-limited, WarmUp, RELATE pairs, breakers) and the inbound resources."""
    from oracle.binding import degrade_rule, local_flow_rule, local_rule
    rng = np.random.default_rng(seed)
    base = np.zeros(N_RES, abi.LOCAL_RULE_DTYPE)
    for r in range(N_RES):
        brk = [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.4, 1, 5, 1000)] if r % 3 == 0 else []
        base[r] = local_rule(0.0, abi.FLOW_GRADE_NONE, brk)
    fr, relate = [], []
    for r in range(N_RES):
        shape = r % 6
        if shape == 0:
            fr.append(local_flow_rule(r, float(rng.integers(3, 30))))
        elif shape == 1:
            fr += [local_flow_rule(r, float(rng.integers(10, 40))), local_flow_rule(r, 4.0, limit_app=1)]
        elif shape == 2:
            fr.append(local_flow_rule(r, float(rng.integers(10, 40)), behavior=abi.CONTROL_WARM_UP, warm_up_sec=3))
        elif shape == 3:  # RELATE: reads another resource's ClusterNode
            ref = int((r + 7) % N_RES)
            fr.append(local_flow_rule(r, float(rng.integers(5, 25)), strategy=abi.STRATEGY_RELATE, ref=ref))
            relate.append((r, ref))
        elif shape == 4:
            fr.append(local_flow_rule(r, float(rng.integers(2, 10)), grade=abi.FLOW_GRADE_THREAD))
    frules = np.array(fr, abi.LOCAL_FLOW_RULE_DTYPE)
    inbound = (rng.random(N_RES) < 0.5).astype(np.uint8)
    return base, frules, relate, inbound


def node_trace(base, frules, inbound, n_batches=3, n=6000, seed=4):
    """Batches of (events, results) of one sequential node replay (entries + the exits of passed entries), and the
    node's metric rows fetched after each batch at its end (the single-chain reference)."""
    from oracle.binding import LocalChain, LocalTraceGen
    from sentinel_amd.workload import zipf_keys
    rng = np.random.default_rng(seed)
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(base)
    ora.load_flow_rules(frules, N_ORIGINS, 0)
    ora.set_entry_types(inbound)
    gen = LocalTraceGen(ora)
    out = []
    for b in range(n_batches):
        t = T0 + 1500 * b
        ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
        ent["ts_ms"] = t + np.sort(rng.integers(0, 1500, n))
        ent["resource"] = zipf_keys(rng, N_RES, n, 1.0, perm_seed=7)
        ent["resource"] |= np.where(rng.random(n) < 0.05, np.uint32(abi.KEY_PRIO), np.uint32(0))
        ent["count"] = 1
        ent["origin"] = rng.integers(0, N_ORIGINS + 1, n)
        rt = rng.integers(0, 60, n).astype(np.int32)
        err = (rng.random(n) < 0.1).astype(np.uint8)
        ev, res = gen.run(ent, rt, err, t + 1500)
        rows = ora.metrics(t + 1500)
        out.append((ev, res, t + 1500, rows))
    return out


def test_local_owners_co_locate_groups():
    base, frules, relate, inbound = node_setup()
    g = local_group_keys(N_RES, relate)
    for a, b in relate:
        assert g[a] == g[b]
    for world in (2, 3, 8):
        own = local_owners(N_RES, relate, world)
        assert own.min() >= 0 and own.max() < world
        for a, b in relate:
            assert own[a] == own[b]


def test_merge_metric_rows_sums_entry_node():
    """Two ranks' raw rows of the same second: ENTRY_NODE rows add up, rt = Σrt // Σsuccess; resource rows pass."""
    rows = np.zeros(4, abi.METRIC_NODE_DTYPE)
    rows[0] = (1000, 3, 1, 2, 0, 50, 0, 5, 0)
    rows[1] = (1000, 2, 0, 1, 1, 40, 0, ENTRY_NODE_RESOURCE, 0)
    rows[2] = (1000, 1, 0, 2, 0, 31, 0, ENTRY_NODE_RESOURCE, 0)
    rows[3] = (2000, 0, 0, 0, 0, 0, 0, ENTRY_NODE_RESOURCE, 0)  # empty: not a valid row
    m = merge_metric_rows([rows[:2], rows[2:]])
    assert len(m) == 2
    assert tuple(m[0])[:6] == (1000, 3, 1, 2, 0, 25) and m[0]["resource"] == 5
    assert tuple(m[1])[:6] == (1000, 3, 0, 3, 1, 23) and m[1]["resource"] == ENTRY_NODE_RESOURCE
    d = DeviceLocalMetricRollup.merge(torch.from_numpy(rows.view(np.int64).reshape(-1, 8).copy()))
    assert np.array_equal(d.numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1), m)


def test_device_merge_equals_host_merge():
    """DeviceLocalMetricRollup.merge (torch, the device rollup's merge) equals merge_metric_rows on random rows of
    three GPUs: resources disjoint per GPU, ENTRY_NODE rows of overlapping seconds (some empty), rows unsorted."""
    rng = np.random.default_rng(9)
    parts = []
    for g in range(3):
        n = 400
        r = np.zeros(n + 6, abi.METRIC_NODE_DTYPE)
        r["timestamp"] = T0 + 1000 * rng.integers(0, 5, n + 6)
        for f in ("pass_qps", "block_qps", "success_qps", "exception_qps", "occupied_pass_qps"):
            r[f] = rng.integers(0, 4, n + 6)
        r["rt"] = rng.integers(0, 500, n + 6)
        r["resource"][:n] = rng.permutation(1000)[:n] * 3 + g
        r["resource"][n:] = ENTRY_NODE_RESOURCE
        r["timestamp"][n:] = T0 + 1000 * (np.arange(6) // 2)   # two GPUs share each second
        r[n + 5]["pass_qps"] = r[n + 5]["block_qps"] = r[n + 5]["success_qps"] = 0
        r[n + 5]["exception_qps"] = r[n + 5]["rt"] = 0
        parts.append(r[rng.permutation(n + 6)])
    want = merge_metric_rows(parts)
    t = torch.from_numpy(np.concatenate(parts).view(np.int64).reshape(-1, 8).copy())
    got = DeviceLocalMetricRollup.merge(t).numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
    assert np.array_equal(got, want)
    parts[1]["timestamp"] += 1000 * (1 << 32)  # rows spanning more than 2^31 ms: the two-sort path
    want = merge_metric_rows(parts)
    t = torch.from_numpy(np.concatenate(parts).view(np.int64).reshape(-1, 8).copy())
    got = DeviceLocalMetricRollup.merge(t).numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
    assert np.array_equal(got, want)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.binding import LocalChain
        base, frules, relate, inbound = node_setup()
        trace = node_trace(base, frules, inbound)
        owners = local_owners(N_RES, relate, world)
        mine_chain = LocalChain(2, 1000, 500)
        mine_chain.load_rules(base)
        mine_chain.load_flow_rules(frules, N_ORIGINS, 0)
        mine_chain.set_entry_types(inbound)
        rollup = LocalMetricRollup("cpu")
        drollup = DeviceLocalMetricRollup("cpu")
        bad = []
        for b, (ev, want, now, rows_want) in enumerate(trace):
            pos = split_local_events(ev, owners, world)[rank]
            got = mine_chain.decide(ev[pos])
            if not np.array_equal(got, want[pos]):
                bad.append(f"batch {b}: {(got != want[pos]).sum()} results differ")
            raw = mine_chain.metrics(now, raw=True)
            rows = rollup.run(raw)
            if not np.array_equal(rows, rows_want):
                bad.append(f"batch {b}: metric rows differ ({len(rows)} vs {len(rows_want)})")
            drows = drollup.run(torch.from_numpy(raw.view(np.int64).reshape(-1, 8).copy()))
            if not np.array_equal(drows.numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1), rows_want):
                bad.append(f"batch {b}: device-rollup rows differ")
            if b == 0 and not (rows_want["resource"] == ENTRY_NODE_RESOURCE).any():
                bad.append("no ENTRY_NODE row in the reference")
        q.put((rank, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_local_chain_equals_node_replay(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad in res:
        assert not bad, f"rank {rank}: {bad}"
