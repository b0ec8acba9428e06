"""Sharded namespace limiter (SURVEY §8(e) exchange step; GlobalRequestLimiter.java:46-55,
ClusterFlowChecker.allowProceed :45-51): every GPU holds a share of the flowIds but the namespace window is
node-wide. Shards count their limited arrivals per millisecond (sg_lim_arrivals), the node gathers them, every
shard is armed with the gathered counts (sg_lim_exchange) and decides its own requests. The results must equal one
oracle replay of the merged batch in the node's arrival order (ts, shard rank, position in the shard's batch),
batch after batch (each shard keeps a replica of the namespace windows), including shards with no requests.
Here the shards are handles in one process and the gather is a device concat; tests/test_dist_gpu.py runs the
same exchange over torch.distributed."""
import numpy as np
import pytest
import torch

from sentinel_amd import abi
from sentinel_amd.cluster import node_order, route_requests, shard_flows

pytestmark = pytest.mark.gpu

N_FLOWS = 3000


def _ns(qps):
    ns = np.zeros(3, abi.NS_DTYPE)
    ns["connected_count"] = [1, 2, 1]
    ns["limiter_enabled"] = [1, 0, 1]
    ns["max_allowed_qps"] = [qps, 0, qps * 3 + 7]
    return ns


def _rules(rng):
    from sentinel_amd.workload import ClusterWorkload
    r = ClusterWorkload(n_flows=N_FLOWS, seed=5).rules()
    r["count"] = rng.integers(1, 400, N_FLOWS).astype(np.float64)
    r["namespace_id"] = rng.integers(0, 3, N_FLOWS)
    return r


def _batches(rng, t0):
    """Time-ordered node batches with many requests per millisecond (the interleaving matters), invalid keys,
    gaps between batches, and one batch whose requests all belong to few flows (some shards get none)."""
    out, t = [], t0
    for b in range(4):
        n = int(rng.integers(20_000, 60_000))
        span = int(rng.integers(80, 1500))
        req = np.zeros(n, abi.REQ_DTYPE)
        req["ts_ms"] = t + np.sort(rng.integers(0, span, n))
        if b == 2:
            req["key"] = rng.integers(0, 2, n).astype(np.uint32)  # two flows only
        else:
            req["key"] = np.minimum(rng.zipf(1.2, n) - 1, N_FLOWS - 1).astype(np.uint32)
            req["key"][rng.random(n) < 0.01] = abi.KEY_NO_RULE
        req["acquire"] = np.where(rng.random(n) < 0.1, rng.integers(2, 5, n), 1)
        req["acquire"][rng.random(n) < 0.005] = 0  # BAD_REQUEST: not a tryPass
        req["key"] |= np.where(rng.random(n) < 0.03, np.uint32(abi.KEY_PRIO), np.uint32(0))
        out.append(req)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 900))
    return out


def _split(req, world, local):
    """Per rank: node indices (arrival order) and the shard batch with shard-local keys (KEY_NO_RULE / BAD keys
    go to flow 0's owner, which answers them as the node would)."""
    keys = (req["key"] & abi.KEY_INDEX).astype(np.int64)
    valid = keys < N_FLOWS
    route = np.where(valid, keys, 0)
    order, counts = route_requests(route, world)
    parts, start = [], 0
    for r in range(world):
        mine = np.sort(order[start:start + counts[r]])
        start += counts[r]
        sub = req[mine].copy()
        k = keys[mine]
        ok = k < N_FLOWS
        sub["key"] = np.where(ok, local[r][np.where(ok, k, 0)], sub["key"] & abi.KEY_INDEX).astype(np.uint32) | \
            (sub["key"] & np.uint32(abi.KEY_PRIO))
        parts.append((mine, sub))
    return parts


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("qps", [0.0, 40.0, 3000.0, 1e12])
def test_sharded_limiter_equals_node_replay(world, qps):
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(world * 1000 + int(qps) % 997)
    rules = _rules(rng)
    ns = _ns(qps)
    shards = [shard_flows(N_FLOWS, r, world) for r in range(world)]
    local = []
    for s in shards:
        m = np.full(N_FLOWS, abi.KEY_NO_RULE, np.int64)
        m[s] = np.arange(len(s))
        local.append(m)
    engs = []
    for r in range(world):
        e = FlowEngine(device=0, max_batch=1 << 16)
        e.set_shard(r, world)
        e.set_namespaces(ns)
        e.load_rules(rules[shards[r]])
        engs.append(e)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    dev = torch.device("cuda:0")
    n_lim = int(ns["limiter_enabled"].sum())
    saw_tmr = False
    for req in _batches(rng, 1_700_000_000_033):
        parts = _split(req, world, local)
        ts = [p[1]["ts_ms"] for p in parts]
        t_base = min(int(t[0]) for t in ts if len(t))
        n_ms = max(int(t[-1]) for t in ts if len(t)) - t_base + 1
        reqs_d = [torch.from_numpy(p[1].view(np.uint8).copy()).to(dev) for p in parts]
        counts = []
        for r in range(world):
            c = torch.zeros(n_lim * n_ms, dtype=torch.int32, device=dev)
            engs[r].lim_arrivals(reqs_d[r].data_ptr() if len(parts[r][1]) else 0, len(parts[r][1]), t_base, n_ms,
                                 c.data_ptr())
            counts.append(c)
        gathered = torch.cat(counts)
        torch.cuda.synchronize()
        got = []
        for r in range(world):
            n = len(parts[r][1])
            out = torch.zeros(max(1, n) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            engs[r].lim_exchange(gathered.data_ptr(), t_base, n_ms)
            engs[r].decide_device(reqs_d[r].data_ptr() if n else 0, n, out.data_ptr())
            got.append(out.cpu().numpy().view(abi.RES_DTYPE)[:n])
        # the oracle decides the merged batch in node order (ts, rank, position)
        cat_idx = np.concatenate([p[0] for p in parts])
        perm = node_order(ts)
        want_node = ora.decide(req[cat_idx[perm]])
        want = np.empty_like(want_node)
        want[perm] = want_node
        got_cat = np.concatenate(got)
        bad = np.nonzero(got_cat != want)[0]
        assert len(bad) == 0, f"{len(bad)} of {len(want)} differ; first {got_cat[bad[:3]]} vs {want[bad[:3]]}"
        saw_tmr |= bool((want["status"] == abi.TOO_MANY_REQUEST).any())
    assert saw_tmr == (qps < 1e6)


def test_sharded_limiter_contract():
    """A sharded handle with a limited namespace decides only through the exchange: a flow batch without an
    armed exchange, the pipelined entry points and requests outside the exchange's range are refused."""
    from sentinel_amd.engine import EngineError, FlowEngine
    rng = np.random.default_rng(3)
    rules = _rules(rng)
    e = FlowEngine(device=0, max_batch=4096)
    e.set_shard(0, 2)
    e.set_namespaces(_ns(100.0))
    mine = rules[shard_flows(N_FLOWS, 0, 2)]
    e.load_rules(mine)
    req = np.zeros(16, abi.REQ_DTYPE)
    req["ts_ms"] = 1_700_000_000_000 + np.arange(16)
    req["acquire"] = 1
    req["key"] = int(np.nonzero(mine["namespace_id"] == 0)[0][0])  # a flow of a limited namespace
    with pytest.raises(EngineError) as ei:
        e.decide_host(req)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    out = e.host_array(len(req), abi.RES_DTYPE)
    with pytest.raises(EngineError) as ei:
        e.submit(req, out)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    dev = torch.device("cuda:0")
    rq = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    c = torch.zeros(2 * 8, dtype=torch.int32, device=dev)
    with pytest.raises(EngineError) as ei:  # the range must hold every limited request
        e.lim_arrivals(rq.data_ptr(), len(req), 1_700_000_000_004, 8, c.data_ptr())
    assert ei.value.code == abi.SG_E_INVAL
    # the same handle unsharded decides without the exchange
    e.set_shard(0, 1)
    assert len(e.decide_host(req)) == len(req)


def test_rejected_shard_batch_keeps_replicas_equal():
    """A shard whose batch is rejected (a batch out of time order → SG_E_TIME on the device; a null output buffer →
    SG_E_INVAL before the device) still walks the node's gathered arrivals, so its replica of the namespace windows
    stays equal to the other shards' and later batches still equal the node replay. The node counted the rejected
    requests as limiter arrivals, so the oracle replays them against stand-in flows of the same namespaces (huge
    thresholds, never compared): their flow windows stay untouched, as on the rejecting shard."""
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import EngineError, FlowEngine
    world = 3
    rng = np.random.default_rng(77)
    rules = _rules(rng)
    ns = _ns(120.0)
    shards = [shard_flows(N_FLOWS, r, world) for r in range(world)]
    local = []
    for s in shards:
        m = np.full(N_FLOWS, abi.KEY_NO_RULE, np.int64)
        m[s] = np.arange(len(s))
        local.append(m)
    engs = []
    for r in range(world):
        e = FlowEngine(device=0, max_batch=1 << 16)
        e.set_shard(r, world)
        e.set_namespaces(ns)
        e.load_rules(rules[shards[r]])
        engs.append(e)
    stand_in = np.zeros(3, abi.RULE_DTYPE)  # one per namespace, after the real flows
    stand_in["flow_id"] = 10_000_000 + np.arange(3)
    stand_in["count"] = 1e15
    stand_in["threshold_type"] = abi.THRESHOLD_GLOBAL
    stand_in["sample_count"], stand_in["window_interval_ms"] = 10, 1000
    stand_in["namespace_id"] = np.arange(3)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(np.concatenate([rules, stand_in]))
    dev = torch.device("cuda:0")
    n_lim = int(ns["limiter_enabled"].sum())
    reject = {1: (0, "unordered"), 2: (1, "null")}  # node batch → (shard, how)
    compared = 0
    for b, req in enumerate(_batches(rng, 1_700_000_000_500)):
        parts = _split(req, world, local)
        ts = [p[1]["ts_ms"] for p in parts]
        t_base = min(int(t[0]) for t in ts if len(t))
        n_ms = max(int(t[-1]) for t in ts if len(t)) - t_base + 1
        rr, how = reject.get(b, (-1, None))
        if rr >= 0 and len(parts[rr][1]) < 3:
            rr = -1
        sub_r = parts[rr][1].copy() if rr >= 0 else None
        if how == "unordered":  # swap the first and last timestamps: same per-millisecond counts
            sub_r["ts_ms"][[0, -1]] = sub_r["ts_ms"][[-1, 0]]
        subs = [sub_r if r == rr else parts[r][1] for r in range(world)]
        reqs_d = [torch.from_numpy(s.view(np.uint8).copy()).to(dev) for s in subs]
        counts = []
        for r in range(world):
            c = torch.zeros(n_lim * n_ms, dtype=torch.int32, device=dev)
            engs[r].lim_arrivals(reqs_d[r].data_ptr() if len(subs[r]) else 0, len(subs[r]), t_base, n_ms, c.data_ptr())
            counts.append(c)
        gathered = torch.cat(counts)
        torch.cuda.synchronize()
        got = []
        for r in range(world):
            n = len(subs[r])
            out = torch.zeros(max(1, n) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            engs[r].lim_exchange(gathered.data_ptr(), t_base, n_ms)
            if r == rr:
                with pytest.raises(EngineError) as ei:
                    engs[r].decide_device(reqs_d[r].data_ptr(), n, 0 if how == "null" else out.data_ptr())
                assert ei.value.code == (abi.SG_E_INVAL if how == "null" else abi.SG_E_TIME)
                got.append(None)
            else:
                engs[r].decide_device(reqs_d[r].data_ptr() if n else 0, n, out.data_ptr())
                got.append(out.cpu().numpy().view(abi.RES_DTYPE)[:n])
        node_req = req.copy()
        if rr >= 0:  # the rejected shard's valid requests → the stand-in flow of their namespace
            mine = parts[rr][0]
            k = (node_req["key"][mine] & abi.KEY_INDEX).astype(np.int64)
            ok = (k < N_FLOWS) & (node_req["acquire"][mine] > 0)
            nsid = rules["namespace_id"][np.where(ok, k, 0)]
            node_req["key"][mine[ok]] = (N_FLOWS + nsid[ok]).astype(np.uint32) | \
                (node_req["key"][mine[ok]] & np.uint32(abi.KEY_PRIO))
        cat_idx = np.concatenate([p[0] for p in parts])
        perm = node_order(ts)
        want_node = ora.decide(node_req[cat_idx[perm]])
        want = np.empty_like(want_node)
        want[perm] = want_node
        off = 0
        for r in range(world):
            n = len(parts[r][1])
            if got[r] is not None:
                bad = np.nonzero(got[r] != want[off:off + n])[0]
                assert len(bad) == 0, f"batch {b} shard {r}: {len(bad)} of {n} differ"
                compared += n
            off += n
    assert compared > 0


def _shard_engines(world, rules, ns, max_batch=1 << 16):
    from sentinel_amd.engine import FlowEngine
    shards = [shard_flows(N_FLOWS, r, world) for r in range(world)]
    local = []
    for s in shards:
        m = np.full(N_FLOWS, abi.KEY_NO_RULE, np.int64)
        m[s] = np.arange(len(s))
        local.append(m)
    engs = []
    for r in range(world):
        e = FlowEngine(device=0, max_batch=max_batch)
        e.set_shard(r, world)
        e.set_namespaces(ns)
        e.load_rules(rules[shards[r]])
        engs.append(e)
    return shards, local, engs


@pytest.mark.parametrize("path", ["enqueue", "submit"])
def test_sharded_limiter_pipelined_equals_node_replay(path):
    """The exchange on the pipelined entry points: per node batch every shard counts, the node gathers, and every
    shard arms its next sg_flow_enqueue (device batches) / sg_flow_submit (pinned host batches) and goes on without
    waiting — batches of one shard overlap (front half beside the previous walkers), each armed with its own
    exchange. Every result equals one oracle replay of the merged batches in node order."""
    from oracle.binding import ClusterTokenService
    world = 2
    rng = np.random.default_rng(91 if path == "enqueue" else 92)
    rules = _rules(rng)
    ns = _ns(60.0)
    shards, local, engs = _shard_engines(world, rules, ns)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    dev = torch.device("cuda:0")
    n_lim = int(ns["limiter_enabled"].sum())
    pending = []  # (tickets per shard, outputs per shard, wanted results per shard)
    keep = []
    batches = _batches(rng, 1_700_000_000_101) + _batches(rng, 1_700_000_020_000)
    for req in batches:
        parts = _split(req, world, local)
        ts = [p[1]["ts_ms"] for p in parts]
        t_base = min(int(t[0]) for t in ts if len(t))
        n_ms = max(int(t[-1]) for t in ts if len(t)) - t_base + 1
        reqs_d = [torch.from_numpy(p[1].view(np.uint8).copy()).to(dev) for p in parts]
        counts = []
        for r in range(world):
            c = torch.zeros(n_lim * n_ms, dtype=torch.int32, device=dev)
            engs[r].lim_arrivals(reqs_d[r].data_ptr() if len(parts[r][1]) else 0, len(parts[r][1]), t_base, n_ms,
                                 c.data_ptr())
            counts.append(c)
        gathered = torch.cat(counts)
        torch.cuda.synchronize()
        tickets, outs = [], []
        for r in range(world):
            n = len(parts[r][1])
            engs[r].lim_exchange(gathered.data_ptr(), t_base, n_ms)
            if path == "enqueue":
                out = torch.zeros(max(1, n) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device=dev)
                tickets.append(engs[r].enqueue_device(reqs_d[r].data_ptr() if n else 0, n, out.data_ptr()))
            else:
                hin = engs[r].host_array(max(1, n), abi.REQ_DTYPE)
                out = engs[r].host_array(max(1, n), abi.RES_DTYPE)
                hin[:n] = parts[r][1]
                tickets.append(engs[r].submit(hin[:n], out[:n]))
                keep.append((engs[r], hin))
            outs.append(out)
        del gathered  # the pipelined calls copied it
        cat_idx = np.concatenate([p[0] for p in parts])
        perm = node_order(ts)
        want_node = ora.decide(req[cat_idx[perm]])
        want = np.empty_like(want_node)
        want[perm] = want_node
        wants, off = [], 0
        for r in range(world):
            n = len(parts[r][1])
            wants.append(want[off:off + n])
            off += n
        pending.append((tickets, outs, wants))
    saw_tmr = False
    for b, (tickets, outs, wants) in enumerate(pending):
        for r in range(world):
            if tickets[r]:
                engs[r].wait(tickets[r])
            n = len(wants[r])
            got = outs[r].cpu().numpy().view(abi.RES_DTYPE)[:n] if path == "enqueue" else outs[r][:n]
            bad = np.nonzero(got != wants[r])[0]
            assert len(bad) == 0, (f"batch {b} shard {r}: {len(bad)} of {n} differ; first (got, want): "
                                   f"{[(tuple(got[i]), tuple(wants[r][i])) for i in bad[:6]]}")
            saw_tmr |= bool((wants[r]["status"] == abi.TOO_MANY_REQUEST).any())
    assert saw_tmr
    for e, a in keep:
        e.free_host(a)


def test_sharded_limiter_cluster_param_equals_node_replay():
    """Cluster param tokens share the namespace limiter (ClusterParamFlowChecker.java:43-45): param rules sharded
    over the shards by rule, sg_lim_arrivals_param counts each shard's param requests, the node gathers them and
    every shard's sg_cparam_decide_batch consumes the exchange. Results equal the oracle's decide_param over the
    merged batch in node order, batch after batch, including a shard without requests."""
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import FlowEngine
    world = 3
    rng = np.random.default_rng(93)
    R = 24
    prules = np.zeros(R, abi.CPARAM_RULE_DTYPE)
    prules["flow_id"] = np.arange(R) * 5 + 3
    prules["count"] = rng.integers(5, 60, R)
    prules["threshold_type"] = abi.THRESHOLD_GLOBAL
    prules["sample_count"], prules["window_interval_ms"] = 10, 1000
    prules["namespace_id"] = rng.integers(0, 3, R)
    ns = _ns(150.0)
    owner = np.arange(R) % world                 # rule r lives on shard r % world
    local = np.zeros(R, np.int64)
    engs = []
    for s in range(world):
        mine = np.nonzero(owner == s)[0]
        local[mine] = np.arange(len(mine))
        e = FlowEngine(device=0, max_batch=1 << 16)
        e.set_shard(s, world)
        e.set_namespaces(ns)
        e.cparam_load_rules(prules[mine], None, 12)
        engs.append(e)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_param_rules(prules)
    dev = torch.device("cuda:0")
    n_lim = int(ns["limiter_enabled"].sum())
    t = 1_700_000_000_000
    saw_tmr = False
    for b in range(4):
        n = int(rng.integers(8_000, 20_000))
        req = np.zeros(n, abi.CPARAM_REQ_DTYPE)
        req["ts_ms"] = t + np.sort(rng.integers(0, int(rng.integers(100, 1500)), n))
        req["key"] = rng.integers(0, R, n) if b != 2 else rng.choice([0, 3], n)  # batch 2: shards 1, 2 get nothing
        req["acquire"] = rng.integers(1, 3, n)
        cnt = np.where(rng.random(n) < 0.2, rng.integers(2, 4, n), 1).astype(np.uint32)
        req["value_count"] = cnt
        req["value_begin"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
        values = (rng.zipf(1.3, int(cnt.sum())) % 500).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        req["acquire"][rng.random(n) < 0.01] = 0  # BAD_REQUEST: not a tryPass
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 700))
        parts = []
        for s in range(world):
            idx = np.nonzero(owner[req["key"]] == s)[0]
            sub = req[idx].copy()
            sub["key"] = local[req["key"][idx]].astype(np.uint32)
            vb = np.concatenate([[0], np.cumsum(sub["value_count"])[:-1]]).astype(np.uint32)
            vals = np.concatenate([values[q["value_begin"]:q["value_begin"] + q["value_count"]] for q in req[idx]]) \
                if len(idx) else np.zeros(0, np.uint64)
            sub["value_begin"] = vb
            parts.append((idx, sub, vals.astype(np.uint64)))
        ts = [p[1]["ts_ms"] for p in parts]
        t_base = min(int(x[0]) for x in ts if len(x))
        n_ms = max(int(x[-1]) for x in ts if len(x)) - t_base + 1
        reqs_d = [torch.from_numpy(p[1].view(np.uint8).copy()).to(dev) for p in parts]
        counts = []
        for s in range(world):
            c = torch.zeros(n_lim * n_ms, dtype=torch.int32, device=dev)
            engs[s].lim_arrivals_param(reqs_d[s].data_ptr() if len(parts[s][1]) else 0, len(parts[s][1]), t_base, n_ms,
                                       c.data_ptr())
            counts.append(c)
        gathered = torch.cat(counts)
        torch.cuda.synchronize()
        got = []
        for s in range(world):
            engs[s].lim_exchange(gathered.data_ptr(), t_base, n_ms)
            got.append(engs[s].cparam_decide_host(parts[s][1], parts[s][2]))
        cat_idx = np.concatenate([p[0] for p in parts])
        perm = node_order(ts)
        node = req[cat_idx[perm]]
        want_node = ora.decide_param(node, values)   # value_begin still indexes the node's value array
        want = np.empty_like(want_node)
        want[perm] = want_node
        off = 0
        for s in range(world):
            k = len(parts[s][1])
            bad = np.nonzero(got[s] != want[off:off + k])[0]
            assert len(bad) == 0, f"batch {b} shard {s}: {len(bad)} of {k} differ"
            off += k
        saw_tmr |= bool((want["status"] == abi.TOO_MANY_REQUEST).any())
    assert saw_tmr
