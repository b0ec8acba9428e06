"""Parity of the node handle's sharded cluster param and concurrent tokens (sg_node_cparam_*, sg_node_conc_*) with one
sequential DefaultTokenService over the node's whole rule set (oracle.binding: ClusterTokenService.decide_param,
ConcurrentTokenService.decide).

A param rule lives on the shard owning its flowId (splitmix64(flowId) mod G); a concurrent acquire goes to the owner
of its flow rule, a release to the shard its node token id names. Every node batch is checked for time order and
value bounds as a whole, split stably by owner on devices[0], decided shard by shard and gathered back into caller
order. Compared exactly: every TokenResult, every (rule, value) window sum, the top values per rule, nowCalls and
the live-token count after expiry. Token ids are the node's own — unique, like the reference's — so the concurrent
test keeps an oracle id → node id map for the releases it sends.
"""
import numpy as np
import pytest

from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _ns(connected=2, limiter=False):
    ns = np.zeros(2, abi.NS_DTYPE)
    ns["connected_count"] = [connected, 1]
    if limiter:
        ns["limiter_enabled"][0] = 1
        ns["max_allowed_qps"][0] = 2000
    return ns


def _prules(rng, n, hot_per_rule=0):
    r = np.zeros(n, abi.CPARAM_RULE_DTYPE)
    r["flow_id"] = 7 + 3 * rng.permutation(20 * n)[:n]
    r["count"] = rng.integers(1, 40, n)
    r["threshold_type"] = np.where(rng.random(n) < 0.7, abi.THRESHOLD_GLOBAL, abi.THRESHOLD_AVG_LOCAL)
    r["sample_count"] = rng.choice([2, 5, 10], n)
    r["window_interval_ms"] = 1000
    r["namespace_id"] = rng.integers(0, 2, n)
    r["hot_begin"] = np.arange(n) * hot_per_rule
    r["hot_count"] = hot_per_rule
    return r


def _ptrace(rng, n, n_rules, n_values, t0, span, multi=0.1, bad=0.005):
    req = np.zeros(n, abi.CPARAM_REQ_DTYPE)
    req["ts_ms"] = t0 + np.sort(rng.integers(0, span, n))
    req["key"] = zipf_keys(rng, n_rules, n, 1.0, perm_seed=int(rng.integers(1 << 30))).astype(np.uint32)
    req["acquire"] = rng.integers(1, 4, n)
    counts = np.where(rng.random(n) < multi, rng.integers(2, 4, n), 1).astype(np.uint32)
    req["value_count"] = counts
    req["value_begin"] = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint32)
    values = zipf_keys(rng, n_values, int(counts.sum()), 1.1, perm_seed=int(rng.integers(1 << 30))).astype(np.uint64)
    values = values * np.uint64(0x9E3779B97F4A7C15)
    u = rng.random(n)
    req["key"][u < bad] = abi.KEY_BAD
    req["acquire"][(u >= bad) & (u < 2 * bad)] = 0
    req["key"][(u >= 2 * bad) & (u < 3 * bad)] = abi.KEY_NO_RULE
    req["key"][(u >= 3 * bad) & (u < 4 * bad)] = n_rules + 3          # past the node's rules
    req["value_count"][(u >= 4 * bad) & (u < 5 * bad)] = 0
    return req, values


def _param_trio(G, rules, hot, ns):
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import FlowEngine, NodeEngine
    node = NodeEngine([0] * G, max_batch=1 << 17)
    node.set_namespaces(ns)
    node.cparam_load_rules(rules, hot, 12)
    single = FlowEngine(device=0, max_batch=1 << 17)
    single.set_namespaces(ns)
    single.cparam_load_rules(rules, hot, 12)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_param_rules(rules, hot)
    return node, single, ora


def _same(got, want, what):
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        raise AssertionError(f"{what}: {len(bad)} differ; first {bad[0]}: oracle={want[bad[0]]} node={got[bad[0]]}")


@pytest.mark.parametrize("G", [1, 2, 3])
def test_node_param_tokens_equal_one_token_service(G):
    rng = np.random.default_rng(200 + G)
    R = 40
    rules = _prules(rng, R, hot_per_rule=2)
    hot = np.zeros(2 * R, abi.PARAM_HOT_DTYPE)
    for i in range(2 * R):
        hot[i] = ((i % 2 + 1) * 0x9E3779B97F4A7C15 % (1 << 64), int(rng.integers(0, 8)), 0)
    node, single, ora = _param_trio(G, rules, hot, _ns(connected=3))
    t = T0 + int(rng.integers(0, 1000))
    for b in range(3):
        req, vals = _ptrace(rng, 30_000, R, 200, t, 1500, multi=0.15)
        want = ora.decide_param(req, vals)
        _same(node.cparam_decide_host(req, vals), want, f"batch {b}")
        _same(single.cparam_decide_host(req, vals), want, f"single batch {b}")
        t = int(req["ts_ms"][-1]) + 1
    assert (want["status"] == abi.OK).any() and (want["status"] == abi.BLOCKED).any()
    now = int(req["ts_ms"][-1])
    keys = sorted({(int(q["key"]), int(v)) for q in req[:3000] if q["key"] < R and q["value_count"]
                   for v in vals[q["value_begin"]: q["value_begin"] + q["value_count"]]})
    for k, v in keys[:200]:
        assert node.cparam_sum(k, v, now) == ora.param_sum(k, v, now), (k, v)
    assert node.cparam_top_values(now, R, 5) == single.cparam_top_values(now, R, 5)


def test_node_param_reload_and_refused_batches():
    """A reload re-partitions the rules (surviving flowIds keep their owner, hence their metric); a batch with a
    value range past the value array, valid requests' ranges that overlap or run against request order (the
    sg_cparam_decide_batch contract), or out of time order is refused whole, leaving every shard untouched."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(210)
    rules = _prules(rng, 24)
    node, _, ora = _param_trio(3, rules, None, _ns())
    req, vals = _ptrace(rng, 20_000, 24, 80, T0, 900)
    _same(node.cparam_decide_host(req, vals), ora.decide_param(req, vals), "first")
    new = np.concatenate([rules[4:16], _prules(rng, 6)])
    new["flow_id"][12:] += 100_000
    node.cparam_load_rules(new, None, 12)
    ora.load_param_rules(new)
    t = int(req["ts_ms"][-1])
    nxt, nvals = _ptrace(rng, 20_000, len(new), 80, t, 900)
    bad = nxt.copy()
    bad["value_begin"][-1] = len(nvals)
    with pytest.raises(EngineError):
        node.cparam_decide_host(bad, nvals)
    valid = np.nonzero((nxt["key"] < len(new)) & (nxt["acquire"] > 0) & (nxt["value_count"] > 0))[0]
    a, b = int(valid[100]), int(valid[101])
    ovl = nxt.copy()  # two valid requests' ranges overlap
    ovl["value_begin"][b] = ovl["value_begin"][a]
    with pytest.raises(EngineError):
        node.cparam_decide_host(ovl, nvals)
    back = nxt.copy()  # two valid requests' ranges out of request order
    back["value_begin"][[a, b]] = back["value_begin"][[b, a]]
    back["value_count"][[a, b]] = 1
    with pytest.raises(EngineError):
        node.cparam_decide_host(back, nvals)
    old = nxt.copy()
    old["ts_ms"][0] = t - 5
    with pytest.raises(EngineError):
        node.cparam_decide_host(old, nvals)
    _same(node.cparam_decide_host(nxt, nvals), ora.decide_param(nxt, nvals), "after reload")
    now = int(nxt["ts_ms"][-1])
    for k in range(len(new)):
        v = int(nvals[0])
        assert node.cparam_sum(k, v, now) == ora.param_sum(k, v, now)


def test_node_param_refuses_namespace_limiter():
    """allowProceed shares the namespace's GlobalRequestLimiter in caller order: the sharded node path refuses rules
    under an enabled limiter (the front handle serves them), and decides nothing."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(211)
    rules = _prules(rng, 8)
    rules["namespace_id"] = 0
    node, _, _ = _param_trio(2, rules, None, _ns(limiter=True))
    req, vals = _ptrace(rng, 1_000, 8, 20, T0, 500)
    with pytest.raises(EngineError) as e:
        node.cparam_decide_host(req, vals)
    assert e.value.code == -4


def _crules(rng, k, fid0=1000):
    r = np.zeros(k, abi.RULE_DTYPE)
    r["flow_id"] = fid0 + rng.permutation(10 * k)[:k]
    r["count"] = rng.integers(1, 40, k).astype(np.float64) + np.where(rng.random(k) < 0.3, 0.5, 0.0)
    r["threshold_type"] = np.where(rng.random(k) < 0.3, abi.THRESHOLD_AVG_LOCAL, abi.THRESHOLD_GLOBAL)
    r["sample_count"], r["window_interval_ms"] = 10, 1000
    return r


class NodeTrace:
    """Acquire / release batches sent to the oracle and the node alike, a release naming the same token in each
    (oracle id ↔ node id); unknown ids are drawn above both id spaces."""

    def __init__(self, seed, k):
        self.rng = np.random.default_rng(seed)
        self.k = k
        self.live = []        # (oracle id, node id)
        self.released = []
        self.t = T0

    def batch(self, n, span):
        rng = self.rng
        q = np.zeros(n, abi.CONC_REQ_DTYPE)
        q["ts_ms"] = self.t + np.sort(rng.integers(0, span, n))
        qn = q.copy()
        for i in range(n):
            if rng.random() < 0.55 or not self.live:
                q[i]["kind"] = abi.CONC_ACQUIRE
                q[i]["key"] = min(int(rng.zipf(1.3)) - 1, self.k + 5) if rng.random() > 0.01 else abi.KEY_BAD
                q[i]["acquire"] = int(rng.integers(1, 4)) if rng.random() > 0.01 else 0
                q[i]["client"] = int(rng.integers(1, 21)) if rng.random() > 0.02 else 0
                qn[i] = q[i]
                continue
            q[i]["kind"] = qn[i]["kind"] = abi.CONC_RELEASE
            u = rng.random()
            if u < 0.8:
                ot, nt = self.live.pop(int(rng.integers(len(self.live))))
            elif u < 0.9 and self.released:
                ot, nt = self.released[int(rng.integers(len(self.released)))]
            elif u < 0.95:
                ot = nt = int(rng.integers(1 << 50, 1 << 51))
            else:
                ot = nt = 0
            q[i]["token_id"], qn[i]["token_id"] = ot, nt
        self.t += span
        return q, qn

    def absorb(self, q, want, got):
        ok = (q["kind"] == abi.CONC_ACQUIRE) & (want["status"] == abi.OK)
        rel = (q["kind"] == abi.CONC_RELEASE) & (want["status"] == abi.RELEASE_OK)
        gone = set(int(x) for x in q["token_id"][rel])
        pairs = list(zip((int(x) for x in want["token_id"][ok]), (int(x) for x in got["token_id"][ok])))
        self.released = (self.released + [p for p in self.live if p[0] in gone])[-200:]
        self.live = [p for p in self.live if p[0] not in gone] + pairs


@pytest.mark.parametrize("G", [1, 2, 3])
def test_node_concurrent_tokens_equal_one_token_service(G):
    from oracle.binding import ConcurrentTokenService
    from sentinel_amd.engine import NodeEngine
    rng = np.random.default_rng(300 + G)
    k = 120
    rules = _crules(rng, k)
    ns = _ns(connected=3)
    timeouts = (rng.integers(200, 3000, k), rng.integers(100, 1500, k))
    node = NodeEngine([0] * G, max_batch=1 << 17)
    node.set_namespaces(ns)
    node.load_rules(rules)
    node.conc_set_rule_timeouts(*timeouts)
    ora = ConcurrentTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    ora.set_rule_timeouts(*timeouts)
    tr = NodeTrace(400 + G, k)
    seen = set()
    for b in range(5):
        q, qn = tr.batch(15_000, 700)
        want = ora.decide(q)
        got = node.conc_decide_host(qn)
        _same(got["status"], want["status"], f"batch {b} status")
        ok = (q["kind"] == abi.CONC_ACQUIRE) & (want["status"] == abi.OK)
        _same(got["token_id"] != 0, want["token_id"] != 0, f"batch {b} token presence")
        ids = got["token_id"][ok]
        assert len(np.unique(ids)) == len(ids) and not set(ids.tolist()) & {p[1] for p in tr.live}
        if G > 1:
            assert len({(int(x) - 1) % G for x in ids}) > 1   # tokens minted by several shards
        tr.absorb(q, want, got)
        seen |= set(want["status"].tolist())
        online = (rng.random(22) < 0.7).astype(np.uint8)
        assert node.conc_expire(tr.t, online) == ora.expire(tr.t, online)
        live = None
        for key in range(k):
            now, live = node.conc_state(key)
            assert now == ora.now_calls(key), f"nowCalls of {key}"
        assert live == ora.live()
    assert {abi.OK, abi.BLOCKED, abi.RELEASE_OK, abi.ALREADY_RELEASE} <= seen
