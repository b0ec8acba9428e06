"""Parity of the node handle (sg_node_*: one token server over G shard handles with routing inside the library) with
one sequential DefaultTokenService over the whole node's rules (oracle.binding.ClusterTokenService).

The node hashes flowIds over its shards (splitmix64(flowId) mod G), runs validation and the namespace limiters over
each node batch in caller order on its front handle, splits the admitted requests by owner (a stable device
multisplit, node.hip), lets every shard decide its slice on its own stream, and gathers the results back. Here the
G shards share device 0 (the one-GPU box); the same code peer-copies slices for shards on other devices. Compared
bit-exactly: every result (BAD_REQUEST / NO_RULE_EXISTS / TOO_MANY_REQUEST / OK / BLOCKED / SHOULD_WAIT, remaining,
wait), every flowId's ClusterMetric ring and occupy counters, across rule reloads; the node's metric snapshot equals
a single handle's that decided the same batches.
"""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu


def _rules(rng, K, fid0=1000):
    r = np.zeros(K, abi.RULE_DTYPE)
    r["flow_id"] = fid0 + rng.permutation(10 * K)[:K]
    r["count"] = rng.integers(1, 40, K)
    r["threshold_type"] = np.where(rng.random(K) < 0.8, abi.THRESHOLD_GLOBAL, 0)
    r["sample_count"] = rng.choice([2, 5, 10], K)
    r["window_interval_ms"] = 1000
    r["namespace_id"] = rng.integers(0, 3, K)
    return r


def _ns(lim_qps):
    ns = np.zeros(3, abi.NS_DTYPE)
    ns["connected_count"] = [2, 1, 4]
    if lim_qps:
        ns["limiter_enabled"][[0, 2]] = 1
        ns["max_allowed_qps"][[0, 2]] = [lim_qps, lim_qps / 2]
    return ns


def _batch(rng, n, K, t, span):
    req = np.zeros(n, abi.REQ_DTYPE)
    req["ts_ms"] = t + np.sort(rng.integers(0, span, n))
    req["key"] = zipf_keys(rng, K, n, 1.0, perm_seed=int(rng.integers(1 << 30))).astype(np.uint32)
    u = rng.random(n)
    req["key"][u < 0.01] = abi.KEY_NO_RULE
    req["key"][(u >= 0.01) & (u < 0.015)] = abi.KEY_BAD
    req["key"] |= np.where(rng.random(n) < 0.05, np.uint32(abi.KEY_PRIO), np.uint32(0))
    acq = np.ones(n, np.int32)
    m = rng.random(n) < 0.1
    acq[m] = rng.integers(2, 5, int(m.sum()))
    acq[rng.random(n) < 0.005] = 0
    req["acquire"] = acq
    return req


def _compare_state(node, cts, rules):
    for k in range(len(rules)):
        S = int(rules["sample_count"][k])
        s_g, c_g, o_g = node.read_state(k, S)
        s_o, c_o, o_o = cts.read_state(k)
        assert np.array_equal(s_g, s_o) and np.array_equal(c_g, c_o) and np.array_equal(o_g, o_o), f"flowId key {k}"


@pytest.mark.parametrize("G", [1, 2, 3])
@pytest.mark.parametrize("lim_qps", [0.0, 3000.0])
def test_node_equals_one_token_service(G, lim_qps):
    from sentinel_amd.engine import FlowEngine, NodeEngine
    rng = np.random.default_rng(10 * G + int(lim_qps > 0))
    K = 300
    rules = _rules(rng, K)
    ns = _ns(lim_qps)
    node = NodeEngine([0] * G, max_batch=1 << 17)
    node.set_namespaces(ns)
    node.load_rules(rules)
    single = FlowEngine(device=0, max_batch=1 << 17)
    single.set_namespaces(ns)
    single.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_rules(rules)
    owners = {node.shard_of(k)[0] for k in range(K)}
    assert owners == set(range(G))
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    for b in range(3):
        req = _batch(rng, 40_000, K, t, 1800)
        want = cts.decide(req)
        got = node.decide_host(req)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"batch {b}: {len(bad)} results differ; first at {bad[0]}: req={req[bad[0]]} "
                                 f"oracle={want[bad[0]]} node={got[bad[0]]}")
        assert np.array_equal(single.decide_host(req), want)
        t = int(req["ts_ms"][-1]) + 1
    _compare_state(node, cts, rules)
    now = t + 5
    assert np.array_equal(node.snapshot(now, K), single.snapshot(now, K).reshape(K, 2))


def test_node_rule_reload_keeps_surviving_metrics():
    """ClusterFlowRuleManager reload (ClusterFlowRuleManager.java:361, putMetricIfAbsent): a surviving flowId keeps its
    owner shard and its ClusterMetric; new flowIds start empty; removed ones disappear."""
    from sentinel_amd.engine import NodeEngine
    rng = np.random.default_rng(5)
    K = 200
    rules = _rules(rng, K)
    ns = _ns(0.0)
    node = NodeEngine([0, 0, 0], max_batch=1 << 16)
    node.set_namespaces(ns)
    node.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_rules(rules)
    t = 1_700_000_000_000
    req = _batch(rng, 20_000, K, t, 900)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    keep = rng.permutation(K)[:120]
    fresh = _rules(rng, 60, fid0=900_000)
    rules2 = np.concatenate([rules[keep], fresh])
    rng.shuffle(rules2)
    rules2["count"] = rng.integers(1, 40, len(rules2))
    node.load_rules(rules2)
    cts.load_rules(rules2)
    t = int(req["ts_ms"][-1]) + 1
    for _ in range(2):
        req = _batch(rng, 20_000, len(rules2), t, 900)
        assert np.array_equal(node.decide_host(req), cts.decide(req))
        t = int(req["ts_ms"][-1]) + 1
    _compare_state(node, cts, rules2)


def test_node_rejects_a_batch_as_a_whole():
    """A batch out of time order is refused before any shard sees it (SG_E_TIME): no state changes."""
    from sentinel_amd.engine import EngineError, NodeEngine
    rng = np.random.default_rng(6)
    rules = _rules(rng, 50)
    node = NodeEngine([0, 0], max_batch=1 << 14)
    node.set_namespaces(_ns(500.0))
    node.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(_ns(500.0))
    cts.load_rules(rules)
    req = _batch(rng, 5000, 50, 10_000, 500)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    late = _batch(rng, 100, 50, 9_000, 10)
    with pytest.raises(EngineError) as ei:
        node.decide_host(late)
    assert ei.value.code == abi.SG_E_TIME
    req = _batch(rng, 5000, 50, 10_600, 500)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    _compare_state(node, cts, rules)


@pytest.mark.parametrize("G", [1, 3])
def test_node_sub_request_path(monkeypatch, G):
    """The sub-request path (shards re-validate their slices and the results are gathered back; the path of shards on
    other devices), forced on one device with SG_NODE_LEGACY: the same answers as the records path."""
    monkeypatch.setenv("SG_NODE_LEGACY", "1")
    test_node_equals_one_token_service(G, 3000.0)


@pytest.mark.parametrize("fail_shard", [0, 2])
def test_node_rule_load_is_all_or_nothing(monkeypatch, fail_shard):
    """sg_node_load_flow_rules validates the node's set before it changes anything (a duplicate flowId: SG_E_INVAL) and
    puts the shards already loaded back when a later one fails (an injected allocation failure): either way the node
    keeps deciding with its previous rules, equal to a token service that never saw the failed loads."""
    from sentinel_amd.engine import EngineError, NodeEngine
    rng = np.random.default_rng(7 + fail_shard)
    K = 150
    rules = _rules(rng, K)
    ns = _ns(2000.0)
    node = NodeEngine([0, 0, 0], max_batch=1 << 16)
    node.set_namespaces(ns)
    node.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_rules(rules)
    t = 1_700_000_000_000
    req = _batch(rng, 20_000, K, t, 900)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    dup = rules.copy()
    dup["flow_id"][5] = dup["flow_id"][6]
    with pytest.raises(EngineError) as ei:
        node.load_rules(dup)
    assert ei.value.code == abi.SG_E_INVAL
    other = _rules(rng, K + 40, fid0=2_000_000)
    monkeypatch.setenv("SG_TEST_NODE_FAIL_SHARD", str(fail_shard))
    with pytest.raises(EngineError) as ei:
        node.load_rules(other)
    assert ei.value.code == abi.SG_E_NOMEM
    monkeypatch.delenv("SG_TEST_NODE_FAIL_SHARD")
    t = int(req["ts_ms"][-1]) + 1
    for _ in range(2):
        req = _batch(rng, 20_000, K, t, 900)
        got, want = node.decide_host(req), cts.decide(req)
        assert np.array_equal(got, want), f"{int((got != want).sum())} results differ after the failed loads"
        t = int(req["ts_ms"][-1]) + 1
    _compare_state(node, cts, rules)


@pytest.mark.parametrize("G", [1, 2, 3])
@pytest.mark.parametrize("lim_qps", [0.0, 3000.0])
def test_node_pipelined_batches_equal_one_token_service(G, lim_qps):
    """sg_node_flow_enqueue / _poll / _wait: five node batches in flight back to back (two node workspaces
    alternating, the front's routing of batch i+1 beside the shards' walkers of batch i), one of them out of time
    order and refused by the front as a whole, equal to the sequential token service batch by batch; then a
    synchronous node batch after the pipeline, and the rings."""
    import torch
    from sentinel_amd.engine import NodeEngine
    rng = np.random.default_rng(70 + 10 * G + int(lim_qps > 0))
    K = 300
    rules = _rules(rng, K)
    ns = _ns(lim_qps)
    node = NodeEngine([0] * G, max_batch=1 << 16)
    node.set_namespaces(ns)
    node.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_rules(rules)
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    reqs, wants = [], []
    for b in range(5):
        n = int(rng.integers(20_000, 40_000))
        if b == 2:  # starts behind the previous batch: refused, no state change
            req = _batch(rng, n, K, t - 50, 600)
            wants.append(None)
        else:
            req = _batch(rng, n, K, t, 900)
            wants.append(cts.decide(req))
            t = int(req["ts_ms"][-1]) + 1
        reqs.append(req)
    dev_req = [torch.from_numpy(r.view(np.uint8).copy()).cuda() for r in reqs]
    dev_out = [torch.zeros(len(r) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for r in reqs]
    torch.cuda.synchronize()
    tickets = [node.enqueue_device(q.data_ptr(), len(r), o.data_ptr()) for q, r, o in zip(dev_req, reqs, dev_out)]
    assert all(tk > 0 for tk in tickets) and len(set(tickets)) == 5
    for b, (tk, o) in enumerate(zip(tickets, dev_out)):
        if wants[b] is None:
            with pytest.raises(Exception):
                node.wait(tk)
            continue
        node.wait(tk)
        got = o.cpu().numpy().view(abi.RES_DTYPE)
        if not np.array_equal(got, wants[b]):
            bad = np.nonzero(got != wants[b])[0]
            raise AssertionError(f"batch {b}: {len(bad)} results differ; first at {bad[0]}: "
                                 f"oracle={wants[b][bad[0]]} node={got[bad[0]]}")
    with pytest.raises(Exception):  # collected already
        node.wait(tickets[0])
    req = _batch(rng, 20_000, K, t, 900)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    _compare_state(node, cts, rules)


def test_node_pipelined_poll_and_interleaved_calls():
    """poll answers 0 / 1 without consuming a running ticket twice; a rule reload or a state read between enqueues
    first completes the batches in flight (their tickets stay collectable)."""
    import torch
    from sentinel_amd.engine import NodeEngine
    rng = np.random.default_rng(91)
    K = 120
    rules = _rules(rng, K)
    ns = _ns(0.0)
    node = NodeEngine([0, 0], max_batch=1 << 16)
    node.set_namespaces(ns)
    node.load_rules(rules)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_rules(rules)
    t = 1_700_000_000_000
    outs, tks, wants = [], [], []
    for b in range(3):
        req = _batch(rng, 30_000, K, t, 700)
        wants.append(cts.decide(req))
        t = int(req["ts_ms"][-1]) + 1
        q = torch.from_numpy(req.view(np.uint8).copy()).cuda()
        o = torch.zeros(len(req) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        tks.append(node.enqueue_device(q.data_ptr(), len(req), o.data_ptr()))
        outs.append((q, o))
        if b == 1:
            _compare_state(node, cts, rules)  # drains the node first
    while not node.poll(tks[2]):
        pass
    for b in range(3):
        if b != 2:
            node.wait(tks[b])
        assert np.array_equal(outs[b][1].cpu().numpy().view(abi.RES_DTYPE), wants[b])
    rules2 = rules.copy()
    rules2["count"] = rng.integers(1, 40, K)
    req = _batch(rng, 30_000, K, t, 700)
    q = torch.from_numpy(req.view(np.uint8).copy()).cuda()
    o = torch.zeros(len(req) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    want = cts.decide(req)
    tk = node.enqueue_device(q.data_ptr(), len(req), o.data_ptr())
    node.load_rules(rules2)  # completes the batch in flight under the old rules
    cts.load_rules(rules2)
    node.wait(tk)
    assert np.array_equal(o.cpu().numpy().view(abi.RES_DTYPE), want)
    t = int(req["ts_ms"][-1]) + 1
    req = _batch(rng, 30_000, K, t, 700)
    assert np.array_equal(node.decide_host(req), cts.decide(req))
    _compare_state(node, cts, rules2)
