"""Parity of cluster-mode flow rules on an embedded token server (sg_local_set_cluster_state(SERVER)) with the oracle.

FlowRuleChecker.passClusterCheck (FlowRuleChecker.java:147-209) on a node whose ClusterStateManager is a server:
pickClusterService → the embedded server (DefaultEmbeddedTokenServer.requestToken → DefaultTokenService.requestToken,
DefaultEmbeddedTokenServer.java:46-51) decides the token against the handle's own cluster flow state, and
applyTokenResult maps it (OK / SHOULD_WAIT pass, BLOCKED blocks, the rest fall back to the local check or pass).

Traces: seeded entries (LocalTraceGen: exits of the passed entries after their sleep + response time) on resources
whose rule sets mix cluster-mode rules (FALLBACK / NO_FALLBACK, flowIds shared between resources, flowIds the server
has no rule for) with local rules, namespaces with and without a GlobalRequestLimiter, interleaved in time with
token-server flow batches on the same flowIds (remote clients). Compared bit-exactly: every result, every flowId's
ClusterMetric ring and occupy counters, every resource's windows and thread count.

The composition of the slot chain with the token server is pinned by the hand-traced KATs of
tests/test_oracle_flow_rules_kat.py (test_embedded_server_*): no reference test drives it (parity unpinned beyond
the restated pieces: ClusterMetricTest, GlobalRequestLimiterTest, FlowRuleCheckerTest).
"""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService, LocalChain, LocalTraceGen, local_flow_rule, local_rule
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

FB, NOFB = abi.CLUSTER_MODE_FALLBACK, abi.CLUSTER_MODE_NO_FALLBACK


def _c3_rules(rng, n_flow, S):
    r = np.zeros(n_flow, abi.RULE_DTYPE)
    r["flow_id"] = 1000 + np.arange(n_flow)
    r["count"] = rng.integers(2, 30, n_flow)
    r["threshold_type"] = abi.THRESHOLD_GLOBAL
    r["sample_count"] = S
    r["window_interval_ms"] = 1000
    r["namespace_id"] = np.arange(n_flow) % 2
    return r


def _rule_set(rng, r, n_flow):
    key = lambda: int(rng.integers(0, n_flow)) if rng.random() < 0.85 else abi.KEY_NO_RULE  # noqa: E731
    c = lambda lo, hi: float(rng.integers(lo, hi + 1))  # noqa: E731
    u = int(rng.integers(0, 7))
    if u == 0:
        return [local_flow_rule(r, c(5, 40))]                                                   # fast path
    if u == 1:
        return [local_flow_rule(r, c(2, 30), cluster_mode=FB, cluster_config=r + 1, cluster_key=key())]
    if u == 2:
        return [local_flow_rule(r, c(2, 30), cluster_mode=NOFB, cluster_config=r + 1, cluster_key=key())]
    if u == 3:
        return [local_flow_rule(r, c(20, 60)),
                local_flow_rule(r, c(2, 30), cluster_mode=FB, cluster_config=r + 1, cluster_key=key())]
    if u == 4:
        return [local_flow_rule(r, c(1, 4), grade=abi.FLOW_GRADE_THREAD),
                local_flow_rule(r, c(2, 30), cluster_mode=NOFB, cluster_config=r + 1, cluster_key=key())]
    if u == 5:
        return [local_flow_rule(r, c(10, 50), behavior=abi.CONTROL_RATE_LIMITER, max_queueing_ms=200),
                local_flow_rule(r, c(2, 30), cluster_mode=FB, cluster_config=r + 1, cluster_key=key())]
    return []


def _setup(rng, n_res, n_flow, S, lim_qps):
    from sentinel_amd.engine import FlowEngine
    ns = np.zeros(2, abi.NS_DTYPE)
    ns["connected_count"] = [3, 1]
    if lim_qps:
        ns["limiter_enabled"][0], ns["max_allowed_qps"][0] = 1, lim_qps
    c3 = _c3_rules(rng, n_flow, S)
    base = np.array([local_rule() for _ in range(n_res)])
    flat = [x for r in range(n_res) for x in _rule_set(rng, r, n_flow)]
    rng.shuffle(flat)
    fr = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE)
    cts = ClusterTokenService(1.0, 1.0)
    cts.set_namespaces(ns)
    cts.load_rules(c3)
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(base)
    kept = ora.load_flow_rules(fr)
    ora.attach_cluster(cts, abi.CLUSTER_SERVER)
    eng = FlowEngine(device=0, max_batch=1 << 18)
    eng.set_namespaces(ns)
    eng.load_rules(c3)
    eng.local_load_rules(base, 2, 1000, 500)
    assert eng.local_load_flow_rules(fr) == kept
    eng.local_set_cluster_state(abi.CLUSTER_SERVER)
    return cts, ora, eng, fr


def _entries(rng, n, n_res, t, span):
    e = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    e["ts_ms"] = t + np.sort(rng.integers(0, span, n))
    e["resource"] = zipf_keys(rng, n_res, n, 0.8, perm_seed=int(rng.integers(1 << 30)))
    e["resource"] |= np.where(rng.random(n) < 0.1, np.uint32(abi.KEY_PRIO), np.uint32(0))
    cnt = np.ones(n, np.int32)
    m = rng.random(n) < 0.1
    cnt[m] = rng.integers(2, 4, int(m.sum()))
    cnt[rng.random(n) < 0.01] = 0                                   # acquireCount 0: BAD_REQUEST → fallback
    e["count"] = cnt
    return e


def _flow_batch(rng, n, n_flow, t_lo, t_hi):
    req = np.zeros(n, abi.REQ_DTYPE)
    req["ts_ms"] = np.sort(rng.integers(t_lo, t_hi + 1, n))
    req["key"] = rng.integers(0, n_flow, n).astype(np.uint32)
    req["key"] |= np.where(rng.random(n) < 0.05, np.uint32(abi.KEY_PRIO), np.uint32(0))
    req["acquire"] = 1
    return req


def _compare(eng, ora, cts, n_res, n_flow):
    stride = eng.state_stride()
    r_g, o_g = eng.export_state(n_flow)
    r_o, o_o = cts.export_state(n_flow, stride)
    assert np.array_equal(r_g, r_o), f"cluster rings differ at flowIds {np.nonzero((r_g != r_o).any((1, 2)))[0]}"
    assert np.array_equal(o_g, o_o), "occupy counters"
    for r in range(n_res):
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g) and np.array_equal(b_o, b_g) and np.array_equal(m_o, m_g), f"windows of {r}"
        assert head[0] == ora.threads(r), f"threads of {r}"


@pytest.mark.parametrize("S,lim_qps", [(2, 0.0), (10, 0.0), (2, 400.0), (10, 150.0)])
@pytest.mark.parametrize("seed", [1, 2])
def test_embedded_server_parity(S, lim_qps, seed):
    rng = np.random.default_rng(seed * 100 + S)
    n_res, n_flow = 40, 10
    cts, ora, eng, fr = _setup(rng, n_res, n_flow, S, lim_qps)
    gen = LocalTraceGen(ora)
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    for b in range(4):
        span = 1500
        ent = _entries(rng, 6000, n_res, t, span)
        rt = rng.integers(0, 60, len(ent)).astype(np.int32)
        err = (rng.random(len(ent)) < 0.05).astype(np.uint8)
        ev, want = gen.run(ent, rt, err, t + span)
        got = eng.local_decide_host(ev)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"batch {b}: {len(bad)} results differ; first at {bad[0]}: ev={ev[bad[0]]} "
                                 f"oracle={want[bad[0]]} gpu={got[bad[0]]}")
        # remote clients' token requests on the same flowIds, between the local events so far and the next batch
        req = _flow_batch(rng, 3000, n_flow, int(ev["ts_ms"][-1]) if len(ev) else t, t + span)
        assert np.array_equal(eng.decide_host(req), cts.decide(req)), f"flow batch {b}"
        t += span
    _compare(eng, ora, cts, n_res, n_flow)


def test_embedded_server_time_order_and_contract():
    """A local batch may not precede the cluster flow batches in time (SG_E_TIME), nor they it; CLIENT state with
    cluster-mode rules stays unsupported."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(9)
    cts, ora, eng, fr = _setup(rng, 6, 4, 2, 0.0)
    req = _flow_batch(rng, 10, 4, 5000, 5000)
    eng.decide_host(req)
    ev = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"] = 4999, 1
    with pytest.raises(EngineError) as ei:
        eng.local_decide_host(ev)
    assert ei.value.code == abi.SG_E_TIME
    ev["ts_ms"] = 6000
    eng.local_decide_host(ev)
    with pytest.raises(EngineError) as ei:
        eng.decide_host(_flow_batch(rng, 4, 4, 5500, 5500))
    assert ei.value.code == abi.SG_E_TIME
    with pytest.raises(EngineError) as ei:
        eng.local_set_cluster_state(abi.CLUSTER_CLIENT)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
