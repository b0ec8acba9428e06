"""Parity of cluster-mode ParamFlowRules (ParamFlowRule.clusterMode + ParamFlowClusterConfig) in the ParamFlowSlot batch
(sg_pslot_decide_batch) and in the whole slot chain (sg_slot_decide_batch) with the oracle.

ParamFlowChecker.passCheck sends a clusterMode QPS rule to passClusterCheck (ParamFlowChecker.java:71-73, :278-303):
with no token service (ClusterStateManager NOT_STARTED) fallbackToLocalOrPass (:305-313) checks the rule locally or
passes it; on an embedded token server (SERVER) the rule requests a param token for all of the argument's values from
the handle's cluster param state (sg_cparam_load_rules → DefaultTokenService.requestParamToken → ClusterParamFlowChecker,
the namespace limiter included), OK passing, BLOCKED throwing, anything else falling back. The rule sets mix local
rules, cluster rules with and without fallback, invalid cluster configs (dropped at load), THREAD-grade cluster rules
(always local), flowIds the server has no rule for, and resources sharing a flowId or a limited namespace (walked as one
key group). Between the ParamFlowSlot batches remote clients request param tokens on the same flowIds
(sg_cparam_decide_batch). Compared exactly: every result, the thread counts, the token states and the cluster param
window sums. The composition is parity-unpinned beyond the hand-traced KATs of tests/test_oracle_pslot_kat.py.
"""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService, ParamFlowSlot
from sentinel_amd import abi
from tests.test_pslot_gpu import Gen, _rules

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
N_CP = 5          # cluster param rules on the server
FLOW_ID0 = 500


def _server(rng, lim_qps):
    ns = np.zeros(2, abi.NS_DTYPE)
    ns["connected_count"] = [2, 1]
    if lim_qps:
        ns["limiter_enabled"][0], ns["max_allowed_qps"][0] = 1, lim_qps
    cp = np.zeros(N_CP, abi.CPARAM_RULE_DTYPE)
    for k in range(N_CP):
        cp[k]["flow_id"] = FLOW_ID0 + k
        cp[k]["count"] = float(rng.integers(3, 25))
        cp[k]["threshold_type"] = abi.THRESHOLD_GLOBAL if rng.random() < 0.7 else abi.THRESHOLD_AVG_LOCAL
        S = int(rng.choice([1, 2, 10]))
        cp[k]["sample_count"], cp[k]["window_interval_ms"] = S, 1000
        cp[k]["namespace_id"] = 0 if k % 2 == 0 else 1
    hot = np.array([(3, 1, 0), (7, 40, 0)], abi.PARAM_HOT_DTYPE)
    cp[1]["hot_begin"], cp[1]["hot_count"] = 0, 2
    return ns, cp, hot


def _cluster_rules(rng, n_res):
    """The local rule sets of tests/test_pslot_gpu.py with cluster-mode rules mixed in."""
    rules, hot = _rules(rng, n_res)
    extra = []
    for res in range(n_res):
        for _ in range(int(rng.integers(0, 3))):
            r = np.zeros((), abi.PSLOT_RULE_DTYPE)
            r["resource"] = res
            r["grade"] = 1 if rng.random() < 0.85 else 0
            r["param_idx"] = int(rng.integers(0, 3))
            r["rule"]["count"] = float(rng.integers(0, 12))
            r["rule"]["duration_sec"] = int(rng.integers(1, 3))
            r["rule"]["behavior"] = 2 if rng.random() < 0.2 else 0
            r["rule"]["max_queueing_ms"] = int(rng.integers(0, 200))
            r["rule"]["capacity_log2"] = 12
            u = rng.random()
            r["cluster_mode"] = (abi.CLUSTER_MODE_FALLBACK if u < 0.5 else abi.CLUSTER_MODE_NO_FALLBACK if u < 0.9
                                 else abi.CLUSTER_MODE_INVALID)
            r["cluster_key"] = int(rng.integers(0, N_CP)) if rng.random() < 0.9 else abi.KEY_NO_RULE
            extra.append(r)
    allr = np.concatenate([rules, np.array(extra, abi.PSLOT_RULE_DTYPE)]) if extra else rules
    perm = rng.permutation(len(allr))                      # cluster and local rules interleaved in load order
    return allr[perm], hot


def _cparam_batch(rng, n, t_lo, t_hi):
    req = np.zeros(n, abi.CPARAM_REQ_DTYPE)
    req["ts_ms"] = np.sort(rng.integers(t_lo, t_hi + 1, n))
    req["key"] = rng.integers(0, N_CP, n).astype(np.uint32)
    req["acquire"] = rng.integers(1, 3, n)
    vals = []
    for i in range(n):
        m = 1 if rng.random() < 0.8 else 2
        req[i]["value_begin"], req[i]["value_count"] = len(vals), m
        vals += [int(x) for x in rng.integers(1, 40, m)]
    return req, np.array(vals, np.uint64)


def _run(seed, state, lim_qps, batches=5):
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(seed)
    n_res = 14
    rules, hot = _cluster_rules(rng, n_res)
    ns, cp, cp_hot = _server(rng, lim_qps)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_param_rules(cp, cp_hot)
    ora = ParamFlowSlot(rules, hot, n_resources=n_res)
    ora.attach_cluster(cts if state == abi.CLUSTER_SERVER else None, state)
    eng = FlowEngine(device=0, max_batch=1 << 17)
    eng.set_namespaces(ns)
    eng.cparam_load_rules(cp, cp_hot)
    eng.local_set_cluster_state(state)
    eng.pslot_load_rules(rules, hot, n_resources=n_res)
    gen = Gen(seed, n_res)
    for b in range(batches):
        ev, args, vals, entries = gen.batch(5000, 1500)
        want = ora.decide(ev, args, vals)
        got = eng.pslot_decide_host(ev, args, vals)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"batch {b}: {len(bad)} differ; first {bad[0]}: ev={ev[bad[0]]} {entries[bad[0]]} "
                                 f"oracle={want[bad[0]]} gpu={got[bad[0]]}")
        gen.absorb(ev, want, entries)
        # remote clients' param tokens on the same flowIds, after this batch's events
        req, rv = _cparam_batch(rng, 800, int(ev["ts_ms"][-1]), gen.t)
        assert np.array_equal(eng.cparam_decide_host(req, rv), cts.decide_param(req, rv)), f"cparam batch {b}"
    for ri in range(len(rules)):
        assert eng.pslot_param_idx(ri) == ora.param_idx(ri), f"paramIdx of rule {ri}"
    for res in range(n_res):
        for idx in range(3):
            for v in range(1, 40):
                assert eng.pslot_thread_count(res, idx, v) == ora.thread_count(res, idx, v), (res, idx, v)
    for ri in range(len(rules)):
        for v in range(1, 40):
            f, lt, tk = ora.token_state(ri, v)
            if f:
                gf, glt, gtk = eng.param_state(ri, v)
                assert (gf, glt if f & 1 else 0, gtk if f & 2 else 0) == (f, lt if f & 1 else 0, tk if f & 2 else 0)
    now = gen.t
    for k in range(N_CP):
        for v in range(1, 40):
            assert eng.cparam_sum(k, v, now) == cts.param_sum(k, v, now), f"cluster param sum of rule {k} value {v}"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_cluster_param_rules_not_started(seed):
    _run(seed, abi.CLUSTER_NOT_STARTED, 0.0)


@pytest.mark.parametrize("lim_qps", [0.0, 300.0])
@pytest.mark.parametrize("seed", [4, 5, 6])
def test_cluster_param_rules_embedded_server(seed, lim_qps):
    _run(seed, abi.CLUSTER_SERVER, lim_qps)


def test_cluster_param_rules_contract():
    """CLIENT with cluster-mode param rules is unsupported (either order); on an embedded server a ParamFlowSlot batch
    may not precede the cluster param batches in time (SG_E_TIME), nor they it."""
    from sentinel_amd.engine import EngineError, FlowEngine
    rng = np.random.default_rng(8)
    ns, cp, cp_hot = _server(rng, 0.0)
    r = np.zeros(1, abi.PSLOT_RULE_DTYPE)
    r["grade"], r["rule"]["count"], r["rule"]["duration_sec"], r["rule"]["capacity_log2"] = 1, 5.0, 1, 10
    r["cluster_mode"], r["cluster_key"] = abi.CLUSTER_MODE_FALLBACK, 0
    eng = FlowEngine(device=0, max_batch=1 << 12)
    eng.set_namespaces(ns)
    eng.cparam_load_rules(cp, cp_hot)
    eng.local_set_cluster_state(abi.CLUSTER_CLIENT)
    with pytest.raises(EngineError) as ei:
        eng.pslot_load_rules(r, n_resources=1)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    eng.local_set_cluster_state(abi.CLUSTER_SERVER)
    eng.pslot_load_rules(r, n_resources=1)
    with pytest.raises(EngineError) as ei:
        eng.local_set_cluster_state(abi.CLUSTER_CLIENT)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    req, rv = _cparam_batch(rng, 4, T0 + 5000, T0 + 5000)
    eng.cparam_decide_host(req, rv)
    ev = np.zeros(1, abi.PSLOT_EVENT_DTYPE)
    ev["ts_ms"], ev["count"], ev["arg_count"] = T0 + 4999, 1, 1
    args = np.array([(0, 1, abi.ARG_VALUE, 0)], abi.PSLOT_ARG_DTYPE)
    with pytest.raises(EngineError) as ei:
        eng.pslot_decide_host(ev, args, np.array([99], np.uint64))
    assert ei.value.code == abi.SG_E_TIME
    ev["ts_ms"] = T0 + 6000
    assert eng.pslot_decide_host(ev, args, np.array([99], np.uint64))["pass"][0] == 1
    with pytest.raises(EngineError) as ei:
        eng.cparam_decide_host(*_cparam_batch(rng, 2, T0 + 5500, T0 + 5500))
    assert ei.value.code == abi.SG_E_TIME


@pytest.mark.parametrize("lim_qps", [0.0, 300.0])
@pytest.mark.parametrize("seed", [1, 2])
def test_cluster_param_rules_in_the_slot_chain(seed, lim_qps):
    """The same rules inside the whole slot chain (ParamFlowSlot before FlowSlot inside StatisticSlot) on an embedded
    server: the resources sharing a flowId or a limited namespace walk as one key group of the chain."""
    from tests.test_oracle_pslot_kat import rule as prule
    from tests.test_slot_chain_gpu import _run as chain_run, _setup as chain_setup
    rng = np.random.default_rng(seed + 40)
    n_res, n_origins, n_ctx = 24, 2, 2
    params = []
    for res in range(n_res):
        u = rng.random()
        if u < 0.3:
            params.append(prule(res=res, idx=0, count=float(rng.integers(2, 12))))
        if u > 0.2:
            r = prule(res=res, idx=int(rng.integers(0, 2)), count=float(rng.integers(0, 8)),
                      behavior=abi.BEHAVIOR_RATE_LIMITER if rng.random() < 0.2 else 0)
            r["cluster_mode"] = abi.CLUSTER_MODE_FALLBACK if rng.random() < 0.6 else abi.CLUSTER_MODE_NO_FALLBACK
            r["cluster_key"] = int(rng.integers(0, N_CP)) if rng.random() < 0.9 else abi.KEY_NO_RULE
            params.append(r)
    params = np.array(params, abi.PSLOT_RULE_DTYPE)
    ora, ps, eng, fr, params = chain_setup(rng, n_res, n_origins, n_ctx, params=params)
    ns, cp, cp_hot = _server(rng, lim_qps)
    cts = ClusterTokenService()
    cts.set_namespaces(ns)
    cts.load_param_rules(cp, cp_hot)
    ora.attach_cluster(cts, abi.CLUSTER_SERVER)     # the node's state: the chain's param rules follow it
    eng.set_namespaces(ns)
    eng.cparam_load_rules(cp, cp_hot)
    eng.local_set_cluster_state(abi.CLUSTER_SERVER)
    t, pool, _ = chain_run(ora, ps, eng, fr, params, n_res, n_origins, n_ctx, [(12_000, 3000), (12_000, 3000)],
                           seed, zipf=0.9)
    for k in range(N_CP):
        for v in range(1, 30):
            assert eng.cparam_sum(k, v, t) == cts.param_sum(k, v, t), f"cluster param sum of rule {k} value {v}"
