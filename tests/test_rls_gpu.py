"""The Envoy RLS front-end on the device against the oracle: the C ABI's sg_rls_should_rate_limit against the oracle's
own restatement of SentinelEnvoyRlsServiceImpl.shouldRateLimit (or_rls_should_rate_limit: overall codes and every
descriptor status, field by field), and the Python shim (sentinel_amd/rls.py over sg_flow_decide_batch) against the
same shim over the oracle's SimpleClusterFlowChecker; identical ClusterMetric windows either way."""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.rls import RateLimitRequest, rls_rules, should_rate_limit

pytestmark = pytest.mark.gpu

T = 1_700_000_000_000


def _req(reqs):
    req = np.zeros(len(reqs), abi.RLS_REQ_DTYPE)
    desc, b = [], 0
    for j, q in enumerate(reqs):
        req[j] = (q.ts_ms, q.hits_addend, b, len(q.descriptors), 0)
        desc += q.descriptors
        b += len(q.descriptors)
    return req, np.array(desc, np.int32)


@pytest.mark.parametrize("seed,exceed,via_abi", [(1, 1.0, False), (2, 1.5, False), (3, 1.0, True), (4, 1.5, True)])
def test_rls_device_matches_oracle(seed, exceed, via_abi):
    """via_abi: the library's sg_rls_should_rate_limit instead of the Python shim over sg_flow_decide_batch."""
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(seed)
    K = 300
    rules = np.zeros(K, abi.RULE_DTYPE)
    rules["flow_id"] = np.arange(1, K + 1) * 13
    rules["count"] = rng.integers(0, 40, K)
    rules["threshold_type"] = rng.integers(0, 2, K)  # ignored by the RLS checker
    rules["sample_count"] = rng.choice([1, 2, 5, 10], K)
    rules["window_interval_ms"] = 1000
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 4
    r = rls_rules(rules)
    eng = FlowEngine(device=0, max_batch=1 << 18, exceed_count=exceed)
    eng.set_namespaces(ns)
    eng.load_rules(r)
    ora = ClusterTokenService(exceed, 1.0)
    ora.set_namespaces(ns)
    ora.load_rules(r)
    p = 1.0 / np.arange(1, K + 1)
    p /= p.sum()
    t = T
    for batch in range(4):
        reqs = []
        for _ in range(20_000):
            t += int(rng.integers(0, 2))
            nd = int(rng.integers(1, 4))
            d = [int(x) if rng.random() < 0.95 else -1 for x in rng.choice(K, nd, p=p)]
            hits = int(rng.choice([0, 1, 1, 1, 2, 5, -1], p=[0.1, 0.5, 0.2, 0.1, 0.05, 0.04, 0.01]))
            reqs.append(RateLimitRequest(t, hits, d))
        if via_abi:
            req, desc = _req(reqs)
            g_all, g_st = eng.rls_should_rate_limit(req, desc)
            w_all, w_st = ora.should_rate_limit(req, desc)
            assert np.array_equal(g_all, w_all), f"batch {batch}: overall codes differ"
            assert np.array_equal(g_st, w_st), f"batch {batch}: descriptor statuses differ"
        else:
            got = should_rate_limit(reqs, rules["count"], eng.decide_host)
            want = should_rate_limit(reqs, rules["count"], ora.decide_rls)
            assert got == want, f"batch {batch}: responses differ"
    for k in range(K):
        s_o, c_o, o_o = ora.read_state(k)
        s_g, c_g, o_g = eng.read_state(k, len(s_o))
        assert np.array_equal(s_o, s_g) and np.array_equal(c_o, c_g), f"window of rule {k} differs"


def test_rls_contract():
    """Rules the cluster path would read differently (AVG_LOCAL, a limited namespace) and batches larger than
    max_batch are refused before any state change."""
    from sentinel_amd.engine import EngineError, FlowEngine
    rules = np.zeros(3, abi.RULE_DTYPE)
    rules["flow_id"], rules["count"], rules["sample_count"], rules["window_interval_ms"] = [1, 2, 3], 5, 2, 1000
    rules["threshold_type"] = [abi.THRESHOLD_GLOBAL, abi.THRESHOLD_AVG_LOCAL, abi.THRESHOLD_GLOBAL]
    rules["namespace_id"] = [0, 0, 1]
    ns = np.zeros(2, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["limiter_enabled"][1], ns["max_allowed_qps"][1] = 1, 100.0
    eng = FlowEngine(device=0, max_batch=8)
    eng.set_namespaces(ns)
    eng.load_rules(rules)
    for bad in (1, 2):
        with pytest.raises(EngineError) as ei:
            eng.rls_should_rate_limit(*_req([RateLimitRequest(T, 1, [0, bad])]))
        assert ei.value.code == abi.SG_E_UNSUPPORTED
    with pytest.raises(EngineError) as ei:
        eng.rls_should_rate_limit(*_req([RateLimitRequest(T, 1, [0] * 5), RateLimitRequest(T, 1, [0] * 5)]))
    assert ei.value.code == abi.SG_E_CAPACITY
    overall, st = eng.rls_should_rate_limit(*_req([RateLimitRequest(T, 1, [0, -1])]))
    assert list(overall) == [abi.RLS_OK] and st["limit_remaining"][0] == 4   # nothing was charged before
