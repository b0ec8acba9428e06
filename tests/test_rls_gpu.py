"""The Envoy RLS front-end on the device (sentinel_amd/rls.py over sg_flow_decide_batch) against the oracle's
SimpleClusterFlowChecker restatement: identical RateLimitResponses and identical ClusterMetric windows."""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.rls import RateLimitRequest, rls_rules, should_rate_limit, should_rate_limit_abi

pytestmark = pytest.mark.gpu

T = 1_700_000_000_000


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
        got = should_rate_limit_abi(eng, reqs) if via_abi else should_rate_limit(reqs, rules["count"], eng.decide_host)
        want = should_rate_limit(reqs, rules["count"], ora.decide_rls)
        assert got == want, f"batch {batch}: responses differ"
    for k in range(K):
        s_o, c_o, o_o = ora.read_state(k)
        s_g, c_g, o_g = eng.read_state(k, len(s_o))
        assert np.array_equal(s_o, s_g) and np.array_equal(c_o, c_g), f"window of rule {k} differs"
