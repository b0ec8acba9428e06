"""The sharded oracle replay used by the full-size parity tests equals one global sequential replay (flowIds
share no state without a namespace limiter), including its state export."""
import numpy as np

from oracle.binding import ClusterTokenService, ShardedClusterTokenService
from sentinel_amd import abi
from sentinel_amd.workload import ClusterWorkload


def test_sharded_replay_equals_sequential_replay():
    wl = ClusterWorkload(n_flows=3000, n_requests=120_000, seed=17, prio_frac=0.2)
    rules = wl.rules()
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    one = ClusterTokenService()
    one.set_namespaces(ns)
    one.load_rules(rules)
    many = ShardedClusterTokenService(rules, ns, 5)
    for b in range(2):
        req = wl.requests(b)
        req["key"][::997] = abi.KEY_NO_RULE
        req["acquire"][::1009] = 0
        assert np.array_equal(one.decide(req), many.decide(req))
    r1, o1 = one.export_state(len(rules), 10)
    r2, o2 = many.export_state(10)
    assert np.array_equal(r1, r2) and np.array_equal(o1, o2)
    s, c, o = one.read_state(123)
    assert np.array_equal(r1[123, :, 0], s) and np.array_equal(o1[123], o)
    live = s != abi.INT64_MIN
    assert np.array_equal(r1[123, live, 1:], c[live])
    many.close()
