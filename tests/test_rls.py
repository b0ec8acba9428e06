"""Envoy RLS front-end (sentinel_amd/rls.py) over the oracle's SimpleClusterFlowChecker restatement: the
reference's SentinelEnvoyRlsServiceImplTest cases (all OK → overall OK; one BLOCKED → overall OVER_LIMIT
with mixed statuses), hitsAddend handling, and the checker's own window arithmetic."""
import numpy as np

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.rls import CODE_OK, CODE_OVER_LIMIT, RateLimitRequest, rls_rules, should_rate_limit

T = 1_700_000_000_000


def _service(counts, exceed=1.0):
    rules = np.zeros(len(counts), abi.RULE_DTYPE)
    rules["flow_id"] = np.arange(1, len(counts) + 1) * 11
    rules["count"] = counts
    rules["threshold_type"] = abi.THRESHOLD_AVG_LOCAL  # ignored by SimpleClusterFlowChecker
    rules["sample_count"] = 10
    rules["window_interval_ms"] = 1000
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 3
    s = ClusterTokenService(exceed, 1.0)
    s.set_namespaces(ns)
    s.load_rules(rls_rules(rules))
    return s, rules


def test_should_rate_limit_pass():  # SentinelEnvoyRlsServiceImplTest.testShouldRateLimitPass
    s, rules = _service([10.0, 10.0])
    (r,) = should_rate_limit([RateLimitRequest(T, 1, [0, 1])], rules["count"], s.decide_rls)
    assert r.overall_code == CODE_OK and [x.code for x in r.statuses] == [CODE_OK, CODE_OK]
    assert [x.limit_remaining for x in r.statuses] == [9, 9] and r.statuses[0].requests_per_unit == 10


def test_should_rate_partial_block():  # SentinelEnvoyRlsServiceImplTest.testShouldRatePartialBlock
    s, rules = _service([0.0, 10.0])
    (r,) = should_rate_limit([RateLimitRequest(T, 1, [0, 1])], rules["count"], s.decide_rls)
    assert r.overall_code == CODE_OVER_LIMIT and len(r.statuses) == 2
    assert [x.code for x in r.statuses] == [CODE_OVER_LIMIT, CODE_OK]


def test_no_rule_passes_and_hits_addend():
    s, rules = _service([2.0])
    out = should_rate_limit([RateLimitRequest(T, 0, [-1, 0]),     # 0 hits → 1; no rule → OK, no limit fields
                             RateLimitRequest(T, 1, [0]),
                             RateLimitRequest(T, 1, [0]),         # threshold 2 reached
                             RateLimitRequest(T, -1, [0])],       # onError
                            rules["count"], s.decide_rls)
    assert out[0].overall_code == CODE_OK and out[0].statuses[0].limit_remaining is None
    assert out[0].statuses[1].limit_remaining == 1
    assert out[1].statuses[0].limit_remaining == 0 and out[1].overall_code == CODE_OK
    assert out[2].overall_code == CODE_OVER_LIMIT
    assert out[3].error and not out[3].statuses


def test_window_slides():
    s, rules = _service([3.0], exceed=2.0)  # threshold count * exceedCount = 6 per 1000 ms window
    req = np.zeros(8, abi.REQ_DTYPE)
    req["ts_ms"] = [T, T, T, T + 500, T + 999, T + 1000, T + 1050, T + 1100]
    req["key"] = 0
    req["acquire"] = [2, 2, 2, 1, 1, 3, 1, 1]
    st = s.decide_rls(req)["status"]
    assert list(st) == [abi.OK, abi.OK, abi.OK, abi.BLOCKED, abi.BLOCKED, abi.OK, abi.OK, abi.OK]


def _req(rows):
    """sg_rls_request records + descriptor array from [(ts, hits, [rule, ...]), ...]."""
    req = np.zeros(len(rows), abi.RLS_REQ_DTYPE)
    desc, b = [], 0
    for j, (ts, hits, d) in enumerate(rows):
        req[j] = (ts, hits, b, len(d), 0)
        desc += d
        b += len(d)
    return req, np.array(desc, np.int32)


def test_oracle_should_rate_limit_restates_the_reference_tests():
    """The oracle's own shouldRateLimit (or_rls_should_rate_limit): SentinelEnvoyRlsServiceImplTest's pass and partial
    block cases, hits_addend 0 / < 0 and a descriptor without a rule, checked field by field."""
    s, _ = _service([10.0, 10.0])
    overall, st = s.should_rate_limit(*_req([(T, 1, [0, 1])]))                      # testShouldRateLimitPass
    assert list(overall) == [abi.RLS_OK] and list(st["code"]) == [abi.RLS_OK] * 2
    assert list(st["limit_remaining"]) == [9, 9] and list(st["requests_per_unit"]) == [10, 10]
    s, _ = _service([0.0, 10.0])
    overall, st = s.should_rate_limit(*_req([(T, 1, [0, 1])]))                      # testShouldRatePartialBlock
    assert list(overall) == [abi.RLS_OVER_LIMIT] and list(st["code"]) == [abi.RLS_OVER_LIMIT, abi.RLS_OK]
    s, _ = _service([2.0])
    overall, st = s.should_rate_limit(*_req([(T, 0, [-1, 0]), (T, 1, [0]), (T, 1, [0]), (T, -1, [0]), (T, 1, [7])]))
    assert list(overall) == [abi.RLS_OK, abi.RLS_OK, abi.RLS_OVER_LIMIT, abi.RLS_ERROR, abi.RLS_OK]
    assert list(st["has_rule"]) == [0, 1, 1, 1, 0, 0]                              # rule 7 does not exist
    assert list(st["limit_remaining"][:3]) == [0, 1, 0] and st["code"][4] == 0      # the failed call: nothing


def test_shim_equals_oracle_mapping():
    """sentinel_amd.rls.should_rate_limit (the shim over any decide()) gives the oracle's mapping on a random trace."""
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 12, 20).astype(np.float64)
    s1, rules = _service(counts, exceed=1.5)
    s2, _ = _service(counts, exceed=1.5)
    rows, t = [], T
    for _ in range(3000):
        t += int(rng.integers(0, 3))
        rows.append((t, int(rng.choice([0, 1, 1, 2, -1])), [int(x) if rng.random() < 0.9 else -1
                                                           for x in rng.integers(0, 20, int(rng.integers(1, 4)))]))
    overall, st = s1.should_rate_limit(*_req(rows))
    shim = should_rate_limit([RateLimitRequest(ts, h, d) for ts, h, d in rows], rules["count"], s2.decide_rls)
    b = 0
    for j, (ts, h, d) in enumerate(rows):
        if h < 0:
            assert overall[j] == abi.RLS_ERROR and shim[j].error
        else:
            assert overall[j] == shim[j].overall_code
            for i, x in enumerate(shim[j].statuses):
                o = st[b + i]
                assert o["code"] == x.code
                if x.limit_remaining is not None:
                    assert o["has_rule"] == 1 and o["limit_remaining"] == x.limit_remaining
                    assert o["requests_per_unit"] == x.requests_per_unit
                else:
                    assert o["has_rule"] == 0
        b += len(d)
