"""Known-answer tests of the hot-parameter checker restatement (oracle), restating
pfT/slots/block/flow/param/ParamFlowDefaultCheckerTest.java and ParamFlowThrottleRateLimitingCheckerTest.java
(paths under sentinel-extension/sentinel-parameter-flow-control/src/test/java/com/alibaba/csp/sentinel/)."""
import numpy as np

from oracle.binding import ParamFlowChecker
from sentinel_amd import abi

VALUE_A = 0x76616C756541  # "valueA"


def _checker(count, burst=0, duration=1, behavior=abi.BEHAVIOR_DEFAULT, max_queue=0, hot=()):
    pf = ParamFlowChecker()
    r = np.zeros(1, abi.PARAM_RULE_DTYPE)
    r[0]["count"] = count
    r[0]["burst"] = burst
    r[0]["duration_sec"] = duration
    r[0]["behavior"] = behavior
    r[0]["max_queueing_ms"] = max_queue
    h = np.zeros(len(hot), abi.PARAM_HOT_DTYPE)
    for i, (v, thr) in enumerate(hot):
        h[i] = (v, thr, 0)
    r[0]["hot_begin"] = 0
    r[0]["hot_count"] = len(hot)
    pf.load_rules(r, h)
    return pf


def _run(pf, t, n, value=VALUE_A):
    return [pf.check(t, 0, value) for _ in range(n)]


def test_check_qps_with_long_interval_and_high_threshold(t0):
    """ParamFlowDefaultCheckerTest.java:45-80: 24 h / 48 h gaps make toAddCount exceed Integer.MAX_VALUE."""
    pf = _checker(25000)
    assert _run(pf, t0, 2) == [True, True]
    t = t0 + 1000 * 60 * 60 * 24
    assert _run(pf, t, 2) == [True, True]
    t += 1000 * 60 * 60 * 48
    assert _run(pf, t, 2) == [True, True]


def test_default_check_single_qps(t0):
    """ParamFlowDefaultCheckerTest.java:82-113: count 5 → 5×T, F; after 3 s again 5×T, F."""
    pf = _checker(5)
    assert _run(pf, t0, 6) == [True] * 5 + [False]
    assert _run(pf, t0 + 3000, 6) == [True] * 5 + [False]


def test_default_check_single_qps_with_burst(t0):
    """ParamFlowDefaultCheckerTest.java:115-176: burst 3 → 8×T, F; refills after 1002 ms / 2000 ms."""
    pf = _checker(5, burst=3)
    t = t0
    assert _run(pf, t, 9) == [True] * 8 + [False]
    t += 1002
    assert _run(pf, t, 6) == [True] * 5 + [False]
    t += 1002
    assert _run(pf, t, 6) == [True] * 5 + [False]
    t += 2000
    assert _run(pf, t, 9) == [True] * 8 + [False]
    t += 1002
    assert _run(pf, t, 6) == [True] * 5 + [False]


def test_default_check_qps_in_different_duration(t0):
    """ParamFlowDefaultCheckerTest.java:178-220: durationInSec 60."""
    pf = _checker(5, duration=60)
    t = t0
    assert _run(pf, t, 6) == [True] * 5 + [False]
    for dt in (1000, 10_000, 30_000):
        t += dt
        assert _run(pf, t, 1) == [False]
    t += 30_000
    assert _run(pf, t, 6) == [True] * 5 + [False]


def test_throttle_single_value(t0):
    """ParamFlowThrottleRateLimitingCheckerTest.java:42-81 on virtual time: one call per ms for 990 ms
    admits exactly `count` requests (cost = round(1000·1·1/5) = 200 ms, no queueing)."""
    pf = _checker(5, behavior=abi.BEHAVIOR_RATE_LIMITER)
    ok = sum(pf.check(t0 + dt, 0, VALUE_A) for dt in range(0, 991))
    assert ok == 5
    t1 = t0 + 991 + 3000
    ok = sum(pf.check(t1 + dt, 0, VALUE_A) for dt in range(0, 991))
    assert ok == 5


def test_throttle_queueing_admits_within_max_wait(t0):
    """passThrottleLocalCheck (:230-250): expected − now < maxQueueingTimeMs admits and books the slot."""
    pf = _checker(10, behavior=abi.BEHAVIOR_RATE_LIMITER, max_queue=250)
    res = [pf.check(t0, 0, VALUE_A) for _ in range(5)]
    # cost 100 ms: slots at +0 (first sight), +100, +200 (wait 200 < 250), +300 is 300 >= 250 → block
    assert res == [True, True, True, False, False]
    assert pf.state(0, VALUE_A)[1] == t0 + 200


def test_hot_items_override_threshold(t0):
    """Hot items (ParamFlowChecker.java:137-141): the value's own threshold; threshold 0 blocks."""
    pf = _checker(5, hot=[(1, 2), (2, 0)])
    assert [pf.check(t0, 0, 1) for _ in range(3)] == [True, True, False]
    assert pf.check(t0, 0, 2) is False
    assert _run(pf, t0, 6, value=99) == [True] * 5 + [False]


def test_acquire_larger_than_max_blocks_and_state_kept(t0):
    pf = _checker(5, burst=1)
    assert pf.check(t0, 0, VALUE_A, acquire=7) is False      # acquireCount > maxCount
    assert pf.size() == 0                                     # rejected before touching the maps
    assert pf.check(t0, 0, VALUE_A, acquire=6) is True        # first sight: tokens = 6 - 6
    assert pf.state(0, VALUE_A) == (3, t0, 0)
    assert pf.check(t0 + 500, 0, VALUE_A) is False
    # refill after > 1000 ms: toAdd = 1001*5/1000 = 5 → min(max, rest + add) - acquire
    assert pf.check(t0 + 1001, 0, VALUE_A, acquire=2) is True
    assert pf.state(0, VALUE_A) == (3, t0 + 1001, 3)
