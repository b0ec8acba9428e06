"""Parity of the device hot-parameter path (sg_param_*) with the oracle's ParamFlowChecker replay:
every pass/block bit and every (rule, value) bucket, bit-exact, for both walkers."""
import numpy as np
import pytest

from oracle.binding import ParamFlowChecker
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY]


def _engine(flags=0, max_batch=1 << 20):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max_batch, flags=flags)


def _rules(specs, cap_log2=16):
    r = np.zeros(len(specs), abi.PARAM_RULE_DTYPE)
    for i, sp in enumerate(specs):
        r[i]["count"] = sp.get("count", 5)
        r[i]["duration_sec"] = sp.get("duration", 1)
        r[i]["burst"] = sp.get("burst", 0)
        r[i]["behavior"] = sp.get("behavior", abi.BEHAVIOR_DEFAULT)
        r[i]["max_queueing_ms"] = sp.get("max_queue", 0)
        r[i]["capacity_log2"] = cap_log2
    return r


def _trace(rng, n, n_rules, n_values, t0, span, zipf=1.1, big_value_frac=0.0, acq_hi=1):
    q = np.zeros(n, abi.PARAM_REQ_DTYPE)
    q["ts_ms"] = t0 + np.sort(rng.integers(0, max(span, 1), n))
    vals = zipf_keys(rng, n_values, n, zipf, perm_seed=int(rng.integers(1 << 30))).astype(np.uint64)
    vals = vals * np.uint64(0x9E3779B97F4A7C15)  # spread over the u64 range
    big = rng.random(n) < big_value_frac
    vals[big] = np.uint64(0xFFFFFFFFFFFFFFFF)
    q["value"] = vals
    q["rule"] = rng.integers(0, n_rules, n)
    q["acquire"] = rng.integers(1, acq_hi + 1, n)
    return q


def _pair(rules, hot=None, flags=0):
    eng = _engine(flags)
    eng.param_load_rules(rules, hot)
    ora = ParamFlowChecker()
    ora.load_rules(rules, hot)
    return eng, ora


def _check(eng, ora, req):
    want = ora.decide(req)
    got = eng.param_decide_host(req)
    if not np.array_equal(want, got):
        bad = np.nonzero(want != got)[0]
        raise AssertionError(f"{len(bad)} differ; first {bad[0]}: req={req[bad[0]]} oracle={want[bad[0]]} gpu={got[bad[0]]}")
    return want


def _check_states(eng, ora, req, limit=300):
    seen = set()
    for r in req[:limit]:
        key = (int(r["rule"]), int(r["value"]))
        if key in seen:
            continue
        seen.add(key)
        assert ora.state(*key) == eng.param_state(*key), key


@pytest.mark.parametrize("flags", WALKERS)
def test_param_default_token_bucket_restated_kats(t0, flags):
    """The ParamFlowDefaultCheckerTest sequences (tests/test_oracle_param_kat.py) through the device."""
    eng, ora = _pair(_rules([{"count": 5, "burst": 3}]), flags=flags)
    seq = [(0, 9), (1002, 6), (2004, 6), (4004, 9), (5006, 6)]
    for dt, k in seq:
        req = np.zeros(k, abi.PARAM_REQ_DTYPE)
        req["ts_ms"] = t0 + dt
        req["value"] = 0x76616C756541
        req["acquire"] = 1
        got = eng.param_decide_host(req)
        assert list(got) == list(ora.decide(req))
        assert list(got) == [1] * (k - 1) + [0]


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("spec", [
    {"count": 5}, {"count": 3, "burst": 4}, {"count": 50, "duration": 2}, {"count": 1},
    {"count": 7, "behavior": abi.BEHAVIOR_RATE_LIMITER},
    {"count": 20, "behavior": abi.BEHAVIOR_RATE_LIMITER, "max_queue": 120},
])
def test_param_random_traces(spec, flags):
    rng = np.random.default_rng(hash(str(spec)) % (1 << 30))
    rules = _rules([spec, {"count": 2}])
    hot = np.zeros(3, abi.PARAM_HOT_DTYPE)
    hot[0] = (np.uint64(0x9E3779B97F4A7C15) * np.uint64(1), 40, 0)   # hot value of rule 0
    hot[1] = (np.uint64(0x9E3779B97F4A7C15) * np.uint64(2), 0, 0)    # threshold 0: always blocked
    hot[2] = (np.uint64(0xFFFFFFFFFFFFFFFF), 9, 0)
    rules[0]["hot_begin"], rules[0]["hot_count"] = 0, 3
    eng, ora = _pair(rules, hot, flags=flags)
    t = 1_700_000_000_000
    for _ in range(3):
        req = _trace(rng, 60_000, 2, 3000, t, int(rng.integers(200, 3500)), big_value_frac=0.01, acq_hi=3)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 1500))
        _check(eng, ora, req)
    _check_states(eng, ora, req)


@pytest.mark.parametrize("flags", WALKERS)
def test_param_hot_value_long_segments(flags):
    """One value taking most requests: the wave walker's zone jumps and refill boundaries."""
    rng = np.random.default_rng(99)
    rules = _rules([{"count": 5}, {"count": 3, "burst": 2, "duration": 1}])
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_123
    for _ in range(4):
        req = _trace(rng, 200_000, 2, 50, t, 2600, zipf=2.2, acq_hi=2)
        t = int(req["ts_ms"][-1]) + 1
        _check(eng, ora, req)
    _check_states(eng, ora, req)


def test_param_unknown_rule_passes_and_time_errors():
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(3)
    eng, ora = _pair(_rules([{"count": 2}]))
    req = _trace(rng, 1000, 1, 10, 1_700_000_000_000, 500)
    req["rule"][::7] = 5
    out = _check(eng, ora, req)
    assert (out[::7] == 1).all()
    bad = _trace(rng, 100, 1, 10, 1_600_000_000_000, 100)
    with pytest.raises(EngineError) as ei:
        eng.param_decide_host(bad)
    assert ei.value.code == abi.SG_E_TIME


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("span", [3_000, 20_000, 100_000])
def test_batch_spans_and_large_acquire(span, flags):
    """The walkers recover each request's timestamp from the batch's millisecond table (request index -> ts, staged in
    LDS up to 4096 ms; longer batches read the timestamps) and its acquireCount from the record's 8-bit code (255 and
    above read the request): spans across both table regimes and past the 65,536-entry table, counts up to 300."""
    rng = np.random.default_rng(span)
    rules = _rules([{"count": 50, "duration": 1, "burst": 20}, {"count": 400, "duration": 2},
                    {"count": 8, "behavior": abi.BEHAVIOR_RATE_LIMITER, "max_queue": 500}])
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_000
    for _ in range(2):
        req = _trace(rng, 40_000, len(rules), 300, t, span, acq_hi=300)
        _check(eng, ora, req)
        t = int(req["ts_ms"][-1]) + 1
