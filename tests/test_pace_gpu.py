"""Parity of the device pace controller (sg_pace_*, RateLimiterController per FlowRule) with the oracle's
sequential canPass replay: every wait / block and every latestPassedTime, bit-exact, for both walkers."""
import numpy as np
import pytest

from oracle.binding import RateLimiterController
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY]


def _engine(flags=0, max_batch=1 << 20):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max_batch, flags=flags)


def _rules(rng, n, zero_frac=0.02):
    r = np.zeros(n, abi.PACE_RULE_DTYPE)
    r["count"] = np.where(rng.random(n) < 0.5, rng.integers(1, 2000, n), rng.random(n) * 50)
    r["count"][rng.random(n) < zero_frac] = 0.0
    r["max_queueing_ms"] = rng.choice([0, 20, 100, 500, 2000], n)
    return r


def _trace(rng, n, n_rules, t0, span, zipf=1.1, acq_hi=3, odd_frac=0.01):
    q = np.zeros(n, abi.PACE_REQ_DTYPE)
    q["ts_ms"] = t0 + np.sort(rng.integers(0, max(span, 1), n))
    q["rule"] = zipf_keys(rng, n_rules, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    q["acquire"] = rng.integers(1, acq_hi + 1, n)
    odd = rng.random(n) < odd_frac
    q["acquire"][odd] = rng.integers(-2, 1, odd.sum())          # acquireCount <= 0 passes
    q["rule"][rng.random(n) < odd_frac] = n_rules + 7           # no rule for the resource
    return q


def _check(eng, ora, req, n_rules):
    want = ora.decide(req)
    got = eng.pace_decide_host(req)
    if not np.array_equal(want, got):
        bad = np.nonzero(want != got)[0]
        raise AssertionError(f"{len(bad)} differ; first {bad[0]}: req={req[bad[0]]} oracle={want[bad[0]]} gpu={got[bad[0]]}")
    for k in range(0, n_rules, max(1, n_rules // 64)):
        assert eng.pace_latest(k) == ora.latest(k), k
    return want


@pytest.mark.parametrize("flags", WALKERS)
def test_pace_random_batches(flags):
    rng = np.random.default_rng(11 + flags)
    n_rules = 500
    rules = _rules(rng, n_rules)
    eng = _engine(flags)
    eng.pace_load_rules(rules)
    ora = RateLimiterController(rules)
    t = 1_700_000_000_000
    seen = np.zeros(0, np.int32)
    for b in range(4):
        req = _trace(rng, 20_000, n_rules, t, 1500)
        seen = np.concatenate([seen, _check(eng, ora, req, n_rules)])
        t = int(req["ts_ms"][-1])
    assert (seen == abi.PACE_BLOCKED).any() and (seen > 0).any() and (seen == 0).any()


@pytest.mark.parametrize("flags", WALKERS)
def test_pace_one_hot_rule_same_instant(flags):
    # the reference's timeout test at scale: one rule, many requests at few instants
    eng = _engine(flags)
    rules = np.zeros(1, abi.PACE_RULE_DTYPE)
    rules[0] = (1000.0, 500, 0)
    eng.pace_load_rules(rules)
    ora = RateLimiterController(rules)
    rng = np.random.default_rng(5)
    req = np.zeros(5000, abi.PACE_REQ_DTYPE)
    req["ts_ms"] = 10_000 + np.sort(rng.integers(0, 4, 5000)) * 700
    req["acquire"] = 1
    w = _check(eng, ora, req, 1)
    assert (w == 0).sum() >= 1 and (w == 500).sum() >= 1 and (w == abi.PACE_BLOCKED).sum() > 2000


def test_pace_large_zipf_batch():
    rng = np.random.default_rng(3)
    n_rules = 100_000
    rules = _rules(rng, n_rules)
    eng = _engine(0, max_batch=1 << 21)
    eng.pace_load_rules(rules)
    ora = RateLimiterController(rules)
    _check(eng, ora, _trace(rng, 1 << 21, n_rules, 5_000, 1000, zipf=1.0), n_rules)


def test_pace_reload_resets_and_time_order():
    from sentinel_amd.engine import EngineError
    eng = _engine(0)
    rules = np.zeros(2, abi.PACE_RULE_DTYPE)
    rules[:] = [(10.0, 0, 0), (5.0, 100, 0)]
    eng.pace_load_rules(rules)
    req = np.zeros(3, abi.PACE_REQ_DTYPE)
    req[:] = [(1000, 0, 1), (1000, 0, 1), (1050, 1, 1)]
    assert list(eng.pace_decide_host(req)) == [0, abi.PACE_BLOCKED, 0]
    assert eng.pace_latest(0) == 1000 and eng.pace_latest(1) == 1050
    eng.pace_load_rules(rules)
    assert eng.pace_latest(0) == -1
    bad = np.zeros(2, abi.PACE_REQ_DTYPE)
    bad[:] = [(900, 0, 1), (800, 0, 1)]
    with pytest.raises(EngineError):
        eng.pace_decide_host(bad)


@pytest.mark.parametrize("flags", WALKERS)
def test_pace_saturated_cost_wraps(flags):
    """A tiny count with a huge acquireCount saturates Math.round at Long.MAX_VALUE, and Java's
    costTime + latestPassedTime wraps negative: the request passes at once (RateLimiterController.java:58-62).
    The wave walker's horizon jump must not skip such requests."""
    eng = _engine(flags)
    rules = np.zeros(2, abi.PACE_RULE_DTYPE)
    rules[:] = [(1e-7, 0, 0), (2e-7, 500, 0)]
    eng.pace_load_rules(rules)
    ora = RateLimiterController(rules)
    rng = np.random.default_rng(9)
    t = 1_700_000_000_000
    for _ in range(2):
        req = np.zeros(4000, abi.PACE_REQ_DTYPE)
        req["ts_ms"] = t + np.sort(rng.integers(0, 3000, len(req)))
        req["rule"] = rng.integers(0, 2, len(req))
        req["acquire"] = np.where(rng.random(len(req)) < 0.05, rng.integers(1 << 29, (1 << 31) - 1, len(req)), 1)
        w = _check(eng, ora, req, 2)
        assert (w[req["acquire"] > 1] == 0).any() and (w[req["acquire"] == 1] == abi.PACE_BLOCKED).any()
        t = int(req["ts_ms"][-1])


@pytest.mark.parametrize("span", [1000, 6000])
def test_pace_bursty_rules_guess_misses(span):
    """The wave walker guesses where its next admissible request lies from the rule's average density over the
    batch; bursty rules (requests packed into a few short windows, idle elsewhere) make the guess land before and
    after the answer. A batch spanning 6 s has no millisecond table in LDS and searches by timestamp instead."""
    rng = np.random.default_rng(21 + span)
    n, n_rules = 200_000, 8
    rules = np.zeros(n_rules, abi.PACE_RULE_DTYPE)
    rules["count"] = [50.0, 7.0, 300.0, 1.5, 64.0, 20.0, 1000.0, 3.0]
    rules["max_queueing_ms"] = [500, 0, 100, 2000, 500, -5, 20, 500]
    eng = _engine(abi.FLAG_WAVE_ONLY)
    eng.pace_load_rules(rules)
    ora = RateLimiterController(rules)
    t = 1_700_000_000_000
    for _ in range(3):
        ts = np.sort(rng.integers(0, span, n))
        rule = rng.integers(0, n_rules, n)
        burst = (ts % 400) < 40                         # rule 0-3 live only in the first 40 ms of every 400
        rule[burst] = rng.integers(0, 4, burst.sum())
        rule[~burst] = rng.integers(4, n_rules, (~burst).sum())
        req = np.zeros(n, abi.PACE_REQ_DTYPE)
        req["ts_ms"] = t + ts
        req["rule"] = rule
        req["acquire"] = np.where(rng.random(n) < 0.1, rng.integers(2, 300, n), 1)
        w = _check(eng, ora, req, n_rules)
        assert (w == abi.PACE_BLOCKED).any() and (w > 0).any() and (w == 0).any()
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 3000))
