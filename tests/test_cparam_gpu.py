"""Parity of the device cluster hot-parameter path (sg_cparam_*: requestParamToken → ClusterParamFlowChecker)
with the oracle (oracle.binding.ClusterTokenService.decide_param, a literal restatement of ClusterParamMetric's
per-flowId LeapArray of value → count maps): every TokenResult and every (rule, value) window sum, bit-exact."""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu


WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY]


def _pair(rules, hot=None, connected=1, cap=12, flags=0):
    from sentinel_amd.engine import FlowEngine
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = connected
    eng = FlowEngine(device=0, max_batch=1 << 20, flags=flags)
    eng.set_namespaces(ns)
    eng.cparam_load_rules(rules, hot, cap)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_param_rules(rules, hot)
    return eng, ora


def _rules(n, rng, S=10, interval=1000, thr=abi.THRESHOLD_GLOBAL, hot_per_rule=0):
    r = np.zeros(n, abi.CPARAM_RULE_DTYPE)
    r["flow_id"] = np.arange(n) * 3 + 7
    r["count"] = rng.integers(1, 40, n)
    r["threshold_type"] = thr
    r["sample_count"] = S
    r["window_interval_ms"] = interval
    r["hot_begin"] = np.arange(n) * hot_per_rule
    r["hot_count"] = hot_per_rule
    return r


def _trace(rng, n, n_rules, n_values, t0, span, multi=0.0, zipf=1.1, acq_hi=3, bad=0.0):
    req = np.zeros(n, abi.CPARAM_REQ_DTYPE)
    req["ts_ms"] = t0 + np.sort(rng.integers(0, max(span, 1), n))
    req["key"] = rng.integers(0, n_rules, n)
    req["acquire"] = rng.integers(1, acq_hi + 1, n)
    counts = np.where(rng.random(n) < multi, rng.integers(2, 4, n), 1).astype(np.uint32)
    req["value_count"] = counts
    req["value_begin"] = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint32)
    values = zipf_keys(rng, n_values, int(counts.sum()), zipf, perm_seed=int(rng.integers(1 << 30))).astype(np.uint64)
    values = values * np.uint64(0x9E3779B97F4A7C15)
    sel = rng.random(n)
    req["key"][sel < bad] = abi.KEY_BAD
    req["acquire"][(sel >= bad) & (sel < 2 * bad)] = 0
    req["key"][(sel >= 2 * bad) & (sel < 3 * bad)] = abi.KEY_NO_RULE
    req["value_count"][(sel >= 3 * bad) & (sel < 4 * bad)] = 0
    return req, values


def _check(eng, ora, req, values):
    want = ora.decide_param(req, values)
    got = eng.cparam_decide_host(req, values)
    if not np.array_equal(want, got):
        bad = np.nonzero(want != got)[0]
        i = bad[0]
        raise AssertionError(f"{len(bad)} differ; first {i}: req={req[i]} oracle={want[i]} gpu={got[i]}")
    return want


def _compare_sums(eng, ora, req, values, now):
    keys = set()
    for q in req[:2000]:
        k = int(q["key"])
        if k < 1 << 20 and q["value_count"] > 0:
            for v in values[q["value_begin"]: q["value_begin"] + q["value_count"]]:
                keys.add((k, int(v)))
    for k, v in sorted(keys)[:300]:
        assert eng.cparam_sum(k, v, now) == ora.param_sum(k, v, now), (k, v)


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("S,interval", [(10, 1000), (2, 1000), (1, 500), (5, 25)])
def test_single_value_requests(S, interval, flags):
    rng = np.random.default_rng(S * 7 + interval)
    rules = _rules(20, rng, S, interval)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_003
    for _ in range(3):
        req, vals = _trace(rng, 50_000, 20, 300, t, int(rng.integers(100, 3 * interval + 500)), bad=0.01)
        out = _check(eng, ora, req, vals)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, interval))
    assert (out["status"] == abi.OK).any() and (out["status"] == abi.BLOCKED).any()
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


@pytest.mark.parametrize("flags", WALKERS)
def test_multi_value_requests_all_or_nothing(flags):
    rng = np.random.default_rng(3)
    rules = _rules(6, rng)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_500
    for _ in range(3):
        req, vals = _trace(rng, 6_000, 6, 40, t, 1500, multi=0.05, bad=0.01)
        out = _check(eng, ora, req, vals)
        t = int(req["ts_ms"][-1]) + 7
    multi = req["value_count"] > 1
    assert (out["remaining"][multi & (out["status"] == abi.OK)] == -1).all()
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def test_hot_items_and_avg_local():
    rng = np.random.default_rng(4)
    rules = _rules(4, rng, thr=abi.THRESHOLD_AVG_LOCAL, hot_per_rule=3)
    hot = np.zeros(12, abi.PARAM_HOT_DTYPE)
    for i in range(12):
        hot[i] = ((i % 3 + 1) * 0x9E3779B97F4A7C15 % (1 << 64), int(rng.integers(0, 6)), 0)
    eng, ora = _pair(rules, hot, connected=3)
    t = 1_700_000_000_000
    for _ in range(2):
        req, vals = _trace(rng, 20_000, 4, 10, t, 2000, zipf=0.8)
        _check(eng, ora, req, vals)
        t = int(req["ts_ms"][-1])


def test_rule_reload_keeps_surviving_metrics():
    rng = np.random.default_rng(5)
    rules = _rules(8, rng)
    eng, ora = _pair(rules)
    req, vals = _trace(rng, 20_000, 8, 50, 1_700_000_000_000, 800)
    _check(eng, ora, req, vals)
    new = np.concatenate([rules[2:6], _rules(3, rng)])
    new["flow_id"][4:] += 1000
    new["count"] = rng.integers(1, 30, len(new))
    new["sample_count"][:2] = 4  # ignored for surviving flowIds: their metric keeps S=10
    eng.cparam_load_rules(new, None, 12)
    ora.load_param_rules(new)
    req, vals = _trace(rng, 20_000, len(new), 50, 1_700_000_000_900, 1200)
    _check(eng, ora, req, vals)
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("seed,multi", [(11, 0.3), (12, 0.8)])
def test_multi_value_heavy_fixed_point(seed, multi, flags):
    """Most requests carry several (possibly repeated) values over a few hot values: the all-or-nothing outcomes
    chain across slots, so the device needs several fixed-point rounds; every result and window sum must still
    equal the sequential replay."""
    rng = np.random.default_rng(seed)
    rules = _rules(5, rng)
    rules["count"] = rng.integers(3, 12, 5)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_250
    rounds = []
    for _ in range(3):
        req, vals = _trace(rng, 30_000, 5, 12, t, 2500, multi=multi, zipf=1.3, bad=0.005)
        _check(eng, ora, req, vals)
        rounds.append(eng.cparam_last_rounds())
        t = int(req["ts_ms"][-1]) + 3
    assert max(rounds) > 1
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def test_serial_fallback(monkeypatch):
    """With no fixed-point rounds allowed every group of linked slots is replayed from the untouched rings — same
    answers."""
    monkeypatch.setenv("SG_CP_MAX_ROUNDS", "0")
    rng = np.random.default_rng(13)
    rules = _rules(4, rng)
    eng, ora = _pair(rules)
    req, vals = _trace(rng, 4_000, 4, 10, 1_700_000_000_000, 1500, multi=0.4, zipf=1.2, bad=0.01)
    _check(eng, ora, req, vals)
    assert eng.cparam_last_rounds() == 1  # max_rounds (0) + 1: the group replay
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


@pytest.mark.parametrize("max_rounds", [1, 2, 4, 5])
def test_round_budget_inside_a_chain(monkeypatch, max_rounds):
    """Round budgets that end inside a chain of three enqueued rounds (r1 = min(round + 3, max)) and the serial
    fallback after rounds > 0 (the linked groups' saved rings restored, k_cpfb_restore): a multi-value-heavy trace
    over a few hot values needs more rounds than the budget, so the groups are replayed — same answers and window
    sums; a batch that converges within the budget reports its rounds."""
    monkeypatch.setenv("SG_CP_MAX_ROUNDS", str(max_rounds))
    rng = np.random.default_rng(40 + max_rounds)
    rules = _rules(5, rng)
    rules["count"] = rng.integers(3, 12, 5)
    eng, ora = _pair(rules)
    t = 1_700_000_000_250
    serial = 0
    for _ in range(3):
        req, vals = _trace(rng, 30_000, 5, 12, t, 2500, multi=0.8, zipf=1.3, bad=0.005)
        _check(eng, ora, req, vals)
        r = eng.cparam_last_rounds()
        assert 1 <= r <= max_rounds + 1
        serial += r == max_rounds + 1
        t = int(req["ts_ms"][-1]) + 3
    assert serial > 0, "the trace should outlast the round budget"
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def _merge(parts):
    """Requests of several traces in one time order (stable), their value lists carried along."""
    req = np.concatenate([r for r, _ in parts])
    vals = [v[int(q["value_begin"]): int(q["value_begin"]) + int(q["value_count"])] for r, v in parts for q in r]
    order = np.argsort(req["ts_ms"], kind="stable")
    req = req[order]
    vals = [vals[i] for i in order]
    req["value_begin"] = np.concatenate([[0], np.cumsum(req["value_count"])[:-1]]).astype(np.uint32)
    return req, np.concatenate(vals).astype(np.uint64)


def _chain(L, key, t0, step_ms, v0=1 << 40):
    """L two-value requests of rule `key`, request k over (c_k, c_k+1): under a threshold of one per window every
    outcome depends on the previous one (they alternate), and the fixed point settles one link per round."""
    req = np.zeros(L, abi.CPARAM_REQ_DTYPE)
    req["ts_ms"] = t0 + step_ms * np.arange(L)
    req["key"] = key
    req["acquire"] = 1
    req["value_count"] = 2
    req["value_begin"] = 2 * np.arange(L)
    c = np.uint64(v0) + np.arange(L + 1, dtype=np.uint64)
    vals = np.stack([c[:-1], c[1:]], axis=1).reshape(-1)
    return req, vals


@pytest.mark.parametrize("L", [100, 300])
def test_deep_chain_replays_the_linked_group(L):
    """A multi-value dependency chain deeper than the 64-round budget among ordinary traffic: the slots the chain
    links are replayed as one group in arrival order (k_cpfb_*), every other slot keeps its walk — same results and
    window sums as the sequential oracle, the alternating chain outcomes included."""
    rng = np.random.default_rng(70 + L)
    rules = _rules(5, rng)
    rules["count"][0] = 1
    eng, ora = _pair(rules)
    t = 1_700_000_000_000
    for b in range(2):
        noise = _trace(rng, 40_000, 4, 400, t, 900, multi=0.1, zipf=1.1)
        noise[0]["key"] += 1  # rules 1..4; rule 0 (threshold 1) carries the chain alone
        req, vals = _merge([noise, _chain(L, 0, t + 50, 1, v0=(1 << 40) + 10_000 * b)])
        want = _check(eng, ora, req, vals)
        assert eng.cparam_last_rounds() == 65  # the budget ran out: the group fallback decided the batch
        st = want["status"][req["key"] == 0]
        assert (st[0::2] == abi.OK).all() and (st[1::2] == abi.BLOCKED).all()
        t = int(req["ts_ms"][-1]) + 1
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def test_limiter_shared_with_flow_tokens():
    """allowProceed → GlobalRequestLimiter.tryPass (ClusterParamFlowChecker.java:45): the namespace's limiter
    admits param and flow requests from one 10 x 100 ms window, so time-ordered flow and param batches interleave."""
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(14)
    ns = np.zeros(2, abi.NS_DTYPE)
    ns["connected_count"] = [2, 1]
    ns["limiter_enabled"] = [1, 0]             # namespace 1: no limiter
    ns["max_allowed_qps"] = [1500, 0]
    prules = _rules(8, rng)
    prules["namespace_id"] = np.arange(8) % 2
    frules = np.zeros(6, abi.RULE_DTYPE)
    frules["flow_id"] = np.arange(6) + 900
    frules["count"] = rng.integers(20, 400, 6)
    frules["threshold_type"] = abi.THRESHOLD_GLOBAL
    frules["sample_count"], frules["window_interval_ms"] = 10, 1000
    eng = FlowEngine(device=0, max_batch=1 << 18)
    eng.set_namespaces(ns)
    eng.load_rules(frules)
    eng.cparam_load_rules(prules, None, 12)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(frules)
    ora.load_param_rules(prules)
    t = 1_700_000_000_040
    seen = set()
    for b in range(4):
        span = int(rng.integers(300, 1500))
        req, vals = _trace(rng, 6_000, 8, 60, t, span, multi=0.2, bad=0.01)
        out = _check(eng, ora, req, vals)
        seen |= set(out["status"].tolist())
        t = int(req["ts_ms"][-1])
        f = np.zeros(3_000, abi.REQ_DTYPE)
        f["ts_ms"] = t + np.sort(rng.integers(0, 400, len(f)))
        f["key"] = rng.integers(0, 6, len(f))
        f["acquire"] = 1
        want, got = ora.decide(f), eng.decide_host(f)
        assert np.array_equal(want, got), f"flow batch {b}"
        seen |= set(want["status"].tolist())
        t = int(f["ts_ms"][-1])
    assert abi.TOO_MANY_REQUEST in seen and abi.OK in seen


def test_value_range_contract():
    """Overlapping, backwards or out-of-range value ranges are SG_E_INVAL and change no state."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(15)
    rules = _rules(3, rng)
    eng, ora = _pair(rules)
    req, vals = _trace(rng, 2_000, 3, 20, 1_700_000_000_000, 900, multi=0.3)
    _check(eng, ora, req, vals)
    t = int(req["ts_ms"][-1])
    nxt, nvals = _trace(rng, 1_000, 3, 20, t, 500, multi=0.3)
    for mutate in ("overlap", "backwards", "outside"):
        bad = nxt.copy()
        if mutate == "overlap":
            bad["value_begin"][10] = bad["value_begin"][9]
        elif mutate == "backwards":  # two requests on one (rule, value) whose positions run backwards
            bad["value_begin"][[20, 21]] = bad["value_begin"][[21, 20]]
            bad["value_count"][[20, 21]] = 1
            bad["key"][21] = bad["key"][20]
            bv = nvals.copy()
            bv[bad["value_begin"][21]] = bv[bad["value_begin"][20]]
        else:
            bad["value_begin"][-1] = len(nvals)
        with pytest.raises(EngineError):
            eng.cparam_decide_host(bad, bv if mutate == "backwards" else nvals)
    _check(eng, ora, nxt, nvals)   # the rejected batches left nothing behind
    _compare_sums(eng, ora, nxt, nvals, int(nxt["ts_ms"][-1]))


@pytest.mark.parametrize("flags", WALKERS)
def test_mixed_window_lengths(flags):
    """Rules of one handle with different window shapes: each distinct windowIntervalMs / sampleCount gets its own
    period table (request index -> window period) in the batch; single- and multi-value requests over all of them."""
    rng = np.random.default_rng(61)
    shapes = [(10, 1000), (2, 1000), (1, 500), (5, 25), (4, 2000), (3, 300), (10, 1000), (2, 1000)]
    rules = _rules(len(shapes) * 3, rng)
    for i in range(len(rules)):
        rules["sample_count"][i], rules["window_interval_ms"][i] = shapes[i % len(shapes)]
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_123
    for _ in range(3):
        req, vals = _trace(rng, 30_000, len(rules), 40, t, 2500, multi=0.15, bad=0.01)
        _check(eng, ora, req, vals)
        t = int(req["ts_ms"][-1]) + 3
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def test_more_than_eight_window_lengths_refused():
    """Nine distinct window lengths do not fit the batch's period tables: SG_E_UNSUPPORTED at load."""
    from sentinel_amd.engine import EngineError, FlowEngine
    rng = np.random.default_rng(62)
    rules = _rules(9, rng, S=1)
    rules["window_interval_ms"] = np.arange(9) * 100 + 100
    eng = FlowEngine(device=0, max_batch=1 << 16)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    eng.set_namespaces(ns)
    with pytest.raises(EngineError):
        eng.cparam_load_rules(rules, None, 10)
    eng.cparam_load_rules(rules[:8], None, 10)  # eight are fine


@pytest.mark.parametrize("flags", WALKERS)
def test_long_spans_and_large_acquire(flags):
    """Value records carry a 7-bit acquire code (127 and above read the request) and the walkers take window periods
    from the batch's period tables — staged in LDS up to 2048 periods, read from memory beyond (4000 here)."""
    rng = np.random.default_rng(63)
    rules = _rules(12, rng)
    rules["count"] = rng.integers(100, 2000, len(rules))
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_000
    for _ in range(2):
        req, vals = _trace(rng, 20_000, len(rules), 30, t, 400_000, multi=0.1, acq_hi=300)
        _check(eng, ora, req, vals)
        t = int(req["ts_ms"][-1]) + 1
    _compare_sums(eng, ora, req, vals, int(req["ts_ms"][-1]))


def test_batch_past_the_period_table_refused():
    """A batch spanning more than 65,536 window periods of some rule is refused before anything is charged."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(64)
    rules = _rules(4, rng, S=10, interval=10)  # 1 ms periods
    eng, ora = _pair(rules)
    req, vals = _trace(rng, 5_000, len(rules), 20, 1_700_000_000_000, 70_000)
    with pytest.raises(EngineError):
        eng.cparam_decide_host(req, vals)
    req, vals = _trace(rng, 5_000, len(rules), 20, 1_700_000_100_000, 30_000)
    _check(eng, ora, req, vals)
