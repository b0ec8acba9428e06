"""Parity of the device flow-rule layer of the local chain (sg_local_load_flow_rules → k_lwalk_cx) with the
oracle (oracle.binding.LocalChain.load_flow_rules): several FlowRules per resource in FlowRuleComparator order,
limitApp origin / "other" rules reading per-origin StatisticNodes, and the WarmUp, RateLimiter and
WarmUpRateLimiter controllers inside the StatisticSlot → FlowSlot → DegradeSlot chain
(FlowRuleChecker.checkFlow, FlowRuleChecker.java:44-145; controller/*.java).

Traces: seeded entries with origins (0 = none) from LocalTraceGen, exits of the passed entries after their
sleep + response time; decided on the device in batches with state carried over. Every result, every
resource's windows / threads / breakers, every origin node of the resources with limitApp rules and every
rule's controller state (storedTokens, lastFilledTime, latestPassedTime) are compared bit-exactly.
"""
import numpy as np
import pytest

from oracle.binding import LocalChain, LocalTraceGen, degrade_rule, local_flow_rule, local_rule
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY]
D, WU, RL, WRL = abi.CONTROL_DEFAULT, abi.CONTROL_WARM_UP, abi.CONTROL_RATE_LIMITER, abi.CONTROL_WARM_UP_RATE_LIMITER
OTHER = abi.LIMIT_APP_OTHER


def _engine(flags=0):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=1 << 20, flags=flags)


def _rule_set(rng, r, n_origins):
    """A random rule list for resource r (one of several shapes)."""
    c = lambda lo, hi: float(rng.integers(lo, hi + 1))  # noqa: E731
    o = lambda: int(rng.integers(1, n_origins + 1))      # noqa: E731
    shape = int(rng.integers(0, 9))
    if shape == 0:
        return [local_flow_rule(r, c(5, 40))]                                             # fast path
    if shape == 1:
        return [local_flow_rule(r, c(10, 60), behavior=WU, warm_up_sec=int(rng.integers(2, 8)))]
    if shape == 2:
        return [local_flow_rule(r, c(10, 80), behavior=RL, max_queueing_ms=int(rng.integers(20, 400)))]
    if shape == 3:
        return [local_flow_rule(r, c(10, 60), behavior=WRL, warm_up_sec=int(rng.integers(2, 8)),
                                max_queueing_ms=int(rng.integers(50, 500)))]
    if shape == 4:
        return [local_flow_rule(r, c(20, 60)), local_flow_rule(r, c(2, 15), limit_app=o())]
    if shape == 5:
        return [local_flow_rule(r, c(5, 20), limit_app=OTHER), local_flow_rule(r, c(3, 10), limit_app=o()),
                local_flow_rule(r, c(30, 80))]
    if shape == 6:
        return [local_flow_rule(r, c(2, 8), grade=abi.FLOW_GRADE_THREAD), local_flow_rule(r, c(10, 40))]
    if shape == 7:
        return [local_flow_rule(r, c(30, 90), behavior=RL, max_queueing_ms=200),
                local_flow_rule(r, c(5, 25), behavior=WU, warm_up_sec=3, limit_app=o()),
                local_flow_rule(r, c(20, 50), limit_app=OTHER)]
    return []                                                                              # no flow rule


def _setup(n_res, rng, n_origins, breakers=False, S=2, interval=1000, flags=0, rule_sets=None):
    base = np.zeros(n_res, abi.LOCAL_RULE_DTYPE)
    for r in range(n_res):
        brk = [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)] if breakers and r % 3 == 0 else []
        base[r] = local_rule(0.0, abi.FLOW_GRADE_NONE, brk)
    if rule_sets is None:
        rule_sets = [_rule_set(rng, r, n_origins) for r in range(n_res)]
    flat = [x for rs in rule_sets for x in rs]
    rng.shuffle(flat)
    frules = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE) if flat else np.zeros(0, abi.LOCAL_FLOW_RULE_DTYPE)
    ora = LocalChain(S, interval, 500)
    ora.load_rules(base)
    kept = ora.load_flow_rules(frules, n_origins)
    eng = _engine(flags)
    eng.local_load_rules(base, S, interval, 500)
    assert eng.local_load_flow_rules(frules, n_origins) == kept
    return ora, eng, frules


def _entries(rng, n, n_res, t_start, span, n_origins, zipf=1.0, prio=0.05, multi=0.1, no_origin=0.3):
    e = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    e["ts_ms"] = t_start + np.sort(rng.integers(0, max(span, 1), n))
    e["resource"] = zipf_keys(rng, n_res, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    cnt = np.ones(n, np.int32)
    m = rng.random(n) < multi
    cnt[m] = rng.integers(2, 5, int(m.sum()))
    e["count"] = cnt
    e["resource"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    if n_origins:
        og = rng.integers(1, n_origins + 1, n).astype(np.int32)
        og[rng.random(n) < no_origin] = 0
        e["origin"] = og
    return e


def _compare(eng, ora, frules, n_res, n_origins):
    for r in range(n_res):
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g), f"second window of {r}:\n{s_o}\nvs\n{s_g}"
        assert np.array_equal(b_o, b_g), f"borrow array of {r}"
        assert np.array_equal(m_o, m_g), f"minute window of {r} differs at {np.nonzero((m_o != m_g).any(1))[0]}"
        assert head[0] == ora.threads(r), f"threads of {r}: {ora.threads(r)} vs {head[0]}"
        for i in range(2):
            st, nr = ora.breaker(r, i)
            if st >= 0:
                assert tuple(head[1 + 6 * i: 6 + 6 * i]) == (st, nr) + ora.breaker_stat(r, i), f"breaker {i} of {r}"
        for o in range(1, n_origins + 1):  # every origin node, whatever the rules (created at the first origin event)
            so, bo, mo, th, ex = ora.origin_dump(r, o)
            sg, bg, mg, hg, gx = eng.local_origin_state(r, o, with_exists=True)
            assert ex == gx, f"origin {o} node of {r}: exists {ex} vs {gx}"
            assert np.array_equal(so, sg), f"origin {o} second window of {r}:\n{so}\nvs\n{sg}"
            assert np.array_equal(bo, bg), f"origin {o} borrow array of {r}"
            assert np.array_equal(mo, mg), f"origin {o} minute window of {r}"
            assert hg[0] == th, f"origin {o} threads of {r}"
    for i in range(len(frules)):
        want = ora.controller(i)
        if want is None:
            continue
        got = eng.local_controller(i)
        assert np.array_equal(want, got), f"controller of rule {i} ({frules[i]}): {want} vs {got}"


def _run(ora, eng, frules, n_res, n_origins, batches, seed, rt_hi=40, err=0.05, **kw):
    rng = np.random.default_rng(seed + 1000)
    gen = LocalTraceGen(ora)
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    for n, span in batches:
        ent = _entries(rng, n, n_res, t, span, n_origins, **kw)
        rt = rng.integers(0, rt_hi + 1, n).astype(np.int32)
        er = (rng.random(n) < err).astype(np.uint8)
        ev, want = gen.run(ent, rt, er, t + span)
        got = eng.local_decide_host(ev)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            i = bad[0]
            raise AssertionError(f"{len(bad)} results differ; first at {i}: ev={ev[i]} oracle={want[i]} gpu={got[i]}")
        t += span
    _compare(eng, ora, frules, n_res, n_origins)
    return t


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("seed", [1, 2])
def test_mixed_rule_sets(flags, seed):
    rng = np.random.default_rng(seed)
    n_res, n_origins = 40, 4
    ora, eng, fr = _setup(n_res, rng, n_origins, breakers=True, flags=flags)
    _run(ora, eng, fr, n_res, n_origins, [(20_000, 3000), (20_000, 4000), (10_000, 2500)], seed, zipf=0.9)


@pytest.mark.parametrize("behavior", [WU, WRL])
def test_warm_up_ramp(behavior):
    """A cold resource under steady load: storedTokens drains through the warning zone over warmUpPeriodSec, the
    admitted rate climbs from count / coldFactor to count (WarmUpController.java:40-60)."""
    rng = np.random.default_rng(3)
    sets = [[local_flow_rule(r, 100.0, behavior=behavior, warm_up_sec=10, max_queueing_ms=300)] for r in range(3)]
    ora, eng, fr = _setup(3, rng, 0, rule_sets=sets)
    _run(ora, eng, fr, 3, 0, [(30_000, 6000), (30_000, 6000), (30_000, 6000)], 3, zipf=0.0, prio=0.0, multi=0.0)


def test_origin_nodes_and_other():
    """limitApp rules per origin and an "other" rule: each origin's StatisticNode sees its own traffic."""
    rng = np.random.default_rng(4)
    n_origins = 6
    sets = [[local_flow_rule(r, 8.0, limit_app=1), local_flow_rule(r, 5.0, limit_app=2),
             local_flow_rule(r, 3.0, limit_app=OTHER), local_flow_rule(r, 40.0)] for r in range(5)]
    sets += [[local_flow_rule(5, 4.0, grade=abi.FLOW_GRADE_THREAD, limit_app=3), local_flow_rule(5, 25.0, limit_app=OTHER)]]
    ora, eng, fr = _setup(6, rng, n_origins, rule_sets=sets)
    _run(ora, eng, fr, 6, n_origins, [(15_000, 2000), (15_000, 2000)], 4, zipf=0.5, prio=0.2, rt_hi=150)


def test_hot_cx_resource():
    """One rate-limited resource taking most of a large batch (one lane walks its long segment)."""
    rng = np.random.default_rng(5)
    sets = [[local_flow_rule(0, 500.0, behavior=RL, max_queueing_ms=500), local_flow_rule(0, 800.0)],
            [local_flow_rule(1, 50.0)], [local_flow_rule(2, 30.0, behavior=WU, warm_up_sec=2)]]
    ora, eng, fr = _setup(3, rng, 0, rule_sets=sets)
    _run(ora, eng, fr, 3, 0, [(100_000, 3000), (50_000, 3000)], 5, zipf=2.0)


def test_reload_keeps_statistics_and_resets_controllers():
    """A reload keeps every resource's statistics and its origin nodes (ClusterNode.originCountMap outlives it) and
    starts fresh controllers. The new rule sets name origins only on resources that named them before: the device
    keeps origin nodes from the first load that names an origin for the resource (the reference from the
    resource's first entry with that origin)."""
    rng = np.random.default_rng(6)
    n_res, n_origins = 12, 3
    sets0 = [_rule_set(rng, r, n_origins) for r in range(n_res)]
    ora, eng, fr = _setup(n_res, rng, n_origins, rule_sets=sets0)
    t = _run(ora, eng, fr, n_res, n_origins, [(10_000, 2000)], 6)
    sets = []
    for rs in sets0:  # same shapes, new thresholds, some resources' rules dropped, shuffled
        if rng.random() < 0.25:
            sets.append([])
            continue
        new = []
        for x in rs:
            y = x.copy()
            y["count"] = float(rng.integers(1, 60))
            new.append(y)
        sets.append(new)
    flat = [x for rs in sets for x in rs]
    rng.shuffle(flat)
    flat = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE)
    assert eng.local_load_flow_rules(flat, n_origins) == ora.load_flow_rules(flat, n_origins)
    gen = LocalTraceGen(ora)
    ent = _entries(rng, 10_000, n_res, t, 2000, n_origins)
    ev, want = gen.run(ent, rng.integers(0, 40, 10_000).astype(np.int32), np.zeros(10_000, np.uint8), t + 2000)
    got = eng.local_decide_host(ev)
    assert np.array_equal(got, want)
    _compare(eng, ora, fr, n_res, n_origins)    # every origin node the first load created
    _compare(eng, ora, flat, n_res, n_origins)  # the new rules' controllers


def test_bad_origin_rejected():
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(7)
    ora, eng, fr = _setup(4, rng, 2)
    ev = np.zeros(2, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"] = [1000, 1001]
    ev["count"] = 1
    ev["origin"] = [0, 3]
    with pytest.raises(EngineError) as ei:
        eng.local_decide_host(ev)
    assert ei.value.code == abi.SG_E_INVAL


def test_pool_growth_failure_leaves_nodes_readable(monkeypatch):
    """A node-pool growth that fails (injected: SG_TEST_POOL_FAIL) refuses the batch; the origin nodes its map
    entries already name have no storage yet and read as empty nodes (no read past the node arrays); once the pool
    can grow, the same batch decides as the oracle does and every node equals the oracle's."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(8)
    n_res, n_origins = 10, 3
    sets = [[local_flow_rule(r, 20.0), local_flow_rule(r, 4.0, limit_app=1)] for r in range(n_res)]
    ora, eng, fr = _setup(n_res, rng, n_origins, rule_sets=sets)
    gen = LocalTraceGen(ora)
    t = 1_700_000_000_000
    ent = _entries(rng, 5_000, n_res, t, 2000, n_origins)
    ev, want = gen.run(ent, rng.integers(0, 40, 5_000).astype(np.int32), np.zeros(5_000, np.uint8), t + 2000)
    monkeypatch.setenv("SG_TEST_POOL_FAIL", "1")
    with pytest.raises(EngineError):
        eng.local_decide_host(ev)
    for r in range(n_res):
        for o in range(1, n_origins + 1):
            s, b, m, h, _ = eng.local_origin_state(r, o, with_exists=True)
            assert not s[:, 1:].any() and not m[:, 1:].any() and not b[:, 1:].any() and h[0] == 0
    monkeypatch.delenv("SG_TEST_POOL_FAIL")
    got = eng.local_decide_host(ev)
    assert np.array_equal(got, want)
    _compare(eng, ora, fr, n_res, n_origins)
