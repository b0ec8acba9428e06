"""Parity of the device local slot chain (sg_local_*: StatisticSlot → FlowSlot/DefaultController →
DegradeSlot) with the oracle's sequential replay (oracle.binding.LocalChain).

Traces come from oracle.binding.LocalTraceGen: seeded time-ordered entries with planned response times and
business errors; each entry that passes exits at ts + waitInMs + rt (a SphU.entry caller only exits the
entries it obtained). The same event stream is then decided on the device in several batches (state carried
across batches) and every result, every resource's second window, borrow array, minute window, thread
count and breaker state/statistics are compared bit-exactly.
"""
import numpy as np
import pytest

from oracle.binding import LocalChain, LocalTraceGen, degrade_rule, local_rule
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY]


def _engine(max_batch=1 << 20, flags=0):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max_batch, flags=flags)


def _entries(rng, n, n_res, t_start, span, zipf=1.0, prio=0.0, multi=0.1):
    e = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    e["ts_ms"] = t_start + np.sort(rng.integers(0, max(span, 1), n))
    e["resource"] = zipf_keys(rng, n_res, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    c = np.ones(n, np.int32)
    m = rng.random(n) < multi
    c[m] = rng.integers(2, 5, int(m.sum()))
    e["count"] = c
    e["resource"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    return e


def _compare(eng, ora, n_res, S):
    for r in range(n_res):
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g), f"second window of {r}:\n{s_o}\nvs\n{s_g}"
        assert np.array_equal(b_o, b_g), f"borrow array of {r}:\n{b_o}\nvs\n{b_g}"
        assert np.array_equal(m_o, m_g), f"minute window of {r} differs at {np.nonzero((m_o != m_g).any(1))[0]}"
        assert head[0] == ora.threads(r), f"threads of {r}: {ora.threads(r)} vs {head[0]}"
        for i in range(2):
            st, nr = ora.breaker(r, i)
            if st < 0:
                continue
            start, bad, total = ora.breaker_stat(r, i)
            got = tuple(head[1 + 6 * i: 6 + 6 * i])
            assert got == (st, nr, start, bad, total), f"breaker {i} of {r}: {(st, nr, start, bad, total)} vs {got}"


def _run(rules, batches, flags=0, S=2, interval=1000, occupy=500, seed=0, rt_hi=40, err=0.05, **kw):
    """batches: list of (n_entries, span_ms) pieces; exits roll over between batches."""
    rng = np.random.default_rng(seed)
    n_res = len(rules)
    ora = LocalChain(S, interval, occupy)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    eng = _engine(flags=flags)
    eng.local_load_rules(rules, S, interval, occupy)
    eng.enable_stats(True)
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    total = 0
    skipped = 0
    for n, span in batches:
        ent = _entries(rng, n, n_res, t, span, **kw)
        rt = rng.integers(0, rt_hi + 1, n).astype(np.int32)
        er = (rng.random(n) < err).astype(np.uint8)
        ev, want = gen.run(ent, rt, er, t + span)
        got = eng.local_decide_host(ev)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            i = bad[0]
            raise AssertionError(f"{len(bad)} results differ; first at {i}: ev={ev[i]} oracle={want[i]} gpu={got[i]}")
        total += len(ev)
        skipped += eng.stats()["skipped_ranges"]
        t += span
    _compare(eng, ora, n_res, S)
    return total, skipped


def _rules(n, rng, grade=abi.FLOW_GRADE_QPS, lo=1, hi=30, breakers=()):
    out = np.zeros(n, abi.LOCAL_RULE_DTYPE)
    for i in range(n):
        out[i] = local_rule(float(rng.integers(lo, hi + 1)), grade, breakers)
    return out


@pytest.mark.parametrize("flags", WALKERS)
def test_qps_rules_no_breakers(flags):
    rng = np.random.default_rng(1)
    rules = _rules(50, rng)
    _run(rules, [(20_000, 1000), (20_000, 1300), (5_000, 200)], flags=flags, seed=1, zipf=1.1)


@pytest.mark.parametrize("flags", WALKERS)
def test_prioritized_occupy_and_borrow_array(flags):
    """DefaultController's prioritized path: tryOccupyNext, addWaitingRequest into the borrow array,
    addOccupiedPass into the minute window, PriorityWaitException (PASS after waitInMs)."""
    rng = np.random.default_rng(2)
    rules = _rules(8, rng, lo=2, hi=12)
    _run(rules, [(6_000, 900), (6_000, 1100), (3_000, 400)], flags=flags, seed=2, zipf=0.8, prio=0.4)


@pytest.mark.parametrize("flags", WALKERS)
def test_thread_grade_and_no_rule(flags):
    rng = np.random.default_rng(3)
    rules = np.concatenate([_rules(10, rng, grade=abi.FLOW_GRADE_THREAD, lo=1, hi=6),
                            _rules(5, rng, grade=abi.FLOW_GRADE_NONE)])
    _run(rules, [(8_000, 800), (8_000, 800)], flags=flags, seed=3, rt_hi=200)


@pytest.mark.parametrize("flags", WALKERS)
def test_circuit_breakers(flags):
    """RT and exception-ratio / exception-count breakers: CLOSED → OPEN on exits, OPEN → HALF_OPEN probe
    after timeWindow, HALF_OPEN → CLOSED / OPEN on the probe's exit, blocked probes back to OPEN."""
    rng = np.random.default_rng(4)
    rules = np.zeros(12, abi.LOCAL_RULE_DTYPE)
    for i in range(12):
        brk = [degrade_rule(abi.DEGRADE_RT, 20, 1, 5, 1000, 0.3),
               degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.2, 1, 5, 500)]
        if i % 3 == 1:
            brk = [degrade_rule(abi.DEGRADE_EXCEPTION_COUNT, 3, 2, 2, 1000)]
        if i % 3 == 2:
            brk = brk[::-1]
        rules[i] = local_rule(float(rng.integers(20, 200)), abi.FLOW_GRADE_QPS if i % 4 else abi.FLOW_GRADE_NONE, brk)
    _run(rules, [(15_000, 1500), (15_000, 2500), (15_000, 3000)], flags=flags, seed=4, zipf=1.0, rt_hi=40, err=0.15)


@pytest.mark.parametrize("flags", WALKERS)
def test_rt_breaker_max_ratio_and_prio_mix(flags):
    rng = np.random.default_rng(5)
    rules = np.zeros(6, abi.LOCAL_RULE_DTYPE)
    for i in range(6):
        rules[i] = local_rule(float(rng.integers(5, 40)), abi.FLOW_GRADE_QPS,
                              [degrade_rule(abi.DEGRADE_RT, 10.5, 1, 3, 300, 1.0)])
    _run(rules, [(10_000, 2000), (10_000, 2000)], flags=flags, seed=5, prio=0.2, rt_hi=25, err=0.0)


@pytest.mark.parametrize("S,interval", [(1, 1000), (4, 1000), (5, 500), (2, 2000), (10, 1000)])
def test_window_shapes(S, interval):
    rng = np.random.default_rng(6 + S)
    rules = _rules(20, rng, breakers=[degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 4, 700)])
    _run(rules, [(12_000, 1700), (12_000, 900)], S=S, interval=interval, seed=6 + S, prio=0.1, err=0.2)


@pytest.mark.parametrize("flags", [0, abi.FLAG_WAVE_ONLY])
def test_hot_resource_long_segments(flags):
    """One resource taking most of the traffic (the wave walker's admit / skip / epoch logic)."""
    rng = np.random.default_rng(7)
    rules = np.zeros(3, abi.LOCAL_RULE_DTYPE)
    rules[0] = local_rule(300.0, abi.FLOW_GRADE_QPS, [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.5, 1, 20, 1000)])
    rules[1] = local_rule(40.0, abi.FLOW_GRADE_QPS)
    rules[2] = local_rule(1000.0, abi.FLOW_GRADE_QPS, [degrade_rule(abi.DEGRADE_RT, 15, 1, 10, 1000, 0.4)])
    _run(rules, [(100_000, 2000), (100_000, 2000)], flags=flags, seed=7, zipf=2.0, err=0.3, rt_hi=30, multi=0.3)


def test_timestamps_rejected():
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(8)
    rules = _rules(4, rng)
    eng = _engine()
    eng.local_load_rules(rules)
    ev = np.zeros(3, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"] = [1000, 900, 1100]
    ev["count"] = 1
    with pytest.raises(EngineError) as ei:
        eng.local_decide_host(ev)
    assert ei.value.code == abi.SG_E_TIME
    # the first event later than the rest by many periods (below the period tables' start)
    ev["ts_ms"] = [90_000, 900, 1100]
    with pytest.raises(EngineError) as ei:
        eng.local_decide_host(ev)
    assert ei.value.code == abi.SG_E_TIME


@pytest.mark.parametrize("flags", [0, abi.FLAG_WAVE_ONLY, abi.FLAG_SERIAL_ONLY])
def test_breakers_near_their_thresholds(flags):
    """Hot resources whose breakers hover around their thresholds: many exits with CLOSED breakers (the wave
    walker's trip search over exit prefix sums), periodic OPEN → HALF_OPEN → CLOSED cycles."""
    rules = np.zeros(4, abi.LOCAL_RULE_DTYPE)
    rules[0] = local_rule(1e6, abi.FLOW_GRADE_QPS, [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.12, 1, 50, 1000)])
    rules[1] = local_rule(1e6, abi.FLOW_GRADE_QPS, [degrade_rule(abi.DEGRADE_RT, 30, 1, 50, 1000, 0.27)])
    rules[2] = local_rule(5e3, abi.FLOW_GRADE_QPS, [degrade_rule(abi.DEGRADE_EXCEPTION_COUNT, 90, 1, 20, 500),
                                                    degrade_rule(abi.DEGRADE_RT, 35, 2, 30, 1000, 0.2)])
    rules[3] = local_rule(1e6, abi.FLOW_GRADE_NONE, [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.1, 1, 10, 250)])
    _run(rules, [(60_000, 3000), (60_000, 3000)], flags=flags, seed=9, zipf=0.5, err=0.1, rt_hi=40)


@pytest.mark.parametrize("breakers", [False, True])
def test_saturated_periods_are_skipped(breakers):
    """Hot resources far above their QPS threshold: once the second window cannot admit even one more
    request, the wave walker jumps to the end of the period (or the resource's next exit) and
    k_lskip_apply adds the skipped entries' BLOCK counts. Results and windows must still match."""
    rng = np.random.default_rng(10)
    brk = [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)] if breakers else []
    rules = _rules(5, rng, lo=5, hi=40, breakers=brk)
    _, skipped = _run(rules, [(200_000, 1000), (200_000, 1700)], seed=10, zipf=1.5, rt_hi=20, err=0.2)
    assert skipped > 0
