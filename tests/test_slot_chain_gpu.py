"""Parity of the whole slot chain on the device (sg_slot_decide_batch: StatisticSlot around ParamFlowSlot → FlowSlot
→ DegradeSlot) with the oracle (oracle.binding.LocalChain + ParamFlowSlot, decide_ext).

Traces: seeded entries from LocalTraceGen.run_ext with a context id and arguments per entry (null args, values,
collections, null arguments), exits of the passed entries after their sleep + response time carrying the same
context and arguments. The resources mix every shape: the fast walkers' single DefaultController rule, shaping
controllers, limitApp origin / "other" rules, CHAIN rules (a context's DefaultNode), RELATE rules (key groups
reading another resource's ClusterNode, including one never entered), cluster-mode rules (fallback or not), param
rules (QPS token bucket, throttle, THREAD grade; collection arguments) and circuit breakers. Compared bit-exactly:
every result (the rule index of a ParamFlowException too), every resource's windows / threads / breakers, every
origin and context node the device keeps, every flow controller's state, every param value's thread count and token
state.
"""
import numpy as np
import pytest

from oracle.binding import LocalChain, LocalTraceGen, ParamFlowSlot, degrade_rule, local_flow_rule, local_rule
from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys
from tests.test_oracle_pslot_kat import QPS, THREAD, rule as prule

pytestmark = pytest.mark.gpu

D, WU, RL, WRL = abi.CONTROL_DEFAULT, abi.CONTROL_WARM_UP, abi.CONTROL_RATE_LIMITER, abi.CONTROL_WARM_UP_RATE_LIMITER
OTHER, RELATE, CHAIN = abi.LIMIT_APP_OTHER, abi.STRATEGY_RELATE, abi.STRATEGY_CHAIN
N_VALUES = 24


def _engine(flags=0):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=1 << 20, flags=flags)


def _flow_rules(rng, r, n_res, n_origins, n_ctx):
    c = lambda lo, hi: float(rng.integers(lo, hi + 1))  # noqa: E731
    o = lambda: int(rng.integers(1, n_origins + 1))      # noqa: E731
    other = lambda: int((r + 1 + rng.integers(0, n_res - 1)) % n_res)  # noqa: E731
    shape = int(rng.integers(0, 12))
    if shape == 0:
        return [local_flow_rule(r, c(5, 40))]                                                # fast path
    if shape == 1:
        return [local_flow_rule(r, c(10, 60), behavior=WU, warm_up_sec=int(rng.integers(2, 8)))]
    if shape == 2:
        return [local_flow_rule(r, c(10, 80), behavior=RL, max_queueing_ms=int(rng.integers(20, 400)))]
    if shape == 3:
        return [local_flow_rule(r, c(20, 60)), local_flow_rule(r, c(2, 15), limit_app=o())]
    if shape == 4:
        return [local_flow_rule(r, c(5, 20), limit_app=OTHER), local_flow_rule(r, c(30, 80))]
    if shape == 5:
        return [local_flow_rule(r, c(2, 8), grade=abi.FLOW_GRADE_THREAD), local_flow_rule(r, c(10, 40))]
    if shape == 6:                                                                            # CHAIN
        return [local_flow_rule(r, c(3, 12), strategy=CHAIN, ref=int(rng.integers(0, n_ctx))), local_flow_rule(r, c(20, 60))]
    if shape == 7:                                                                            # RELATE
        return [local_flow_rule(r, c(5, 30), strategy=RELATE, ref=other())]
    if shape == 8:                                                                            # RELATE + origin
        return [local_flow_rule(r, c(5, 30), strategy=RELATE, ref=other(), limit_app=o()),
                local_flow_rule(r, c(20, 50), behavior=RL, max_queueing_ms=150)]
    if shape == 9:                                                                            # cluster mode
        return [local_flow_rule(r, c(5, 30), cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=r + 1),
                local_flow_rule(r, c(1, 3), cluster_mode=abi.CLUSTER_MODE_NO_FALLBACK, cluster_config=r + 1000),
                local_flow_rule(r, c(20, 80))]
    if shape == 10:                                                                           # CHAIN + WarmUp
        return [local_flow_rule(r, c(10, 40), strategy=CHAIN, ref=int(rng.integers(0, n_ctx)), behavior=WU,
                                warm_up_sec=3)]
    return []


def _param_rules(rng, n_res):
    out = []
    for r in range(n_res):
        u = rng.random()
        if u < 0.25:
            out.append(prule(res=r, idx=0, count=float(rng.integers(2, 12)), grade=QPS))
        elif u < 0.4:
            out.append(prule(res=r, idx=1, count=float(rng.integers(1, 4)), grade=THREAD))
            out.append(prule(res=r, idx=0, count=float(rng.integers(4, 20)), grade=QPS, dur=2))
        elif u < 0.5:
            out.append(prule(res=r, idx=-1, count=float(rng.integers(5, 20)), grade=QPS, behavior=abi.BEHAVIOR_RATE_LIMITER,
                             max_q=int(rng.integers(0, 300))))
    return np.array(out, abi.PSLOT_RULE_DTYPE)


class Pool:
    """The argument pool every ext record indexes (grows over the batches; the device gets all of it)."""

    def __init__(self):
        self.args = [(0, 0, abi.ARG_NULL, 0)]
        self.values = [0]

    def draw(self, rng, n):
        ext = np.zeros(n, abi.SLOT_EXT_DTYPE)
        for i in range(n):
            if rng.random() < 0.1:
                ext[i]["args_null"] = 1
                continue
            na = int(rng.choice([1, 2, 2, 3]))
            b = len(self.args)
            for _ in range(na):
                u = rng.random()
                if u < 0.1:
                    self.args.append((0, 0, abi.ARG_NULL, 0))
                elif u < 0.3:
                    m = int(rng.integers(1, 4))
                    self.args.append((len(self.values), m, abi.ARG_COLLECTION, 0))
                    self.values += [int(min(rng.zipf(1.3), N_VALUES)) for _ in range(m)]
                else:
                    self.args.append((len(self.values), 1, abi.ARG_VALUE, 0))
                    self.values.append(int(min(rng.zipf(1.3), N_VALUES)))
            ext[i]["arg_begin"], ext[i]["arg_count"] = b, na
        return ext

    def arrays(self):
        return np.array(self.args, abi.PSLOT_ARG_DTYPE), np.array(self.values, np.uint64)


def _setup(rng, n_res, n_origins, n_ctx, flags=0, breakers=True, rule_sets=None, params=None):
    base = np.zeros(n_res, abi.LOCAL_RULE_DTYPE)
    for r in range(n_res):
        brk = [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)] if breakers and r % 4 == 0 else []
        base[r] = local_rule(0.0, abi.FLOW_GRADE_NONE, brk)
    if rule_sets is None:
        rule_sets = [_flow_rules(rng, r, n_res, n_origins, n_ctx) for r in range(n_res)]
    flat = [x for rs in rule_sets for x in rs]
    rng.shuffle(flat)
    frules = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE) if flat else np.zeros(0, abi.LOCAL_FLOW_RULE_DTYPE)
    params = _param_rules(rng, n_res) if params is None else params
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(base)
    kept = ora.load_flow_rules(frules, n_origins, n_ctx)
    ps = ParamFlowSlot(params, n_resources=n_res)
    ora.attach_params(ps)
    eng = _engine(flags)
    eng.local_load_rules(base, 2, 1000, 500)
    assert eng.local_load_flow_rules(frules, n_origins, n_ctx) == kept
    eng.pslot_load_rules(params, n_resources=n_res)
    return ora, ps, eng, frules, params


def _entries(rng, n, n_res, t_start, span, n_origins, zipf=1.0, prio=0.05, multi=0.1):
    e = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    e["ts_ms"] = t_start + np.sort(rng.integers(0, max(span, 1), n))
    e["resource"] = zipf_keys(rng, n_res, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    cnt = np.ones(n, np.int32)
    m = rng.random(n) < multi
    cnt[m] = rng.integers(2, 4, int(m.sum()))
    e["count"] = cnt
    e["resource"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    og = rng.integers(1, n_origins + 1, n).astype(np.int32) if n_origins else np.zeros(n, np.int32)
    og[rng.random(n) < 0.3] = 0
    e["origin"] = og
    return e


def _compare(eng, ora, ps, frules, params, n_res, n_origins, n_ctx, pool):
    for r in range(n_res):
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g), f"second window of {r}:\n{s_o}\nvs\n{s_g}"
        assert np.array_equal(b_o, b_g), f"borrow array of {r}"
        assert np.array_equal(m_o, m_g), f"minute window of {r}"
        assert head[0] == ora.threads(r), f"threads of {r}: {ora.threads(r)} vs {head[0]}"
        for i in range(2):
            st, nr = ora.breaker(r, i)
            if st >= 0:
                assert tuple(head[1 + 6 * i: 6 + 6 * i]) == (st, nr) + ora.breaker_stat(r, i), f"breaker {i} of {r}"
        for o in range(1, n_origins + 1):  # every origin node and DefaultNode, whatever the rules
            so, bo, mo, th, ex = ora.origin_dump(r, o)
            sg, bg, mg, hg, gx = eng.local_origin_state(r, o, with_exists=True)
            assert ex == gx, f"origin {o} node of {r}: exists {ex} vs {gx}"
            assert np.array_equal(so, sg) and np.array_equal(bo, bg) and np.array_equal(mo, mg), \
                f"origin {o} node of {r}"
            assert hg[0] == th, f"origin {o} threads of {r}"
        for c in range(n_ctx):
            so, bo, mo, th, ex = ora.context_dump(r, c)
            sg, bg, mg, hg, gx = eng.local_context_state(r, c, with_exists=True)
            assert ex == gx, f"context {c} node of {r}: exists {ex} vs {gx}"
            assert np.array_equal(so, sg) and np.array_equal(bo, bg) and np.array_equal(mo, mg), \
                f"context {c} node of {r}"
            assert hg[0] == th, f"context {c} threads of {r}"
    for i in range(len(frules)):
        want = ora.controller(i)
        if want is not None:
            assert np.array_equal(want, eng.local_controller(i)), f"controller of rule {i}"
    for ri in range(len(params)):
        assert eng.pslot_param_idx(ri) == ps.param_idx(ri), f"paramIdx of param rule {ri}"
    vals = sorted(set(int(v) for v in pool.values))
    for r in np.unique(params["resource"]):
        for idx in range(3):
            for v in vals:
                assert eng.pslot_thread_count(int(r), idx, v) == ps.thread_count(int(r), idx, v), \
                    f"thread count of resource {r} idx {idx} value {v}"
    for ri in range(len(params)):
        for v in vals:
            f, lt, tk = ps.token_state(ri, v)
            gf, glt, gtk = eng.param_state(ri, v)
            assert (gf, glt if f & 1 else 0, gtk if f & 2 else 0) == (f, lt if f & 1 else 0, tk if f & 2 else 0), \
                f"token state of param rule {ri} value {v}"


def _run(ora, ps, eng, frules, params, n_res, n_origins, n_ctx, batches, seed, pool=None, gen=None, t=None,
         compare=True, rt_hi=40, err=0.05, **kw):
    rng = np.random.default_rng(seed + 1000)
    pool = pool or Pool()
    gen = gen or LocalTraceGen(ora)
    t = t if t is not None else 1_700_000_000_000 + int(rng.integers(0, 1000))
    for n, span in batches:
        ent = _entries(rng, n, n_res, t, span, n_origins, **kw)
        ext = pool.draw(rng, n)
        ext["context"] = rng.integers(0, max(n_ctx, 1), n)
        args, values = pool.arrays()
        rt = rng.integers(0, rt_hi + 1, n).astype(np.int32)
        er = (rng.random(n) < err).astype(np.uint8)
        ev, xo, want = gen.run_ext(ent, ext, rt, er, t + span, args, values)
        got = eng.slot_decide_host(ev, xo, args, values)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            i = bad[0]
            raise AssertionError(f"{len(bad)} results differ; first at {i}: ev={ev[i]} ext={xo[i]} "
                                 f"oracle={want[i]} gpu={got[i]}")
        t += span
    if compare:
        _compare(eng, ora, ps, frules, params, n_res, n_origins, n_ctx, pool)
    return t, pool, gen


@pytest.mark.parametrize("flags", [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mixed_slot_chain(flags, seed):
    rng = np.random.default_rng(seed)
    n_res, n_origins, n_ctx = 36, 3, 3
    ora, ps, eng, fr, params = _setup(rng, n_res, n_origins, n_ctx, flags=flags)
    _run(ora, ps, eng, fr, params, n_res, n_origins, n_ctx, [(15_000, 3000), (15_000, 3000), (8_000, 2000)], seed,
         zipf=0.9)


def test_hot_resources_with_params():
    """A few hot resources take most of the events (long segments on one lane), each with param rules."""
    rng = np.random.default_rng(11)
    n_res = 6
    sets = [[local_flow_rule(0, 400.0), local_flow_rule(0, 40.0, limit_app=1)],
            [local_flow_rule(1, 300.0, behavior=RL, max_queueing_ms=300)],
            [local_flow_rule(2, 50.0, strategy=RELATE, ref=0)],
            [local_flow_rule(3, 30.0, strategy=CHAIN, ref=1)], [local_flow_rule(4, 200.0)], []]
    params = np.array([prule(res=0, idx=0, count=20.0), prule(res=1, idx=1, count=3.0, grade=THREAD),
                       prule(res=2, idx=0, count=15.0, behavior=abi.BEHAVIOR_RATE_LIMITER, max_q=100),
                       prule(res=3, idx=0, count=8.0), prule(res=4, idx=0, count=30.0),  # + the fast-path rule
                       prule(res=5, idx=0, count=5.0)], abi.PSLOT_RULE_DTYPE)
    ora, ps, eng, fr, params = _setup(rng, n_res, 2, 2, rule_sets=sets, params=params)
    _run(ora, ps, eng, fr, params, n_res, 2, 2, [(60_000, 3000), (60_000, 3000)], 11, zipf=1.5)


@pytest.mark.parametrize("env", [{}, {"SG_CXW_MIN": "17"}, {"SG_CXW": "0"}, {"SG_TEST_CXSIDE_POISON": "1"}],
                         ids=["default", "cxw17", "lanes", "cxside_poison"])
@pytest.mark.parametrize("flags", [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY])
def test_dead_periods(flags, env, monkeypatch):
    """Hot cx resources whose window periods saturate, with no prioritized entry and no context tracking: the cx
    walkers' dead periods (the wave walker's chunks, the lane walker's per-entry path) decide the rest of each period —
    origin-limitApp, "other", lone WarmUp and one-QPS-param-rule resources (token buckets and a throttle over Zipf
    values, null and collection arguments among them), with the wave walker on the short classes too (SG_CXW_MIN=17)
    or off (SG_CXW=0); with the side words poisoned before k_lcx_side writes them (SG_TEST_CXSIDE_POISON: a walker
    ordered before that kernel would read garbage slot indices)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SG_DEBUG", "64")  # the wave walker's counters (local.hip cx_wave; results unchanged)
    rng = np.random.default_rng(21)
    n_res, n_origins = 12, 3
    sets = [[local_flow_rule(0, 30.0), local_flow_rule(0, 6.0, limit_app=1)],
            [local_flow_rule(1, 25.0, behavior=WU, warm_up_sec=3)],
            [local_flow_rule(2, 40.0)],
            [local_flow_rule(3, 20.0), local_flow_rule(3, 4.0, limit_app=OTHER)],
            [local_flow_rule(4, 15.0)],
            [local_flow_rule(5, 12.0, behavior=WU, warm_up_sec=2)],
            [local_flow_rule(6, 50.0)],
            [local_flow_rule(7, 8.0), local_flow_rule(7, 2.0, limit_app=2)],
            [local_flow_rule(8, 5.0)], [local_flow_rule(9, 60.0)], [], [local_flow_rule(11, 3.0)]]
    params = np.array([prule(res=2, idx=0, count=8.0), prule(res=4, idx=0, count=3.0, dur=2),
                       prule(res=6, idx=0, count=20.0, behavior=abi.BEHAVIOR_RATE_LIMITER, max_q=50),
                       prule(res=9, idx=1, count=5.0), prule(res=10, idx=0, count=4.0)], abi.PSLOT_RULE_DTYPE)
    ora, ps, eng, fr, params = _setup(rng, n_res, n_origins, 0, flags=flags, rule_sets=sets, params=params)
    _run(ora, ps, eng, fr, params, n_res, n_origins, 0, [(60_000, 3000), (60_000, 2500), (30_000, 4000)], 21,
         zipf=1.2, prio=0.0)
    if flags != abi.FLAG_SERIAL_ONLY and env.get("SG_CXW") != "0":  # the wave walker decided dead chunks
        d = eng.debug_copy(5, np.uint64, 32)
        assert d[20] > 0 and d[23] > 0, f"wave walker segments {d[20]}, dead chunks {d[23]}"


def test_relate_to_a_resource_never_entered():
    """RELATE to a resource with no entry yet: no ClusterNode, the rule passes (even at count 0); once that
    resource is entered, its ClusterNode is read."""
    rng = np.random.default_rng(12)
    sets = [[local_flow_rule(0, 0.0, strategy=RELATE, ref=1)], [], [local_flow_rule(2, 10.0)]]
    ora, ps, eng, fr, params = _setup(rng, 3, 1, 1, rule_sets=sets, params=np.zeros(0, abi.PSLOT_RULE_DTYPE))
    ev = np.zeros(3, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["resource"], ev["count"] = 1_700_000_000_000, [0, 1, 0], 1
    ext = np.zeros(3, abi.SLOT_EXT_DTYPE)
    ext["args_null"] = 1
    want = ora.decide_ext(ev, ext, np.zeros(1, abi.PSLOT_ARG_DTYPE), np.zeros(1, np.uint64))
    got = eng.slot_decide_host(ev, ext, None, None)
    assert np.array_equal(got, want)
    assert want["status"].tolist() == [abi.LOCAL_PASS, abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW]


def test_reload_keeps_origin_and_context_nodes():
    """A flow-rule reload keeps the origin nodes and context DefaultNodes (ClusterNode.originCountMap and
    NodeSelectorSlot's nodes outlive it) and the param state; the new rules read them at once."""
    rng = np.random.default_rng(13)
    n_res, n_origins, n_ctx = 20, 3, 3
    sets = [_flow_rules(rng, r, n_res, n_origins, n_ctx) for r in range(n_res)]
    ora, ps, eng, fr, params = _setup(rng, n_res, n_origins, n_ctx, rule_sets=sets)
    t, pool, gen = _run(ora, ps, eng, fr, params, n_res, n_origins, n_ctx, [(10_000, 2000)], 13)
    # same shapes with new counts, rules shuffled, some resources' rules dropped
    sets2 = []
    for r, rs in enumerate(sets):
        if rng.random() < 0.25:
            sets2.append([])
            continue
        new = []
        for x in rs:
            y = x.copy()
            y["count"] = float(rng.integers(1, 50))
            new.append(y)
        sets2.append(new)
    flat = [x for rs in sets2 for x in rs]
    rng.shuffle(flat)
    fr2 = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE)
    assert eng.local_load_flow_rules(fr2, n_origins, n_ctx) == ora.load_flow_rules(fr2, n_origins, n_ctx)
    _run(ora, ps, eng, fr2, params, n_res, n_origins, n_ctx, [(10_000, 2000), (10_000, 2000)], 14, pool=pool, gen=gen,
         t=t)


@pytest.mark.parametrize("seed", [21, 22])
def test_reload_adds_origin_and_chain_rules_to_plain_resources(seed):
    """Resources that had only the fast path's one rule (or none) get limitApp-origin, THREAD-grade origin, "other"
    and CHAIN rules mid-stream, with entries in flight across the reload. The origin nodes and the DefaultNodes have
    counted every event since the resources' first entries (ClusterBuilderSlot.java:99-102, NodeSelectorSlot
    .java:156-170), so the new rules read the windows and curThreadNum the reference's nodes hold — including
    threads of entries admitted before the reload that exit after it."""
    rng = np.random.default_rng(seed)
    n_res, n_origins, n_ctx = 24, 3, 3
    plain = [[local_flow_rule(r, float(rng.integers(20, 80)))] if r % 3 else [] for r in range(n_res)]
    ora, ps, eng, fr, params = _setup(rng, n_res, n_origins, n_ctx, rule_sets=plain,
                                      params=np.zeros(0, abi.PSLOT_RULE_DTYPE), breakers=False)
    # long response times keep entries in flight across the reload
    t, pool, gen = _run(ora, ps, eng, fr, params, n_res, n_origins, n_ctx, [(12_000, 2000), (12_000, 2000)], seed,
                        rt_hi=900)
    o = lambda: int(rng.integers(1, n_origins + 1))  # noqa: E731
    sets2 = []
    for r in range(n_res):
        u = r % 6
        if u == 0:
            sets2.append([local_flow_rule(r, float(rng.integers(1, 4)), grade=abi.FLOW_GRADE_THREAD, limit_app=o()),
                          local_flow_rule(r, 60.0)])
        elif u == 1:
            sets2.append([local_flow_rule(r, float(rng.integers(2, 10)), limit_app=o())])
        elif u == 2:
            sets2.append([local_flow_rule(r, float(rng.integers(2, 6)), grade=abi.FLOW_GRADE_THREAD, limit_app=OTHER)])
        elif u == 3:
            sets2.append([local_flow_rule(r, float(rng.integers(2, 10)), strategy=CHAIN, ref=int(rng.integers(0, n_ctx)))])
        elif u == 4:
            sets2.append([local_flow_rule(r, float(rng.integers(1, 4)), grade=abi.FLOW_GRADE_THREAD, strategy=CHAIN,
                                          ref=int(rng.integers(0, n_ctx))), local_flow_rule(r, 5.0, limit_app=o())])
        else:
            sets2.append(plain[r])
    flat = [x for rs in sets2 for x in rs]
    rng.shuffle(flat)
    fr2 = np.array(flat, abi.LOCAL_FLOW_RULE_DTYPE)
    assert eng.local_load_flow_rules(fr2, n_origins, n_ctx) == ora.load_flow_rules(fr2, n_origins, n_ctx)
    _run(ora, ps, eng, fr2, params, n_res, n_origins, n_ctx, [(12_000, 2000), (12_000, 2000)], seed + 50, pool=pool,
         gen=gen, t=t, rt_hi=900)


def test_origins_declared_later_and_context_tracking_contract():
    """Origin ids can be declared at a later load (no earlier event could carry them, so the origin nodes are exact
    from their first event); context tracking cannot start after a batch (the DefaultNodes would miss the entries
    before it): SG_E_UNSUPPORTED on the device and in the oracle."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(23)
    n_res = 10
    plain = [[local_flow_rule(r, 30.0)] for r in range(n_res)]
    ora, ps, eng, fr, params = _setup(rng, n_res, 0, 0, rule_sets=plain, params=np.zeros(0, abi.PSLOT_RULE_DTYPE))
    t, pool, gen = _run(ora, ps, eng, fr, params, n_res, 0, 0, [(5_000, 1500)], 23, rt_hi=600)
    with pytest.raises(EngineError) as ei:
        eng.local_load_flow_rules(fr, 0, 2)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    with pytest.raises(ValueError, match=str(abi.SG_E_UNSUPPORTED)):
        ora.load_flow_rules(fr, 0, 2)
    fr2 = np.array([local_flow_rule(r, 3.0, grade=abi.FLOW_GRADE_THREAD, limit_app=1 + r % 2) for r in range(n_res)] +
                   [local_flow_rule(r, 40.0) for r in range(n_res)], abi.LOCAL_FLOW_RULE_DTYPE)
    assert eng.local_load_flow_rules(fr2, 2, 0) == ora.load_flow_rules(fr2, 2, 0)
    _run(ora, ps, eng, fr2, params, n_res, 2, 0, [(5_000, 1500), (5_000, 1500)], 24, pool=pool, gen=gen, t=t, rt_hi=600)


def test_cluster_state_contract():
    """Cluster-mode rules are decided on a node that is neither token client nor server, or on an embedded token
    server (tests/test_embedded_server_gpu.py); a token client's tokens come over the network: unsupported."""
    from sentinel_amd.engine import EngineError
    eng = _engine()
    eng.local_load_rules(np.array([local_rule()]), 2, 1000, 500)
    cr = np.array([local_flow_rule(0, 5.0, cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=1)])
    assert eng.local_load_flow_rules(cr) == 1
    with pytest.raises(EngineError) as ei:
        eng.local_set_cluster_state(abi.CLUSTER_CLIENT)
    assert ei.value.code == abi.SG_E_UNSUPPORTED
    eng.local_set_cluster_state(abi.CLUSTER_SERVER)
    eng.local_load_flow_rules(np.array([local_flow_rule(0, 5.0)]))
    eng.local_set_cluster_state(abi.CLUSTER_CLIENT)
    with pytest.raises(EngineError) as ei:
        eng.local_load_flow_rules(cr)
    assert ei.value.code == abi.SG_E_UNSUPPORTED


def test_out_of_range_context_and_args_rejected():
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(14)
    ora, ps, eng, fr, params = _setup(rng, 4, 1, 2, params=np.array([prule(res=0, idx=0, count=5.0)],
                                                                     abi.PSLOT_RULE_DTYPE))
    ev = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"] = 1000, 1
    ext = np.zeros(1, abi.SLOT_EXT_DTYPE)
    ext["context"] = 2
    with pytest.raises(EngineError) as ei:
        eng.slot_decide_host(ev, ext, None, None)
    assert ei.value.code == abi.SG_E_INVAL
    ext["context"], ext["arg_begin"], ext["arg_count"] = 0, 0, 3          # args beyond the (empty) arg array
    with pytest.raises(EngineError) as ei:
        eng.slot_decide_host(ev, ext, None, None)
    assert ei.value.code == abi.SG_E_INVAL
