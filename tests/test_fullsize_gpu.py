"""Full-size parity: every BASELINE.json configuration at the size bench.py / bench_configs.py time it,
decided on the device through the C ABI and compared bit-exactly with the oracle's sequential replay.

  C1  HelloWorld: one resource, QPS FlowRule count=20, S=2/1000 ms + minute window, 1M entries (Poisson
      arrivals at 1000/s over 1000 s, FlowQpsDemo.java:45-70 / README.md:96-121), each passed entry exits at
      once; plus the behavioural bound the README shows (<= 20 passes per second).
  C2  10k resources x QPS FlowRule (count U{1..64}), 16M entries per 1000 ms batch, Zipf(1.0), two batches.
  C3  1M flowIds x ClusterFlowRule (GLOBAL, count U{1..32}, S=10/1000 ms), 16M requests per batch (Zipf 1.0,
      1 % prioritized, 10 % acquire U{2..4}), two batches, every result and every flowId's window; then the
      same config with the namespace limiter on (maxAllowedQps 1e12 as SURVEY §8d specifies, and a binding cap).
  C4  one ParamFlowRule (count 5, 1 s) over 10M distinct values (Zipf 1.1) in a 2^25-slot table, 16M requests.
  C5  1M resources x (QPS FlowRule + RT breaker + exception-ratio breaker), 16M entries + the exits of the
      passed ones (rt lognormal, 5 % errors), one batch.

The oracle's C3 replay is sharded by flowId over the host's threads (flowIds share no state without a
namespace limiter, so per-shard sequential replay equals the global one); every other oracle run is a single
sequential replay. Sizes are the BASELINE ones, so this file takes a few minutes on the GPU box.
"""
import os

import numpy as np
import pytest

from oracle.binding import (LocalChain, LocalTraceGen, ClusterTokenService, ParamFlowChecker,
                            ShardedClusterTokenService, degrade_rule)
from sentinel_amd import abi
from sentinel_amd.workload import ClusterWorkload, zipf_keys

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
N_BIG = 16_000_000


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def _engine(max_batch, **kw):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max_batch, **kw)


def _same(want, got, what, ctx=None):
    if not np.array_equal(want, got):
        bad = np.nonzero(want != got)[0]
        i = bad[0]
        extra = f" input={ctx[i]}" if ctx is not None else ""
        raise AssertionError(f"{what}: {len(bad)} of {len(want)} differ; first at {i}: oracle={want[i]} gpu={got[i]}{extra}")


def _ns(limiter=False, qps=30000.0):
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["limiter_enabled"] = 1 if limiter else 0
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = qps
    return ns


def _compare_flow_state(eng, ora_ring, ora_occ, K):
    ring, occ = eng.export_state(K)
    assert ring.shape == ora_ring.shape
    # counters of never-created slots are not state (the Java slot is null)
    live_o = ora_ring[:, :, 0] != abi.INT64_MIN
    live_g = ring[:, :, 0] != abi.INT64_MIN
    _same(live_o.reshape(-1), live_g.reshape(-1), "created buckets")
    m = live_o[:, :, None]
    diff = np.nonzero(((np.where(m, ora_ring, 0) != np.where(m, ring, 0)).any(axis=(1, 2))))[0]
    assert diff.size == 0, f"{diff.size} flowIds' windows differ, first {diff[0]}:\n{ora_ring[diff[0]]}\nvs\n{ring[diff[0]]}"
    _same(ora_occ.reshape(-1), occ.reshape(-1), "occupy counters")


# ------------------------------------------------------------------------------------------------ C3

def test_c3_full_size_two_batches():
    wl = ClusterWorkload(n_flows=1_000_000, n_requests=N_BIG)
    rules, ns = wl.rules(), _ns()
    eng = _engine(N_BIG)
    eng.set_namespaces(ns)
    eng.load_rules(rules)
    ora = ShardedClusterTokenService(rules, ns, _threads())
    try:
        for b in range(2):
            req = wl.requests(b)
            want = ora.decide(req)
            got = eng.decide_host(req)
            _same(want, got, f"C3 batch {b} results", req)
            st = want["status"]
            # the workload exercises every outcome of ClusterFlowChecker
            assert (st == abi.OK).any() and (st == abi.BLOCKED).any() and (st == abi.SHOULD_WAIT).any()
        ring, occ = ora.export_state(eng.state_stride())
        _compare_flow_state(eng, ring, occ, len(rules))
    finally:
        ora.close()


@pytest.mark.parametrize("qps", [1e12, 6e6])
def test_c3_full_size_namespace_limiter(qps):
    """SURVEY §8d C3's second run: the GlobalRequestLimiter pre-pass on (1e12 admits everything but still runs
    the exact per-100 ms quota arithmetic; 6e6 < 16M/s makes it bind: TOO_MANY_REQUEST leaves flows untouched)."""
    wl = ClusterWorkload(n_flows=1_000_000, n_requests=N_BIG, seed=31)
    rules, ns = wl.rules(), _ns(limiter=True, qps=qps)
    eng = _engine(N_BIG)
    eng.set_namespaces(ns)
    eng.load_rules(rules)
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    req = wl.requests(0)
    want = ora.decide(req)
    got = eng.decide_host(req)
    _same(want, got, "C3 + limiter results", req)
    n_tmr = int((want["status"] == abi.TOO_MANY_REQUEST).sum())
    assert (n_tmr == 0) if qps > 1e9 else (n_tmr > N_BIG // 2)
    ring, occ = ora.export_state(len(rules), eng.state_stride())
    _compare_flow_state(eng, ring, occ, len(rules))


# ------------------------------------------------------------------------------------------------ C2

def test_c2_full_size_10k_resources():
    K = 10_000
    rng = np.random.default_rng(2)
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    eng = _engine(N_BIG)
    eng.local_load_rules(rules, 2, 1000, 500)
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(rules)
    for b in range(2):
        ev = np.zeros(N_BIG, abi.LOCAL_EVENT_DTYPE)
        ev["ts_ms"] = T0 + 1000 * b + np.sort(rng.integers(0, 1000, N_BIG))
        ev["resource"] = zipf_keys(rng, K, N_BIG, 1.0, perm_seed=2)
        c = np.ones(N_BIG, np.int32)
        m = rng.random(N_BIG) < 0.1
        c[m] = rng.integers(2, 5, int(m.sum()))
        ev["count"] = c
        want = ora.decide(ev)
        got = eng.local_decide_host(ev)
        _same(want, got, f"C2 batch {b} results", ev)
    for r in range(K):
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g) and np.array_equal(b_o, b_g) and np.array_equal(m_o, m_g), f"resource {r}"
        assert head[0] == ora.threads(r)


# ------------------------------------------------------------------------------------------------ C1

def test_c1_helloworld_qps20():
    """FlowQpsDemo: 'HelloWorld' QPS=20 (README.md:96-121 shows ~20 passes per second). Every entry that
    passes exits immediately (the demo's finally { entry.exit() })."""
    rng = np.random.default_rng(1)
    n = 1_000_000
    gaps = rng.exponential(1.0, n)                      # Poisson arrivals at 1000/s
    ts = T0 + np.floor(np.cumsum(gaps)).astype(np.int64)
    ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    ent["ts_ms"] = ts
    ent["count"] = 1
    rules = np.zeros(1, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = 20.0
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    eng = _engine(2 * n + 16)
    eng.local_load_rules(rules, 2, 1000, 500)
    t_end = int(ts[-1]) + 1
    ev, want = gen.run(ent, np.zeros(n, np.int32), np.zeros(n, np.uint8), t_end)
    # 100 s batches, state carried
    bounds = np.searchsorted(ev["ts_ms"], T0 + 100_000 * np.arange(1, 11))
    lo = 0
    for hi in list(bounds) + [len(ev)]:
        if hi > lo:
            _same(want[lo:hi], eng.local_decide_host(ev[lo:hi]), "C1 results", ev[lo:hi])
        lo = hi
    s_o, b_o, m_o = ora.dump(0)
    s_g, b_g, m_g, _ = eng.local_state(0)
    assert np.array_equal(s_o, s_g) and np.array_equal(m_o, m_g)
    # behaviour: the second window is 2 x 500 ms buckets; every entry is checked against both buckets, so the
    # passes of any two consecutive buckets -- every aligned 1000 ms span [500 k, 500 k + 1000) -- are <= 20
    # (a sliding window of arbitrary alignment can hold up to 40: 20 at the end of one bucket pair, 20 more
    # at the start of the next).
    entries = ev["kind"] == abi.LOCAL_ENTRY
    passed = entries & (want["status"] == abi.LOCAL_PASS)
    half = (ev["ts_ms"][passed] - T0) // 500
    per_half = np.bincount(half)
    pair = per_half[:-1] + per_half[1:]
    assert pair.max() <= 20
    per_sec = np.bincount((ev["ts_ms"][passed] - T0) // 1000)
    assert per_sec.max() <= 20 and np.median(per_sec) == 20  # ~1000 arrivals/s: every second saturates


# ------------------------------------------------------------------------------------------------ C4

def test_c4_full_size_10m_values():
    V, n = 10_000_000, N_BIG
    rng = np.random.default_rng(4)
    rules = np.zeros(1, abi.PARAM_RULE_DTYPE)
    rules["count"], rules["duration_sec"], rules["behavior"], rules["capacity_log2"] = 5, 1, abi.BEHAVIOR_DEFAULT, 25
    eng = _engine(n)
    eng.param_load_rules(rules)
    ora = ParamFlowChecker()
    ora.load_rules(rules)
    keys = zipf_keys(rng, V, n, 1.1, perm_seed=4).astype(np.uint64)
    req = np.zeros(n, abi.PARAM_REQ_DTYPE)
    req["ts_ms"] = T0 + np.sort(rng.integers(0, 1000, n))
    req["value"] = keys * np.uint64(0x9E3779B1) + np.uint64(17)
    req["rule"] = 0
    req["acquire"] = 1
    want = ora.decide(req)
    got = eng.param_decide_host(req)
    _same(want, got, "C4 pass bits", req)
    assert 0 < want.sum() < n
    vals = np.unique(req["value"])
    sample = np.concatenate([vals[:: max(1, len(vals) // 5000)], req["value"][:200]])
    for v in sample:
        assert ora.state(0, int(v)) == eng.param_state(0, int(v)), f"value {v}"


# ------------------------------------------------------------------------------------------------ C5

def test_c5_full_size_1m_resources_breakers():
    K, n = 1_000_000, N_BIG
    rng = np.random.default_rng(5)
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    rules["n_breakers"] = 2
    b = np.zeros(2, abi.DEGRADE_RULE_DTYPE)
    b[0] = degrade_rule(abi.DEGRADE_RT, 100, 10, 5, 1000, 0.5)
    b[1] = degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.5, 10, 5, 1000)
    rules["breakers"] = b
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    ent["ts_ms"] = T0 + np.sort(rng.integers(0, 1000, n))
    ent["resource"] = zipf_keys(rng, K, n, 1.0, perm_seed=5)
    ent["count"] = 1
    rt = np.minimum(np.round(np.exp(rng.normal(2.5, 0.8, n))), 10_000).astype(np.int32)
    err = (rng.random(n) < 0.05).astype(np.uint8)
    ev, want = gen.run(ent, rt, err, T0 + 1000)
    eng = _engine(len(ev))
    eng.local_load_rules(rules, 2, 1000, 500)
    got = eng.local_decide_host(ev)
    _same(want, got, "C5 results", ev)
    assert (ev["kind"] != abi.LOCAL_ENTRY).sum() > 100_000
    res = ev["resource"] & abi.KEY_INDEX
    hot = np.argsort(np.bincount(res, minlength=K))[::-1][:300]
    sample = np.unique(np.concatenate([hot, rng.integers(0, K, 1500)]))
    for r in sample:
        r = int(r)
        s_o, b_o, m_o = ora.dump(r)
        s_g, b_g, m_g, head = eng.local_state(r)
        assert np.array_equal(s_o, s_g) and np.array_equal(m_o, m_g), f"windows of resource {r}"
        assert head[0] == ora.threads(r)
        for i in range(2):
            st, nr = ora.breaker(r, i)
            start, bad, total = ora.breaker_stat(r, i)
            assert tuple(head[1 + 6 * i: 6 + 6 * i]) == (st, nr, start, bad, total), f"breaker {i} of {r}"
