"""Parity of the HIP engine (through the C ABI) with the oracle: bit-exact TokenResults and windows.

Every case replays the same seeded trace through oracle.binding.ClusterTokenService (sequential
restatement of DefaultTokenService → ClusterFlowChecker) and through libsentinel_gpu.so, then compares
every (status, remaining, waitInMs) and every flowId's bucket ring + occupy counters.
"""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.workload import ClusterWorkload, zipf_keys

pytestmark = pytest.mark.gpu


# default split, every flow serial, every flow by a wave, short walker re-reading the ring (no register snapshot)
WALKERS = [0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY, abi.FLAG_RING_REREAD]


def _engine(max_batch=1 << 20, exceed=1.0, occ_ratio=1.0, flags=0):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max_batch, exceed_count=exceed, max_occupy_ratio=occ_ratio, flags=flags)


def _ns(connected=1):
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = connected
    ns["max_allowed_qps"] = 30000
    return ns


def _pair(rules, ns=None, exceed=1.0, occ_ratio=1.0, max_batch=1 << 20, flags=0):
    ns = _ns() if ns is None else ns
    eng = _engine(max_batch, exceed, occ_ratio, flags)
    eng.set_namespaces(ns)
    eng.load_rules(rules)
    ora = ClusterTokenService(exceed, occ_ratio)
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    return eng, ora


def _compare_state(eng, ora, rules, keys=None):
    keys = range(len(rules)) if keys is None else keys
    for k in keys:
        s_o, c_o, o_o = ora.read_state(int(k))
        s_g, c_g, o_g = eng.read_state(int(k), len(s_o))
        assert np.array_equal(s_o, s_g), f"starts differ for key {k}: {s_o} vs {s_g}"
        assert np.array_equal(c_o, c_g), f"counters differ for key {k}:\n{c_o}\nvs\n{c_g}"
        assert np.array_equal(o_o, o_g), f"occupy differs for key {k}: {o_o} vs {o_g}"


def _compare_results(out_o, out_g, req):
    if not np.array_equal(out_o, out_g):
        bad = np.nonzero(out_o != out_g)[0]
        i = bad[0]
        raise AssertionError(f"{len(bad)} results differ; first at {i}: req={req[i]} oracle={out_o[i]} gpu={out_g[i]}")


def _rules(n, rng, counts=None, S=10, interval=1000, thr_type=abi.THRESHOLD_GLOBAL):
    r = np.zeros(n, abi.RULE_DTYPE)
    r["flow_id"] = np.arange(1, n + 1) * 7 + 100
    r["count"] = rng.integers(1, 33, n) if counts is None else counts
    r["threshold_type"] = thr_type
    r["sample_count"] = S
    r["window_interval_ms"] = interval
    return r


def _trace(rng, n, n_keys, t_start, span, zipf=1.0, prio=0.01, multi=0.1, big=0.0):
    req = np.zeros(n, abi.REQ_DTYPE)
    req["ts_ms"] = t_start + np.sort(rng.integers(0, max(span, 1), n))
    req["key"] = zipf_keys(rng, n_keys, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    acq = np.ones(n, np.int32)
    m = rng.random(n) < multi
    acq[m] = rng.integers(2, 5, int(m.sum()))
    b = rng.random(n) < big
    acq[b] = rng.integers(1, 2**31 - 1, int(b.sum()))
    req["acquire"] = acq
    req["key"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    return req


@pytest.mark.parametrize("flags", WALKERS)
def test_cluster_flow_checker_occupy_pass_gpu(t0, flags):
    """The hand-traced ClusterFlowCheckerTest sequence (tests/test_oracle_kat.py), one request per batch
    (state carried across batches) and again as a single batch."""
    rules = _rules(1, np.random.default_rng(0), counts=np.array([5.0]), S=5, interval=1000)
    steps = [(0, False), (0, False), (200, False), (400, True), (400, False), (400, True), (600, False),
             (600, False), (800, False), (800, True), (800, False), (1000, False)]
    req = np.zeros(len(steps), abi.REQ_DTYPE)
    for i, (dt, p) in enumerate(steps):
        req[i] = (t0 + dt, abi.KEY_PRIO if p else 0, 1)
    want = [(0, 4, 0), (0, 3, 0), (0, 2, 0), (0, 1, 0), (0, 0, 0), (1, 0, 0), (1, 0, 0), (1, 0, 0), (1, 0, 0),
            (2, 0, 200), (1, 0, 0), (0, 0, 0)]
    eng, ora = _pair(rules, flags=flags)
    got = [tuple(eng.decide_host(req[i:i + 1])[0]) for i in range(len(req))]
    assert got == want
    eng2, _ = _pair(rules, flags=flags)
    assert [tuple(x) for x in eng2.decide_host(req)] == want
    ora.decide(req)
    _compare_state(eng, ora, rules)
    _compare_state(eng2, ora, rules)


@pytest.mark.parametrize("n_keys,n,zipf,prio,S,interval", [
    (1, 1000, 1.0, 0.0, 10, 1000),
    (1, 5000, 1.0, 0.3, 10, 1000),
    (7, 20_000, 1.2, 0.05, 5, 1000),
    (100, 50_000, 1.0, 0.01, 10, 1000),
    (1000, 100_000, 1.0, 0.01, 10, 1000),
    (3000, 60_000, 0.6, 0.5, 2, 1000),
    (50, 30_000, 1.0, 1.0, 10, 1000),
    (20, 30_000, 1.0, 0.2, 1, 1000),
    (20, 30_000, 1.0, 0.2, 64, 6400),
    (40, 30_000, 1.1, 0.2, 3, 1500),
    (40, 30_000, 1.1, 0.2, 5, 25),
    (40, 30_000, 1.1, 0.2, 60, 60000),
    (40, 30_000, 1.1, 0.2, 4, 2000),   # power-of-two intervals other than 1 s: the average's exact-reciprocal path
    (40, 30_000, 1.1, 0.2, 2, 500),
])
@pytest.mark.parametrize("flags", WALKERS)
def test_random_traces_match_oracle(n_keys, n, zipf, prio, S, interval, flags):
    rng = np.random.default_rng(n_keys * 1000 + n + S)
    rules = _rules(n_keys, rng, S=S, interval=interval)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_017
    for batch in range(3):
        span = int(rng.integers(1, 3 * interval))
        req = _trace(rng, n, n_keys, t, span, zipf=zipf, prio=prio)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 2 * interval))
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


@pytest.mark.parametrize("seg_mark,csum", [("0", "1"), ("1", "0"), ("0", "0")])
def test_sort_variants(monkeypatch, seg_mark, csum):
    """The non-default sort paths stay exact: segment marks fused into the last scatter pass (SG_SEG_MARK=0) and the
    k_colsum pass instead of the histogram kernels' atomic column sums (SG_CSUM_ATOMIC=0)."""
    monkeypatch.setenv("SG_SEG_MARK", seg_mark)
    monkeypatch.setenv("SG_CSUM_ATOMIC", csum)
    rng = np.random.default_rng(int(seg_mark) * 2 + int(csum) + 90)
    rules = _rules(3000, rng, S=10, interval=1000)
    eng, ora = _pair(rules)
    t = 1_700_000_000_003
    for batch in range(3):
        req = _trace(rng, 200_000, 3000, t, 1500, zipf=1.0, prio=0.02)
        t = int(req["ts_ms"][-1]) + 7
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


@pytest.mark.parametrize("flags", WALKERS)
def test_fractional_thresholds_and_exceed(flags):
    """Non-integer count and exceedCount: the double comparisons of ClusterFlowChecker.java:67-71."""
    rng = np.random.default_rng(5)
    rules = _rules(64, rng, counts=rng.random(64) * 40 + 0.3, S=4, interval=1000)
    eng, ora = _pair(rules, exceed=1.37, occ_ratio=0.55, flags=flags)
    t = 1_700_000_000_500
    for _ in range(3):
        req = _trace(rng, 40_000, 64, t, 1700, prio=0.3, multi=0.4)
        t = int(req["ts_ms"][-1])
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


def test_avg_local_threshold_and_connected_count():
    rng = np.random.default_rng(6)
    rules = _rules(32, rng, thr_type=abi.THRESHOLD_AVG_LOCAL)
    eng, ora = _pair(rules, ns=_ns(connected=3))
    req = _trace(rng, 20_000, 32, 1_700_000_000_000, 1000, prio=0.1)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    ns0 = _ns(connected=0)
    eng.set_namespaces(ns0)
    ora.set_namespaces(ns0)
    req = _trace(rng, 5_000, 32, 1_700_000_001_000, 1000, prio=0.1)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


@pytest.mark.parametrize("flags", WALKERS)
def test_large_acquire_counts_and_huge_thresholds(flags):
    """acquireCount beyond the packed field (escape path) and thresholds beyond int (remaining saturates)."""
    rng = np.random.default_rng(7)
    counts = np.where(rng.random(16) < 0.5, 1e12, rng.integers(1, 1000, 16).astype(float))
    rules = _rules(16, rng, counts=counts)
    eng, ora = _pair(rules, flags=flags)
    req = _trace(rng, 20_000, 16, 1_700_000_000_000, 1500, prio=0.2, big=0.05)
    out_o = ora.decide(req)
    _compare_results(out_o, eng.decide_host(req), req)
    assert (out_o["remaining"] == 2**31 - 1).any()
    _compare_state(eng, ora, rules)


def test_invalid_requests_interleaved():
    rng = np.random.default_rng(8)
    rules = _rules(10, rng)
    eng, ora = _pair(rules)
    req = _trace(rng, 10_000, 10, 1_700_000_000_000, 1000)
    sel = rng.random(len(req))
    req["acquire"][sel < 0.05] = 0
    req["acquire"][(sel >= 0.05) & (sel < 0.08)] = -7
    req["key"][(sel >= 0.08) & (sel < 0.11)] = abi.KEY_BAD
    req["key"][(sel >= 0.11) & (sel < 0.14)] = abi.KEY_NO_RULE
    req["key"][(sel >= 0.14) & (sel < 0.16)] = 10 | abi.KEY_PRIO
    out_o = ora.decide(req)
    _compare_results(out_o, eng.decide_host(req), req)
    assert set(np.unique(out_o["status"])) >= {abi.BAD_REQUEST, abi.NO_RULE_EXISTS, abi.OK, abi.BLOCKED}
    _compare_state(eng, ora, rules)


def test_timestamp_violations_rejected_without_side_effects():
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(9)
    rules = _rules(10, rng)
    eng, ora = _pair(rules)
    req = _trace(rng, 1000, 10, 1_700_000_000_000, 1000)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    bad = _trace(rng, 1000, 10, 1_700_000_000_500, 100)  # older than the previous batch's last request
    with pytest.raises(EngineError) as ei:
        eng.decide_host(bad)
    assert ei.value.code == abi.SG_E_TIME
    unsorted = _trace(rng, 1000, 10, 1_700_000_002_000, 1000)
    unsorted["ts_ms"][500] -= 300
    with pytest.raises(EngineError):
        eng.decide_host(unsorted)
    # the first request later than the rest by many window periods: every later period lies before the batch's
    # first one (the period tables must not be written below their start)
    first_late = _trace(rng, 1000, 10, 1_700_000_002_000, 1000)
    first_late["ts_ms"][0] += 20_000
    with pytest.raises(EngineError) as ei:
        eng.decide_host(first_late)
    assert ei.value.code == abi.SG_E_TIME
    _compare_state(eng, ora, rules)
    nxt = _trace(rng, 1000, 10, 1_700_000_003_000, 1000)
    _compare_results(ora.decide(nxt), eng.decide_host(nxt), nxt)


def test_rule_reload_keeps_surviving_metrics():
    """ClusterFlowRuleManager.applyClusterFlowRule (:325-375): surviving flowIds keep their metric (even
    with a new window config), new ones start empty, removed ones are dropped."""
    rng = np.random.default_rng(10)
    rules = _rules(20, rng)
    eng, ora = _pair(rules)
    req = _trace(rng, 20_000, 20, 1_700_000_000_000, 800, prio=0.1)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    new = np.concatenate([rules[5:15], _rules(6, rng, S=4, interval=2000)])
    new["flow_id"][10:] += 99_999
    new["sample_count"][:3] = 2          # ignored for surviving flows: their metric keeps S=10
    new["count"] = rng.integers(1, 40, len(new))
    eng.load_rules(new)
    ora.load_rules(new)
    req = _trace(rng, 20_000, len(new), 1_700_000_000_900, 1500, prio=0.1)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, new)


@pytest.mark.parametrize("flags", WALKERS)
def test_hot_flow_long_segment_prio_heavy(flags):
    """One flow taking most of the traffic: the wave walker's admit / skip / occupy modes."""
    rng = np.random.default_rng(11)
    rules = _rules(3, rng, counts=np.array([25.0, 3.0, 1000.0]), S=10, interval=1000)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_000
    for _ in range(4):
        req = _trace(rng, 120_000, 3, t, 2500, zipf=2.0, prio=0.35, multi=0.5)
        t = int(req["ts_ms"][-1]) + 50
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


@pytest.mark.parametrize("flags", WALKERS)
def test_north_star_shape_small(flags):
    """The C3 workload shape (Zipf(1.0), counts U{1..32}, S=10/1000 ms, 1 % prioritized) at 20k flows."""
    wl = ClusterWorkload(n_flows=20_000, n_requests=400_000, seed=12)
    rules = wl.rules()
    eng, ora = _pair(rules, flags=flags)
    for b in range(2):
        req = wl.requests(b)
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules, keys=range(0, len(rules), 7))


def test_snapshot_matches_oracle_avg():
    rng = np.random.default_rng(13)
    rules = _rules(50, rng, S=5, interval=1000)
    eng, ora = _pair(rules)
    req = _trace(rng, 30_000, 50, 1_700_000_000_000, 1800, prio=0.3)
    ora.decide(req)
    eng.decide_host(req)
    now = int(req["ts_ms"][-1]) + 150
    snap = eng.snapshot(now, len(rules))
    for k in range(len(rules)):
        assert snap[k, 0] == ora.avg(k, now, abi.EV_PASS)
        assert snap[k, 1] == ora.avg(k, now, abi.EV_BLOCK)


def _host_records(req, n_rules, max_batch):
    kbits = max(1, int(n_rules).bit_length())
    ibits = int(max_batch - 1).bit_length()
    abits = min(8, 64 - kbits - ibits)  # acquire field: 7 bits + prio, larger acquires escape to the request
    key = (req["key"] & abi.KEY_INDEX).astype(np.uint64)
    bad = (key == abi.KEY_BAD) | (req["acquire"] <= 0)
    norule = (~bad) & (key >= n_rules)
    acq = np.minimum(req["acquire"].astype(np.int64), (1 << (abits - 1)) - 1).astype(np.uint64)
    ac = (acq << np.uint64(1)) | (req["key"] >> np.uint64(31)).astype(np.uint64)
    rec = (key << np.uint64(64 - kbits)) | (np.arange(len(req), dtype=np.uint64) << np.uint64(abits)) | ac
    rec[bad | norule] = np.uint64(n_rules) << np.uint64(64 - kbits)
    return rec, 64 - kbits


@pytest.mark.parametrize("n_keys,n", [(1, 100), (7, 20_000), (3000, 4096 * 3 + 17), (1 << 20, 300_000)])
def test_radix_sort_is_stable_partition_by_flow(n_keys, n):
    """The hand-written LSD radix sort (sort.hip) against numpy's stable argsort of the same records."""
    rng = np.random.default_rng(n_keys + n)
    rules = _rules(n_keys, rng)
    max_batch = 1 << 20
    eng, _ = _pair(rules, max_batch=max_batch)
    req = _trace(rng, n, n_keys, 1_700_000_000_000, 1000, zipf=1.1)
    req["key"][rng.random(n) < 0.01] = abi.KEY_NO_RULE
    eng.decide_host(req)
    rec, kshift = _host_records(req, n_keys, max_batch)
    want = rec[np.argsort(rec >> np.uint64(kshift), kind="stable")]
    got = eng.debug_copy(1, np.uint64, n)
    assert_stable_partition(got, want, kshift)


def assert_stable_partition(got, want, kshift):
    """`got` holds every flowId's records contiguous and in arrival order (the two-pass sort: in flowId order; the binned
    front half: regular bins in flowId order, then one segment per hot flowId)."""
    keys = got >> np.uint64(kshift)
    runs = 1 + int(np.count_nonzero(keys[1:] != keys[:-1])) if len(keys) else 0
    assert runs == len(np.unique(keys)), "a flowId's records are split"
    assert np.array_equal(got[np.argsort(keys, kind="stable")], want)


def _ns_multi(specs):
    """specs: list of (limiter_enabled, max_allowed_qps, connected_count)."""
    ns = np.zeros(len(specs), abi.NS_DTYPE)
    for i, (en, q, c) in enumerate(specs):
        ns[i] = (1 if en else 0, c, q)
    return ns


@pytest.mark.parametrize("flags", WALKERS)
@pytest.mark.parametrize("qps", [0.0, 1.0, 7.5, 300.0, 5000.0, 1e12])
def test_namespace_limiter_matches_oracle(qps, flags):
    """GlobalRequestLimiter.tryPass (GlobalRequestLimiter.java:46-55) before every flow check:
    TOO_MANY_REQUEST leaves the flow metric untouched; the limiter window persists across batches."""
    rng = np.random.default_rng(int(qps * 10) % 1000 + 31)
    rules = _rules(200, rng, counts=rng.integers(1, 200, 200).astype(float))
    rules["namespace_id"] = rng.integers(0, 3, len(rules))
    ns = _ns_multi([(True, qps, 1), (False, 0, 2), (True, qps * 2 + 3, 1)])
    eng, ora = _pair(rules, ns=ns, flags=flags)
    t = 1_700_000_000_050
    for _ in range(3):
        req = _trace(rng, 30_000, 200, t, int(rng.integers(50, 2500)), prio=0.05)
        req["key"][rng.random(len(req)) < 0.02] = abi.KEY_NO_RULE
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 700))
        out_o = ora.decide(req)
        _compare_results(out_o, eng.decide_host(req), req)
    _compare_state(eng, ora, rules)
    if 0 < qps < 1e6:
        assert (out_o["status"] == abi.TOO_MANY_REQUEST).any()


def test_namespace_limiter_config_changes():
    """applyMaxQpsChange keeps the window; switching a limiter off and on again starts it empty."""
    rng = np.random.default_rng(41)
    rules = _rules(50, rng)
    rules["namespace_id"] = rng.integers(0, 2, len(rules))
    eng, ora = _pair(rules, ns=_ns_multi([(True, 40, 1), (True, 900, 1)]))
    t = 1_700_000_000_000
    for cfg in ([(True, 40, 1), (True, 900, 1)], [(True, 55.5, 1), (True, 10, 1)],
                [(False, 0, 1), (True, 10, 1)], [(True, 20, 1), (True, 10, 1)]):
        ns = _ns_multi(cfg)
        eng.set_namespaces(ns)
        ora.set_namespaces(ns)
        req = _trace(rng, 8000, 50, t, 900, prio=0.1)
        t = int(req["ts_ms"][-1]) + 30
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


@pytest.mark.parametrize("prio", [0.0, 0.01, 0.2])
def test_hot_flow_saturated_periods_are_skipped_exactly(prio):
    """A flow far above its threshold: once a window period can admit nothing (not even acquire 1, and no
    prioritized request can occupy), the wave walker jumps to the period's end and k_skip_apply adds the
    skipped requests' BLOCK counts. Results and windows must still match the sequential replay."""
    rng = np.random.default_rng(int(prio * 100) + 77)
    rules = _rules(3, rng, counts=np.array([10.0, 2.0, 7.5]), S=10, interval=1000)
    eng, ora = _pair(rules, flags=abi.FLAG_WAVE_ONLY)
    eng.enable_stats(True)
    t = 1_700_000_000_010
    skipped = 0
    for _ in range(3):
        req = _trace(rng, 300_000, 3, t, 2300, zipf=1.5, prio=prio, multi=0.2)
        t = int(req["ts_ms"][-1]) + 1
        _compare_results(ora.decide(req), eng.decide_host(req), req)
        skipped += eng.stats()["skipped_ranges"]
        _compare_state(eng, ora, rules)
    assert skipped > 0


@pytest.mark.parametrize("n_keys,n,S", [(1000, 100_000, 10), (3000, 60_000, 2), (200_000, 400_000, 10)])
def test_tiny_walker_opt_in_matches_oracle(monkeypatch, n_keys, n, S):
    """SG_DEBUG=128 walks length class 0 with k_walk_tiny (off by default: slower in the r03 A/B)."""
    monkeypatch.setenv("SG_DEBUG", "128")
    rng = np.random.default_rng(n_keys + n)
    rules = _rules(n_keys, rng, S=S)
    eng, ora = _pair(rules)
    t = 1_700_000_000_017
    for _ in range(3):
        req = _trace(rng, n, n_keys, t, int(rng.integers(1, 3000)), zipf=0.8, prio=0.05)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 2000))
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)
