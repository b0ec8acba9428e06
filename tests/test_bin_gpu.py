"""The binned front half of the cluster flow path (engine.hip k_bin_sort / k_hot_update, SG_BIN): one scatter pass by
bin digit — a hot flowId's own bin or its key range — and the regular bins sorted in LDS. Every case replays the same
seeded traces through the oracle (ClusterFlowChecker.acquireClusterToken, srv/flow/ClusterFlowChecker.java:55-112) and
through the library with the binned path forced (SG_BIN=2) at small flowId counts, so hot sets form, change and reset
(rule reloads, refused batches) within a few batches; and compares against the two-pass sort (SG_BIN=0)."""
import numpy as np
import pytest

from sentinel_amd import abi
from sentinel_amd.workload import ClusterWorkload
from test_flow_gpu import (WALKERS, _compare_results, _compare_state, _host_records, _pair, _rules, _trace,
                           assert_stable_partition)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_keys,n,zipf,prio,S", [
    (1, 3000, 1.0, 0.1, 10),
    (7, 20_000, 1.2, 0.05, 5),
    (300, 60_000, 1.3, 0.02, 10),
    (3000, 120_000, 1.0, 0.2, 2),
    (5000, 200_000, 1.5, 0.01, 10),
])
@pytest.mark.parametrize("flags", WALKERS)
def test_forced_bins_match_oracle(monkeypatch, n_keys, n, zipf, prio, S, flags):
    monkeypatch.setenv("SG_BIN", "2")
    rng = np.random.default_rng(n_keys * 7 + n + S)
    rules = _rules(n_keys, rng, S=S, interval=1000)
    eng, ora = _pair(rules, flags=flags)
    t = 1_700_000_000_011
    for _ in range(4):  # the hot set of batch i is batch i-1's longest segments
        req = _trace(rng, n, n_keys, t, int(rng.integers(200, 2500)), zipf=zipf, prio=prio)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 300))
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


def test_hot_set_changes_between_batches(monkeypatch):
    """Each batch takes a different popularity permutation: last batch's hot flowIds are this batch's cold ones (a
    stale hot set only costs speed) and the hot-looking flowIds of this batch sit in regular bins."""
    monkeypatch.setenv("SG_BIN", "2")
    rng = np.random.default_rng(77)
    rules = _rules(4000, rng)
    eng, ora = _pair(rules)
    t = 1_700_000_000_000
    for _ in range(5):
        req = _trace(rng, 150_000, 4000, t, 900, zipf=1.4, prio=0.05)
        t = int(req["ts_ms"][-1]) + 40
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, rules)


def test_reload_and_refused_batch_reset_the_hot_set(monkeypatch):
    from sentinel_amd.engine import EngineError
    monkeypatch.setenv("SG_BIN", "2")
    rng = np.random.default_rng(78)
    rules = _rules(2000, rng)
    eng, ora = _pair(rules)
    t = 1_700_000_000_000
    req = _trace(rng, 100_000, 2000, t, 800, zipf=1.3)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    bad = _trace(rng, 1000, 2000, t, 100)  # older than the previous batch: refused, decides nothing
    with pytest.raises(EngineError):
        eng.decide_host(bad)
    t = int(req["ts_ms"][-1]) + 10
    req = _trace(rng, 100_000, 2000, t, 800, zipf=1.3)
    _compare_results(ora.decide(req), eng.decide_host(req), req)
    new = rules[::-1].copy()  # flowIds renumbered: rule index k is another flowId now
    new["count"] = rng.integers(1, 40, len(new))
    eng.load_rules(new)
    ora.load_rules(new)
    for _ in range(2):
        t = int(req["ts_ms"][-1]) + 10
        req = _trace(rng, 100_000, 2000, t, 800, zipf=1.3)
        _compare_results(ora.decide(req), eng.decide_host(req), req)
    _compare_state(eng, ora, new)


def test_binned_layout_is_a_stable_partition(monkeypatch):
    monkeypatch.setenv("SG_BIN", "2")
    rng = np.random.default_rng(79)
    n_keys, n, max_batch = 3000, 4096 * 5 + 33, 1 << 20
    rules = _rules(n_keys, rng)
    eng, _ = _pair(rules, max_batch=max_batch)
    for b in range(3):
        req = _trace(rng, n, n_keys, 1_700_000_000_000 + 2000 * b, 1000, zipf=1.2)
        req["key"][rng.random(n) < 0.01] = abi.KEY_NO_RULE
        eng.decide_host(req)
        rec, kshift = _host_records(req, n_keys, max_batch)
        valid = (rec >> np.uint64(kshift)) < n_keys
        want = rec[np.argsort(rec >> np.uint64(kshift), kind="stable")]
        got = eng.debug_copy(1, np.uint64, n)
        # rejected requests (sentinel key) lie in their own bin: compare the valid records' partition
        gv = got[(got >> np.uint64(kshift)) < n_keys]
        assert len(gv) == int(valid.sum())
        assert_stable_partition(gv, want[(want >> np.uint64(kshift)) < n_keys], kshift)


@pytest.mark.parametrize("prio", [0.01, 0.3])
def test_binned_equals_two_pass(monkeypatch, prio):
    """The C3 shape at 40k flowIds (the binned path's default range): binned and two-pass engines give identical
    results and windows, batch after batch, and both equal the oracle."""
    wl = ClusterWorkload(n_flows=40_000, n_requests=600_000, seed=13, prio_frac=prio)
    rules = wl.rules()
    monkeypatch.setenv("SG_BIN", "1")
    eng, ora = _pair(rules)
    monkeypatch.setenv("SG_BIN", "0")
    eng0, _ = _pair(rules)
    for b in range(3):
        req = wl.requests(b)
        out = eng.decide_host(req)
        assert np.array_equal(out, eng0.decide_host(req))
        _compare_results(ora.decide(req), out, req)
    _compare_state(eng, ora, rules, keys=range(0, len(rules), 5))
    _compare_state(eng0, ora, rules, keys=range(0, len(rules), 5))
