"""Parity of the device concurrent-token path (sg_conc_*: ConcurrentClusterFlowChecker over nowCalls per flowId
and the token table) with the oracle's sequential replay (oracle.binding.ConcurrentTokenService): acquires and
releases in time order — releases of tokens from earlier batches, of tokens acquired earlier in the same batch
(even ones that were blocked), double releases and unknown ids —, token expiry (RegularExpireStrategy) between
batches, and a rule reload that keeps surviving flowIds' counters. Every result, token id, nowCalls and the
number of live tokens are compared exactly."""
import numpy as np
import pytest

from sentinel_amd import abi

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _rules(rng, k, fid0=1000):
    r = np.zeros(k, abi.RULE_DTYPE)
    r["flow_id"] = fid0 + np.arange(k)
    r["count"] = rng.integers(1, 40, k).astype(np.float64) + np.where(rng.random(k) < 0.3, 0.5, 0.0)
    r["threshold_type"] = np.where(rng.random(k) < 0.3, abi.THRESHOLD_AVG_LOCAL, abi.THRESHOLD_GLOBAL)
    r["sample_count"], r["window_interval_ms"] = 10, 1000
    return r


def _ns():
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 3
    ns["max_allowed_qps"] = 30000
    return ns


class Trace:
    """Seeded acquire/release batches; token ids follow the ABI's rule (1 + requests decided before)."""

    def __init__(self, seed, k):
        self.rng = np.random.default_rng(seed)
        self.k = k
        self.seq = 0
        self.live = []       # tokens believed live (from the oracle's answers)
        self.released = []   # recently released (double releases)
        self.t = T0

    def batch(self, n, span, hot=None):
        rng = self.rng
        q = np.zeros(n, abi.CONC_REQ_DTYPE)
        q["ts_ms"] = self.t + np.sort(rng.integers(0, span, n))
        acq_idx = []
        for i in range(n):
            if rng.random() < 0.55 or not (self.live or acq_idx):
                q[i]["kind"] = abi.CONC_ACQUIRE
                u = rng.random()
                if hot is not None and u < hot:
                    q[i]["key"] = 0
                else:
                    q[i]["key"] = min(int(rng.zipf(1.3)) - 1, self.k + 5)   # a few keys beyond the rules
                if rng.random() < 0.01:
                    q[i]["key"] = abi.KEY_BAD
                q[i]["acquire"] = int(rng.integers(1, 4)) if rng.random() > 0.01 else 0
                q[i]["client"] = int(rng.integers(1, 21)) if rng.random() > 0.02 else 0
                acq_idx.append(i)
            else:
                q[i]["kind"] = abi.CONC_RELEASE
                u = rng.random()
                if u < 0.45 and self.live:
                    q[i]["token_id"] = self.live.pop(int(rng.integers(len(self.live))))
                elif u < 0.8 and acq_idx:
                    q[i]["token_id"] = self.seq + acq_idx[int(rng.integers(len(acq_idx)))] + 1
                elif u < 0.9 and self.released:
                    q[i]["token_id"] = self.released[int(rng.integers(len(self.released)))]
                elif u < 0.95:
                    q[i]["token_id"] = int(rng.integers(1, 1 << 40))
                else:
                    q[i]["token_id"] = 0
        self.t += span
        return q

    def absorb(self, q, out):
        self.seq += len(q)
        ok = (q["kind"] == abi.CONC_ACQUIRE) & (out["status"] == abi.OK)
        rel = (q["kind"] == abi.CONC_RELEASE) & (out["status"] == abi.RELEASE_OK)
        gone = set(int(x) for x in q["token_id"][rel])
        self.released = (self.released + list(gone))[-200:]
        fresh = [int(x) for x in out["token_id"][ok] if int(x) not in gone]
        self.live = [x for x in self.live if x not in gone] + fresh


def _pair(rules, timeouts=None):
    from oracle.binding import ConcurrentTokenService
    from sentinel_amd.engine import FlowEngine
    eng = FlowEngine(device=0, max_batch=1 << 18)
    eng.set_namespaces(_ns())
    eng.load_rules(rules)
    ora = ConcurrentTokenService()
    ora.set_namespaces(_ns())
    ora.load_rules(rules)
    if timeouts is not None:
        eng.conc_set_rule_timeouts(*timeouts)
        ora.set_rule_timeouts(*timeouts)
    return eng, ora


def _check_state(eng, ora, k):
    live = None
    for key in range(k):
        now, live = eng.conc_state(key)
        assert now == ora.now_calls(key), f"nowCalls of {key}: {ora.now_calls(key)} vs {now}"
    assert live == ora.live()


def _step(eng, ora, tr, q):
    want = ora.decide(q)
    got = eng.conc_decide_host(q)
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        i = bad[0]
        raise AssertionError(f"{len(bad)} differ; first {i}: req={q[i]} oracle={want[i]} gpu={got[i]}")
    tr.absorb(q, want)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_acquire_release_batches(seed):
    rng = np.random.default_rng(seed)
    k = 150
    rules = _rules(rng, k)
    timeouts = (rng.integers(200, 3000, k), rng.integers(100, 1500, k))
    eng, ora = _pair(rules, timeouts)
    tr = Trace(seed, k)
    for b in range(6):
        _step(eng, ora, tr, tr.batch(20_000, 700))
        online = (rng.random(22) < 0.7).astype(np.uint8)
        assert eng.conc_expire(tr.t, online) == ora.expire(tr.t, online)
        _check_state(eng, ora, k)


def test_reload_keeps_surviving_counters():
    rng = np.random.default_rng(4)
    k = 60
    rules = _rules(rng, k)
    eng, ora = _pair(rules)
    tr = Trace(4, k)
    _step(eng, ora, tr, tr.batch(8_000, 500))
    new = np.concatenate([rules[10:40], _rules(rng, 20, fid0=5000)])   # 30 survive (re-indexed), 20 new
    eng.load_rules(new)
    ora.load_rules(new)
    tr.k = len(new)
    _check_state(eng, ora, len(new))
    _step(eng, ora, tr, tr.batch(8_000, 500))        # releases of tokens whose rule is gone: NO_RULE_EXISTS
    _check_state(eng, ora, len(new))


def test_two_reloads_in_a_row():
    """Two rule reloads with no concurrent call between them (the counters of the first reload are still
    host-side when the second remaps them): grow the rule set, then permute it; nowCalls and the releases of the
    live tokens must follow their flowIds."""
    rng = np.random.default_rng(6)
    k = 50
    rules = _rules(rng, k)
    eng, ora = _pair(rules)
    tr = Trace(6, k)
    _step(eng, ora, tr, tr.batch(6_000, 500))
    grown = np.concatenate([rules, _rules(rng, 30, fid0=7000)])
    perm = grown[rng.permutation(len(grown))]
    for new in (grown, perm):
        eng.load_rules(new)
        ora.load_rules(new)
    tr.k = len(perm)
    _check_state(eng, ora, len(perm))
    _step(eng, ora, tr, tr.batch(6_000, 500))
    _check_state(eng, ora, len(perm))


def test_hot_flow_large_batch():
    """One flowId takes most of a 200k-request batch (one lane walks its segment)."""
    rng = np.random.default_rng(5)
    rules = _rules(rng, 20)
    rules["count"][0] = 500
    eng, ora = _pair(rules)
    tr = Trace(5, 20)
    for _ in range(2):
        _step(eng, ora, tr, tr.batch(200_000, 1000, hot=0.8))
    _check_state(eng, ora, 20)


def test_easy_acquire_and_release_on_device():
    """ConcurrentClusterFlowCheckerTest.testEasyAcquireAndRelease on the device path."""
    rules = np.zeros(1, abi.RULE_DTYPE)
    rules["flow_id"], rules["count"], rules["threshold_type"] = 111, 10, abi.THRESHOLD_GLOBAL
    rules["sample_count"], rules["window_interval_ms"] = 10, 1000
    eng, _ = _pair(rules, ([1000], [500]))
    q = np.zeros(20, abi.CONC_REQ_DTYPE)
    q["ts_ms"], q["kind"], q["key"], q["acquire"], q["client"] = T0, abi.CONC_ACQUIRE, 0, 1, 1
    out = eng.conc_decide_host(q)
    assert (out["status"][:10] == abi.OK).all() and (out["status"][10:] == abi.BLOCKED).all()
    r = np.zeros(10, abi.CONC_REQ_DTYPE)
    r["ts_ms"], r["kind"], r["token_id"] = T0, abi.CONC_RELEASE, out["token_id"][:10]
    assert (eng.conc_decide_host(r)["status"] == abi.RELEASE_OK).all()
    assert eng.conc_state(0) == (0, 0)
    # testReleaseExpiredToken: 10 tokens of an online client expire after 2 x resourceTimeout
    eng.conc_decide_host(q[:10].copy())
    assert eng.conc_expire(T0 + 1000, np.array([0, 1], np.uint8)) == 0
    assert eng.conc_expire(T0 + 2000, np.array([0, 1], np.uint8)) == 10
    assert eng.conc_state(0) == (0, 0)
