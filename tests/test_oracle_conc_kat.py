"""Known-answer tests of the concurrent-token oracle (oracle.binding.ConcurrentTokenService), restating the
reference's own tests on the sequential replay model:

  ConcurrentClusterFlowCheckerTest.{testEasyAcquireAndRelease, testConcurrentAcquireAndRelease,
  testReleaseExpiredToken}   sentinel-cluster/sentinel-cluster-server-default/src/test/.../flow/
                             ConcurrentClusterFlowCheckerTest.java:36-118
  DefaultTokenService.requestConcurrentToken validation           …/flow/DefaultTokenService.java:66-93

The reference's concurrent test runs 1000 acquire-then-release tasks on 100 threads; any interleaving keeps
nowCalls <= count and ends at 0 with no tokens left, which the sequential replay checks for several orders.
"""
import numpy as np
import pytest

from oracle.binding import ConcurrentTokenService
from sentinel_amd import abi

T0 = 1_700_000_000_000


def _svc(count=10, threshold=abi.THRESHOLD_GLOBAL, connected=1, resource_timeout=500, client_offline=1000):
    s = ConcurrentTokenService()
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = connected
    s.set_namespaces(ns)
    r = np.zeros(1, abi.RULE_DTYPE)
    r["flow_id"], r["count"], r["threshold_type"] = 111, count, threshold
    r["sample_count"], r["window_interval_ms"] = 10, 1000
    s.load_rules(r)
    s.set_rule_timeouts([client_offline], [resource_timeout])
    return s


def _req(events):
    q = np.zeros(len(events), abi.CONC_REQ_DTYPE)
    for i, (ts, kind, key_or_tok, acq, client) in enumerate(events):
        q[i]["ts_ms"], q[i]["kind"], q[i]["acquire"], q[i]["client"] = ts, kind, acq, client
        if kind == abi.CONC_ACQUIRE:
            q[i]["key"] = key_or_tok
        else:
            q[i]["token_id"] = key_or_tok
    return q


def test_easy_acquire_and_release():
    s = _svc()
    out = s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 1, 1)] * 10))
    assert (out["status"] == abi.OK).all() and (out["token_id"] != 0).all()
    blocked = s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 1, 1)] * 10))
    assert (blocked["status"] == abi.BLOCKED).all()
    rel = s.decide(_req([(T0, abi.CONC_RELEASE, int(t), 0, 0) for t in out["token_id"]]))
    assert (rel["status"] == abi.RELEASE_OK).all()
    assert s.now_calls(0) == 0 and s.live() == 0


@pytest.mark.parametrize("seed", range(4))
def test_acquire_release_interleavings(seed):
    """1000 tasks (acquire, and release when OK) in a random interleaving of their two steps."""
    rng = np.random.default_rng(seed)
    s = _svc()
    pending = []  # tokens acquired and not yet released
    steps = 0
    todo = 1000
    while todo or pending:
        if todo and (not pending or rng.random() < 0.5):
            r = s.decide(_req([(T0 + steps, abi.CONC_ACQUIRE, 0, 1, 1)]))[0]
            todo -= 1
            assert s.now_calls(0) <= 10
            if r["status"] == abi.OK:
                pending.append(int(r["token_id"]))
        else:
            t = pending.pop(int(rng.integers(len(pending))))
            assert s.decide(_req([(T0 + steps, abi.CONC_RELEASE, t, 0, 0)]))[0]["status"] == abi.RELEASE_OK
        steps += 1
    assert s.now_calls(0) == 0 and s.live() == 0


def test_release_expired_token():
    s = _svc()
    s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 1, 1)] * 10))
    online = np.array([0, 1], np.uint8)  # client 1 ("127.0.0.1") connected
    # the clear task runs every second: by T0 + 1000 nothing is past 2 x resourceTimeout yet
    assert s.expire(T0 + 1000, online) == 0 and s.now_calls(0) == 10
    assert s.expire(T0 + 2000, online) == 10
    assert s.now_calls(0) == 0 and s.live() == 0


def test_offline_client_tokens_expire_after_client_timeout():
    s = _svc(resource_timeout=100_000, client_offline=1000)
    s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 2, 1), (T0, abi.CONC_ACQUIRE, 0, 3, 2)]))
    online = np.array([0, 1, 0], np.uint8)  # client 2 went offline
    assert s.expire(T0 + 1000, online) == 0             # clientTimeout - now < 0 is strict
    assert s.expire(T0 + 1001, online) == 1 and s.now_calls(0) == 2


def test_validation_and_release_statuses():
    s = _svc(count=2.5)
    out = s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 1, 0),                 # null client address
                         (T0, abi.CONC_ACQUIRE, abi.KEY_BAD, 1, 1),       # flowId null / <= 0
                         (T0, abi.CONC_ACQUIRE, 0, 0, 1),                 # acquireCount <= 0
                         (T0, abi.CONC_ACQUIRE, 5, 1, 1),                 # no rule
                         (T0, abi.CONC_ACQUIRE, 0, 2, 1),                 # 0 + 2 <= 2.5
                         (T0, abi.CONC_ACQUIRE, 0, 1, 1),                 # 2 + 1 > 2.5
                         (T0, abi.CONC_RELEASE, 12345, 0, 0),             # unknown token
                         (T0, abi.CONC_RELEASE, 0, 0, 0)]))               # null token
    assert list(out["status"]) == [abi.BAD_REQUEST, abi.BAD_REQUEST, abi.BAD_REQUEST, abi.NO_RULE_EXISTS, abi.OK,
                                   abi.BLOCKED, abi.ALREADY_RELEASE, abi.BAD_REQUEST]
    tok = int(out["token_id"][4])
    assert tok == 5  # 1 + requests decided before it
    assert [r["status"] for r in s.decide(_req([(T0, abi.CONC_RELEASE, tok, 0, 0)] * 2))] == \
        [abi.RELEASE_OK, abi.ALREADY_RELEASE]


def test_avg_local_threshold_and_reload():
    s = _svc(count=3, threshold=abi.THRESHOLD_AVG_LOCAL, connected=2)   # 3 x 2 connected clients
    out = s.decide(_req([(T0, abi.CONC_ACQUIRE, 0, 1, 1)] * 7))
    assert list(out["status"]) == [abi.OK] * 6 + [abi.BLOCKED]
    # a reload keeps the counter of a surviving flowId; a removed flowId's tokens answer NO_RULE_EXISTS
    r = np.zeros(2, abi.RULE_DTYPE)
    r["flow_id"] = [222, 111]
    r["count"], r["threshold_type"], r["sample_count"], r["window_interval_ms"] = 10, abi.THRESHOLD_GLOBAL, 10, 1000
    s.load_rules(r)
    assert s.now_calls(1) == 6 and s.now_calls(0) == 0
    s.load_rules(r[:1])
    rel = s.decide(_req([(T0, abi.CONC_RELEASE, int(out["token_id"][0]), 0, 0)]))
    assert rel["status"][0] == abi.NO_RULE_EXISTS and s.live() == 6
