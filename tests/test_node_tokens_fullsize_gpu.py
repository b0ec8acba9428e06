"""The node handle's sharded param and concurrent tokens at the cparam workload's size: 1000 ClusterParamFlowRules,
16M requests per 1000 ms batch (Zipf rules, Zipf values, 10 % with 2-3 values), decided by one handle and by the
node over 2 and 3 shards of this GPU — every TokenResult equal, batch after batch, and a sample of (rule, value)
window sums equal; concurrent tokens at 4M acquires / releases per batch over 100k flow rules — every status equal
and nowCalls equal for every rule. (The oracle replays the smaller cases in test_node_tokens_gpu.py; here the
single handle, itself oracle-checked at these sizes by test_fullsize_gpu.py and the benches, is the reference.)"""
import numpy as np
import pytest

from sentinel_amd import abi
from sentinel_amd.workload import zipf_keys

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _cparam_batch(rng, n, R, V, t0):
    req = np.zeros(n, abi.CPARAM_REQ_DTYPE)
    req["ts_ms"] = t0 + np.sort(rng.integers(0, 1000, n))
    req["key"] = zipf_keys(rng, R, n, 1.0, perm_seed=7).astype(np.uint32)
    req["acquire"] = 1
    cnt = np.where(rng.random(n) < 0.1, rng.integers(2, 4, n), 1).astype(np.uint32)
    req["value_count"] = cnt
    req["value_begin"] = (np.cumsum(cnt) - cnt).astype(np.uint32)
    owner = np.repeat(req["key"].astype(np.uint64), cnt)
    vals = zipf_keys(rng, V, int(cnt.sum()), 1.1, perm_seed=8).astype(np.uint64) * np.uint64(0x9E3779B1) \
        + owner * np.uint64(0x85EBCA77) + np.uint64(11)
    return req, vals


@pytest.mark.timeout(600)
@pytest.mark.parametrize("G", [2, 3])
def test_node_param_tokens_full_size(G):
    from sentinel_amd.engine import FlowEngine, NodeEngine
    rng = np.random.default_rng(500 + G)
    R, n, V = 1000, 16_000_000, 50_000
    rules = np.zeros(R, abi.CPARAM_RULE_DTYPE)
    rules["flow_id"] = np.arange(R) + 1
    rules["count"] = rng.integers(1, 41, R)
    rules["threshold_type"] = abi.THRESHOLD_GLOBAL
    rules["sample_count"], rules["window_interval_ms"] = 10, 1000
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    single = FlowEngine(device=0, max_batch=1 << 25)
    node = NodeEngine([0] * G, max_batch=1 << 25)
    for e in (single, node):
        e.set_namespaces(ns)
        e.cparam_load_rules(rules, None, 17)
    for b in range(2):
        req, vals = _cparam_batch(rng, n, R, V, T0 + 1000 * b)
        want = single.cparam_decide_host(req, vals)
        got = node.cparam_decide_host(req, vals)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"G={G} batch {b}: {len(bad)} of {n} differ; first {bad[0]}: {want[bad[0]]} vs {got[bad[0]]}")
        assert (want["status"] == abi.OK).any() and (want["status"] == abi.BLOCKED).any()
    now = T0 + 1999
    for i in rng.integers(0, n, 200):
        k, v = int(req["key"][i]), int(vals[req["value_begin"][i]])
        assert node.cparam_sum(k, v, now) == single.cparam_sum(k, v, now), (k, v)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("G", [2, 3])
def test_node_concurrent_tokens_full_size(G):
    from sentinel_amd.engine import FlowEngine, NodeEngine
    rng = np.random.default_rng(600 + G)
    K, n = 100_000, 4_000_000
    rules = np.zeros(K, abi.RULE_DTYPE)
    rules["flow_id"] = np.arange(K) + 10
    rules["count"] = rng.integers(1, 40, K).astype(np.float64)
    rules["threshold_type"] = abi.THRESHOLD_GLOBAL
    rules["sample_count"], rules["window_interval_ms"] = 10, 1000
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    single = FlowEngine(device=0, max_batch=1 << 23)
    node = NodeEngine([0] * G, max_batch=1 << 23)
    for e in (single, node):
        e.set_namespaces(ns)
        e.load_rules(rules)
    live_s, live_n = np.zeros(0, np.uint64), np.zeros(0, np.uint64)  # the same tokens, each engine's ids
    for b in range(3):
        q = np.zeros(n, abi.CONC_REQ_DTYPE)
        q["ts_ms"] = T0 + 1000 * b + np.sort(rng.integers(0, 1000, n))
        rel = np.zeros(n, bool)
        if len(live_s):
            m = min(len(live_s), n // 3)
            pick = rng.choice(len(live_s), m, replace=False)
            pos = np.sort(rng.choice(n, m, replace=False))
            rel[pos] = True
        q["kind"] = np.where(rel, abi.CONC_RELEASE, abi.CONC_ACQUIRE)
        q["key"][~rel] = zipf_keys(rng, K, int((~rel).sum()), 1.0, perm_seed=9).astype(np.uint32)
        q["acquire"][~rel] = 1
        q["client"][~rel] = rng.integers(1, 50, int((~rel).sum()))
        qs, qn = q.copy(), q.copy()
        if len(live_s):
            qs["token_id"][rel] = live_s[pick]
            qn["token_id"][rel] = live_n[pick]
            keep = np.ones(len(live_s), bool)
            keep[pick] = False
            live_s, live_n = live_s[keep], live_n[keep]
        ws = single.conc_decide_host(qs)
        wn = node.conc_decide_host(qn)
        assert np.array_equal(ws["status"], wn["status"]), f"G={G} batch {b}: {(ws['status'] != wn['status']).sum()} differ"
        ok = (q["kind"] == abi.CONC_ACQUIRE) & (ws["status"] == abi.OK)
        live_s = np.concatenate([live_s, ws["token_id"][ok]])
        live_n = np.concatenate([live_n, wn["token_id"][ok]])
        assert len(np.unique(wn["token_id"][ok])) == int(ok.sum())
    for k in rng.integers(0, K, 300):
        assert node.conc_state(int(k)) == single.conc_state(int(k)), int(k)
