"""Generate the committed golden fixtures (TEST INFRASTRUCTURE): seeded small versions of every BASELINE
configuration plus the pace and cluster-param paths, replayed through the oracle (oracle/liboracle.so, the
sequential C restatement of the reference, pinned by the reference's own JUnit expectations in
tests/test_oracle_*kat.py). Each case is one .npz of inputs (rules, events in batches) and expected outputs
(decisions, state dumps); MANIFEST.json records the seed, the parameters and the SHA-256 of every file.

    python tests/golden/make_golden.py          # rewrite the fixtures (only when the oracle changes on purpose)

tests/test_golden.py re-derives every expected output from the inputs through the oracle and checks the
hashes (CPU); tests/test_golden_gpu.py decides the same inputs on the device (GPU)."""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.binding import (ClusterTokenService, LocalChain, LocalTraceGen, ParamFlowChecker,  # noqa: E402
                            RateLimiterController, degrade_rule, local_rule)
from sentinel_amd import abi  # noqa: E402
from sentinel_amd.workload import zipf_keys  # noqa: E402

T0 = 1_700_000_000_000


def _local_dump(ora, n_res, sample):
    sec, bor, mnt, head = [], [], [], []
    for r in sample:
        s, b, m = ora.dump(int(r))
        h = np.zeros(14, np.int64)
        h[0] = ora.threads(int(r))
        for i in range(2):
            st, nr = ora.breaker(int(r), i)
            if st >= 0:
                start, bad, total = ora.breaker_stat(int(r), i)
                h[1 + 6 * i: 6 + 6 * i] = (st, nr, start, bad, total)
        sec.append(s)
        bor.append(b)
        mnt.append(m)
        head.append(h)
    return {"state_res": np.asarray(sample, np.uint32), "state_second": np.stack(sec), "state_borrow": np.stack(bor),
            "state_minute": np.stack(mnt), "state_head": np.stack(head)}


def local_case(rules, cfg, batches, seed, sample):
    """batches: list of (entries, rt, err, t_end); events come from the oracle's client model."""
    ora = LocalChain(*cfg)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    evs, res, bounds = [], [], [0]
    for ent, rt, err, t_end in batches:
        ev, r = gen.run(ent, rt, err, t_end)
        evs.append(ev)
        res.append(r)
        bounds.append(bounds[-1] + len(ev))
    out = {"rules": rules, "events": np.concatenate(evs), "results": np.concatenate(res),
           "bounds": np.asarray(bounds, np.int64)}
    out.update(_local_dump(ora, len(rules), sample))
    return out


def entries(rng, n, n_res, t, span, zipf=1.0, prio=0.0, multi=0.1):
    e = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    e["ts_ms"] = t + np.sort(rng.integers(0, span, n))
    e["resource"] = zipf_keys(rng, n_res, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    c = np.ones(n, np.int32)
    m = rng.random(n) < multi
    c[m] = rng.integers(2, 5, int(m.sum()))
    e["count"] = c
    e["resource"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    return e


def case_c1():
    rng = np.random.default_rng(1)
    n = 60_000
    ts = T0 + np.floor(np.cumsum(rng.exponential(1.0, n))).astype(np.int64)
    ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
    ent["ts_ms"], ent["count"] = ts, 1
    rules = np.zeros(1, abi.LOCAL_RULE_DTYPE)
    rules[0] = local_rule(20.0, abi.FLOW_GRADE_QPS)
    half = n // 2
    b = [(ent[:half], np.zeros(half, np.int32), np.zeros(half, np.uint8), int(ts[half - 1]) + 1),
         (ent[half:], np.zeros(n - half, np.int32), np.zeros(n - half, np.uint8), int(ts[-1]) + 1)]
    return {"kind": "local", "cfg": [2, 1000, 500], "seed": 1,
            "what": "C1 HelloWorld: 1 resource QPS=20, Poisson 1000/s for 60 s, exits at once"}, \
        local_case(rules, (2, 1000, 500), b, 1, [0])


def case_c2():
    rng = np.random.default_rng(2)
    K = 200
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    b = []
    for i in range(2):
        e = entries(rng, 30_000, K, T0 + 1000 * i, 1000)
        b.append((e, np.zeros(len(e), np.int32), np.zeros(len(e), np.uint8), 0))  # no exits (t_end before)
    return {"kind": "local", "cfg": [2, 1000, 500], "seed": 2,
            "what": "C2 shape: 200 resources QPS count U{1..64}, 2 x 30k entries Zipf 1.0, no exits"}, \
        local_case(rules, (2, 1000, 500), b, 2, np.arange(K))


def case_c5():
    rng = np.random.default_rng(5)
    K = 1000
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    rules["n_breakers"] = 2
    br = np.zeros(2, abi.DEGRADE_RULE_DTYPE)
    br[0] = degrade_rule(abi.DEGRADE_RT, 30, 1, 5, 1000, 0.5)
    br[1] = degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)
    rules["breakers"] = br
    b = []
    for i in range(3):
        e = entries(rng, 20_000, K, T0 + 1000 * i, 1000, prio=0.05)
        rt = np.minimum(np.round(np.exp(rng.normal(2.5, 0.8, len(e)))), 10_000).astype(np.int32)
        b.append((e, rt, (rng.random(len(e)) < 0.15).astype(np.uint8), T0 + 1000 * (i + 1)))
    return {"kind": "local", "cfg": [2, 1000, 500], "seed": 5,
            "what": "C5 shape: 1000 resources QPS + RT + exception-ratio breakers, 3 x 20k entries + exits"}, \
        local_case(rules, (2, 1000, 500), b, 5, np.arange(0, K, 5))


def cluster_case(rules, ns, batches, exceed=1.0, ratio=1.0):
    ora = ClusterTokenService(exceed, ratio)
    ora.set_namespaces(ns)
    ora.load_rules(rules)
    res = [ora.decide(q) for q in batches]
    stride = int(rules["sample_count"].max())
    ring, occ = ora.export_state(len(rules), stride)
    bounds = np.cumsum([0] + [len(q) for q in batches]).astype(np.int64)
    return {"rules": rules, "ns": ns, "requests": np.concatenate(batches), "results": np.concatenate(res),
            "bounds": bounds, "state_ring": ring, "state_occ": occ}


def flow_rules(rng, n, S=10, interval=1000):
    r = np.zeros(n, abi.RULE_DTYPE)
    r["flow_id"] = np.arange(1, n + 1, dtype=np.int64) + 10_000_000
    r["count"] = rng.integers(1, 33, n).astype(np.float64)
    r["threshold_type"] = abi.THRESHOLD_GLOBAL
    r["sample_count"] = S
    r["window_interval_ms"] = interval
    return r


def flow_requests(rng, n, K, t, span, prio=0.05, multi=0.1, zipf=1.0):
    q = np.zeros(n, abi.REQ_DTYPE)
    q["ts_ms"] = t + np.sort(rng.integers(0, span, n))
    q["key"] = zipf_keys(rng, K, n, zipf, perm_seed=int(rng.integers(1 << 30)))
    a = np.ones(n, np.int32)
    m = rng.random(n) < multi
    a[m] = rng.integers(2, 5, int(m.sum()))
    q["acquire"] = a
    q["key"] |= np.where(rng.random(n) < prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
    sel = rng.random(n)
    q["key"][sel < 0.002] = abi.KEY_NO_RULE
    q["acquire"][(sel >= 0.002) & (sel < 0.003)] = 0
    return q


def case_c3():
    rng = np.random.default_rng(3)
    K = 5000
    rules = flow_rules(rng, K)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"], ns["max_allowed_qps"] = 1, 30000
    b = [flow_requests(rng, 60_000, K, T0 + 1000 * i, 1000) for i in range(2)]
    return {"kind": "cluster", "exceed": 1.0, "ratio": 1.0, "seed": 3,
            "what": "C3 shape: 5000 flowIds GLOBAL count U{1..32} S=10/1000, 2 x 60k requests, 5 % prioritized"}, \
        cluster_case(rules, ns, b)


def case_c3_limiter():
    rng = np.random.default_rng(33)
    K = 2000
    rules = flow_rules(rng, K)
    rules["namespace_id"] = rng.integers(0, 3, K)
    ns = np.zeros(3, abi.NS_DTYPE)
    ns[0] = (1, 1, 4000.0)
    ns[1] = (0, 2, 0.0)
    ns[2] = (1, 1, 1500.5)
    b = [flow_requests(rng, 20_000, K, T0 + 1300 * i, 1300) for i in range(2)]
    return {"kind": "cluster", "exceed": 1.2, "ratio": 0.7, "seed": 33,
            "what": "C3 + GlobalRequestLimiter: 2000 flowIds over 3 namespaces (2 limited), 2 x 20k requests"}, \
        cluster_case(rules, ns, b, 1.2, 0.7)


def case_c4():
    rng = np.random.default_rng(4)
    rules = np.zeros(2, abi.PARAM_RULE_DTYPE)
    rules[0] = (5.0, 1, 0, abi.BEHAVIOR_DEFAULT, 0, 0, 0, 16)
    rules[1] = (20.0, 2, 3, abi.BEHAVIOR_RATE_LIMITER, 100, 0, 4, 16)
    hot = np.zeros(4, abi.PARAM_HOT_DTYPE)
    for i in range(4):
        hot[i] = (np.uint64(i + 1) * np.uint64(0x9E3779B1) + np.uint64(17), int(rng.integers(0, 50)), 0)
    n, V = 60_000, 100_000
    q = np.zeros(n, abi.PARAM_REQ_DTYPE)
    q["ts_ms"] = T0 + np.sort(rng.integers(0, 2500, n))
    q["value"] = zipf_keys(rng, V, n, 1.1, perm_seed=4).astype(np.uint64) * np.uint64(0x9E3779B1) + np.uint64(17)
    q["rule"] = (rng.random(n) < 0.3).astype(np.uint32)
    q["acquire"] = rng.integers(1, 3, n)
    ora = ParamFlowChecker()
    ora.load_rules(rules, hot)
    half = n // 2
    res = np.concatenate([ora.decide(q[:half]), ora.decide(q[half:])])
    vals = np.unique(q["value"])[::50]
    st = np.array([[r, *ora.state(r, int(v))] for r in range(2) for v in vals], np.int64)
    return {"kind": "param", "seed": 4,
            "what": "C4 shape: token bucket count 5/1 s + throttle with hot items, 60k requests over 100k values"}, \
        {"rules": rules, "hot": hot, "requests": q, "results": res, "bounds": np.array([0, half, n], np.int64),
         "state_values": np.tile(vals, 2), "state": st}


def case_pace():
    rng = np.random.default_rng(6)
    K = 500
    rules = np.zeros(K, abi.PACE_RULE_DTYPE)
    rules["count"] = np.where(rng.random(K) < 0.5, rng.integers(1, 2000, K), rng.random(K) * 50)
    rules["max_queueing_ms"] = rng.choice([0, 20, 100, 500, 2000], K)
    n = 40_000
    q = np.zeros(n, abi.PACE_REQ_DTYPE)
    q["ts_ms"] = T0 + np.sort(rng.integers(0, 3000, n))
    q["rule"] = zipf_keys(rng, K, n, 1.1, perm_seed=6)
    q["acquire"] = rng.integers(1, 4, n)
    ora = RateLimiterController(rules)
    half = n // 2
    res = np.concatenate([ora.decide(q[:half]), ora.decide(q[half:])])
    latest = np.array([ora.latest(k) for k in range(K)], np.int64)
    return {"kind": "pace", "seed": 6, "what": "RateLimiterController: 500 rules, 40k canPass over 3 s"}, \
        {"rules": rules, "requests": q, "results": res, "bounds": np.array([0, half, n], np.int64), "latest": latest}


def case_cparam():
    rng = np.random.default_rng(7)
    K = 20
    rules = np.zeros(K, abi.CPARAM_RULE_DTYPE)
    rules["flow_id"] = np.arange(K) * 3 + 7
    rules["count"] = rng.integers(1, 40, K)
    rules["threshold_type"] = abi.THRESHOLD_GLOBAL
    rules["sample_count"] = 10
    rules["window_interval_ms"] = 1000
    n = 30_000
    q = np.zeros(n, abi.CPARAM_REQ_DTYPE)
    q["ts_ms"] = T0 + np.sort(rng.integers(0, 2000, n))
    q["key"] = rng.integers(0, K, n)
    q["acquire"] = rng.integers(1, 4, n)
    cnt = np.where(rng.random(n) < 0.03, rng.integers(2, 4, n), 1).astype(np.uint32)
    q["value_count"] = cnt
    q["value_begin"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint32)
    values = zipf_keys(rng, 300, int(cnt.sum()), 1.1, perm_seed=7).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_param_rules(rules)
    res = ora.decide_param(q, values)
    return {"kind": "cparam", "seed": 7, "what": "ClusterParamFlowChecker: 20 rules, 30k requests, 3 % multi-value"}, \
        {"rules": rules, "ns": ns, "requests": q, "values": values, "results": res,
         "bounds": np.array([0, n], np.int64)}


CASES = {"c1_helloworld": case_c1, "c2_local": case_c2, "c3_cluster": case_c3, "c3_limiter": case_c3_limiter,
         "c4_param": case_c4, "c5_breakers": case_c5, "pace": case_pace, "cparam": case_cparam}


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/sentinel_oracle.c", "cases": {}}
    for name, fn in CASES.items():
        meta, arrays = fn()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrays)
        meta["file"] = name + ".npz"
        meta["sha256"] = sha256(path)
        manifest["cases"][name] = meta
        print(f"{name}: {os.path.getsize(path) / 1e3:.0f} kB  {meta['what']}")
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
