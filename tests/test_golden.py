"""The committed golden fixtures (tests/golden, made by tests/golden/make_golden.py): every file matches the
SHA-256 in MANIFEST.json, and the oracle re-derives every stored decision and state dump from the stored
inputs (so a change to the oracle that moves any result shows up here, on the CPU)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle.binding import ClusterTokenService, LocalChain, ParamFlowChecker, RateLimiterController
from sentinel_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "MANIFEST.json")))
CASES = sorted(MANIFEST["cases"])


def load_case(name):
    meta = MANIFEST["cases"][name]
    path = os.path.join(GOLDEN, meta["file"])
    return meta, dict(np.load(path, allow_pickle=False))


def batches(d, key):
    b = d["bounds"]
    return [d[key][b[i]:b[i + 1]] for i in range(len(b) - 1)]


@pytest.mark.parametrize("name", CASES)
def test_fixture_hash(name):
    meta = MANIFEST["cases"][name]
    with open(os.path.join(GOLDEN, meta["file"]), "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == meta["sha256"]


def _local_state_check(ora, d):
    for j, r in enumerate(d["state_res"]):
        s, b, m = ora.dump(int(r))
        assert np.array_equal(s, d["state_second"][j]) and np.array_equal(b, d["state_borrow"][j])
        assert np.array_equal(m, d["state_minute"][j])
        assert ora.threads(int(r)) == d["state_head"][j][0]


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_fixture(name):
    meta, d = load_case(name)
    kind = meta["kind"]
    if kind == "local":
        ora = LocalChain(*meta["cfg"])
        ora.load_rules(d["rules"])
        got = np.concatenate([ora.decide(ev) for ev in batches(d, "events")])
        assert np.array_equal(got, d["results"])
        _local_state_check(ora, d)
    elif kind == "cluster":
        ora = ClusterTokenService(meta["exceed"], meta["ratio"])
        ora.set_namespaces(d["ns"])
        ora.load_rules(d["rules"])
        got = np.concatenate([ora.decide(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        ring, occ = ora.export_state(len(d["rules"]), d["state_ring"].shape[1])
        assert np.array_equal(ring, d["state_ring"]) and np.array_equal(occ, d["state_occ"])
    elif kind == "param":
        ora = ParamFlowChecker()
        ora.load_rules(d["rules"], d["hot"])
        got = np.concatenate([ora.decide(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        for (r, f, lt, tk), v in zip(d["state"], d["state_values"]):
            assert ora.state(int(r), int(v)) == (f, lt, tk)
    elif kind == "pace":
        ora = RateLimiterController(d["rules"])
        got = np.concatenate([ora.decide(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        assert [ora.latest(k) for k in range(len(d["rules"]))] == list(d["latest"])
    elif kind == "cparam":
        ora = ClusterTokenService()
        ora.set_namespaces(d["ns"])
        ora.load_param_rules(d["rules"])
        assert np.array_equal(ora.decide_param(d["requests"], d["values"]), d["results"])
    else:
        raise AssertionError(kind)


def test_fixture_coverage():
    """The fixtures exercise every outcome the paths have."""
    _, c3 = load_case("c3_cluster")
    st = c3["results"]["status"]
    for s in (abi.OK, abi.BLOCKED, abi.SHOULD_WAIT, abi.NO_RULE_EXISTS, abi.BAD_REQUEST):
        assert (st == s).any(), s
    _, lim = load_case("c3_limiter")
    assert (lim["results"]["status"] == abi.TOO_MANY_REQUEST).any()
    _, c5 = load_case("c5_breakers")
    st = c5["results"]["status"]
    for s in (abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW, abi.LOCAL_BLOCK_DEGRADE, abi.LOCAL_PASS_WAIT):
        assert (st == s).any(), s
    _, c1 = load_case("c1_helloworld")
    ev, res = c1["events"], c1["results"]
    passed = (ev["kind"] == abi.LOCAL_ENTRY) & (res["status"] == abi.LOCAL_PASS)
    per_sec = np.bincount((ev["ts_ms"][passed] - ev["ts_ms"][0] + (ev["ts_ms"][0] % 1000)) // 1000)
    assert per_sec.max() <= 20
