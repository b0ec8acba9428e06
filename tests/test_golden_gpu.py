"""The committed golden fixtures decided on the device through the C ABI: every decision and every stored
state dump must equal the fixture (which the oracle reproduces on the CPU, tests/test_golden.py)."""
import numpy as np
import pytest

from test_golden import CASES, batches, load_case

pytestmark = pytest.mark.gpu


def _eng(n, **kw):
    from sentinel_amd.engine import FlowEngine
    return FlowEngine(device=0, max_batch=max(n, 16), **kw)


@pytest.mark.parametrize("name", CASES)
def test_device_reproduces_fixture(name):
    meta, d = load_case(name)
    kind = meta["kind"]
    if kind == "local":
        eng = _eng(len(d["events"]))
        S, interval, occ = meta["cfg"]
        eng.local_load_rules(d["rules"], S, interval, occ)
        got = np.concatenate([eng.local_decide_host(ev) for ev in batches(d, "events")])
        assert np.array_equal(got, d["results"])
        for j, r in enumerate(d["state_res"]):
            s, b, m, head = eng.local_state(int(r))
            assert np.array_equal(s, d["state_second"][j]) and np.array_equal(b, d["state_borrow"][j])
            assert np.array_equal(m, d["state_minute"][j])
            nb = int(d["rules"][int(r)]["n_breakers"])  # the fixture holds zeros for absent breakers
            want = d["state_head"][j]
            assert head[0] == want[0] and np.array_equal(head[1:1 + 6 * nb], want[1:1 + 6 * nb]), (r, head, want)
    elif kind == "cluster":
        eng = _eng(len(d["requests"]), exceed_count=meta["exceed"], max_occupy_ratio=meta["ratio"])
        eng.set_namespaces(d["ns"])
        eng.load_rules(d["rules"])
        got = np.concatenate([eng.decide_host(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        ring, occ = eng.export_state(len(d["rules"]))
        assert ring.shape == d["state_ring"].shape
        live = d["state_ring"][:, :, :1] != np.iinfo(np.int64).min
        assert np.array_equal(ring[:, :, 0], d["state_ring"][:, :, 0])
        assert np.array_equal(np.where(live, ring, 0), np.where(live, d["state_ring"], 0))
        assert np.array_equal(occ, d["state_occ"])
    elif kind == "param":
        eng = _eng(len(d["requests"]))
        eng.param_load_rules(d["rules"], d["hot"])
        got = np.concatenate([eng.param_decide_host(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        for (r, f, lt, tk), v in zip(d["state"], d["state_values"]):
            assert eng.param_state(int(r), int(v)) == (f, lt, tk)
    elif kind == "pace":
        eng = _eng(len(d["requests"]))
        eng.pace_load_rules(d["rules"])
        got = np.concatenate([eng.pace_decide_host(q) for q in batches(d, "requests")])
        assert np.array_equal(got, d["results"])
        assert [eng.pace_latest(k) for k in range(len(d["rules"]))] == list(d["latest"])
    elif kind == "cparam":
        eng = _eng(len(d["requests"]))
        eng.set_namespaces(d["ns"])
        eng.cparam_load_rules(d["rules"], None, 12)
        assert np.array_equal(eng.cparam_decide_host(d["requests"], d["values"]), d["results"])
    else:
        raise AssertionError(kind)
