"""The asynchronous host pipeline (sg_flow_submit / sg_flow_poll / sg_flow_wait, include/sentinel_gpu.h):
batches submitted from pinned or pageable host memory with up to 3 in flight decide exactly as the
synchronous path and the oracle; a rejected batch reports its error on its own ticket and changes nothing;
every other call completes the batches in flight first."""
import numpy as np
import pytest

from sentinel_amd import abi

pytestmark = pytest.mark.gpu


def _setup(n_flows=3000, n_req=100_000, seed=31):
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import FlowEngine
    from sentinel_amd.workload import ClusterWorkload
    wl = ClusterWorkload(n_flows=n_flows, n_requests=n_req, seed=seed, prio_frac=0.05)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    eng = FlowEngine(device=0, max_batch=n_req)
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules())
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(wl.rules())
    return wl, eng, ora


@pytest.mark.parametrize("pinned", [True, False])
def test_pipelined_batches_equal_oracle(pinned):
    wl, eng, ora = _setup()
    nb = 7  # more batches than pipeline slots: the 4th submit completes the oldest
    reqs = [wl.requests(b) for b in range(nb)]
    if pinned:
        ins = [eng.host_array(len(r), abi.REQ_DTYPE) for r in reqs]
        outs = [eng.host_array(len(r), abi.RES_DTYPE) for r in reqs]
        for a, r in zip(ins, reqs):
            a[:] = r
    else:
        ins = reqs
        outs = [np.zeros(len(r), abi.RES_DTYPE) for r in reqs]
    tickets = [eng.submit(i, o) for i, o in zip(ins, outs)]
    done = [False] * nb
    while not all(done):  # poll in any order
        for k in reversed(range(nb)):
            if not done[k]:
                done[k] = eng.poll(tickets[k])
    for b in range(nb):
        want = ora.decide(reqs[b])
        assert np.array_equal(outs[b], want), f"batch {b}: {(outs[b] != want).sum()} differ"
    ring, occ = eng.export_state(len(wl.rules()))
    ring_o, occ_o = ora.export_state(len(wl.rules()), ring.shape[1])
    assert np.array_equal(ring, ring_o) and np.array_equal(occ, occ_o)


def test_rejected_batch_reports_on_its_ticket():
    from sentinel_amd.engine import EngineError
    wl, eng, ora = _setup()
    r0, r1, r2 = wl.requests(0), wl.requests(1), wl.requests(2)
    bad = r1.copy()
    bad["ts_ms"][10] = bad["ts_ms"][9] - 5  # not time-ordered
    o0, o1, o2 = (np.zeros(len(r), abi.RES_DTYPE) for r in (r0, bad, r2))
    t0 = eng.submit(r0, o0)
    t1 = eng.submit(bad, o1)
    t2 = eng.submit(r1, o2)  # the good version of batch 1
    eng.wait(t0)
    with pytest.raises(EngineError) as ei:
        eng.wait(t1)
    assert ei.value.code == abi.SG_E_TIME
    eng.wait(t2)
    assert np.array_equal(o0, ora.decide(r0))
    assert np.array_equal(o2, ora.decide(r1))


def test_other_calls_drain_the_pipeline():
    wl, eng, ora = _setup()
    reqs = [wl.requests(b) for b in range(3)]
    outs = [np.zeros(len(r), abi.RES_DTYPE) for r in reqs]
    tickets = [eng.submit(r, o) for r, o in zip(reqs, outs)]
    snap = eng.snapshot(int(reqs[-1]["ts_ms"][-1]) + 1, len(wl.rules()))  # completes all three first
    for t in tickets:
        eng.wait(t)  # statuses are kept until collected
    for r, o in zip(reqs, outs):
        assert np.array_equal(o, ora.decide(r))
    now = int(reqs[-1]["ts_ms"][-1]) + 1
    want = np.array([[ora.avg(k, now, abi.EV_PASS), ora.avg(k, now, abi.EV_BLOCK)] for k in range(len(wl.rules()))])
    assert np.array_equal(snap, want)
