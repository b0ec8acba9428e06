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


@pytest.mark.parametrize("d2h", ["0", "1"])
@pytest.mark.parametrize("offset,trim", [(1, 0), (4, 3), (0, 1)])
def test_pinned_outputs_any_alignment_and_length(monkeypatch, d2h, offset, trim):
    """Results into views of pinned buffers, by the copy engine (SG_D2H=0, the default) or the shader copy
    (SG_D2H=1): a 12-B offset (not 16-B aligned: the copy engine takes it either way), a 48-B offset, and batch
    lengths whose result bytes are not a multiple of 16 (the copy kernel's 4-B tail)."""
    monkeypatch.setenv("SG_D2H", d2h)
    wl, eng, ora = _setup(seed=35)
    reqs = [wl.requests(b)[: 100_000 - trim - b] for b in range(4)]
    bufs = [eng.host_array(len(r) + offset, abi.RES_DTYPE) for r in reqs]
    outs = [bf[offset:offset + len(r)] for bf, r in zip(bufs, reqs)]
    for bf in bufs:
        bf["status"] = -7  # sentinel: every slot must be overwritten
    tickets = [eng.submit(r, o) for r, o in zip(reqs, outs)]
    for t in tickets:
        eng.wait(t)
    for b, (r, o, bf) in enumerate(zip(reqs, outs, bufs)):
        assert np.array_equal(o, ora.decide(r)), f"batch {b}"
        assert (bf["status"][:offset] == -7).all()  # nothing written before the view


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


def _dev(arr):
    import torch
    return torch.from_numpy(arr.view(np.uint8).copy()).to("cuda:0")


def test_device_enqueue_pipelined_equal_oracle():
    """sg_flow_enqueue: device batches back to back (more than the 4 slots), each batch's sort beside the previous
    batch's walkers; decisions and the final window state equal the oracle's sequential replay."""
    import torch
    wl, eng, ora = _setup(seed=33)
    nb = 9
    reqs = [wl.requests(b) for b in range(nb)]
    d_in = [_dev(r) for r in reqs]
    d_out = [torch.empty(len(r) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0") for r in reqs]
    torch.cuda.synchronize()
    tickets = [eng.enqueue_device(i.data_ptr(), len(r), o.data_ptr()) for i, o, r in zip(d_in, d_out, reqs)]
    for t in tickets:
        eng.wait(t)
    for b in range(nb):
        got = d_out[b].cpu().numpy().view(abi.RES_DTYPE)
        want = ora.decide(reqs[b])
        assert np.array_equal(got, want), f"batch {b}: {(got != want).sum()} differ"
    ring, occ = eng.export_state(len(wl.rules()))
    ring_o, occ_o = ora.export_state(len(wl.rules()), ring.shape[1])
    assert np.array_equal(ring, ring_o) and np.array_equal(occ, occ_o)


def test_device_enqueue_cross_batch_time_check():
    """A batch starting before the previous batch's last timestamp is rejected on its own ticket although its
    front half ran before the previous batch finished; the batches around it decide as the oracle."""
    import torch
    from sentinel_amd.engine import EngineError
    wl, eng, ora = _setup(seed=35)
    r0, r1, r2 = wl.requests(0), wl.requests(1), wl.requests(2)
    late = r0.copy()  # batch 0's timestamps again: older than batch 0's last
    bufs = [(_dev(r), torch.empty(len(r) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0"))
            for r in (r0, late, r1, r2)]
    torch.cuda.synchronize()
    t = [eng.enqueue_device(i.data_ptr(), len(i) // abi.REQ_DTYPE.itemsize, o.data_ptr()) for i, o in bufs]
    eng.wait(t[0])
    with pytest.raises(EngineError) as ei:
        eng.wait(t[1])
    assert ei.value.code == abi.SG_E_TIME
    eng.wait(t[2])
    eng.wait(t[3])
    for (i, o), r in zip([bufs[0], bufs[2], bufs[3]], [r0, r1, r2]):
        assert np.array_equal(o.cpu().numpy().view(abi.RES_DTYPE), ora.decide(r))


def test_device_enqueue_with_limiter_and_sync_calls_between():
    """Pipelined batches with a namespace limiter (each front half checks the time order against the previous front
    half's, so the limiter pre-pass sees accepted batches only, without waiting for the previous walkers) mixed with
    synchronous calls, which drain the pipeline first."""
    import torch
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import FlowEngine
    from sentinel_amd.workload import ClusterWorkload
    wl = ClusterWorkload(n_flows=2000, n_requests=60_000, seed=37, prio_frac=0.05)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 20_000
    ns["limiter_enabled"] = 1
    eng = FlowEngine(device=0, max_batch=60_000)
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules())
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(wl.rules())
    reqs = [wl.requests(b) for b in range(6)]
    outs = {}
    pend = []
    for b, r in enumerate(reqs):
        if b == 3:  # synchronous call in between
            outs[b] = eng.decide_host(r)
            continue
        i, o = _dev(r), torch.empty(len(r) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0")
        pend.append((b, i, o, eng.enqueue_device(i.data_ptr(), len(r), o.data_ptr())))
        if b == 2:
            for bb, _, oo, t in pend:
                eng.wait(t)
                outs[bb] = oo.cpu().numpy().view(abi.RES_DTYPE)
            pend = []
    for bb, _, oo, t in pend:
        eng.wait(t)
        outs[bb] = oo.cpu().numpy().view(abi.RES_DTYPE)
    for b, r in enumerate(reqs):
        want = ora.decide(r)
        assert np.array_equal(outs[b], want), f"batch {b}: {(outs[b] != want).sum()} differ"


@pytest.mark.parametrize("lim_pipe", ["1", "0"])
def test_device_enqueue_with_limiter_rejects_a_late_batch(monkeypatch, lim_pipe):
    """Four limiter batches in flight, the second older than the first: it is refused on its own ticket, its
    requests never reach the namespace limiter (the following batches' TOO_MANY_REQUEST answers equal the oracle's,
    which never saw it), and the flowIds' rings equal the oracle's. SG_LIM_PIPE=0: the front halves wait for the
    previous back half (the round-4 order), same answers."""
    import torch
    from oracle.binding import ClusterTokenService
    from sentinel_amd.engine import EngineError, FlowEngine
    from sentinel_amd.workload import ClusterWorkload
    monkeypatch.setenv("SG_LIM_PIPE", lim_pipe)
    wl = ClusterWorkload(n_flows=1500, n_requests=50_000, seed=41, prio_frac=0.05)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30_000
    ns["limiter_enabled"] = 1
    eng = FlowEngine(device=0, max_batch=50_000)
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules())
    ora = ClusterTokenService()
    ora.set_namespaces(ns)
    ora.load_rules(wl.rules())
    r0, r1, r2 = wl.requests(0), wl.requests(1), wl.requests(2)
    late = r0.copy()
    bufs = [(_dev(r), torch.empty(len(r) * abi.RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda:0"))
            for r in (r0, late, r1, r2)]
    torch.cuda.synchronize()
    t = [eng.enqueue_device(i.data_ptr(), len(i) // abi.REQ_DTYPE.itemsize, o.data_ptr()) for i, o in bufs]
    eng.wait(t[0])
    with pytest.raises(EngineError) as ei:
        eng.wait(t[1])
    assert ei.value.code == abi.SG_E_TIME
    eng.wait(t[2])
    eng.wait(t[3])
    for (i, o), r in zip([bufs[0], bufs[2], bufs[3]], [r0, r1, r2]):
        want = ora.decide(r)
        got = o.cpu().numpy().view(abi.RES_DTYPE)
        assert (want["status"] == abi.TOO_MANY_REQUEST).any()
        assert np.array_equal(got, want), f"{(got != want).sum()} results differ"
    ring, occ = eng.export_state(len(wl.rules()))
    ring_o, occ_o = ora.export_state(len(wl.rules()), ring.shape[1])
    assert np.array_equal(ring, ring_o) and np.array_equal(occ, occ_o)
