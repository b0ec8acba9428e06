"""Parity of the pipelined local slot chain (sg_local_enqueue / sg_local_wait) with the oracle's sequential replay.

Batches are enqueued back to back on device buffers, so the front half of batch i+1 (validation, sort, segment and
exit lists) runs beside the walkers of batch i and the two batch workspaces alternate. Every result and every
resource's windows, thread count and breaker state must equal oracle.binding.LocalChain replaying the same events
one at a time (the traces come from LocalTraceGen as in test_local_gpu.py), including a batch rejected in the middle
of the pipeline (its first timestamp older than the batch before: checked in the back half, after that batch has
advanced the last timestamp) and batches the pipeline does not take (origin tracking: decided synchronously).
"""
import numpy as np
import pytest

from oracle.binding import LocalChain, LocalTraceGen, degrade_rule, local_flow_rule
from sentinel_amd import abi

from test_local_gpu import WALKERS, _compare, _engine, _entries, _rules

pytestmark = pytest.mark.gpu


def _trace(rules, batches, S, interval, occupy, seed, rt_hi=40, err=0.05, **kw):
    """The oracle decides the batches in order: [(events, oracle results)], the oracle, its state after them."""
    rng = np.random.default_rng(seed)
    ora = LocalChain(S, interval, occupy)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    out = []
    for n, span in batches:
        ent = _entries(rng, n, len(rules), t, span, **kw)
        rt = rng.integers(0, rt_hi + 1, n).astype(np.int32)
        er = (rng.random(n) < err).astype(np.uint8)
        ev, want = gen.run(ent, rt, er, t + span)
        out.append((ev, want))
        t += span
    return out, ora


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to("cuda")


def _enqueue_all(eng, evs):
    """Every batch on the pipeline before the first wait, each with its own out buffer."""
    import torch
    bufs = []
    for ev in evs:
        d_ev = _dev(ev)
        d_out = torch.zeros(len(ev) * abi.LOCAL_RES_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        bufs.append((d_ev, d_out, eng.local_enqueue(d_ev.data_ptr(), len(ev), d_out.data_ptr())))
    return bufs


def _results(d_out):
    return d_out.cpu().numpy().view(abi.LOCAL_RES_DTYPE)


def _check(got, want, b):
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        raise AssertionError(f"batch {b}: {len(bad)} results differ; first at {bad[0]}: oracle={want[bad[0]]} "
                             f"gpu={got[bad[0]]}")


@pytest.mark.parametrize("flags", WALKERS)
def test_pipelined_batches_equal_the_oracle(flags):
    """Six batches in flight on the two workspaces (four device tickets: the fifth enqueue completes the first)."""
    rng = np.random.default_rng(21)
    rules = _rules(40, rng, lo=2, hi=40, breakers=[degrade_rule(abi.DEGRADE_RT, 20, 1, 5, 1000, 0.3),
                                                    degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.2, 1, 5, 500)])
    trace, ora = _trace(rules, [(20_000, 700), (25_000, 900), (5_000, 150), (30_000, 1200), (20_000, 500),
                                (10_000, 800)], 2, 1000, 500, seed=21, zipf=1.2, err=0.15)
    eng = _engine(flags=flags)
    eng.local_load_rules(rules, 2, 1000, 500)
    bufs = _enqueue_all(eng, [ev for ev, _ in trace])
    for b, ((_, want), (_, d_out, ticket)) in enumerate(zip(trace, bufs)):
        eng.local_wait(ticket)
        _check(_results(d_out), want, b)
    _compare(eng, ora, len(rules), 2)


def test_pipelined_saturated_hot_resources_and_prio():
    """Hot resources far above their threshold (dead-period skips on both workspaces) and prioritized entries."""
    rng = np.random.default_rng(22)
    rules = _rules(6, rng, lo=5, hi=40, breakers=[degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)])
    trace, ora = _trace(rules, [(150_000, 1000), (150_000, 1000), (100_000, 700)], 2, 1000, 500, seed=22,
                        zipf=1.5, rt_hi=20, err=0.2, prio=0.05)
    eng = _engine()
    eng.local_load_rules(rules, 2, 1000, 500)
    bufs = _enqueue_all(eng, [ev for ev, _ in trace])
    for b, ((_, want), (_, d_out, ticket)) in enumerate(zip(trace, bufs)):
        eng.local_wait(ticket)
        _check(_results(d_out), want, b)
    _compare(eng, ora, len(rules), 2)


def test_pipelined_rejects_an_older_batch_as_a_whole():
    """A batch whose first event is older than the previous batch's last is rejected (SG_E_TIME on its ticket)
    after the front half of the next batch has already run beside it; the batches around it decide as if it had
    never been sent. A batch out of order inside itself is rejected too (k_local_prep)."""
    from sentinel_amd.engine import EngineError
    rng = np.random.default_rng(23)
    rules = _rules(30, rng, lo=2, hi=25, breakers=[degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.25, 1, 5, 800)])
    trace, ora = _trace(rules, [(15_000, 800), (15_000, 800), (15_000, 800)], 2, 1000, 500, seed=23, err=0.2)
    older = trace[0][0].copy()          # batch 0 again: its first timestamp is older than batch 0's last
    unordered = trace[1][0].copy()
    unordered["ts_ms"][10] = unordered["ts_ms"][11] + 1  # event 10 later than event 11
    evs = [trace[0][0], older, trace[1][0], unordered, trace[2][0]]
    eng = _engine()
    eng.local_load_rules(rules, 2, 1000, 500)
    bufs = _enqueue_all(eng, evs)
    codes = []
    for _, _, ticket in bufs:
        try:
            eng.local_wait(ticket)
            codes.append(0)
        except EngineError as e:
            codes.append(e.code)
    assert codes == [0, abi.SG_E_TIME, 0, abi.SG_E_TIME, 0]
    for b, (want_idx, buf_idx) in enumerate([(0, 0), (1, 2), (2, 4)]):
        _check(_results(bufs[buf_idx][1]), trace[want_idx][1], b)
    _compare(eng, ora, len(rules), 2)


def test_pipelined_with_synchronous_calls_between():
    """Synchronous decisions and state reads between enqueues complete the batches in flight first."""
    rng = np.random.default_rng(24)
    rules = _rules(25, rng, lo=3, hi=30)
    trace, ora = _trace(rules, [(10_000, 600), (10_000, 600), (10_000, 600), (10_000, 600)], 2, 1000, 500, seed=24)
    eng = _engine()
    eng.local_load_rules(rules, 2, 1000, 500)
    bufs = _enqueue_all(eng, [trace[0][0], trace[1][0]])
    got2 = eng.local_decide_host(trace[2][0])   # after both enqueued batches
    _check(got2, trace[2][1], 2)
    bufs += _enqueue_all(eng, [trace[3][0]])
    for b, (i, (_, d_out, ticket)) in enumerate(zip([0, 1, 3], bufs)):
        eng.local_wait(ticket)
        _check(_results(d_out), trace[i][1], i)
    _compare(eng, ora, len(rules), 2)


def test_batches_the_pipeline_does_not_take_are_decided_synchronously():
    """With origin nodes tracked a batch syncs with the host mid-way: sg_local_enqueue decides it synchronously and
    its ticket carries the status (here against the plain oracle: the flow rules name no origin)."""
    rng = np.random.default_rng(25)
    rules = _rules(20, rng, lo=3, hi=30)
    trace, ora = _trace(rules, [(8_000, 600), (8_000, 600)], 2, 1000, 500, seed=25)
    eng = _engine()
    eng.local_load_rules(rules, 2, 1000, 500)
    frules = np.array([local_flow_rule(r, float(rules["flow_count"][r])) for r in range(len(rules))])
    eng.local_load_flow_rules(frules, n_origins=2)
    bufs = _enqueue_all(eng, [ev for ev, _ in trace])
    for b, ((_, want), (_, d_out, ticket)) in enumerate(zip(trace, bufs)):
        eng.local_wait(ticket)
        _check(_results(d_out), want, b)
    _compare(eng, ora, len(rules), 2)
