"""Parity of the device metric snapshots with the oracle:

  sg_local_metrics      MetricTimerListener.run / StatisticNode.metrics() rows of every resource after batches of
                        local-chain traffic, called repeatedly (lastFetchTime) — rows and the minute windows after
                        the call (currentWindow's side effect) compared exactly;
  sg_cparam_top_values  ClusterParamMetric.getTopValues(5) of every cluster param rule (ties by value).
"""
import numpy as np
import pytest

from oracle.binding import ClusterTokenService, LocalChain, LocalTraceGen, degrade_rule, local_rule
from sentinel_amd import abi

from test_cparam_gpu import _pair as cp_pair
from test_cparam_gpu import _rules as cp_rules
from test_cparam_gpu import _check as cp_check
from test_cparam_gpu import _trace as cp_trace
from test_local_gpu import _entries

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("S,interval,inbound", [(2, 1000, False), (4, 1000, True), (5, 500, True)])
def test_local_metric_rows(S, interval, inbound):
    """inbound: a third of the resources are EntryType.IN, so the rows end with Constants.ENTRY_NODE's
    (__total_inbound_traffic__, MetricTimerListener.java:46): the device sums the inbound resources' buckets, the
    oracle keeps the ENTRY_NODE as its own StatisticNode."""
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(40 + S)
    n_res = 40
    rules = np.zeros(n_res, abi.LOCAL_RULE_DTYPE)
    for i in range(n_res):
        brk = [degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.3, 1, 5, 1000)] if i % 4 == 0 else []
        rules[i] = local_rule(float(rng.integers(5, 60)), abi.FLOW_GRADE_QPS, brk)
    ora = LocalChain(S, interval, 500)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    eng = FlowEngine(device=0, max_batch=1 << 20)
    eng.local_load_rules(rules, S, interval, 500)
    if inbound:
        ib = (np.arange(n_res) % 3 == 0).astype(np.uint8)
        ora.set_entry_types(ib)
        eng.local_set_entry_types(ib)
    entry_rows = 0
    t = 1_700_000_000_000 + int(rng.integers(0, 1000))
    for b, (n, span) in enumerate([(20_000, 2500), (20_000, 1800), (5_000, 65_000), (10_000, 900)]):
        ent = _entries(rng, n, n_res, t, span, prio=0.1)
        ev, want = gen.run(ent, rng.integers(0, 50, n).astype(np.int32), (rng.random(n) < 0.1).astype(np.uint8), t + span)
        got = eng.local_decide_host(ev)
        assert np.array_equal(got, want)
        t += span
        last_ts = int(ev["ts_ms"].max())
        for now in (t - 400, t + 300, t + 300):  # a repeat at the same time reports nothing new
            w_rows = ora.metrics(now)
            g_rows = eng.local_metrics(now)
            if now < last_ts:
                # the ENTRY_NODE row is exact when fetched at or after the latest event (as MetricTimerListener
                # does): behind it, a slot the ENTRY_NODE already moved to a later second may still hold an
                # older second in some resource (include/sentinel_gpu.h, sg_local_metrics)
                w_rows = w_rows[w_rows["resource"] != abi.ENTRY_NODE_RESOURCE]
                g_rows = g_rows[g_rows["resource"] != abi.ENTRY_NODE_RESOURCE]
            assert np.array_equal(w_rows, g_rows), f"batch {b} now {now}: {len(w_rows)} vs {len(g_rows)} rows"
            entry_rows += int((w_rows["resource"] == abi.ENTRY_NODE_RESOURCE).sum())
        for r in range(0, n_res, 7):
            assert np.array_equal(ora.dump(r)[2], eng.local_state(r)[2]), f"minute window of {r}"
    assert (entry_rows > 0) == inbound


def test_cparam_top_values():
    rng = np.random.default_rng(50)
    rules = cp_rules(30, rng, S=5, interval=1000)
    eng, ora = cp_pair(rules)
    t = 1_700_000_000_000
    for b in range(3):
        req, values = cp_trace(rng, 30_000, 30, 400, t, 900, zipf=1.2)
        cp_check(eng, ora, req, values)
        t += 900
        # at the current time: not behind the batch (the per-value rings equal the bucket maps only from the latest
        # request on) and not ahead of the next one (getTopValues' currentWindow would open a future bucket)
        for now in (t,) if b < 2 else (t, t + 400):
            got = eng.cparam_top_values(now, len(rules), 5)
            for k in range(len(rules)):
                assert got[k] == ora.param_top(k, now, 5), f"rule {k} at {now}: {got[k]} vs {ora.param_top(k, now, 5)}"
