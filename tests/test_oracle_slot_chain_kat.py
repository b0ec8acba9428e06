"""Known-answer tests of the whole slot chain in the oracle (oracle.binding.LocalChain with an attached
ParamFlowSlot: sg_slot_decide_batch's semantics). No reference test drives ParamFlowSlot together with FlowSlot /
DegradeSlot through SphU.entry, so each case below is traced by hand through the Java text:

  StatisticSlot.entry / exit      sentinel-core/.../slots/statistic/StatisticSlot.java:55-165 (checks first; a pass
                                  raises threads + PASS and runs the entry callbacks' onPass; a BlockException of any
                                  slot — ParamFlowException included — adds BLOCK; exits only for passed entries)
  ParamFlowSlot (@Spi -3000)      sentinel-extension/.../param/ParamFlowSlot.java:38-93 (runs before FlowSlot -2000)
  ParamFlowStatisticEntryCallback.onPass / ExitCallback.onExit
                                  sentinel-extension/.../slots/statistic/ParamFlowStatistic{Entry,Exit}Callback.java
                                  (param thread counts rise only when the whole chain passed)
"""
import numpy as np
import pytest

from oracle.binding import LocalChain, ParamFlowSlot, local_flow_rule, local_rule
from sentinel_amd import abi
from tests.test_oracle_pslot_kat import QPS, THREAD, rule

T0S = [1_700_000_000_000, 1_700_000_000_437, 86_400_000 * 365 + 17]


class Chain:
    """One LocalChain + ParamFlowSlot; calls carry (context, args) like sg_slot_ext."""

    def __init__(self, n_res, flow_rules, param_rules, n_contexts=0, n_origins=0):
        self.c = LocalChain()
        self.c.load_rules(np.array([local_rule() for _ in range(n_res)]))
        if flow_rules:
            self.c.load_flow_rules(np.array(flow_rules), n_origins=n_origins, n_contexts=n_contexts)
        self.ps = ParamFlowSlot(np.array(param_rules), n_resources=n_res)
        self.c.attach_params(self.ps)
        self.args, self.values = [], []

    def _args(self, args):
        b = len(self.args)
        for a in args:
            if a is None:
                self.args.append((0, 0, abi.ARG_NULL, 0))
            elif isinstance(a, (list, tuple)):
                self.args.append((len(self.values), len(a), abi.ARG_COLLECTION, 0))
                self.values += list(a)
            else:
                self.args.append((len(self.values), 1, abi.ARG_VALUE, 0))
                self.values.append(a)
        return b

    def event(self, t, res, kind, args, create=0, ctx=0, count=1, origin=0):
        ev = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
        ev[0] = (t, create, res, count, kind, origin)
        x = np.zeros(1, abi.SLOT_EXT_DTYPE)
        x[0] = (ctx, self._args(args), len(args), 0)
        a = np.array(self.args, abi.PSLOT_ARG_DTYPE) if self.args else np.zeros(0, abi.PSLOT_ARG_DTYPE)
        r = self.c.decide_ext(ev, x, a, np.array(self.values, np.uint64))[0]
        return int(r["status"]), int(r["wait_ms"])

    def entry(self, t, *args, res=0, **kw):
        return self.event(t, res, abi.LOCAL_ENTRY, args, **kw)

    def exit(self, t, create, *args, res=0, **kw):
        return self.event(t, res, abi.LOCAL_EXIT, args, create=create, **kw)


@pytest.mark.parametrize("t0", T0S)
def test_param_thread_count_rises_only_when_the_whole_chain_passes(t0):
    """A THREAD-grade param rule (count 1 per value) with a QPS flow rule (count 1): an entry that passes
    ParamFlowSlot but is blocked by FlowSlot does not raise the value's thread count (onPass never runs)."""
    ch = Chain(1, [local_flow_rule(0, count=1)], [rule(idx=0, count=1, grade=THREAD)])
    assert ch.entry(t0, 7) == (abi.LOCAL_PASS, 0)
    assert ch.ps.thread_count(0, 0, 7) == 1
    assert ch.entry(t0, 8)[0] == abi.LOCAL_BLOCK_FLOW           # param passes, flow blocks
    assert ch.entry(t0, 8)[0] == abi.LOCAL_BLOCK_FLOW           # still 0 threads for value 8
    assert ch.ps.thread_count(0, 0, 8) == 0
    assert ch.entry(t0, 7) == (abi.LOCAL_BLOCK_PARAM, 0)        # value 7 holds its one thread: rule 0 throws
    # StatisticSlot counted every BlockException, the ParamFlowException too
    assert ch.c.second_sum(0, t0, 0) == 1 and ch.c.second_sum(0, t0, 1) == 3
    assert ch.c.threads(0) == 1
    ch.exit(t0 + 5, t0, 7)                                      # ParamFlowStatisticExitCallback
    assert ch.ps.thread_count(0, 0, 7) == 0 and ch.c.threads(0) == 0


@pytest.mark.parametrize("t0", T0S)
def test_param_tokens_are_spent_before_flow_slot_runs(t0):
    """ParamFlowSlot runs before FlowSlot: a token bucket pays for an entry FlowSlot then blocks, and an entry
    ParamFlowSlot blocks never reaches the flow rule's controller (its latestPassedTime stays)."""
    ch = Chain(1, [local_flow_rule(0, count=10, behavior=abi.CONTROL_RATE_LIMITER, max_queueing_ms=1)],
               [rule(idx=0, count=2, grade=QPS)])
    assert ch.entry(t0, 5) == (abi.LOCAL_PASS, 0)               # tokens 2 - 1; latestPassedTime = t0
    assert ch.entry(t0, 5)[0] == abi.LOCAL_BLOCK_FLOW           # tokens 1 - 1; the limiter would wait 100 ms
    assert ch.ps.token_state(0, 5)[2] == 0
    assert ch.entry(t0, 5) == (abi.LOCAL_BLOCK_PARAM, 0)        # no token left: the limiter is not asked
    assert ch.c.controller(0)[2] == t0
    assert ch.entry(t0 + 100, 6)[0] == abi.LOCAL_PASS           # another value, the limiter's next slot


@pytest.mark.parametrize("t0", T0S)
def test_param_block_reports_the_rule_and_reaches_origin_and_context_nodes(t0):
    """The second param rule of the resource throws (wait_ms carries its index); the block lands on the
    ClusterNode, the origin node and the context's DefaultNode (StatisticSlot.java:96-113)."""
    fr = [local_flow_rule(0, count=100, limit_app=1), local_flow_rule(0, count=100, strategy=abi.STRATEGY_CHAIN, ref=1)]
    ch = Chain(1, fr, [rule(idx=0, count=100, grade=QPS), rule(idx=1, count=1, grade=QPS)], n_contexts=2, n_origins=1)
    assert ch.entry(t0, 1, 9, origin=1, ctx=1)[0] == abi.LOCAL_PASS
    assert ch.entry(t0, 1, 9, origin=1, ctx=1) == (abi.LOCAL_BLOCK_PARAM, 1)
    so = ch.c.origin_dump(0, 1)
    sc = ch.c.context_dump(0, 1)
    for d in (so, sc):
        assert d[0][:, 1].sum() == 1 and d[0][:, 2].sum() == 1 and d[3] == 1
    assert ch.c.second_sum(0, t0, 1) == 1


@pytest.mark.parametrize("t0", T0S)
def test_null_args_skip_param_flow_slot(t0):
    """args == null: ParamFlowSlot.checkFlow returns at once and the callbacks do nothing (addThreadCount /
    decreaseThreadCount return on null args)."""
    ch = Chain(1, [], [rule(idx=0, count=0, grade=QPS)])
    ev = np.zeros(2, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"] = t0, 1
    x = np.zeros(2, abi.SLOT_EXT_DTYPE)
    x["args_null"] = 1
    out = ch.c.decide_ext(ev, x, np.zeros(0, abi.PSLOT_ARG_DTYPE), np.zeros(0, np.uint64))
    assert (out["status"] == abi.LOCAL_PASS).all()
    assert ch.entry(t0, 3)[0] == abi.LOCAL_BLOCK_PARAM         # count 0: tokenCount 0 blocks any value


@pytest.mark.parametrize("t0", T0S)
def test_degrade_slot_runs_after_param_and_flow(t0):
    """An OPEN breaker rejects an entry only after ParamFlowSlot passed it (so the token is spent)."""
    c = LocalChain()
    brk = np.zeros((), abi.DEGRADE_RULE_DTYPE)
    brk["grade"], brk["count"], brk["time_window_sec"] = abi.DEGRADE_EXCEPTION_COUNT, 0, 10
    brk["min_request_amount"], brk["stat_interval_ms"] = 1, 1000
    c.load_rules(np.array([local_rule(0.0, abi.FLOW_GRADE_NONE, [brk])]))
    ps = ParamFlowSlot(np.array([rule(idx=0, count=3, grade=QPS)]), n_resources=1)
    c.attach_params(ps)
    ch = Chain.__new__(Chain)
    ch.c, ch.ps, ch.args, ch.values = c, ps, [], []
    assert ch.entry(t0, 4)[0] == abi.LOCAL_PASS                 # tokens 3 - 1
    ev = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
    ev[0] = (t0 + 1, t0, 0, 1, abi.LOCAL_EXIT_ERROR, 0)         # one error opens the breaker (count > 0)
    x = np.zeros(1, abi.SLOT_EXT_DTYPE)
    x[0] = (0, 0, 1, 0)
    c.decide_ext(ev, x, np.array(ch.args, abi.PSLOT_ARG_DTYPE), np.array(ch.values, np.uint64))
    assert ch.entry(t0 + 2, 4)[0] == abi.LOCAL_BLOCK_DEGRADE    # tokens 2 - 1, then DegradeException
    assert ps.token_state(0, 4)[2] == 1
