"""Known-answer tests of the ParamFlowSlot oracle (oracle.binding.ParamFlowSlot), restating the reference's tests
on the replay model (a mocked thread count is produced by entries that passed and did not exit yet):

  ParamFlowCheckerTest.{testHotParamCheckerPassCheckExceedArgs, testSingleValueCheckQpsWithExceptionItems,
  testSingleValueCheckThreadCountWithExceptionItems, testPassLocalCheckForCollection, testPassLocalCheckForArray,
  testPassLocalCheckForComplexParam}     sentinel-extension/sentinel-parameter-flow-control/src/test/.../param/
                                        ParamFlowCheckerTest.java:47-212
  ParamFlowSlotTest.testNegativeParamIdx                                    …/param/ParamFlowSlotTest.java:51-77
"""
import numpy as np

from oracle.binding import ParamFlowSlot
from sentinel_amd import abi

T0 = 1_700_000_000_000
QPS, THREAD = 1, 0


def rule(res=0, idx=0, count=10.0, grade=QPS, behavior=0, hot_begin=0, hot_count=0, dur=1, max_q=0):
    r = np.zeros((), abi.PSLOT_RULE_DTYPE)
    r["rule"]["count"], r["rule"]["duration_sec"], r["rule"]["behavior"] = count, dur, behavior
    r["rule"]["max_queueing_ms"], r["rule"]["hot_begin"], r["rule"]["hot_count"] = max_q, hot_begin, hot_count
    r["resource"], r["param_idx"], r["grade"] = res, idx, grade
    return r


class Calls:
    """Builds events / args / values for a sequence of SphU.entry(resource, count, args...) calls."""

    def __init__(self):
        self.ev, self.args, self.values = [], [], []

    def arg(self, a):
        if a is None:
            return (0, 0, abi.ARG_NULL, 0)
        if isinstance(a, (list, tuple)):
            b = len(self.values)
            self.values += list(a)
            return (b, len(a), abi.ARG_COLLECTION, 0)
        self.values.append(a)
        return (len(self.values) - 1, 1, abi.ARG_VALUE, 0)

    def call(self, t, *args, res=0, count=1, kind=abi.LOCAL_ENTRY, null_args=False):
        b = len(self.args)
        self.args += [self.arg(a) for a in args]
        self.ev.append((t, res, count, kind, b, len(args), 1 if null_args else 0))
        return self

    def arrays(self):
        ev = np.array(self.ev, abi.PSLOT_EVENT_DTYPE)
        args = np.array(self.args, abi.PSLOT_ARG_DTYPE) if self.args else np.zeros(0, abi.PSLOT_ARG_DTYPE)
        return ev, args, np.array(self.values, np.uint64)


def run(ps, calls):
    return ps.decide(*calls.arrays())


def test_pass_check_exceed_args():
    ps = ParamFlowSlot(np.array([rule(idx=1, count=10)]))
    assert run(ps, Calls().call(T0, 7))["pass"][0] == 1   # paramIdx 1 beyond the one argument


def test_single_value_qps_with_exception_items():
    A, B = 11, 12
    hot = np.array([(B, 0, 0), (14, 7, 0)], abi.PARAM_HOT_DTYPE)   # valueB threshold 0, valueD 7
    ps = ParamFlowSlot(np.array([rule(count=5, behavior=2, hot_count=2)]), hot)
    out = run(ps, Calls().call(T0, A).call(T0, B))
    assert list(out["pass"]) == [1, 0] and list(out["rule"]) == [-1, 0]


def test_single_value_thread_count_with_exception_items():
    A, B, C, D = 1, 2, 3, 4
    hot = np.array([(B, 3, 0), (D, 7, 0)], abi.PARAM_HOT_DTYPE)
    ps = ParamFlowSlot(np.array([rule(count=5, grade=THREAD, hot_count=2)]), hot)
    c = Calls()
    for v, k in ((A, 4), (B, 3), (C, 4), (D, 6)):      # threads in flight (no exits yet)
        for _ in range(k):
            c.call(T0, v)
    pre = run(ps, c)
    assert list(pre["pass"]) == [1] * 17
    # A: ++4 <= 5, B: ++3 > 3 (hot 3), C: ++4 <= 5, D: ++6 <= 7 (hot 7)
    out = run(ps, Calls().call(T0 + 1, A).call(T0 + 1, B).call(T0 + 1, C).call(T0 + 1, D))
    assert list(out["pass"]) == [1, 0, 1, 1]
    # now A = 5, C = 5, D = 7: all at their thresholds
    out = run(ps, Calls().call(T0 + 2, A).call(T0 + 2, C).call(T0 + 2, D))
    assert list(out["pass"]) == [0, 0, 0]
    # exits give the threads back
    out = run(ps, Calls().call(T0 + 3, A, kind=abi.LOCAL_EXIT).call(T0 + 3, A))
    assert ps.thread_count(0, 0, A) == 5 and list(out["pass"]) == [1, 1]


def test_pass_local_check_collection_and_array():
    for behavior in (0, 2):   # token bucket (collection) and throttle (array)
        ps = ParamFlowSlot(np.array([rule(count=1, behavior=behavior)]))
        out = run(ps, Calls().call(T0, [101, 102, 103]).call(T0, [101, 102, 103]))
        assert list(out["pass"]) == [1, 0]


def test_collection_early_exit_keeps_earlier_elements_state():
    ps = ParamFlowSlot(np.array([rule(count=1)]))
    out = run(ps, Calls().call(T0, [5]).call(T0, [6, 5, 7]))
    assert list(out["pass"]) == [1, 0]
    assert ps.token_state(0, 6)[0] == 3 and ps.token_state(0, 6)[2] == 0     # 6 consumed its token
    assert ps.token_state(0, 7)[0] == 0                                        # 7 was never checked


def test_complex_param_first_arg():
    ps = ParamFlowSlot(np.array([rule(count=1)]))
    out = run(ps, Calls().call(T0, 999, 10, 77).call(T0, 999, 10, 77))  # paramFlowKey() of the User: its name
    assert list(out["pass"]) == [1, 0]


def test_negative_param_idx():
    ps = ParamFlowSlot(np.array([rule(idx=-1, count=1)]))
    run(ps, Calls().call(T0, 1, 2, 3))
    assert ps.param_idx(0) == 2
    ps = ParamFlowSlot(np.array([rule(idx=-1, count=1)]))
    run(ps, Calls().call(T0, null_args=True))        # null args: no conversion
    assert ps.param_idx(0) == -1
    ps = ParamFlowSlot(np.array([rule(idx=-100, count=1)]))
    run(ps, Calls().call(T0, 1, 2, 3))
    assert ps.param_idx(0) == 100
    ps = ParamFlowSlot(np.array([rule(idx=0, count=1)]))
    run(ps, Calls().call(T0, 1, 2, 3))
    assert ps.param_idx(0) == 0


def test_several_rules_first_failure_wins():
    """Two rules on different arguments: the second rule is only reached when the first passes."""
    ps = ParamFlowSlot(np.array([rule(idx=0, count=2), rule(idx=1, count=1)]))
    out = run(ps, Calls().call(T0, 1, 50).call(T0, 1, 50).call(T0, 1, 51).call(T0, 2, 51))
    assert list(out["pass"]) == [1, 0, 0, 1] and list(out["rule"]) == [-1, 1, 0, -1]
    assert ps.token_state(1, 51)[0] == 3   # only the 4th call reached rule 1 with value 51
