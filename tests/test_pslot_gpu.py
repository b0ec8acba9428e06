"""Parity of the device ParamFlowSlot chain (sg_pslot_*) with the oracle (oracle.binding.ParamFlowSlot): several
param rules per resource (QPS token bucket and throttle, THREAD grade, hot items, negative paramIdx), arguments
that are null, single values or collections / arrays (checked element by element with early exit), and the exits
of passed entries lowering the thread counts. Every result, the rule that blocked, the thread counts, the
resolved paramIdx and the token state of the touched (rule, value) pairs are compared exactly."""
import numpy as np
import pytest

from oracle.binding import ParamFlowSlot
from sentinel_amd import abi

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _rules(rng, n_res):
    rules, hot = [], []
    for res in range(n_res):
        for _ in range(int(rng.integers(1, 4))):
            r = np.zeros((), abi.PSLOT_RULE_DTYPE)
            grade = 0 if rng.random() < 0.3 else 1
            r["resource"], r["grade"] = res, grade
            r["param_idx"] = int(rng.integers(0, 3)) if rng.random() < 0.8 else -int(rng.integers(1, 4))
            r["rule"]["count"] = float(rng.integers(1, 6)) if grade == 0 else float(rng.integers(2, 30))
            r["rule"]["duration_sec"] = int(rng.integers(1, 3))
            r["rule"]["burst"] = int(rng.integers(0, 3))
            r["rule"]["behavior"] = 2 if (grade == 1 and rng.random() < 0.3) else 0
            r["rule"]["max_queueing_ms"] = int(rng.integers(0, 300))
            r["rule"]["capacity_log2"] = 12
            k = int(rng.integers(0, 3))
            r["rule"]["hot_begin"], r["rule"]["hot_count"] = len(hot), k
            for _ in range(k):
                hot.append((int(rng.integers(1, 40)), int(rng.integers(0, 8)), 0))
            rules.append(r)
    # a rule's hot items need distinct values
    out_hot = []
    for r in rules:
        b, k = int(r["rule"]["hot_begin"]), int(r["rule"]["hot_count"])
        seen = {}
        for v, t, _ in hot[b:b + k]:
            seen[v] = t
        r["rule"]["hot_begin"], r["rule"]["hot_count"] = len(out_hot), len(seen)
        out_hot += [(v, t, 0) for v, t in seen.items()]
    return np.array(rules, abi.PSLOT_RULE_DTYPE), np.array(out_hot, abi.PARAM_HOT_DTYPE)


class Gen:
    def __init__(self, seed, n_res):
        self.rng = np.random.default_rng(seed)
        self.n_res = n_res
        self.open = []  # (resource, args tuple) of passed entries not exited yet
        self.t = T0

    def _arg(self):
        u = self.rng.random()
        if u < 0.1:
            return None
        if u < 0.45:
            return [int(x) for x in self.rng.integers(1, 40, int(self.rng.integers(1, 5)))]
        return int(self.rng.integers(1, 40))

    def batch(self, n, span):
        ev, args, vals, entries = [], [], [], []
        ts = self.t + np.sort(self.rng.integers(0, span, n))
        for i in range(n):
            if self.open and self.rng.random() < 0.35:
                res, a = self.open.pop(int(self.rng.integers(len(self.open))))
                kind, nulla = abi.LOCAL_EXIT, 0
            else:
                res = int(self.rng.integers(0, self.n_res + 1))   # one unknown resource
                a = tuple(self._arg() for _ in range(int(self.rng.integers(0, 4))))
                kind, nulla = abi.LOCAL_ENTRY, int(self.rng.random() < 0.03)
            b = len(args)
            for x in a:
                if x is None:
                    args.append((0, 0, abi.ARG_NULL, 0))
                elif isinstance(x, list):
                    args.append((len(vals), len(x), abi.ARG_COLLECTION, 0))
                    vals += x
                else:
                    args.append((len(vals), 1, abi.ARG_VALUE, 0))
                    vals.append(x)
            ev.append((int(ts[i]), res, int(self.rng.integers(1, 3)), kind, b, len(a), nulla))
            entries.append((res, tuple(tuple(x) if isinstance(x, list) else x for x in a)))
        self.t += span
        ev = np.array(ev, abi.PSLOT_EVENT_DTYPE)
        args = np.array(args, abi.PSLOT_ARG_DTYPE) if args else np.zeros(0, abi.PSLOT_ARG_DTYPE)
        return ev, args, np.array(vals, np.uint64), entries

    def absorb(self, ev, res_out, entries):
        for e, r, (res, a) in zip(ev, res_out, entries):
            if e["kind"] == abi.LOCAL_ENTRY and r["pass"] == 1 and res < self.n_res and not e["args_null"]:
                self.open.append((res, tuple(list(x) if isinstance(x, tuple) else x for x in a)))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_param_slot_chain(seed):
    from sentinel_amd.engine import FlowEngine
    rng = np.random.default_rng(seed)
    n_res = 12
    rules, hot = _rules(rng, n_res)
    ora = ParamFlowSlot(rules, hot, n_resources=n_res)
    eng = FlowEngine(device=0, max_batch=1 << 17)
    eng.pslot_load_rules(rules, hot, n_resources=n_res)
    gen = Gen(seed, n_res)
    for b in range(5):
        ev, args, vals, entries = gen.batch(6000, 1500)
        want = ora.decide(ev, args, vals)
        got = eng.pslot_decide_host(ev, args, vals)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"batch {b}: {len(bad)} differ; first {bad[0]}: ev={ev[bad[0]]} {entries[bad[0]]} "
                                 f"oracle={want[bad[0]]} gpu={got[bad[0]]}")
        gen.absorb(ev, want, entries)
    for ri in range(len(rules)):
        assert eng.pslot_param_idx(ri) == ora.param_idx(ri)
    for res in range(n_res):
        for idx in range(3):
            for v in range(1, 40):
                assert eng.pslot_thread_count(res, idx, v) == ora.thread_count(res, idx, v), (res, idx, v)
    for ri in range(len(rules)):
        for v in range(1, 40):
            f, lt, tk = ora.token_state(ri, v)
            if f:
                gf, glt, gtk = eng.param_state(ri, v)
                assert (gf, glt if f & 1 else 0, gtk if f & 2 else 0) == (f, lt if f & 1 else 0, tk if f & 2 else 0)
