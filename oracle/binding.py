"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product path (sentinel_amd) never does.
"""
import ctypes as C
import os

import numpy as np

from sentinel_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

# leap array kinds (sentinel_oracle.h)
LEAP_BUCKET, LEAP_OCCUPIABLE, LEAP_FUTURE, LEAP_UNARY, LEAP_CLUSTER = range(5)
# MetricEvent ordinals
M_PASS, M_BLOCK, M_EXCEPTION, M_SUCCESS, M_RT, M_OCCUPIED_PASS = range(6)

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u32, u64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
    sig = {
        "or_d2i": (i32, [d]), "or_d2l": (i64, [d]), "or_math_round": (i64, [d]),
        "or_leap_new": (vp, [C.c_int, C.c_int, C.c_int]), "or_leap_free": (None, [vp]),
        "or_leap_current_window": (C.c_int, [vp, i64]),
        "or_leap_slot_start": (i64, [vp, C.c_int]), "or_leap_slot_get": (i64, [vp, C.c_int, C.c_int]),
        "or_leap_slot_add": (None, [vp, C.c_int, C.c_int, i64]),
        "or_leap_slot_min_rt": (i64, [vp, C.c_int]), "or_leap_slot_add_rt": (None, [vp, C.c_int, i64]),
        "or_leap_add": (None, [vp, i64, C.c_int, i64]),
        "or_leap_values": (C.c_int, [vp, i64, vp]), "or_leap_get_sum": (i64, [vp, i64, C.c_int]),
        "or_leap_valid_head": (C.c_int, [vp, i64]), "or_leap_previous_window": (C.c_int, [vp, i64]),
        "or_leap_window_value": (C.c_int, [vp, i64]), "or_leap_interval_sec": (d, [vp]),
        "or_leap_current_waiting": (i64, [vp, i64]), "or_leap_add_waiting": (None, [vp, i64, C.c_int]),
        "or_leap_borrow": (vp, [vp]),
        "or_cluster_metric_new": (vp, [C.c_int, C.c_int]),
        "or_cluster_metric_add": (None, [vp, i64, C.c_int, i64]),
        "or_cluster_metric_get_sum": (i64, [vp, i64, C.c_int]),
        "or_cluster_metric_get_avg": (d, [vp, i64, C.c_int]),
        "or_cluster_metric_try_occupy_next": (C.c_int, [vp, i64, C.c_int, C.c_int, d]),
        "or_cluster_metric_occupied": (i64, [vp, C.c_int]),
        "or_limiter_new": (vp, [d]), "or_limiter_free": (None, [vp]),
        "or_limiter_add": (None, [vp, i64, C.c_int]), "or_limiter_get_sum": (i64, [vp, i64]),
        "or_limiter_get_qps": (d, [vp, i64]), "or_limiter_can_pass": (C.c_int, [vp, i64]),
        "or_limiter_try_pass": (C.c_int, [vp, i64]), "or_limiter_set_qps_allowed": (None, [vp, d]),
        "or_limiter_get_qps_allowed": (d, [vp]),
        "or_cts_new": (vp, [d, d]), "or_cts_free": (None, [vp]),
        "or_cts_set_namespaces": (C.c_int, [vp, vp, u32]),
        "or_cts_load_rules": (C.c_int, [vp, vp, u32]),
        "or_cts_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_cts_read_state": (C.c_int, [vp, u32, vp, vp, vp]),
        "or_cts_sample_count": (C.c_int, [vp, u32]),
        "or_cts_avg": (d, [vp, u32, i64, C.c_int]),
        "or_cts_export_state": (C.c_int, [vp, C.c_int, vp, vp]),
        "or_pf_new": (vp, []), "or_pf_free": (None, [vp]),
        "or_pf_load_rules": (C.c_int, [vp, vp, u32, vp, u32]),
        "or_pf_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_pf_read_state": (C.c_int, [vp, u32, u64, vp, vp]),
        "or_pf_size": (u64, [vp]),
        "or_pace_new": (vp, []), "or_pace_free": (None, [vp]),
        "or_pace_load_rules": (C.c_int, [vp, vp, u32]),
        "or_pace_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_pace_latest": (i64, [vp, u32]),
        "or_local_new": (vp, [C.c_int, C.c_int, C.c_int]), "or_local_free": (None, [vp]),
        "or_local_load_rules": (C.c_int, [vp, vp, u32]),
        "or_local_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_local_second_sum": (i64, [vp, u32, i64, C.c_int]),
        "or_local_minute_sum": (i64, [vp, u32, i64, C.c_int]),
        "or_local_thread_num": (i64, [vp, u32]), "or_local_waiting": (i64, [vp, u32, i64]),
        "or_local_breaker_state": (C.c_int, [vp, u32, C.c_int, vp]),
        "or_local_dump": (C.c_int, [vp, u32, vp, vp, vp]),
        "or_cts_load_param_rules": (C.c_int, [vp, vp, u32, vp, u32]),
        "or_cts_decide_param": (C.c_int, [vp, vp, u64, vp, vp]),
        "or_cts_param_sum": (i64, [vp, u32, u64, i64]),
        "or_cpm_new": (vp, [C.c_int, C.c_int]), "or_cpm_free": (None, [vp]),
        "or_cpm_add": (None, [vp, i64, u64, C.c_int]), "or_cpm_get_sum": (i64, [vp, i64, u64]),
        "or_cpm_get_avg": (C.c_double, [vp, i64, u64]),
        "or_local_breaker_stat": (C.c_int, [vp, u32, C.c_int, vp, vp, vp]),
        "or_local_load_flow_rules": (C.c_int, [vp, vp, u32, C.c_int32, C.c_int32]),
        "or_local_decide_ext": (C.c_int, [vp, vp, vp, u64, vp, vp, vp]),
        "or_local_attach_pslot": (None, [vp, vp]),
        "or_local_attach_cluster": (C.c_int, [vp, vp, C.c_int]),
        "or_local_set_entry_types": (C.c_int, [vp, vp, u32]),
        "or_local_context_dump": (C.c_int, [vp, u32, C.c_int, vp, vp, vp, vp]),
        "or_lgen_run_ext": (u64, [vp, vp, vp, vp, vp, u64, i64, vp, vp, vp, u64, vp, vp]),
        "or_local_set_cold_factor": (None, [vp, C.c_int]),
        "or_local_origin_dump": (C.c_int, [vp, u32, C.c_int, vp, vp, vp, vp]),
        "or_local_controller": (C.c_int, [vp, u32, vp]),
        "or_local_rule_order": (C.c_int, [vp, u32, vp, u32]),
        "or_local_metrics": (i64, [vp, i64, vp, u64]),
        "or_local_metrics_raw": (i64, [vp, i64, vp, u64, C.c_int]),
        "or_cts_param_top": (C.c_int, [vp, u32, i64, C.c_int, vp, vp]),
        "or_cpm_top": (C.c_int, [vp, i64, C.c_int, vp, vp]),
        "or_pslot_new": (vp, []), "or_pslot_free": (None, [vp]),
        "or_pslot_load_rules": (C.c_int, [vp, vp, u32, vp, u32, u32]),
        "or_pslot_decide": (C.c_int, [vp, vp, u64, vp, vp, vp]),
        "or_pslot_thread_count": (i64, [vp, u32, C.c_int32, u64]),
        "or_pslot_param_idx": (C.c_int32, [vp, u32]),
        "or_pslot_token_state": (C.c_int, [vp, u32, u64, vp, vp]),
        "or_pslot_attach_cluster": (C.c_int, [vp, vp, C.c_int]),
        "or_conc_new": (vp, []), "or_conc_free": (None, [vp]),
        "or_conc_set_namespaces": (C.c_int, [vp, vp, u32]), "or_conc_load_rules": (C.c_int, [vp, vp, u32]),
        "or_conc_set_rule_timeouts": (C.c_int, [vp, vp, vp, u32]),
        "or_conc_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_conc_expire": (u64, [vp, i64, vp, u32]),
        "or_conc_now_calls": (C.c_int32, [vp, u32]), "or_conc_live": (u64, [vp]),
        "or_ctl_new": (vp, [vp, C.c_int]), "or_ctl_free": (None, [vp]), "or_ctl_state": (None, [vp, vp]),
        "or_ctl_warning_token": (C.c_int32, [vp]), "or_ctl_max_token": (C.c_int32, [vp]),
        "or_warm_can_pass": (C.c_int, [vp, i64, d, d, C.c_int]),
        "or_warm_rl_can_pass": (C.c_int, [vp, i64, d, C.c_int, vp]),
        "or_select_node": (C.c_int, [vp, u32, u32, C.c_int, C.c_int, C.c_int]),
        "or_lgen_new": (vp, [vp]), "or_lgen_free": (None, [vp]), "or_lgen_pending": (u64, [vp]),
        "or_lgen_run": (u64, [vp, vp, vp, vp, u64, i64, vp, vp, u64]),
        "or_rls_decide": (C.c_int, [vp, vp, u64, vp]),
        "or_rls_should_rate_limit": (C.c_int, [vp, vp, u32, vp, u64, vp, vp]),
        "or_codec_decode_flow": (None, [vp, vp, vp, u64, vp, u32, vp, vp, vp]),
        "or_codec_encode_flow": (None, [vp, vp, vp, u64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class Leap:
    """A LeapArray of the given kind (explicit time on every call)."""

    def __init__(self, kind, sample_count, interval_ms, handle=None, owner=None):
        self._owner = owner
        if handle is None:
            handle = lib().or_leap_new(kind, sample_count, interval_ms)
            if not handle:
                raise ValueError("invalid window config")
            self._own = True
        else:
            self._own = False
        self.h = handle

    def __del__(self):
        if getattr(self, "_own", False) and self.h:
            lib().or_leap_free(self.h)
            self.h = None

    def current_window(self, t):
        return lib().or_leap_current_window(self.h, t)

    def start(self, slot):
        return lib().or_leap_slot_start(self.h, slot)

    def get(self, slot, ev):
        return lib().or_leap_slot_get(self.h, slot, ev)

    def slot_add(self, slot, ev, n):
        lib().or_leap_slot_add(self.h, slot, ev, n)

    def add(self, t, ev, n):
        lib().or_leap_add(self.h, t, ev, n)

    def values(self, t):
        out = (C.c_int * 64)()
        k = lib().or_leap_values(self.h, t, out)
        return list(out[:k])

    def get_sum(self, t, ev):
        return lib().or_leap_get_sum(self.h, t, ev)

    def valid_head(self, t):
        return lib().or_leap_valid_head(self.h, t)

    def previous_window(self, t):
        return lib().or_leap_previous_window(self.h, t)

    def window_value(self, t):
        return lib().or_leap_window_value(self.h, t)

    def current_waiting(self, t):
        return lib().or_leap_current_waiting(self.h, t)

    def add_waiting(self, t, n):
        lib().or_leap_add_waiting(self.h, t, n)

    def borrow(self):
        return Leap(None, None, None, handle=lib().or_leap_borrow(self.h), owner=self)


class ClusterMetric(Leap):
    """srv/flow/statistic/metric/ClusterMetric.java with explicit time."""

    def __init__(self, sample_count, interval_ms):
        h = lib().or_cluster_metric_new(sample_count, interval_ms)
        if not h:
            raise ValueError("invalid window config")
        super().__init__(None, None, None, handle=h)
        self._own = True

    def add_event(self, t, ev, n):
        lib().or_cluster_metric_add(self.h, t, ev, n)

    def get_sum_event(self, t, ev):
        return lib().or_cluster_metric_get_sum(self.h, t, ev)

    def get_avg(self, t, ev):
        return lib().or_cluster_metric_get_avg(self.h, t, ev)

    def try_occupy_next(self, t, ev, acquire, threshold):
        return lib().or_cluster_metric_try_occupy_next(self.h, t, ev, acquire, threshold)

    def occupied(self, ev):
        return lib().or_cluster_metric_occupied(self.h, ev)


class RequestLimiter:
    """srv/flow/statistic/limit/RequestLimiter.java with explicit time."""

    def __init__(self, qps_allowed):
        self.h = lib().or_limiter_new(qps_allowed)

    def __del__(self):
        if self.h:
            lib().or_limiter_free(self.h)
            self.h = None

    def add(self, t, x):
        lib().or_limiter_add(self.h, t, x)

    def get_sum(self, t):
        return lib().or_limiter_get_sum(self.h, t)

    def get_qps(self, t):
        return lib().or_limiter_get_qps(self.h, t)

    def can_pass(self, t):
        return bool(lib().or_limiter_can_pass(self.h, t))

    def try_pass(self, t):
        return bool(lib().or_limiter_try_pass(self.h, t))

    def set_qps_allowed(self, q):
        lib().or_limiter_set_qps_allowed(self.h, q)

    def qps_allowed(self):
        return lib().or_limiter_get_qps_allowed(self.h)


class ClusterTokenService:
    """Sequential replay of DefaultTokenService.requestToken → ClusterFlowChecker for a rule set."""

    def __init__(self, exceed_count=1.0, max_occupy_ratio=1.0):
        self.h = lib().or_cts_new(exceed_count, max_occupy_ratio)

    def __del__(self):
        if self.h:
            lib().or_cts_free(self.h)
            self.h = None

    def set_namespaces(self, ns: np.ndarray):
        ns = np.ascontiguousarray(ns, dtype=abi.NS_DTYPE)
        rc = lib().or_cts_set_namespaces(self.h, abi.ptr(ns), len(ns))
        assert rc == 0

    def load_rules(self, rules: np.ndarray):
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        rc = lib().or_cts_load_rules(self.h, abi.ptr(rules), len(rules))
        if rc != 0:
            raise ValueError(f"invalid rules ({rc})")

    def decide(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.REQ_DTYPE)
        out = np.zeros(len(req), dtype=abi.RES_DTYPE)
        lib().or_cts_decide(self.h, abi.ptr(req), len(req), abi.ptr(out))
        return out

    def avg(self, key, now, ev):
        return lib().or_cts_avg(self.h, key, now, ev)

    def decide_rls(self, req: np.ndarray) -> np.ndarray:
        """Envoy RLS path: SimpleClusterFlowChecker.acquireClusterToken per request (no limiter, no occupy)."""
        req = np.ascontiguousarray(req, dtype=abi.REQ_DTYPE)
        out = np.zeros(max(len(req), 1), dtype=abi.RES_DTYPE)
        lib().or_rls_decide(self.h, abi.ptr(req), len(req), abi.ptr(out))
        return out[:len(req)]

    def should_rate_limit(self, req: np.ndarray, desc_rule: np.ndarray):
        """SentinelEnvoyRlsServiceImpl.shouldRateLimit over sg_rls_request records (the oracle's own restatement of
        the descriptor mapping): (overall codes per request, sg_rls_status per descriptor)."""
        req = np.ascontiguousarray(req, dtype=abi.RLS_REQ_DTYPE)
        desc_rule = np.ascontiguousarray(desc_rule, dtype=np.int32)
        overall = np.zeros(max(len(req), 1), np.int32)
        status = np.zeros(max(len(desc_rule), 1), abi.RLS_STATUS_DTYPE)
        rc = lib().or_rls_should_rate_limit(self.h, abi.ptr(req), len(req), abi.ptr(desc_rule), len(desc_rule),
                                            abi.ptr(overall), abi.ptr(status))
        if rc:
            raise ValueError(f"or_rls_should_rate_limit: {rc}")
        return overall[:len(req)], status[:len(desc_rule)]

    # ---- requestParamToken → ClusterParamFlowChecker
    def load_param_rules(self, rules: np.ndarray, hot: np.ndarray = None):
        rules = np.ascontiguousarray(rules, dtype=abi.CPARAM_RULE_DTYPE)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        rc = lib().or_cts_load_param_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot), len(hot))
        if rc != 0:
            raise ValueError(f"invalid param rules ({rc})")

    def decide_param(self, req: np.ndarray, values: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.CPARAM_REQ_DTYPE)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.zeros(len(req), dtype=abi.RES_DTYPE)
        lib().or_cts_decide_param(self.h, abi.ptr(req), len(req), abi.ptr(values), abi.ptr(out))
        return out

    def param_sum(self, key, value, now):
        return lib().or_cts_param_sum(self.h, key, int(value), now)

    def param_top(self, key, now, number=5):
        """ClusterParamMetric.getTopValues(number): [(value, qps), ...] by count, ties by value."""
        vals = np.zeros(number, np.uint64)
        qps = np.zeros(number, np.float64)
        k = lib().or_cts_param_top(self.h, key, now, number, abi.ptr(vals), abi.ptr(qps))
        assert k >= 0
        return [(int(vals[i]), float(qps[i])) for i in range(k)]

    def export_state(self, n_rules, stride):
        """(ring [K][stride][8] {start, 7 counters}, occ [K][2]) — same layout as FlowEngine.export_state."""
        ring = np.zeros((n_rules, stride, 8), np.int64)
        occ = np.zeros((n_rules, 2), np.int64)
        assert lib().or_cts_export_state(self.h, stride, abi.ptr(ring), abi.ptr(occ)) == 0
        return ring, occ

    def read_state(self, key):
        S = lib().or_cts_sample_count(self.h, key)
        starts = np.zeros(S, np.int64)
        counters = np.zeros(S * abi.NUM_EVENTS, np.int64)
        occ = np.zeros(2, np.int64)
        rc = lib().or_cts_read_state(self.h, key, abi.ptr(starts), abi.ptr(counters), abi.ptr(occ))
        assert rc == 0
        return starts, counters.reshape(S, abi.NUM_EVENTS), occ


class ShardedClusterTokenService:
    """The oracle's ClusterTokenService over T independent shards (flowId key % T), replayed on T host threads
    (ctypes releases the GIL inside or_cts_decide). Exact for rule sets without a namespace limiter: flowIds
    share no state then, so per-shard sequential replay equals one global sequential replay."""

    def __init__(self, rules, ns, threads, exceed_count=1.0, max_occupy_ratio=1.0):
        from concurrent.futures import ThreadPoolExecutor
        ns = np.ascontiguousarray(ns, dtype=abi.NS_DTYPE)
        assert not ns["limiter_enabled"].any(), "a namespace limiter couples flowIds: replay sequentially"
        self.T, self.K = threads, len(rules)
        self.pool = ThreadPoolExecutor(max_workers=threads)
        self.shards = []
        for t in range(threads):
            s = ClusterTokenService(exceed_count, max_occupy_ratio)
            s.set_namespaces(ns)
            s.load_rules(np.ascontiguousarray(rules[t::threads]))
            self.shards.append(s)

    def decide(self, req):
        req = np.ascontiguousarray(req, dtype=abi.REQ_DTYPE)
        key = req["key"] & abi.KEY_INDEX
        valid = (key < self.K)
        shard = np.where(valid, key % self.T, np.arange(len(req)) % self.T)
        out = np.zeros(len(req), abi.RES_DTYPE)
        idx = [np.nonzero(shard == t)[0] for t in range(self.T)]

        def run(t):
            part = req[idx[t]].copy()
            k = part["key"] & abi.KEY_INDEX
            inb = k < self.K
            # local rule index; out-of-range keys (BAD / NO_RULE) keep their reserved values
            part["key"] = np.where(inb, (part["key"] & np.uint32(abi.KEY_PRIO)) | (k // self.T).astype(np.uint32),
                                   part["key"])
            # a local index can collide with a reserved key only for K >= 2^31 * T: not reachable here
            out[idx[t]] = self.shards[t].decide(part)

        list(self.pool.map(run, range(self.T)))
        return out

    def export_state(self, stride):
        ring = np.zeros((self.K, stride, 8), np.int64)
        occ = np.zeros((self.K, 2), np.int64)
        for t, s in enumerate(self.shards):
            n = len(range(t, self.K, self.T))
            r, o = s.export_state(n, stride)
            ring[t::self.T] = r
            occ[t::self.T] = o
        return ring, occ

    def close(self):
        self.pool.shutdown()


class ParamFlowSlot:
    """Sequential replay of ParamFlowSlot.checkFlow over every param rule of a resource (collection / array
    arguments, THREAD grade, negative paramIdx resolution)."""

    def __init__(self, rules, hot=None, n_resources=None):
        self.h = lib().or_pslot_new()
        rules = np.ascontiguousarray(rules, dtype=abi.PSLOT_RULE_DTYPE).reshape(-1)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        n_res = int(rules["resource"].max()) + 1 if n_resources is None else n_resources
        lib().or_pslot_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot) if len(hot) else None, len(hot), n_res)

    def __del__(self):
        if self.h:
            lib().or_pslot_free(self.h)
            self.h = None

    def decide(self, ev, args, values):
        ev = np.ascontiguousarray(ev, dtype=abi.PSLOT_EVENT_DTYPE).reshape(-1)
        args = np.ascontiguousarray(args, dtype=abi.PSLOT_ARG_DTYPE).reshape(-1)
        values = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1)
        out = np.zeros(len(ev), abi.PSLOT_RES_DTYPE)
        lib().or_pslot_decide(self.h, abi.ptr(ev), len(ev), abi.ptr(args) if len(args) else None,
                              abi.ptr(values) if len(values) else None, abi.ptr(out))
        return out

    def attach_cluster(self, cts, state):
        """ClusterStateManager state for the cluster-mode param rules; SERVER: param tokens from `cts` (a
        ClusterTokenService with param rules), kept referenced here."""
        self._cts = cts
        rc = lib().or_pslot_attach_cluster(self.h, cts.h if cts is not None else None, state)
        if rc:
            raise ValueError(f"or_pslot_attach_cluster: {rc}")

    def thread_count(self, res, idx, value):
        return int(lib().or_pslot_thread_count(self.h, res, idx, int(value)))

    def param_idx(self, rule):
        return int(lib().or_pslot_param_idx(self.h, rule))

    def token_state(self, rule, value):
        lt, tk = C.c_int64(), C.c_int64()
        f = lib().or_pslot_token_state(self.h, rule, int(value), C.byref(lt), C.byref(tk))
        return f, lt.value, tk.value


class ConcurrentTokenService:
    """Sequential replay of DefaultTokenService.requestConcurrentToken / releaseConcurrentToken
    (ConcurrentClusterFlowChecker + CurrentConcurrencyManager + TokenCacheNodeManager)."""

    def __init__(self):
        self.h = lib().or_conc_new()

    def __del__(self):
        if self.h:
            lib().or_conc_free(self.h)
            self.h = None

    def set_namespaces(self, ns):
        ns = np.ascontiguousarray(ns, dtype=abi.NS_DTYPE)
        lib().or_conc_set_namespaces(self.h, abi.ptr(ns), len(ns))

    def load_rules(self, rules):
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        lib().or_conc_load_rules(self.h, abi.ptr(rules), len(rules))

    def set_rule_timeouts(self, client_offline_ms, resource_timeout_ms):
        a = np.ascontiguousarray(client_offline_ms, dtype=np.int64)
        b = np.ascontiguousarray(resource_timeout_ms, dtype=np.int64)
        assert lib().or_conc_set_rule_timeouts(self.h, abi.ptr(a), abi.ptr(b), len(a)) == 0

    def decide(self, req):
        req = np.ascontiguousarray(req, dtype=abi.CONC_REQ_DTYPE)
        out = np.zeros(len(req), abi.CONC_RES_DTYPE)
        lib().or_conc_decide(self.h, abi.ptr(req), len(req), abi.ptr(out))
        return out

    def expire(self, now, online):
        online = np.ascontiguousarray(online, dtype=np.uint8)
        return int(lib().or_conc_expire(self.h, now, abi.ptr(online) if len(online) else None, len(online)))

    def now_calls(self, k):
        return int(lib().or_conc_now_calls(self.h, k))

    def live(self):
        return int(lib().or_conc_live(self.h))


class ClusterParamMetric:
    """ClusterParamMetric (ClusterParamMetric.java) with explicit time; values are u64."""

    def __init__(self, sample_count, interval_ms):
        self.h = lib().or_cpm_new(sample_count, interval_ms)
        assert self.h

    def __del__(self):
        if self.h:
            lib().or_cpm_free(self.h)
            self.h = None

    def add_value(self, t, value, count):
        lib().or_cpm_add(self.h, t, int(value), count)

    def get_sum(self, t, value):
        return lib().or_cpm_get_sum(self.h, t, int(value))

    def get_avg(self, t, value):
        return lib().or_cpm_get_avg(self.h, t, int(value))

    def top_values(self, t, number):
        """getTopValues(number) → {value: qps}; raises for number <= 0 (AssertUtil)."""
        vals = np.zeros(max(1, number), np.uint64)
        qps = np.zeros(max(1, number), np.float64)
        k = lib().or_cpm_top(self.h, t, number, abi.ptr(vals), abi.ptr(qps))
        if k < 0:
            raise ValueError("number must be positive")
        return {int(vals[i]): float(qps[i]) for i in range(k)}


class ParamFlowChecker:
    """Sequential replay of ParamFlowChecker.passSingleValueCheck (QPS default / throttle), exact maps."""

    def __init__(self):
        self.h = lib().or_pf_new()

    def __del__(self):
        if self.h:
            lib().or_pf_free(self.h)
            self.h = None

    def load_rules(self, rules, hot=None):
        rules = np.ascontiguousarray(rules, dtype=abi.PARAM_RULE_DTYPE)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        assert lib().or_pf_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot), len(hot)) == 0

    def decide(self, req):
        req = np.ascontiguousarray(req, dtype=abi.PARAM_REQ_DTYPE)
        out = np.zeros(len(req), np.int32)
        lib().or_pf_decide(self.h, abi.ptr(req), len(req), abi.ptr(out))
        return out

    def check(self, t, rule, value, acquire=1):
        r = np.zeros(1, abi.PARAM_REQ_DTYPE)
        r[0] = (t, value, rule, acquire)
        return bool(self.decide(r)[0])

    def state(self, rule, value):
        lt, tk = C.c_int64(), C.c_int64()
        flags = lib().or_pf_read_state(self.h, rule, value, C.byref(lt), C.byref(tk))
        return flags, lt.value, tk.value

    def size(self):
        return lib().or_pf_size(self.h)


class RateLimiterController:
    """Sequential replay of RateLimiterController.canPass, one controller per rule (latestPassedTime -1).
    decide() returns the sleep in ms per request, or abi.PACE_BLOCKED."""

    def __init__(self, rules=None):
        self.h = lib().or_pace_new()
        if rules is not None:
            self.load_rules(rules)

    def __del__(self):
        if self.h:
            lib().or_pace_free(self.h)
            self.h = None

    def load_rules(self, rules):
        rules = np.ascontiguousarray(rules, dtype=abi.PACE_RULE_DTYPE)
        if lib().or_pace_load_rules(self.h, abi.ptr(rules), len(rules)) != 0:
            raise ValueError("invalid pace rule (count must be >= 0)")

    def decide(self, req):
        req = np.ascontiguousarray(req, dtype=abi.PACE_REQ_DTYPE)
        out = np.zeros(len(req), np.int32)
        lib().or_pace_decide(self.h, abi.ptr(req), len(req), abi.ptr(out))
        return out

    def can_pass(self, t, rule=0, acquire=1):
        r = np.zeros(1, abi.PACE_REQ_DTYPE)
        r[0] = (t, rule, acquire)
        return int(self.decide(r)[0])

    def latest(self, rule):
        return lib().or_pace_latest(self.h, rule)


def pace_rule(count, max_queueing_ms=500):
    r = np.zeros((), abi.PACE_RULE_DTYPE)
    r["count"] = count
    r["max_queueing_ms"] = max_queueing_ms
    return r


def degrade_rule(grade, count, time_window_sec, min_request_amount=5, stat_interval_ms=1000,
                 slow_ratio_threshold=1.0):
    r = np.zeros((), abi.DEGRADE_RULE_DTYPE)
    r["grade"], r["count"], r["time_window_sec"] = grade, count, time_window_sec
    r["min_request_amount"], r["stat_interval_ms"] = min_request_amount, stat_interval_ms
    r["slow_ratio_threshold"] = slow_ratio_threshold
    return r


def local_flow_rule(resource=0, count=0.0, grade=abi.FLOW_GRADE_QPS, behavior=abi.CONTROL_DEFAULT,
                    limit_app=abi.LIMIT_APP_DEFAULT, warm_up_sec=10, max_queueing_ms=500, strategy=abi.STRATEGY_DIRECT,
                    ref=-1, cluster_mode=abi.CLUSTER_MODE_OFF, cluster_config=0, cluster_key=abi.KEY_NO_RULE):
    """sg_local_flow_rule: FlowRule defaults (FlowRule.java: warmUpPeriodSec 10, maxQueueingTimeMs 500; refResource
    null = -1; clusterMode false). cluster_key: the flowId's rule index on an embedded token server."""
    r = np.zeros((), abi.LOCAL_FLOW_RULE_DTYPE)
    r["resource"], r["grade"], r["count"], r["control_behavior"] = resource, grade, count, behavior
    r["limit_app"], r["strategy"], r["warm_up_period_sec"], r["max_queueing_ms"] = (limit_app, strategy, warm_up_sec,
                                                                                   max_queueing_ms)
    r["ref_resource"], r["cluster_mode"], r["cluster_config"] = ref, cluster_mode, cluster_config
    r["cluster_key"] = cluster_key
    return r


class Controller:
    """One WarmUpController / WarmUpRateLimiterController on its own (the reference's controller tests mock the
    node's passQps and previousPassQps)."""

    def __init__(self, count, warm_up_sec, cold_factor=3, behavior=abi.CONTROL_WARM_UP, max_queueing_ms=500):
        r = local_flow_rule(count=count, behavior=behavior, warm_up_sec=warm_up_sec, max_queueing_ms=max_queueing_ms)
        r = np.ascontiguousarray(r.reshape(1))
        self.h = lib().or_ctl_new(abi.ptr(r), cold_factor)

    def __del__(self):
        if self.h:
            lib().or_ctl_free(self.h)
            self.h = None

    def warm_can_pass(self, now, pass_qps, prev_qps, acquire=1):
        return bool(lib().or_warm_can_pass(self.h, now, float(pass_qps), float(prev_qps), acquire))

    def warm_rl_can_pass(self, now, prev_qps, acquire=1):
        w = C.c_int64()
        ok = lib().or_warm_rl_can_pass(self.h, now, float(prev_qps), acquire, C.byref(w))
        return bool(ok), w.value

    def state(self):
        out = np.zeros(3, np.int64)
        lib().or_ctl_state(self.h, abi.ptr(out))
        return out

    @property
    def warning_token(self):
        return lib().or_ctl_warning_token(self.h)

    @property
    def max_token(self):
        return lib().or_ctl_max_token(self.h)


def select_node(rules, i, origin, context=0, ref_exists=True):
    """FlowRuleChecker.selectNodeByRequesterAndStrategy / selectReferenceNode: 0 ClusterNode, 1 origin node,
    2 the DefaultNode of the context (CHAIN), 3 the referenced ClusterNode (RELATE), None."""
    rules = np.ascontiguousarray(rules, dtype=abi.LOCAL_FLOW_RULE_DTYPE).reshape(-1)
    r = lib().or_select_node(abi.ptr(rules), len(rules), i, origin, context, 1 if ref_exists else 0)
    return None if r < 0 else r


def local_rule(flow_count=0.0, flow_grade=abi.FLOW_GRADE_NONE, breakers=()):
    r = np.zeros((), abi.LOCAL_RULE_DTYPE)
    r["flow_count"], r["flow_grade"], r["n_breakers"] = flow_count, flow_grade, len(breakers)
    for i, b in enumerate(breakers):
        r["breakers"][i] = b
    return r


class LocalChain:
    """Sequential replay of the local slot chain (StatisticSlot → FlowSlot/DefaultController → DegradeSlot)
    for one resource per rule. Events: entries and exits with explicit times."""

    def __init__(self, sample_count=2, interval_ms=1000, occupy_timeout_ms=500, cold_factor=3):
        self.h = lib().or_local_new(sample_count, interval_ms, occupy_timeout_ms)
        lib().or_local_set_cold_factor(self.h, cold_factor)
        self.S = sample_count

    def __del__(self):
        if self.h:
            lib().or_local_free(self.h)
            self.h = None

    def load_rules(self, rules):
        rules = np.ascontiguousarray(rules, dtype=abi.LOCAL_RULE_DTYPE).reshape(-1)
        assert lib().or_local_load_rules(self.h, abi.ptr(rules), len(rules)) == 0

    def attach_cluster(self, cts, state):
        """ClusterStateManager state of the node; with CLUSTER_SERVER the cluster-mode rules request tokens from
        `cts` (a ClusterTokenService: the embedded token server's DefaultTokenService)."""
        self._cts = cts
        rc = lib().or_local_attach_cluster(self.h, cts.h if cts is not None else None, state)
        if rc < 0:
            raise ValueError(f"or_local_attach_cluster: {rc}")

    def load_flow_rules(self, rules, n_origins=0, n_contexts=0):
        """FlowRuleManager.loadRules: returns the number of rules kept."""
        rules = np.ascontiguousarray(rules, dtype=abi.LOCAL_FLOW_RULE_DTYPE).reshape(-1)
        rc = lib().or_local_load_flow_rules(self.h, abi.ptr(rules), len(rules), n_origins, n_contexts)
        if rc < 0:
            raise ValueError(f"or_local_load_flow_rules: {rc}")
        return rc

    def decide(self, events):
        ev = np.ascontiguousarray(events, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        out = np.zeros(len(ev), abi.LOCAL_RES_DTYPE)
        rc = lib().or_local_decide(self.h, abi.ptr(ev), len(ev), abi.ptr(out))
        if rc != 0:
            raise ValueError(f"or_local_decide: {rc}")
        return out

    def entry(self, t, res=0, count=1, prio=False, origin=0):
        e = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
        e[0] = (t, 0, res | (0x80000000 if prio else 0), count, abi.LOCAL_ENTRY, origin)
        r = self.decide(e)[0]
        return int(r["status"]), int(r["wait_ms"])

    def exit(self, t, create_ts, res=0, count=1, error=False, origin=0):
        e = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
        e[0] = (t, create_ts, res, count, abi.LOCAL_EXIT_ERROR if error else abi.LOCAL_EXIT, origin)
        self.decide(e)

    def set_entry_types(self, inbound):
        v = np.ascontiguousarray(inbound, dtype=np.uint8)
        assert lib().or_local_set_entry_types(self.h, abi.ptr(v), len(v)) == 0

    def attach_params(self, pslot):
        """The ParamFlowSlot of the chain: a ParamSlot whose rules name this chain's resources."""
        self._ps = pslot
        lib().or_local_attach_pslot(self.h, pslot.h)

    def decide_ext(self, events, ext, args, values):
        """The whole slot chain (sg_slot_decide_batch): events with their context / argument records."""
        ev = np.ascontiguousarray(events, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        ext = np.ascontiguousarray(ext, dtype=abi.SLOT_EXT_DTYPE).reshape(-1)
        args = np.ascontiguousarray(args, dtype=abi.PSLOT_ARG_DTYPE).reshape(-1)
        values = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1)
        if len(args) == 0:
            args = np.zeros(1, abi.PSLOT_ARG_DTYPE)
        if len(values) == 0:
            values = np.zeros(1, np.uint64)
        out = np.zeros(len(ev), abi.LOCAL_RES_DTYPE)
        rc = lib().or_local_decide_ext(self.h, abi.ptr(ev), abi.ptr(ext), len(ev), abi.ptr(args), abi.ptr(values),
                                       abi.ptr(out))
        if rc != 0:
            raise ValueError(f"or_local_decide_ext: {rc}")
        return out

    def context_dump(self, res, context):
        """(second, borrow, minute, threads, exists) of the DefaultNode of (res, context)."""
        sec = np.zeros((self.S, 8), np.int64)
        bor = np.zeros((self.S, 2), np.int64)
        mnt = np.zeros((60, 8), np.int64)
        th = C.c_int64()
        rc = lib().or_local_context_dump(self.h, res, context, abi.ptr(sec), abi.ptr(bor), abi.ptr(mnt), C.byref(th))
        assert rc >= 0
        return sec, bor, mnt, th.value, rc == 1

    def origin_dump(self, res, origin):
        """(second, borrow, minute, threads, exists) of the origin node of (res, origin)."""
        sec = np.zeros((self.S, 8), np.int64)
        bor = np.zeros((self.S, 2), np.int64)
        mnt = np.zeros((60, 8), np.int64)
        th = C.c_int64()
        rc = lib().or_local_origin_dump(self.h, res, origin, abi.ptr(sec), abi.ptr(bor), abi.ptr(mnt), C.byref(th))
        assert rc >= 0
        return sec, bor, mnt, th.value, rc == 1

    def metrics(self, now, raw=False):
        """StatisticNode.metrics() rows of every resource at now (MetricTimerListener.run), time-sorted (raw: rt as
        the bucket's sum, as sg_local_metrics_raw)."""
        n = int(lib().or_local_metrics_raw(self.h, now, None, 0, int(raw)))
        out = np.zeros(max(1, n), abi.METRIC_NODE_DTYPE)
        m = int(lib().or_local_metrics_raw(self.h, now, abi.ptr(out), len(out), int(raw)))
        assert m == n
        return out[:n]

    def rule_order(self, res):
        out = np.zeros(256, np.int32)
        k = lib().or_local_rule_order(self.h, res, abi.ptr(out), len(out))
        assert k >= 0
        return [int(x) for x in out[:k]]

    def controller(self, i):
        out = np.zeros(3, np.int64)
        if lib().or_local_controller(self.h, i, abi.ptr(out)) != 0:
            return None
        return out

    def second_sum(self, res, t, ev):
        return lib().or_local_second_sum(self.h, res, t, ev)

    def minute_sum(self, res, t, ev):
        return lib().or_local_minute_sum(self.h, res, t, ev)

    def threads(self, res):
        return lib().or_local_thread_num(self.h, res)

    def waiting(self, res, t):
        return lib().or_local_waiting(self.h, res, t)

    def breaker(self, res, i):
        nr = C.c_int64()
        st = lib().or_local_breaker_state(self.h, res, i, C.byref(nr))
        return st, nr.value

    def dump(self, res):
        sec = np.zeros((self.S, 8), np.int64)
        bor = np.zeros((self.S, 2), np.int64)
        mnt = np.zeros((60, 8), np.int64)
        assert lib().or_local_dump(self.h, res, abi.ptr(sec), abi.ptr(bor), abi.ptr(mnt)) == 0
        return sec, bor, mnt


    def breaker_stat(self, res, i):
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        assert lib().or_local_breaker_stat(self.h, res, i, C.byref(a), C.byref(b), C.byref(c)) == 0
        return a.value, b.value, c.value


class LocalTraceGen:
    """Client model over a LocalChain (test infrastructure): time-ordered entries with planned response
    times and business errors; each entry that passes exits at ts + waitInMs + rt (SphU.entry callers
    only exit entries they obtained). run() returns the merged event stream up to t_end and the oracle's
    decision for every event; exits due later stay pending for the next call."""

    def __init__(self, chain):
        self.chain = chain
        self.h = lib().or_lgen_new(chain.h)

    def __del__(self):
        if self.h:
            lib().or_lgen_free(self.h)
            self.h = None

    def pending(self):
        return int(lib().or_lgen_pending(self.h))

    def run(self, entries, rt, err, t_end):
        entries = np.ascontiguousarray(entries, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        rt = np.ascontiguousarray(rt, dtype=np.int32)
        err = np.ascontiguousarray(err, dtype=np.uint8)
        cap = 2 * len(entries) + self.pending() + 16
        out = np.zeros(cap, abi.LOCAL_EVENT_DTYPE)
        res = np.zeros(cap, abi.LOCAL_RES_DTYPE)
        k = lib().or_lgen_run(self.h, abi.ptr(entries), abi.ptr(rt), abi.ptr(err), len(entries), int(t_end),
                              abi.ptr(out), abi.ptr(res), cap)
        assert k != 2**64 - 1
        return out[:k].copy(), res[:k].copy()

    def run_ext(self, entries, ext, rt, err, t_end, args, values):
        """run() for the whole slot chain: each entry's context / argument record (ext) travels to its exit; args /
        values are the argument pool the records index (the same pool for every call)."""
        entries = np.ascontiguousarray(entries, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        ext = np.ascontiguousarray(ext, dtype=abi.SLOT_EXT_DTYPE).reshape(-1)
        rt = np.ascontiguousarray(rt, dtype=np.int32)
        err = np.ascontiguousarray(err, dtype=np.uint8)
        args = np.ascontiguousarray(args, dtype=abi.PSLOT_ARG_DTYPE).reshape(-1)
        values = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1)
        cap = 2 * len(entries) + self.pending() + 16
        out = np.zeros(cap, abi.LOCAL_EVENT_DTYPE)
        xo = np.zeros(cap, abi.SLOT_EXT_DTYPE)
        res = np.zeros(cap, abi.LOCAL_RES_DTYPE)
        k = lib().or_lgen_run_ext(self.h, abi.ptr(entries), abi.ptr(ext), abi.ptr(rt), abi.ptr(err), len(entries),
                                  int(t_end), abi.ptr(out), abi.ptr(xo), abi.ptr(res), cap, abi.ptr(args),
                                  abi.ptr(values))
        assert k != 2**64 - 1
        return out[:k].copy(), xo[:k].copy(), res[:k].copy()


# ---- token-server wire codec (DefaultRequestEntityDecoder / FlowRequestDataDecoder / DefaultResponseEntityWriter)
def codec_decode_flow(payload: np.ndarray, offsets: np.ndarray, ts_ms: np.ndarray, flow_ids: np.ndarray):
    """Frame payloads → (sg_req records, xids, kinds), as the default token server decodes them."""
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    if len(payload) == 0:
        payload = np.zeros(1, np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    ts_ms = np.ascontiguousarray(ts_ms, dtype=np.int64)
    flow_ids = np.ascontiguousarray(flow_ids, dtype=np.int64)
    n = len(offsets) - 1
    req = np.zeros(max(n, 1), abi.REQ_DTYPE)
    xid = np.zeros(max(n, 1), np.int32)
    kind = np.zeros(max(n, 1), np.uint8)
    lib().or_codec_decode_flow(abi.ptr(payload), abi.ptr(offsets), abi.ptr(ts_ms), n, abi.ptr(flow_ids),
                               len(flow_ids), abi.ptr(req), abi.ptr(xid), abi.ptr(kind))
    return req[:n], xid[:n], kind[:n]


def codec_encode_flow(xid: np.ndarray, kind: np.ndarray, res: np.ndarray) -> np.ndarray:
    """16-byte response frames (length-prefixed), zeros where the kind is not a flow request."""
    xid = np.ascontiguousarray(xid, dtype=np.int32)
    kind = np.ascontiguousarray(kind, dtype=np.uint8)
    res = np.ascontiguousarray(res, dtype=abi.RES_DTYPE)
    out = np.zeros(max(len(xid), 1) * 16, np.uint8)
    lib().or_codec_encode_flow(abi.ptr(xid), abi.ptr(kind), abi.ptr(res), len(xid), abi.ptr(out))
    return out[:len(xid) * 16]
