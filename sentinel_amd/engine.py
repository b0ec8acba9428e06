"""Thin ctypes handle over libsentinel_gpu.so (the C ABI in include/sentinel_gpu.h).

There is no CPU fallback: if the HIP library is missing, constructing a FlowEngine raises.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(_HERE, "libsentinel_gpu.so")  # override: A/B tuning runs

EXPORTS = ["sg_create", "sg_destroy", "sg_last_error", "sg_set_namespaces", "sg_set_shard", "sg_lim_arrivals", "sg_lim_arrivals_param",
           "sg_lim_exchange", "sg_lim_slots", "sg_load_flow_rules",
           "sg_flow_decide_batch", "sg_flow_decide_batch_host", "sg_flow_submit", "sg_flow_enqueue", "sg_flow_poll", "sg_flow_wait",
           "sg_host_alloc", "sg_host_free", "sg_enable_stats", "sg_get_stats",
           "sg_flow_read_state", "sg_flow_export_state", "sg_flow_import_state", "sg_snapshot_metrics", "sg_snapshot_metrics_device", "sg_snapshot_metrics_enqueue", "sg_debug_copy", "sg_build_info",
           "sg_param_load_rules", "sg_param_decide_batch", "sg_param_decide_batch_host", "sg_param_read_state",
           "sg_cparam_load_rules", "sg_cparam_decide_batch", "sg_cparam_decide_batch_host", "sg_cparam_read_sum",
           "sg_local_load_rules", "sg_local_decide_batch", "sg_local_decide_batch_host", "sg_local_read_state",
           "sg_local_load_flow_rules", "sg_local_read_origin_state", "sg_local_read_controller",
           "sg_local_read_context_state", "sg_local_set_cluster_state", "sg_slot_decide_batch", "sg_local_set_entry_types",
           "sg_slot_decide_batch_host",
           "sg_codec_decode_flow", "sg_codec_encode_flow",
           "sg_conc_set_rule_timeouts", "sg_conc_decide_batch", "sg_conc_decide_batch_host", "sg_conc_expire",
           "sg_conc_read_state", "sg_local_metrics", "sg_cparam_top_values", "sg_cparam_last_rounds",
           "sg_pslot_load_rules", "sg_pslot_decide_batch", "sg_pslot_decide_batch_host", "sg_pslot_thread_count",
           "sg_pslot_param_idx", "sg_rls_should_rate_limit", "sg_local_enqueue", "sg_local_poll", "sg_local_wait",
           "sg_pace_load_rules", "sg_pace_decide_batch", "sg_pace_decide_batch_host", "sg_pace_read_state",
           "sg_node_create", "sg_node_destroy", "sg_node_last_error", "sg_node_set_namespaces", "sg_node_load_flow_rules",
           "sg_node_flow_decide_batch", "sg_node_flow_decide_batch_host", "sg_node_flow_read_state",
           "sg_node_snapshot_metrics", "sg_node_shard_of", "sg_node_flow_enqueue", "sg_node_flow_poll",
           "sg_node_flow_wait", "sg_local_metrics_raw", "sg_local_owners", "sg_node_cparam_load_rules",
           "sg_node_cparam_decide_batch", "sg_node_cparam_decide_batch_host", "sg_node_cparam_read_sum",
           "sg_node_cparam_top_values", "sg_node_conc_set_rule_timeouts", "sg_node_conc_decide_batch",
           "sg_node_conc_decide_batch_host", "sg_node_conc_expire", "sg_node_conc_read_state",
           "sg_local_metrics_raw_device", "sg_local_metrics_raw_enqueue"]

_lib = None


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sentinel_gpu error {code}: {msg}")
        self.code = code


def load_library():
    """Load the HIP library (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C sentinel_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int64
    sig = {
        "sg_create": (C.c_int, [C.POINTER(abi.sg_config), C.POINTER(vp)]),
        "sg_destroy": (None, [vp]),
        "sg_last_error": (C.c_char_p, [vp]),
        "sg_set_namespaces": (C.c_int, [vp, vp, u32]),
        "sg_set_shard": (C.c_int, [vp, C.c_int32, C.c_int32]),
        "sg_lim_arrivals": (C.c_int, [vp, vp, u64, i64, u32, vp, u64, vp]),
        "sg_lim_arrivals_param": (C.c_int, [vp, vp, u64, i64, u32, vp, u64, vp]),
        "sg_lim_exchange": (C.c_int, [vp, vp, u64, i64, u32]),
        "sg_lim_slots": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
        "sg_load_flow_rules": (C.c_int, [vp, vp, u32]),
        "sg_flow_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_flow_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_flow_submit": (C.c_int, [vp, vp, u64, vp, C.POINTER(u64)]),
        "sg_flow_enqueue": (C.c_int, [vp, vp, u64, vp, C.POINTER(u64)]),
        "sg_flow_poll": (C.c_int, [vp, u64]),
        "sg_flow_wait": (C.c_int, [vp, u64]),
        "sg_host_alloc": (vp, [vp, u64]),
        "sg_host_free": (None, [vp, vp]),
        "sg_enable_stats": (C.c_int, [vp, C.c_int]),
        "sg_get_stats": (C.c_int, [vp, C.POINTER(abi.sg_batch_stats)]),
        "sg_flow_read_state": (C.c_int, [vp, u32, vp, vp, vp]),
        "sg_flow_export_state": (C.c_int, [vp, vp, u64, vp, u64, vp]),
        "sg_flow_import_state": (C.c_int, [vp, vp, u64, vp, u64]),
        "sg_snapshot_metrics": (C.c_int, [vp, i64, vp, u64]),
        "sg_snapshot_metrics_device": (C.c_int, [vp, i64, vp, u64, vp]),
        "sg_snapshot_metrics_enqueue": (C.c_int, [vp, i64, vp, u64, C.POINTER(u64)]),
        "sg_debug_copy": (C.c_int, [vp, C.c_int, vp, u64]),
        "sg_param_load_rules": (C.c_int, [vp, vp, u32, vp, u32]),
        "sg_param_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_param_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_param_read_state": (C.c_int, [vp, u32, u64, vp, vp]),
        "sg_build_info": (C.c_char_p, []),
        "sg_local_load_rules": (C.c_int, [vp, vp, vp, u32]),
        "sg_cparam_load_rules": (C.c_int, [vp, vp, u32, vp, u32, C.c_int32]),
        "sg_cparam_decide_batch": (C.c_int, [vp, vp, u64, vp, u64, vp, vp]),
        "sg_cparam_decide_batch_host": (C.c_int, [vp, vp, u64, vp, u64, vp]),
        "sg_cparam_read_sum": (C.c_int, [vp, u32, u64, i64, vp]),
        "sg_local_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_local_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_local_enqueue": (C.c_int, [vp, vp, u64, vp, C.POINTER(u64)]),
        "sg_local_poll": (C.c_int, [vp, u64]),
        "sg_local_wait": (C.c_int, [vp, u64]),
        "sg_local_read_state": (C.c_int, [vp, u32, vp, vp, vp, vp]),
        "sg_local_load_flow_rules": (C.c_int, [vp, vp, u32, C.c_int32, C.c_int32]),
        "sg_local_read_context_state": (C.c_int, [vp, u32, C.c_int32, vp, vp, vp, vp]),
        "sg_local_set_cluster_state": (C.c_int, [vp, C.c_int32]),
        "sg_local_set_entry_types": (C.c_int, [vp, vp, u32]),
        "sg_slot_decide_batch": (C.c_int, [vp, vp, vp, u64, vp, u64, vp, u64, vp, vp]),
        "sg_slot_decide_batch_host": (C.c_int, [vp, vp, vp, u64, vp, u64, vp, u64, vp]),
        "sg_local_read_origin_state": (C.c_int, [vp, u32, C.c_int32, vp, vp, vp, vp]),
        "sg_local_read_controller": (C.c_int, [vp, u32, vp]),
        "sg_codec_decode_flow": (C.c_int, [vp, vp, vp, vp, u64, vp, vp, vp, vp]),
        "sg_conc_set_rule_timeouts": (C.c_int, [vp, vp, vp, u32]),
        "sg_local_metrics": (C.c_int, [vp, i64, vp, u64, C.POINTER(u64)]),
        "sg_pslot_load_rules": (C.c_int, [vp, vp, u32, vp, u32, u32]),
        "sg_pslot_decide_batch": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp]),
        "sg_pslot_decide_batch_host": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp]),
        "sg_pslot_thread_count": (C.c_int, [vp, u32, C.c_int32, u64, C.POINTER(i64)]),
        "sg_pslot_param_idx": (C.c_int, [vp, u32, C.POINTER(C.c_int32)]),
        "sg_cparam_top_values": (C.c_int, [vp, i64, u32, vp, vp, vp]),
        "sg_cparam_last_rounds": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
        "sg_conc_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_conc_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_conc_expire": (C.c_int, [vp, i64, vp, u32, C.POINTER(u64)]),
        "sg_conc_read_state": (C.c_int, [vp, u32, C.POINTER(C.c_int32), C.POINTER(u64)]),
        "sg_codec_encode_flow": (C.c_int, [vp, vp, vp, vp, u64, vp, vp]),
        "sg_pace_load_rules": (C.c_int, [vp, vp, u32]),
        "sg_pace_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_pace_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_pace_read_state": (C.c_int, [vp, u32, vp]),
        "sg_rls_should_rate_limit": (C.c_int, [vp, vp, u32, vp, u64, vp, vp]),
        "sg_node_create": (C.c_int, [C.POINTER(abi.sg_config), vp, u32, C.POINTER(vp)]),
        "sg_node_destroy": (None, [vp]),
        "sg_node_last_error": (C.c_char_p, [vp]),
        "sg_node_set_namespaces": (C.c_int, [vp, vp, u32]),
        "sg_node_load_flow_rules": (C.c_int, [vp, vp, u32]),
        "sg_node_flow_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_node_flow_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_node_flow_read_state": (C.c_int, [vp, u32, vp, vp, vp]),
        "sg_node_snapshot_metrics": (C.c_int, [vp, i64, vp, u64]),
        "sg_node_shard_of": (C.c_int, [vp, u32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "sg_node_flow_enqueue": (C.c_int, [vp, vp, u64, vp, C.POINTER(C.c_uint64)]),
        "sg_node_flow_poll": (C.c_int, [vp, u64]),
        "sg_node_flow_wait": (C.c_int, [vp, u64]),
        "sg_local_metrics_raw": (C.c_int, [vp, i64, vp, u64, C.POINTER(C.c_uint64)]),
        "sg_local_metrics_raw_device": (C.c_int, [vp, i64, vp, u64, C.POINTER(C.c_uint64)]),
        "sg_local_metrics_raw_enqueue": (C.c_int, [vp, i64, vp, u64, vp, vp]),
        "sg_local_owners": (C.c_int, [vp, u32, vp, u32]),
        "sg_node_cparam_load_rules": (C.c_int, [vp, vp, u32, vp, u32, C.c_int32]),
        "sg_node_cparam_decide_batch": (C.c_int, [vp, vp, u64, vp, u64, vp, vp]),
        "sg_node_cparam_decide_batch_host": (C.c_int, [vp, vp, u64, vp, u64, vp]),
        "sg_node_cparam_read_sum": (C.c_int, [vp, u32, u64, i64, vp]),
        "sg_node_cparam_top_values": (C.c_int, [vp, i64, u32, vp, vp, vp]),
        "sg_node_conc_set_rule_timeouts": (C.c_int, [vp, vp, vp, u32]),
        "sg_node_conc_decide_batch": (C.c_int, [vp, vp, u64, vp, vp]),
        "sg_node_conc_decide_batch_host": (C.c_int, [vp, vp, u64, vp]),
        "sg_node_conc_expire": (C.c_int, [vp, i64, vp, u32, C.POINTER(u64)]),
        "sg_node_conc_read_state": (C.c_int, [vp, u32, C.POINTER(C.c_int32), C.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("SG_LIB_PATH") and not hasattr(L, name):
            continue  # an older build under A/B (tuning only): the product library must export every entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class NodeEngine:
    """One sg_node: a token server's cluster flow rules over G shard handles (devices[g] per shard; one device may
    hold several), with routing by flowId owner inside the library."""

    def __init__(self, devices, max_batch=1 << 20, exceed_count=1.0, max_occupy_ratio=1.0, flags=0):
        L = load_library()
        cfg = abi.sg_config(device=int(devices[0]), flags=flags, exceed_count=exceed_count,
                            max_occupy_ratio=max_occupy_ratio, max_batch=max_batch)
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = C.c_void_p()
        rc = L.sg_node_create(C.byref(cfg), abi.ptr(devs), len(devs), C.byref(h))
        if rc != 0:
            raise EngineError(rc, "sg_node_create failed")
        self._L, self.h, self.G = L, h, len(devs)
        self._S = {}

    def __del__(self):
        if getattr(self, "h", None):
            self._L.sg_node_destroy(self.h)
            self.h = None

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, self._L.sg_node_last_error(self.h).decode())

    def set_namespaces(self, ns: np.ndarray):
        ns = np.ascontiguousarray(ns, dtype=abi.NS_DTYPE)
        self._check(self._L.sg_node_set_namespaces(self.h, abi.ptr(ns), len(ns)))

    def load_rules(self, rules: np.ndarray):
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        self._check(self._L.sg_node_load_flow_rules(self.h, abi.ptr(rules), len(rules)))
        self._S = {int(k): int(s) for k, s in enumerate(rules["sample_count"])} if len(rules) else {}

    def decide_host(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.REQ_DTYPE)
        out = np.zeros(len(req), dtype=abi.RES_DTYPE)
        self._check(self._L.sg_node_flow_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def decide_device(self, req_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        self._check(self._L.sg_node_flow_decide_batch(self.h, req_ptr, n, out_ptr, stream_ptr))

    def enqueue_device(self, req_ptr: int, n: int, out_ptr: int) -> int:
        """sg_node_flow_enqueue: a device-resident node batch on the node pipeline; returns the ticket."""
        t = C.c_uint64()
        self._check(self._L.sg_node_flow_enqueue(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr), C.byref(t)))
        return t.value

    def poll(self, ticket) -> bool:
        r = self._L.sg_node_flow_poll(self.h, ticket)
        if r < 0:
            self._check(r)
        return r == 1

    def wait(self, ticket):
        self._check(self._L.sg_node_flow_wait(self.h, ticket))

    def shard_of(self, key):
        s, lk = C.c_uint32(), C.c_uint32()
        self._check(self._L.sg_node_shard_of(self.h, key, C.byref(s), C.byref(lk)))
        return s.value, lk.value

    def read_state(self, key, sample_count):
        starts = np.zeros(sample_count, np.int64)
        counters = np.zeros(sample_count * abi.NUM_EVENTS, np.int64)
        occ = np.zeros(2, np.int64)
        self._check(self._L.sg_node_flow_read_state(self.h, key, abi.ptr(starts), abi.ptr(counters), abi.ptr(occ)))
        return starts, counters.reshape(sample_count, abi.NUM_EVENTS), occ

    def snapshot(self, now_ms, n_rules):
        out = np.zeros(2 * max(n_rules, 1), np.float64)
        self._check(self._L.sg_node_snapshot_metrics(self.h, now_ms, abi.ptr(out), len(out)))
        return out[:2 * n_rules].reshape(n_rules, 2)

    # ---- cluster param and concurrent tokens sharded over the node (FlowEngine's cparam_* / conc_* shapes)
    def cparam_load_rules(self, rules: np.ndarray, hot: np.ndarray = None, capacity_log2=0):
        rules = np.ascontiguousarray(rules, dtype=abi.CPARAM_RULE_DTYPE)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        self._check(self._L.sg_node_cparam_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot), len(hot),
                                                      capacity_log2))

    def cparam_decide_host(self, req: np.ndarray, values: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.CPARAM_REQ_DTYPE)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.zeros(len(req), abi.RES_DTYPE)
        self._check(self._L.sg_node_cparam_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(values),
                                                              len(values), abi.ptr(out)))
        return out

    def cparam_decide_device(self, req_ptr: int, n: int, values_ptr: int, n_values: int, out_ptr: int,
                             stream_ptr: int = 0):
        self._check(self._L.sg_node_cparam_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(values_ptr),
                                                        n_values, C.c_void_p(out_ptr), C.c_void_p(stream_ptr)))

    def cparam_top_values(self, now_ms, n_rules, number=5):
        vals = np.zeros(max(1, n_rules * number), np.uint64)
        qps = np.zeros(max(1, n_rules * number), np.float64)
        cnt = np.zeros(max(1, n_rules), np.uint32)
        self._check(self._L.sg_node_cparam_top_values(self.h, now_ms, number, abi.ptr(vals), abi.ptr(qps),
                                                      abi.ptr(cnt)))
        return [[(int(vals[r * number + i]), float(qps[r * number + i])) for i in range(int(cnt[r]))]
                for r in range(n_rules)]

    def cparam_sum(self, rule, value, now):
        v = C.c_int64()
        self._check(self._L.sg_node_cparam_read_sum(self.h, rule, int(value), now, C.byref(v)))
        return v.value

    def conc_set_rule_timeouts(self, client_offline_ms, resource_timeout_ms):
        a = np.ascontiguousarray(client_offline_ms, dtype=np.int64)
        b = np.ascontiguousarray(resource_timeout_ms, dtype=np.int64)
        self._check(self._L.sg_node_conc_set_rule_timeouts(self.h, abi.ptr(a), abi.ptr(b), len(a)))

    def conc_decide_host(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.CONC_REQ_DTYPE)
        out = np.zeros(len(req), abi.CONC_RES_DTYPE)
        self._check(self._L.sg_node_conc_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def conc_decide_device(self, req_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        self._check(self._L.sg_node_conc_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr),
                                                      C.c_void_p(stream_ptr)))

    def conc_expire(self, now_ms, online) -> int:
        online = np.ascontiguousarray(online, dtype=np.uint8)
        rm = C.c_uint64()
        self._check(self._L.sg_node_conc_expire(self.h, now_ms, abi.ptr(online) if len(online) else None,
                                                len(online), C.byref(rm)))
        return rm.value

    def conc_state(self, key):
        now, live = C.c_int32(), C.c_uint64()
        self._check(self._L.sg_node_conc_read_state(self.h, key, C.byref(now), C.byref(live)))
        return now.value, live.value


class FlowEngine:
    """One sg_handle: the cluster flow rules of a token server on one GPU."""

    def __init__(self, device=0, max_batch=1 << 20, exceed_count=1.0, max_occupy_ratio=1.0, flags=0):
        self._world = 1
        L = load_library()
        cfg = abi.sg_config(device=device, flags=flags, exceed_count=exceed_count,
                            max_occupy_ratio=max_occupy_ratio, max_batch=max_batch)
        h = C.c_void_p()
        rc = L.sg_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise EngineError(rc, "sg_create failed")
        self._L = L
        self.h = h
        self.max_batch = max_batch
        self.sample_counts = None

    def close(self):
        if getattr(self, "h", None):
            for p in getattr(self, "_pinned", {}).values():
                self._L.sg_host_free(self.h, C.c_void_p(p))
            self._pinned = {}
            self._L.sg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise EngineError(rc, self._L.sg_last_error(self.h).decode())

    def set_namespaces(self, ns: np.ndarray):
        ns = np.ascontiguousarray(ns, dtype=abi.NS_DTYPE)
        self._check(self._L.sg_set_namespaces(self.h, abi.ptr(ns), len(ns)))

    def set_shard(self, rank: int, world: int):
        """This handle decides shard `rank` of `world`. With world > 1 and a namespace QPS limiter every flow
        batch (decide_device / decide_host / enqueue_device / submit) must follow lim_arrivals + lim_exchange, and
        every cluster param batch lim_arrivals_param + lim_exchange (cluster.LimiterExchange)."""
        self._check(self._L.sg_set_shard(self.h, rank, world))
        self._world = world

    def lim_slots(self) -> int:
        """The handle's limiter-slot count n_lim (limiter-enabled namespaces)."""
        n = C.c_uint32(0)
        self._check(self._L.sg_lim_slots(self.h, C.byref(n)))
        return int(n.value)

    def lim_arrivals(self, req_ptr: int, n: int, t_base: int, n_ms: int, counts_ptr: int, stream_ptr: int = 0,
                     counts_words: int = None):
        """This shard's limited arrivals per (limiter slot, millisecond) into device counts[n_lim][n_ms]
        (counts_words: the buffer's uint32 count, n_lim * n_ms by default; the library checks it)."""
        if counts_words is None:
            counts_words = self.lim_slots() * n_ms
        self._check(self._L.sg_lim_arrivals(self.h, req_ptr, n, t_base, n_ms, counts_ptr, counts_words, stream_ptr))

    def lim_arrivals_param(self, req_ptr: int, n: int, t_base: int, n_ms: int, counts_ptr: int, stream_ptr: int = 0,
                           counts_words: int = None):
        """sg_lim_arrivals over a device batch of sg_cparam_req (cluster param tokens share the namespace limiter)."""
        if counts_words is None:
            counts_words = self.lim_slots() * n_ms
        self._check(self._L.sg_lim_arrivals_param(self.h, req_ptr, n, t_base, n_ms, counts_ptr, counts_words,
                                                  stream_ptr))

    def lim_exchange(self, gathered_ptr: int, t_base: int, n_ms: int, gathered_words: int = None):
        """Arm the next flow batch with the node's gathered arrivals (device [world][n_lim][n_ms]; gathered_words
        defaults to world * n_lim * n_ms with the world of set_shard)."""
        if gathered_words is None:
            gathered_words = self._world * self.lim_slots() * n_ms
        self._check(self._L.sg_lim_exchange(self.h, gathered_ptr, gathered_words, t_base, n_ms))

    def load_rules(self, rules: np.ndarray):
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        self._check(self._L.sg_load_flow_rules(self.h, abi.ptr(rules), len(rules)))

    def decide_device(self, req_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        """req_ptr/out_ptr: device addresses of n sg_req / sg_result records (e.g. torch data_ptr())."""
        self._check(self._L.sg_flow_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr),
                                                 C.c_void_p(stream_ptr)))

    def codec_decode(self, payload_ptr: int, offsets_ptr: int, ts_ptr: int, n: int, req_ptr: int, xid_ptr: int,
                     kind_ptr: int, stream_ptr: int = 0):
        """Device addresses: frame payloads, offsets[n + 1] (u32), arrival ms (i64) → sg_req, xid (i32), kind (u8)."""
        self._check(self._L.sg_codec_decode_flow(self.h, C.c_void_p(payload_ptr), C.c_void_p(offsets_ptr),
                                                 C.c_void_p(ts_ptr), n, C.c_void_p(req_ptr), C.c_void_p(xid_ptr),
                                                 C.c_void_p(kind_ptr), C.c_void_p(stream_ptr)))

    def codec_encode(self, xid_ptr: int, kind_ptr: int, res_ptr: int, n: int, frames_ptr: int, stream_ptr: int = 0):
        """Device addresses: xid (i32), kind (u8), sg_result → n 16-byte response frames."""
        self._check(self._L.sg_codec_encode_flow(self.h, C.c_void_p(xid_ptr), C.c_void_p(kind_ptr),
                                                 C.c_void_p(res_ptr), n, C.c_void_p(frames_ptr),
                                                 C.c_void_p(stream_ptr)))

    def decide_host(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.REQ_DTYPE)
        out = np.zeros(len(req), abi.RES_DTYPE)
        self._check(self._L.sg_flow_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def rls_should_rate_limit(self, req: np.ndarray, desc_rule: np.ndarray):
        """sg_rls_should_rate_limit: (overall codes per request, sg_rls_status per descriptor)."""
        req = np.ascontiguousarray(req, dtype=abi.RLS_REQ_DTYPE)
        desc_rule = np.ascontiguousarray(desc_rule, dtype=np.int32)
        overall = np.zeros(len(req), np.int32)
        status = np.zeros(len(desc_rule), abi.RLS_STATUS_DTYPE)
        self._check(self._L.sg_rls_should_rate_limit(self.h, abi.ptr(req), len(req), abi.ptr(desc_rule), len(desc_rule),
                                                     abi.ptr(overall), abi.ptr(status)))
        return overall, status

    # ---- asynchronous host pipeline (pinned buffers, tickets)
    def host_array(self, n, dtype):
        """A numpy array of n `dtype` records in pinned host memory (freed with the engine or free_host)."""
        dtype = np.dtype(dtype)
        p = self._L.sg_host_alloc(self.h, max(1, n * dtype.itemsize))
        if not p:
            raise EngineError(abi.SG_E_NOMEM, "sg_host_alloc")
        buf = (C.c_uint8 * (n * dtype.itemsize)).from_address(p)
        arr = np.frombuffer(buf, dtype=dtype, count=n)
        self._pinned = getattr(self, "_pinned", {})
        self._pinned[arr.__array_interface__["data"][0]] = p
        return arr

    def free_host(self, arr):
        p = self._pinned.pop(arr.__array_interface__["data"][0], None)
        if p:
            self._L.sg_host_free(self.h, C.c_void_p(p))

    def submit(self, req: np.ndarray, out: np.ndarray) -> int:
        """sg_flow_submit over host arrays (pinned ones from host_array overlap); returns the ticket."""
        t = C.c_uint64()
        self._check(self._L.sg_flow_submit(self.h, C.c_void_p(req.ctypes.data), len(req), C.c_void_p(out.ctypes.data),
                                           C.byref(t)))
        return t.value

    def enqueue_device(self, req_ptr: int, n: int, out_ptr: int) -> int:
        """sg_flow_enqueue: a device-resident batch on the pipelined path (front half beside the previous batch's
        walkers); returns the ticket for poll / wait. The buffers must stay untouched until it completes."""
        t = C.c_uint64()
        self._check(self._L.sg_flow_enqueue(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr), C.byref(t)))
        return t.value

    def poll(self, ticket) -> bool:
        r = self._L.sg_flow_poll(self.h, ticket)
        if r < 0:
            self._check(r)
        return r == 1

    def wait(self, ticket):
        self._check(self._L.sg_flow_wait(self.h, ticket))

    def enable_stats(self, on=True):
        self._check(self._L.sg_enable_stats(self.h, 1 if on else 0))

    def stats(self):
        s = abi.sg_batch_stats()
        self._check(self._L.sg_get_stats(self.h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in abi.sg_batch_stats._fields_}

    def read_state(self, key, sample_count):
        starts = np.zeros(sample_count, np.int64)
        counters = np.zeros(sample_count * abi.NUM_EVENTS, np.int64)
        occ = np.zeros(2, np.int64)
        self._check(self._L.sg_flow_read_state(self.h, key, abi.ptr(starts), abi.ptr(counters), abi.ptr(occ)))
        return starts, counters.reshape(sample_count, abi.NUM_EVENTS), occ

    def state_stride(self):
        st = C.c_int32()
        self._check(self._L.sg_flow_export_state(self.h, None, 0, None, 0, C.byref(st)))
        return st.value

    def export_state(self, n_rules):
        """(ring [K][stride][8] {start, 7 ClusterFlowEvent counters}, occ [K][2]) of every flowId."""
        stride = self.state_stride()
        ring = np.zeros((n_rules, stride, 8), np.int64)
        occ = np.zeros((n_rules, 2), np.int64)
        st = C.c_int32()
        self._check(self._L.sg_flow_export_state(self.h, abi.ptr(ring), ring.size, abi.ptr(occ), occ.size,
                                                 C.byref(st)))
        return ring, occ

    def import_state(self, ring, occ):
        ring = np.ascontiguousarray(ring, dtype=np.int64)
        occ = np.ascontiguousarray(occ, dtype=np.int64)
        self._check(self._L.sg_flow_import_state(self.h, abi.ptr(ring), ring.size, abi.ptr(occ), occ.size))

    def snapshot_device(self, now_ms, out_ptr, n_rules, stream_ptr=0):
        """{passQps, blockQps} per flowId into device memory at out_ptr (2*n_rules doubles)."""
        self._check(self._L.sg_snapshot_metrics_device(self.h, now_ms, C.c_void_p(out_ptr), 2 * n_rules,
                                                       C.c_void_p(stream_ptr)))

    def snapshot_enqueue(self, now_ms, out_ptr, n_rules) -> int:
        """{passQps, blockQps} per flowId into device memory at out_ptr, ordered after every batch enqueued so far
        (sg_snapshot_metrics_enqueue); returns the ticket for wait."""
        t = C.c_uint64()
        self._check(self._L.sg_snapshot_metrics_enqueue(self.h, now_ms, C.c_void_p(out_ptr), 2 * n_rules, C.byref(t)))
        return t.value

    def debug_copy(self, what, dtype, count):
        """Testing aid: an internal buffer of the last batch (see sg_debug_copy)."""
        out = np.zeros(count, dtype)
        self._check(self._L.sg_debug_copy(self.h, what, abi.ptr(out), out.nbytes))
        return out

    # ---- hot-parameter flow control (ParamFlowChecker.passSingleValueCheck, QPS rules)
    def param_load_rules(self, rules: np.ndarray, hot: np.ndarray = None):
        rules = np.ascontiguousarray(rules, dtype=abi.PARAM_RULE_DTYPE)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        self._check(self._L.sg_param_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot), len(hot)))

    def param_decide_host(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.PARAM_REQ_DTYPE)
        out = np.zeros(len(req), np.int32)
        self._check(self._L.sg_param_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def param_decide_device(self, req_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        self._check(self._L.sg_param_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr),
                                                  C.c_void_p(stream_ptr)))

    def param_state(self, rule, value):
        lt, tk = C.c_int64(), C.c_int64()
        flags = self._L.sg_param_read_state(self.h, rule, value, C.byref(lt), C.byref(tk))
        if flags < 0:
            self._check(flags)
        return flags, lt.value, tk.value

    # ---- pace controller (RateLimiterController.canPass per CONTROL_BEHAVIOR_RATE_LIMITER FlowRule)
    def pace_load_rules(self, rules: np.ndarray):
        rules = np.ascontiguousarray(rules, dtype=abi.PACE_RULE_DTYPE)
        self._check(self._L.sg_pace_load_rules(self.h, abi.ptr(rules), len(rules)))

    def pace_decide_host(self, req: np.ndarray) -> np.ndarray:
        """wait ms per request, abi.PACE_BLOCKED (-1) when canPass is false."""
        req = np.ascontiguousarray(req, dtype=abi.PACE_REQ_DTYPE)
        out = np.zeros(len(req), np.int32)
        self._check(self._L.sg_pace_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def pace_decide_device(self, req_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        self._check(self._L.sg_pace_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr),
                                                 C.c_void_p(stream_ptr)))

    def pace_latest(self, rule):
        v = C.c_int64()
        self._check(self._L.sg_pace_read_state(self.h, rule, C.byref(v)))
        return v.value

    def snapshot(self, now_ms, n_rules):
        out = np.zeros(2 * n_rules, np.float64)
        self._check(self._L.sg_snapshot_metrics(self.h, now_ms, abi.ptr(out), len(out)))
        return out.reshape(n_rules, 2)

    # ---- ParamFlowSlot chain (every param rule of a resource, collection args, THREAD grade)
    def pslot_load_rules(self, rules, hot=None, n_resources=None):
        rules = np.ascontiguousarray(rules, dtype=abi.PSLOT_RULE_DTYPE).reshape(-1)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        n_res = int(rules["resource"].max()) + 1 if n_resources is None else n_resources
        self._check(self._L.sg_pslot_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot) if len(hot) else None,
                                                len(hot), n_res))

    def pslot_decide_host(self, ev, args, values):
        ev = np.ascontiguousarray(ev, dtype=abi.PSLOT_EVENT_DTYPE).reshape(-1)
        args = np.ascontiguousarray(args, dtype=abi.PSLOT_ARG_DTYPE).reshape(-1)
        values = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1)
        out = np.zeros(len(ev), abi.PSLOT_RES_DTYPE)
        self._check(self._L.sg_pslot_decide_batch_host(self.h, abi.ptr(ev), len(ev), abi.ptr(args) if len(args) else None,
                                                       len(args), abi.ptr(values) if len(values) else None,
                                                       len(values), abi.ptr(out)))
        return out

    def pslot_thread_count(self, res, idx, value):
        v = C.c_int64()
        self._check(self._L.sg_pslot_thread_count(self.h, res, idx, int(value), C.byref(v)))
        return v.value

    def pslot_param_idx(self, rule):
        v = C.c_int32()
        self._check(self._L.sg_pslot_param_idx(self.h, rule, C.byref(v)))
        return v.value

    # ---- concurrent cluster tokens (requestConcurrentToken / releaseConcurrentToken)
    def conc_set_rule_timeouts(self, client_offline_ms, resource_timeout_ms):
        a = np.ascontiguousarray(client_offline_ms, dtype=np.int64)
        b = np.ascontiguousarray(resource_timeout_ms, dtype=np.int64)
        self._check(self._L.sg_conc_set_rule_timeouts(self.h, abi.ptr(a), abi.ptr(b), len(a)))

    def conc_decide_host(self, req: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.CONC_REQ_DTYPE)
        out = np.zeros(len(req), abi.CONC_RES_DTYPE)
        self._check(self._L.sg_conc_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(out)))
        return out

    def conc_expire(self, now_ms, online) -> int:
        online = np.ascontiguousarray(online, dtype=np.uint8)
        rm = C.c_uint64()
        self._check(self._L.sg_conc_expire(self.h, now_ms, abi.ptr(online) if len(online) else None, len(online),
                                           C.byref(rm)))
        return rm.value

    def conc_state(self, key):
        """(nowCalls of rule key, live tokens)."""
        now, live = C.c_int32(), C.c_uint64()
        self._check(self._L.sg_conc_read_state(self.h, key, C.byref(now), C.byref(live)))
        return now.value, live.value

    # ---- local slot chain (StatisticSlot → FlowSlot/DefaultController → DegradeSlot)
    def local_load_rules(self, rules: np.ndarray, sample_count=2, interval_ms=1000, occupy_timeout_ms=500,
                         cold_factor=3):
        rules = np.ascontiguousarray(rules, dtype=abi.LOCAL_RULE_DTYPE).reshape(-1)
        cfg = abi.sg_local_config(sample_count=sample_count, interval_ms=interval_ms,
                                  occupy_timeout_ms=occupy_timeout_ms, cold_factor=cold_factor)
        self._check(self._L.sg_local_load_rules(self.h, C.byref(cfg), abi.ptr(rules), len(rules)))
        self.local_S = sample_count
        self.local_K = len(rules)

    def local_decide_host(self, ev: np.ndarray) -> np.ndarray:
        ev = np.ascontiguousarray(ev, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        out = np.zeros(len(ev), abi.LOCAL_RES_DTYPE)
        self._check(self._L.sg_local_decide_batch_host(self.h, abi.ptr(ev), len(ev), abi.ptr(out)))
        return out

    def local_decide_device(self, ev_ptr: int, n: int, out_ptr: int, stream_ptr: int = 0):
        self._check(self._L.sg_local_decide_batch(self.h, C.c_void_p(ev_ptr), n, C.c_void_p(out_ptr),
                                                  C.c_void_p(stream_ptr)))

    def local_enqueue(self, ev_ptr: int, n: int, out_ptr: int) -> int:
        """sg_local_enqueue: a device-resident local batch on the pipelined path (its front half beside the previous
        batch's walkers); returns the ticket for local_wait. The buffers must stay untouched until it completes."""
        t = C.c_uint64()
        self._check(self._L.sg_local_enqueue(self.h, C.c_void_p(ev_ptr), n, C.c_void_p(out_ptr), C.byref(t)))
        return t.value

    def local_wait(self, ticket):
        self._check(self._L.sg_local_wait(self.h, ticket))

    def local_poll(self, ticket) -> bool:
        r = self._L.sg_local_poll(self.h, ticket)
        if r < 0:
            self._check(r)
        return r == 1

    def local_state(self, res):
        """(second [S][8], borrow [S][2], minute [60][8], head[14]) — see sg_local_read_state."""
        S = self.local_S
        sec = np.zeros((S, 8), np.int64)
        bor = np.zeros((S, 2), np.int64)
        mnt = np.zeros((60, 8), np.int64)
        head = np.zeros(14, np.int64)
        self._check(self._L.sg_local_read_state(self.h, res, abi.ptr(sec), abi.ptr(bor), abi.ptr(mnt), abi.ptr(head)))
        return sec, bor, mnt, head

    def local_metrics(self, now_ms) -> np.ndarray:
        """MetricTimerListener.run: every resource's new minute-bucket rows (sg_metric_node), time-sorted."""
        n = C.c_uint64()
        rc = self._L.sg_local_metrics(self.h, now_ms, None, 0, C.byref(n))
        if rc not in (0, abi.SG_E_CAPACITY):
            self._check(rc)
        out = np.zeros(max(1, n.value), abi.METRIC_NODE_DTYPE)
        self._check(self._L.sg_local_metrics(self.h, now_ms, abi.ptr(out), len(out), C.byref(n)))
        return out[:n.value]

    def local_metrics_raw(self, now_ms) -> np.ndarray:
        """sg_local_metrics_raw: this GPU's share of the node's rows, rt as the raw sum (LocalMetricRollup merges)."""
        n = C.c_uint64()
        rc = self._L.sg_local_metrics_raw(self.h, now_ms, None, 0, C.byref(n))
        if rc not in (0, abi.SG_E_CAPACITY):
            self._check(rc)
        out = np.zeros(max(1, n.value), abi.METRIC_NODE_DTYPE)
        self._check(self._L.sg_local_metrics_raw(self.h, now_ms, abi.ptr(out), len(out), C.byref(n)))
        return out[:n.value]

    def local_metrics_raw_device(self, now_ms, out) -> int:
        """sg_local_metrics_raw_device: this GPU's raw rows into `out` (a device tensor of at least cap x 64 B, as
        int64 [cap, 8]), unsorted; returns the row count."""
        n = C.c_uint64()
        cap = out.numel() * out.element_size() // abi.METRIC_NODE_DTYPE.itemsize
        self._check(self._L.sg_local_metrics_raw_device(self.h, now_ms, C.c_void_p(out.data_ptr()), cap, C.byref(n)))
        return n.value

    def local_metrics_raw_enqueue(self, now_ms, out, count, stream_ptr: int = 0):
        """sg_local_metrics_raw_enqueue: the rows into `out` (device int64 [cap, 8]) and their number into `count`
        (a device int64 tensor of one element), after the batches enqueued so far; `stream_ptr` waits for them."""
        cap = out.numel() * out.element_size() // abi.METRIC_NODE_DTYPE.itemsize
        self._check(self._L.sg_local_metrics_raw_enqueue(self.h, now_ms, C.c_void_p(out.data_ptr()), cap,
                                                         C.c_void_p(count.data_ptr()), C.c_void_p(stream_ptr)))

    def local_owners(self, world) -> np.ndarray:
        """sg_local_owners: the GPU of `world` that owns each resource (key groups co-located)."""
        out = np.zeros(max(1, self.local_K), np.uint32)
        self._check(self._L.sg_local_owners(self.h, world, abi.ptr(out), self.local_K))
        return out[:self.local_K]

    def local_load_flow_rules(self, rules: np.ndarray, n_origins=0, n_contexts=0) -> int:
        """FlowRuleManager.loadRules for the local chain; returns the number of rules kept."""
        rules = np.ascontiguousarray(rules, dtype=abi.LOCAL_FLOW_RULE_DTYPE).reshape(-1)
        rc = self._L.sg_local_load_flow_rules(self.h, abi.ptr(rules), len(rules), n_origins, n_contexts)
        self._check(min(rc, 0))
        return rc

    def local_set_entry_types(self, inbound):
        """EntryType of each resource's entries (1 = IN: counted by Constants.ENTRY_NODE); default OUT."""
        v = np.ascontiguousarray(inbound, dtype=np.uint8)
        self._check(self._L.sg_local_set_entry_types(self.h, abi.ptr(v), len(v)))

    def local_set_cluster_state(self, state):
        """ClusterStateManager state (CLUSTER_NOT_STARTED -1 is the one the device decides cluster rules in)."""
        self._check(self._L.sg_local_set_cluster_state(self.h, state))

    def slot_decide_host(self, ev, ext, args, values) -> np.ndarray:
        """The whole slot chain (sg_slot_decide_batch_host): StatisticSlot around ParamFlowSlot → FlowSlot →
        DegradeSlot for HOST events with their context / argument records (ext may be None)."""
        ev = np.ascontiguousarray(ev, dtype=abi.LOCAL_EVENT_DTYPE).reshape(-1)
        out = np.zeros(len(ev), abi.LOCAL_RES_DTYPE)
        if len(ev) == 0:
            return out
        xp = None
        if ext is not None:
            ext = np.ascontiguousarray(ext, dtype=abi.SLOT_EXT_DTYPE).reshape(-1)
            xp = abi.ptr(ext)
        args = np.ascontiguousarray(np.zeros(0, abi.PSLOT_ARG_DTYPE) if args is None else args,
                                    dtype=abi.PSLOT_ARG_DTYPE).reshape(-1)
        values = np.ascontiguousarray(np.zeros(0, np.uint64) if values is None else values, dtype=np.uint64).reshape(-1)
        self._check(self._L.sg_slot_decide_batch_host(self.h, abi.ptr(ev), xp, len(ev),
                                                      abi.ptr(args) if len(args) else None, len(args),
                                                      abi.ptr(values) if len(values) else None, len(values),
                                                      abi.ptr(out)))
        return out

    def slot_decide_device(self, ev_ptr: int, ext_ptr: int, n: int, args_ptr: int, n_args: int, values_ptr: int,
                           n_values: int, out_ptr: int, stream_ptr: int = 0):
        """DEVICE pointers (ext_ptr 0: no ext)."""
        self._check(self._L.sg_slot_decide_batch(self.h, C.c_void_p(ev_ptr), C.c_void_p(ext_ptr or None), n,
                                                 C.c_void_p(args_ptr or None), n_args, C.c_void_p(values_ptr or None),
                                                 n_values, C.c_void_p(out_ptr), C.c_void_p(stream_ptr)))

    def local_context_state(self, res, context, with_exists=False):
        """The DefaultNode of (res, context): (second, borrow, minute, head) as local_state (+ whether an event created
        it yet, with_exists)."""
        return self._pool_node_state(self._L.sg_local_read_context_state, res, context, with_exists)

    def local_origin_state(self, res, origin, with_exists=False):
        """The origin node of (res, origin): (second, borrow, minute, head) as local_state (+ exists)."""
        return self._pool_node_state(self._L.sg_local_read_origin_state, res, origin, with_exists)

    def _pool_node_state(self, fn, res, ident, with_exists):
        S = self.local_S
        sec = np.zeros((S, 8), np.int64)
        bor = np.zeros((S, 2), np.int64)
        mnt = np.zeros((60, 8), np.int64)
        head = np.zeros(14, np.int64)
        rc = fn(self.h, res, ident, abi.ptr(sec), abi.ptr(bor), abi.ptr(mnt), abi.ptr(head))
        if rc < 0:
            self._check(rc)
        return (sec, bor, mnt, head, rc == 1) if with_exists else (sec, bor, mnt, head)

    def local_controller(self, rule):
        """{storedTokens, lastFilledTime, latestPassedTime} of input flow rule `rule`."""
        out = np.zeros(3, np.int64)
        self._check(self._L.sg_local_read_controller(self.h, rule, abi.ptr(out)))
        return out

    # ---- cluster hot-parameter tokens (requestParamToken → ClusterParamFlowChecker)
    def cparam_load_rules(self, rules: np.ndarray, hot: np.ndarray = None, capacity_log2=0):
        rules = np.ascontiguousarray(rules, dtype=abi.CPARAM_RULE_DTYPE)
        hot = np.ascontiguousarray(np.zeros(0, abi.PARAM_HOT_DTYPE) if hot is None else hot, dtype=abi.PARAM_HOT_DTYPE)
        self._check(self._L.sg_cparam_load_rules(self.h, abi.ptr(rules), len(rules), abi.ptr(hot), len(hot),
                                                 capacity_log2))

    def cparam_decide_device(self, req_ptr: int, n: int, values_ptr: int, n_values: int, out_ptr: int,
                             stream_ptr: int = 0):
        """DEVICE pointers: n sg_cparam_req, n_values u64 values, n sg_result."""
        self._check(self._L.sg_cparam_decide_batch(self.h, C.c_void_p(req_ptr), n, C.c_void_p(values_ptr), n_values,
                                                   C.c_void_p(out_ptr), C.c_void_p(stream_ptr)))

    def cparam_last_rounds(self) -> int:
        """Fixed-point rounds the last sg_cparam_decide_batch needed (max_rounds + 1: decided serially)."""
        r = C.c_uint32()
        self._check(self._L.sg_cparam_last_rounds(self.h, C.byref(r)))
        return r.value

    def cparam_decide_host(self, req: np.ndarray, values: np.ndarray) -> np.ndarray:
        req = np.ascontiguousarray(req, dtype=abi.CPARAM_REQ_DTYPE)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.zeros(len(req), abi.RES_DTYPE)
        self._check(self._L.sg_cparam_decide_batch_host(self.h, abi.ptr(req), len(req), abi.ptr(values), len(values),
                                                         abi.ptr(out)))
        return out

    def cparam_top_values(self, now_ms, n_rules, number=5):
        """ClusterParamMetric.getTopValues(number) of every cluster param rule: list of [(value, qps), ...]."""
        vals = np.zeros(n_rules * number, np.uint64)
        qps = np.zeros(n_rules * number, np.float64)
        cnt = np.zeros(max(1, n_rules), np.uint32)
        self._check(self._L.sg_cparam_top_values(self.h, now_ms, number, abi.ptr(vals), abi.ptr(qps), abi.ptr(cnt)))
        return [[(int(vals[r * number + i]), float(qps[r * number + i])) for i in range(int(cnt[r]))]
                for r in range(n_rules)]

    def cparam_sum(self, rule, value, now):
        v = C.c_int64()
        self._check(self._L.sg_cparam_read_sum(self.h, rule, int(value), now, C.byref(v)))
        return v.value
