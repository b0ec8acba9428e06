"""ctypes mirror of include/sentinel_gpu.h (the C ABI of libsentinel_gpu.so).

Struct layouts here must match the header byte for byte; tests/test_abi.py checks the sizes.
Status codes follow TokenResultStatus (sentinel-core/.../cluster/TokenResultStatus.java:27-53).
"""
import ctypes as C

import numpy as np

SG_OK = 0
SG_E_INVAL = -1
SG_E_DEVICE = -2
SG_E_NOMEM = -3
SG_E_UNSUPPORTED = -4
SG_E_TIME = -5
SG_E_CAPACITY = -6

BAD_REQUEST = -4
TOO_MANY_REQUEST = -2
FAIL = -1
OK = 0
BLOCKED = 1
SHOULD_WAIT = 2
NO_RULE_EXISTS = 3

THRESHOLD_AVG_LOCAL = 0
THRESHOLD_GLOBAL = 1

# ClusterFlowEvent ordinals (srv/flow/statistic/data/ClusterFlowEvent.java:22-52)
EV_PASS, EV_BLOCK, EV_PASS_REQUEST, EV_BLOCK_REQUEST, EV_OCCUPIED_PASS, EV_OCCUPIED_BLOCK, EV_WAITING = range(7)
NUM_EVENTS = 7

KEY_PRIO = 0x80000000

# token-server wire codec (include/sentinel_gpu.h SG_FRAME_*, SG_MSG_TYPE_*)
MSG_TYPE_PING, MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW = 0, 1, 2
FRAME_FLOW, FRAME_SHORT, FRAME_NO_DATA, FRAME_OTHER = 0, 1, 2, 3
RESPONSE_FRAME_BYTES = 16
KEY_INDEX = 0x7FFFFFFF
KEY_NO_RULE = 0x7FFFFFFF
KEY_BAD = 0x7FFFFFFE

MAX_SAMPLE_COUNT = 64
FLAG_SERIAL_ONLY = 1
FLAG_WAVE_ONLY = 2
FLAG_RING_REREAD = 4
INT64_MIN = -(1 << 63)


class sg_config(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_int32), ("exceed_count", C.c_double),
                ("max_occupy_ratio", C.c_double), ("max_batch", C.c_uint64)]


class sg_flow_rule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32), ("namespace_id", C.c_int32)]


class sg_namespace(C.Structure):
    _fields_ = [("limiter_enabled", C.c_int32), ("connected_count", C.c_int32), ("max_allowed_qps", C.c_double)]


class sg_req(C.Structure):
    _fields_ = [("ts_ms", C.c_int64), ("key", C.c_uint32), ("acquire", C.c_int32)]


class sg_result(C.Structure):
    _fields_ = [("status", C.c_int32), ("remaining", C.c_int32), ("wait_ms", C.c_int32)]


class sg_batch_stats(C.Structure):
    _fields_ = [("total_ms", C.c_float), ("walk_ms", C.c_float), ("sort_ms", C.c_float),
                ("touched_keys", C.c_uint64), ("long_segments", C.c_uint64), ("skipped_ranges", C.c_uint64)]


# numpy views of the request / result records (same layout as the C structs)
REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("key", "<u4"), ("acquire", "<i4")], align=True)
# sg_rls_request / sg_rls_status (Envoy RLS entry point)
RLS_REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("hits_addend", "<i4"), ("desc_begin", "<u4"), ("desc_count", "<u4"),
                          ("pad", "<u4")], align=True)
RLS_STATUS_DTYPE = np.dtype([("code", "<i4"), ("limit_remaining", "<i4"), ("requests_per_unit", "<i4"),
                             ("has_rule", "<i4")], align=True)
RLS_OK, RLS_OVER_LIMIT, RLS_ERROR = 1, 2, -1
RES_DTYPE = np.dtype([("status", "<i4"), ("remaining", "<i4"), ("wait_ms", "<i4")], align=True)
RULE_DTYPE = np.dtype([("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"), ("sample_count", "<i4"),
                       ("window_interval_ms", "<i4"), ("namespace_id", "<i4")], align=True)
NS_DTYPE = np.dtype([("limiter_enabled", "<i4"), ("connected_count", "<i4"), ("max_allowed_qps", "<f8")],
                    align=True)

PARAM_RULE_DTYPE = np.dtype([("count", "<f8"), ("duration_sec", "<i8"), ("burst", "<i4"), ("behavior", "<i4"),
                             ("max_queueing_ms", "<i4"), ("hot_begin", "<u4"), ("hot_count", "<u4"),
                             ("capacity_log2", "<i4")], align=True)
PARAM_HOT_DTYPE = np.dtype([("value", "<u8"), ("threshold", "<i4"), ("reserved", "<i4")], align=True)
PARAM_REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("value", "<u8"), ("rule", "<u4"), ("acquire", "<i4")], align=True)
PACE_RULE_DTYPE = np.dtype([("count", "<f8"), ("max_queueing_ms", "<i4"), ("reserved", "<i4")], align=True)
PACE_REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("rule", "<u4"), ("acquire", "<i4")], align=True)
PACE_BLOCKED = -1
CPARAM_RULE_DTYPE = np.dtype([("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"), ("sample_count", "<i4"),
                              ("window_interval_ms", "<i4"), ("namespace_id", "<i4"), ("hot_begin", "<u4"),
                              ("hot_count", "<u4")], align=True)
CPARAM_REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("key", "<u4"), ("acquire", "<i4"), ("value_begin", "<u4"),
                             ("value_count", "<u4")], align=True)
BEHAVIOR_DEFAULT = 0
BEHAVIOR_RATE_LIMITER = 2

# ParamFlowSlot chain (sg_pslot_*)
PSLOT_RULE_DTYPE = np.dtype([("rule", PARAM_RULE_DTYPE), ("resource", "<u4"), ("param_idx", "<i4"), ("grade", "<i4"),
                             ("cluster_mode", "<i4"), ("cluster_key", "<u4"),
                             ("reserved", "<i4")], align=True)
PSLOT_ARG_DTYPE = np.dtype([("value_begin", "<u4"), ("value_count", "<u4"), ("kind", "<i4"), ("reserved", "<i4")],
                           align=True)
PSLOT_EVENT_DTYPE = np.dtype([("ts_ms", "<i8"), ("resource", "<u4"), ("count", "<i4"), ("kind", "<i4"),
                              ("arg_begin", "<u4"), ("arg_count", "<u4"), ("args_null", "<i4")], align=True)
PSLOT_RES_DTYPE = np.dtype([("pass", "<i4"), ("rule", "<i4")], align=True)
ARG_NULL, ARG_VALUE, ARG_COLLECTION = 0, 1, 2

# metric snapshots (sg_local_metrics)
METRIC_NODE_DTYPE = np.dtype([("timestamp", "<i8"), ("pass_qps", "<i8"), ("block_qps", "<i8"), ("success_qps", "<i8"),
                              ("exception_qps", "<i8"), ("rt", "<i8"), ("occupied_pass_qps", "<i8"),
                              ("resource", "<u4"), ("concurrency", "<i4")], align=True)

# concurrent cluster tokens (sg_conc_*)
CONC_REQ_DTYPE = np.dtype([("ts_ms", "<i8"), ("token_id", "<u8"), ("key", "<u4"), ("acquire", "<i4"),
                           ("client", "<u4"), ("kind", "<i4")], align=True)
CONC_RES_DTYPE = np.dtype([("status", "<i4"), ("reserved", "<i4"), ("token_id", "<u8")], align=True)
CONC_ACQUIRE, CONC_RELEASE = 0, 1
RELEASE_OK, ALREADY_RELEASE = 6, 7

# local slot chain (sg_local_*)
DEGRADE_RULE_DTYPE = np.dtype([("grade", "<i4"), ("time_window_sec", "<i4"), ("count", "<f8"),
                               ("slow_ratio_threshold", "<f8"), ("min_request_amount", "<i4"),
                               ("stat_interval_ms", "<i4")], align=True)
LOCAL_RULE_DTYPE = np.dtype([("flow_count", "<f8"), ("flow_grade", "<i4"), ("n_breakers", "<i4"),
                             ("breakers", DEGRADE_RULE_DTYPE, (2,))], align=True)
LOCAL_EVENT_DTYPE = np.dtype([("ts_ms", "<i8"), ("create_ts", "<i8"), ("resource", "<u4"), ("count", "<i4"),
                              ("kind", "<i4"), ("origin", "<i4")], align=True)
LOCAL_RES_DTYPE = np.dtype([("status", "<i4"), ("wait_ms", "<i4")], align=True)
DEGRADE_RT, DEGRADE_EXCEPTION_RATIO, DEGRADE_EXCEPTION_COUNT = 0, 1, 2
FLOW_GRADE_THREAD, FLOW_GRADE_QPS, FLOW_GRADE_NONE = 0, 1, -1
LOCAL_ENTRY, LOCAL_EXIT, LOCAL_EXIT_ERROR = 0, 1, 2
LOCAL_PASS, LOCAL_BLOCK_FLOW, LOCAL_BLOCK_DEGRADE, LOCAL_PASS_WAIT = 0, 1, 2, 3
# sg_local_flow_rule (FlowRule of the local chain)
LOCAL_FLOW_RULE_DTYPE = np.dtype([("resource", "<u4"), ("grade", "<i4"), ("count", "<f8"),
                                  ("control_behavior", "<i4"), ("limit_app", "<i4"), ("strategy", "<i4"),
                                  ("warm_up_period_sec", "<i4"), ("max_queueing_ms", "<i4"),
                                  ("ref_resource", "<i4"), ("cluster_mode", "<i4"), ("cluster_config", "<i4"),
                                  ("cluster_key", "<u4")],
                                 align=True)
CLUSTER_MODE_OFF, CLUSTER_MODE_FALLBACK, CLUSTER_MODE_NO_FALLBACK, CLUSTER_MODE_INVALID = 0, 1, 2, -1
CLUSTER_CLIENT, CLUSTER_SERVER, CLUSTER_NOT_STARTED = 0, 1, -1
# the whole slot chain (sg_slot_decide_batch): per-event context and arguments
SLOT_EXT_DTYPE = np.dtype([("context", "<u4"), ("arg_begin", "<u4"), ("arg_count", "<u4"), ("args_null", "<i4")],
                          align=True)
LOCAL_BLOCK_PARAM = 4
ENTRY_NODE_RESOURCE = 0xFFFFFFFF  # sg_local_metrics rows of Constants.ENTRY_NODE
CONTROL_DEFAULT, CONTROL_WARM_UP, CONTROL_RATE_LIMITER, CONTROL_WARM_UP_RATE_LIMITER = 0, 1, 2, 3
LIMIT_APP_DEFAULT, LIMIT_APP_OTHER = 0, -1
STRATEGY_DIRECT, STRATEGY_RELATE, STRATEGY_CHAIN = 0, 1, 2

class sg_local_config(C.Structure):
    _fields_ = [("sample_count", C.c_int32), ("interval_ms", C.c_int32), ("occupy_timeout_ms", C.c_int32),
                ("cold_factor", C.c_int32)]


assert REQ_DTYPE.itemsize == C.sizeof(sg_req) == 16
assert RES_DTYPE.itemsize == C.sizeof(sg_result) == 12
assert RULE_DTYPE.itemsize == C.sizeof(sg_flow_rule) == 32
assert NS_DTYPE.itemsize == C.sizeof(sg_namespace) == 16
assert CPARAM_RULE_DTYPE.itemsize == 40 and CPARAM_REQ_DTYPE.itemsize == 24
assert DEGRADE_RULE_DTYPE.itemsize == 32 and LOCAL_RULE_DTYPE.itemsize == 80
assert LOCAL_EVENT_DTYPE.itemsize == 32 and LOCAL_RES_DTYPE.itemsize == 8
assert LOCAL_FLOW_RULE_DTYPE.itemsize == 56 and SLOT_EXT_DTYPE.itemsize == 16
assert CONC_REQ_DTYPE.itemsize == 32 and CONC_RES_DTYPE.itemsize == 16
assert METRIC_NODE_DTYPE.itemsize == 64
assert PSLOT_RULE_DTYPE.itemsize == PARAM_RULE_DTYPE.itemsize + 24 and PSLOT_EVENT_DTYPE.itemsize == 32


def ptr(a: np.ndarray) -> C.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)
