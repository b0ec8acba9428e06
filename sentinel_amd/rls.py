"""Envoy RLS front-end over the device engine.

Mirrors sentinel-cluster-server-envoy-rls's SentinelEnvoyRlsServiceImpl.shouldRateLimit
(service/v3/SentinelEnvoyRlsServiceImpl.java:34-85) for a batch of RateLimitRequests: every descriptor is one
SimpleClusterFlowChecker.acquireClusterToken call (flow/SimpleClusterFlowChecker.java:33-65), which is the
token server's ClusterFlowChecker without the namespace limiter and without prioritized occupy. So the shim
submits each descriptor as a non-prioritized request of its rule to sg_flow_decide_batch (rules loaded with
the GLOBAL threshold, count * exceedCount, as SimpleClusterFlowChecker computes it; no namespace limiter)
and maps the TokenResults back to Envoy codes. The descriptor → rule lookup
(EnvoySentinelRuleConverter.generateFlowId over domain + descriptor entries) is string work the caller does;
here a descriptor arrives as its rule index, or -1 when no rule exists.

`should_rate_limit` builds the descriptor batch in Python over any decide() (the device engine or the oracle);
`should_rate_limit_abi` calls the library's own entry point, sg_rls_should_rate_limit (the same mapping in C++ for
C++ / JNI callers), and returns the same responses.
"""
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

from . import abi

CODE_OK = 1          # envoy.service.ratelimit.v3.RateLimitResponse.Code.OK
CODE_OVER_LIMIT = 2  # ... Code.OVER_LIMIT


@dataclass
class RateLimitRequest:
    ts_ms: int                 # TimeUtil.currentTimeMillis() when the call is served
    hits_addend: int           # RateLimitRequest.hits_addend (0 = not present → 1)
    descriptors: List[int]     # rule index of each descriptor, -1 = no rule for it


@dataclass
class DescriptorStatus:
    code: int
    limit_remaining: Optional[int] = None  # set when the descriptor has a rule (:67-73)
    requests_per_unit: Optional[int] = None


@dataclass
class RateLimitResponse:
    overall_code: int = CODE_OK
    statuses: List[DescriptorStatus] = field(default_factory=list)
    error: Optional[str] = None  # responseObserver.onError (hits_addend < 0, :36-40)


def rls_rules(rules: np.ndarray) -> np.ndarray:
    """The flow rules as the RLS checker reads them: threshold count * exceedCount for every type (:42)."""
    r = np.array(rules, dtype=abi.RULE_DTYPE, copy=True)
    r["threshold_type"] = abi.THRESHOLD_GLOBAL
    return r


def should_rate_limit(requests: List[RateLimitRequest], rule_counts: np.ndarray,
                      decide: Callable[[np.ndarray], np.ndarray]) -> List[RateLimitResponse]:
    """Serve a time-ordered batch of RLS requests with one decide() call over all their descriptors.
    decide: sg_req records → TokenResults (the device engine's decide_host, or the oracle's decide_rls)."""
    reqs, owner = [], []
    out = [RateLimitResponse() for _ in requests]
    for j, q in enumerate(requests):
        if q.hits_addend < 0:
            out[j].error = f"acquireCount should be positive, but actual: {q.hits_addend}"
            continue
        acquire = 1 if q.hits_addend == 0 else q.hits_addend  # :41-44
        for d in q.descriptors:
            key = abi.KEY_NO_RULE if d < 0 else int(d)          # checkToken: rule == null → NO_RULE_EXISTS
            reqs.append((q.ts_ms, key, acquire))
            owner.append((j, d))
    if not reqs:
        return out
    batch = np.zeros(len(reqs), abi.REQ_DTYPE)
    batch["ts_ms"] = [r[0] for r in reqs]
    batch["key"] = [r[1] for r in reqs]
    batch["acquire"] = [r[2] for r in reqs]
    res = decide(batch)
    for (j, d), r in zip(owner, res):
        status = int(r["status"])
        if status == abi.NO_RULE_EXISTS:  # the request passes when the descriptor has no rule (:55-58)
            status = abi.OK
        code = CODE_OK if status == abi.OK else CODE_OVER_LIMIT
        st = DescriptorStatus(code)
        if d >= 0:
            st.requests_per_unit = int(rule_counts[d])  # (int) rule.getCount()
            st.limit_remaining = int(r["remaining"])
        out[j].statuses.append(st)
        if code != CODE_OK:
            out[j].overall_code = CODE_OVER_LIMIT
    return out


def should_rate_limit_abi(eng, requests: List[RateLimitRequest]) -> List[RateLimitResponse]:
    """The same responses through sg_rls_should_rate_limit (one call for the whole batch)."""
    req = np.zeros(len(requests), abi.RLS_REQ_DTYPE)
    desc, begin = [], 0
    for j, q in enumerate(requests):
        req[j] = (q.ts_ms, q.hits_addend, begin, len(q.descriptors), 0)
        desc.extend(q.descriptors)
        begin += len(q.descriptors)
    overall, status = eng.rls_should_rate_limit(req, np.array(desc, np.int32))
    out = []
    for j, q in enumerate(requests):
        if overall[j] == abi.RLS_ERROR:
            out.append(RateLimitResponse(error=f"acquireCount should be positive, but actual: {q.hits_addend}"))
            continue
        r = RateLimitResponse(overall_code=int(overall[j]))
        b = int(req[j]["desc_begin"])
        for st in status[b:b + len(q.descriptors)]:
            if st["has_rule"]:
                r.statuses.append(DescriptorStatus(int(st["code"]), int(st["limit_remaining"]),
                                                   int(st["requests_per_unit"])))
            else:
                r.statuses.append(DescriptorStatus(int(st["code"])))
        out.append(r)
    return out
