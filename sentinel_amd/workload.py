"""Seeded synthetic workloads for the flow-decision engine.

A workload is a rule table (sg_flow_rule records) plus time-ordered token requests (sg_req records):
keys follow a Zipf law over the flowIds (rank → flowId through a seeded permutation, so hot flows are
spread over the key space), timestamps are uniform over the simulated span and sorted, ties keep
arrival order.
"""
from dataclasses import dataclass

import numpy as np

from . import abi


@dataclass
class ClusterWorkload:
    """C3 (north star): cluster token server, FLOW_THRESHOLD_GLOBAL rules, S=10 / 1000 ms windows."""
    n_flows: int = 1_000_000
    n_requests: int = 16_000_000
    span_ms: int = 1000
    zipf_s: float = 1.0
    count_lo: int = 1
    count_hi: int = 32
    prio_frac: float = 0.01
    multi_acquire_frac: float = 0.10   # acquire ~ U{2..4} for this fraction, else 1
    sample_count: int = 10
    interval_ms: int = 1000
    t0: int = 1_700_000_000_000
    seed: int = 3

    def rules(self) -> np.ndarray:
        rng = np.random.default_rng(self.seed)
        r = np.zeros(self.n_flows, abi.RULE_DTYPE)
        r["flow_id"] = np.arange(1, self.n_flows + 1, dtype=np.int64) + 10_000_000
        r["count"] = rng.integers(self.count_lo, self.count_hi + 1, self.n_flows).astype(np.float64)
        r["threshold_type"] = abi.THRESHOLD_GLOBAL
        r["sample_count"] = self.sample_count
        r["window_interval_ms"] = self.interval_ms
        r["namespace_id"] = 0
        return r

    def requests(self, batch: int = 0) -> np.ndarray:
        """Batch `batch` covers [t0 + batch*span, t0 + (batch+1)*span)."""
        rng = np.random.default_rng((self.seed, batch))
        n = self.n_requests
        req = np.zeros(n, abi.REQ_DTYPE)
        start = self.t0 + batch * self.span_ms
        req["ts_ms"] = start + np.sort(rng.integers(0, self.span_ms, n, dtype=np.int64))
        req["key"] = zipf_keys(rng, self.n_flows, n, self.zipf_s, perm_seed=self.seed)
        acq = np.ones(n, np.int32)
        multi = rng.random(n) < self.multi_acquire_frac
        acq[multi] = rng.integers(2, 5, int(multi.sum()), dtype=np.int32)
        req["acquire"] = acq
        prio = rng.random(n) < self.prio_frac
        req["key"] |= np.where(prio, np.uint32(abi.KEY_PRIO), np.uint32(0))
        return req


_zipf_cache = {}


def zipf_keys(rng, n_keys, n, s, perm_seed=0):
    """n draws of key indices with P(rank r) ∝ r^-s, ranks mapped to keys by a seeded permutation."""
    ck = (n_keys, s, perm_seed)
    if ck not in _zipf_cache:
        w = 1.0 / np.power(np.arange(1, n_keys + 1, dtype=np.float64), s)
        cdf = np.cumsum(w)
        cdf /= cdf[-1]
        perm = np.random.default_rng(perm_seed + 7919).permutation(n_keys).astype(np.uint32)
        _zipf_cache[ck] = (cdf, perm)
    cdf, perm = _zipf_cache[ck]
    ranks = np.searchsorted(cdf, rng.random(n), side="right")
    np.minimum(ranks, n_keys - 1, out=ranks)
    return perm[ranks]


def touched_keys(req: np.ndarray, n_flows: int) -> int:
    k = req["key"] & abi.KEY_INDEX
    k = k[k < n_flows]
    return int(np.unique(k).size)
