// cparam_dev.h — ClusterParamMetric / ClusterParamFlowChecker steps on the device, shared by the cluster param walkers
// (cparam.hip) and the embedded token server of the ParamFlowSlot (pslot_dev.h): the exact (rule, value) table and
// the per-value window sum (srv/flow/statistic/metric/ClusterParamMetric.java:49-63, ClusterParamFlowChecker.java:96-116).
#pragma once
#include "engine.h"

namespace sg {

constexpr uint64_t kCpEmpty = ~0ull;

// ParamFlowRule.retrieveExclusiveItemCount(value) ?? count, × connectedCount for AVG_LOCAL (thr_scale)
__device__ __forceinline__ double cp_threshold(const CPArgs& c, const CPRule& r, uint64_t v) {
    uint32_t lo = r.hot_begin, hi = r.hot_begin + r.hot_count;  // sorted by value
    double count = r.count;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t hv = c.hot[mid].value;
        if (hv == v) {
            count = (double)c.hot[mid].threshold;
            break;
        }
        if (hv < v) lo = mid + 1;
        else hi = mid;
    }
    return r.global ? count : count * (double)r.connected;
}

__device__ __forceinline__ uint64_t cp_slot(const CPArgs& c, const CPRule& r, uint64_t v) {
    if (v == kCpEmpty) return r.table_base + r.table_mask + 1;  // side slot for the marker value
    uint64_t h = v + 0x9E3779B97F4A7C15ull;
    h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
    h ^= h >> 31;
    uint64_t i = h & r.table_mask;
    for (uint64_t probes = 0; probes <= r.table_mask; ++probes) {
        unsigned long long* vw = (unsigned long long*)&c.keys[r.table_base + i];
        // a plain (L2-cached) load: a slot only ever goes from empty to its value, so a stale read can only say
        // "empty", and the CAS below then returns the value that is there (an agent-scope atomic load bypassed
        // the XCD's L2 on every probe, also for the hot values that repeat throughout a batch)
        const unsigned long long cur = *vw;
        if (cur == v) return r.table_base + i;
        if (cur == kCpEmpty) {
            const unsigned long long old = atomicCAS(vw, (unsigned long long)kCpEmpty, (unsigned long long)v);
            if (old == kCpEmpty || old == v) return r.table_base + i;
        }
        i = (i + 1) & r.table_mask;
    }
    return ~0ull;
}

__device__ __forceinline__ uint32_t cp_rule_of_slot(const CPArgs& c, uint64_t g) {
    return (uint32_t)(g / c.per);  // every rule's sub-table has the same size
}

// Σ of the value's counts over the window at period P (slot I = P % S is current or stale; the others
// count iff their period is one of the S - 1 before P), plus slot I's count if it is already period P.
__device__ __forceinline__ int64_t cp_window(const CPBucket* ring, int S, int64_t wl, int64_t P, int64_t* cur_count) {
    const int I = (int)(P % S);
    const int64_t ws = P * wl, lo = ws - (int64_t)(S - 1) * wl;
    int64_t sum = 0;
    for (int j = 0; j < S; ++j) {
        const CPBucket b = ring[j];
        if (j == I) {
            *cur_count = b.start == ws ? b.count : 0;
        } else if (b.start != INT64_MIN && b.start >= lo) {
            sum += b.count;
        }
    }
    return sum;
}

// The slot of (rule, value) when the value is in the table, else ~0 (ClusterParamMetric.getSum of an absent value: 0).
__device__ __forceinline__ uint64_t cp_find(const CPArgs& c, const CPRule& r, uint64_t v) {
    if (v == kCpEmpty) return r.table_base + r.table_mask + 1;
    uint64_t h = v + 0x9E3779B97F4A7C15ull;
    h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
    h ^= h >> 31;
    uint64_t i = h & r.table_mask;
    for (uint64_t probes = 0; probes <= r.table_mask; ++probes) {
        const uint64_t cur = c.keys[r.table_base + i];
        if (cur == v) return r.table_base + i;
        if (cur == kCpEmpty) return ~0ull;
        i = (i + 1) & r.table_mask;
    }
    return ~0ull;
}

}  // namespace sg
