// pslot_dev.h — device steps of hot-parameter flow control shared by the ParamFlowSlot walkers (param.hip) and the
// whole slot chain's walker (local.hip): ParamFlowChecker.passDefaultLocalCheck / passThrottleLocalCheck
// (sentinel-extension/sentinel-parameter-flow-control/.../slots/block/flow/param/ParamFlowChecker.java:127-254) over the
// exact per-rule value tables, ParameterMetric's thread counts (ParameterMetric.java:125-239) and ParamFlowSlot.checkFlow
// (ParamFlowSlot.java:66-93).
#pragma once
#include "cparam_dev.h"
#include "engine.h"

namespace sg {

constexpr uint64_t kEmptyValue = ~0ull;

__device__ __forceinline__ int64_t java_math_round(double a) {
    // java.lang.Math.round(double), exact floor(a + 1/2) (JDK 7u+)
    const int64_t bits = __double_as_longlong(a);
    const int64_t biased_exp = (bits & 0x7FF0000000000000LL) >> 52;
    const int64_t shift = (52 - 1 + 1023) - biased_exp;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000FFFFFFFFFFFFFLL) | 0x0010000000000000LL;
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    if (a != a) return 0;
    if (a >= 9223372036854775807.0) return INT64_MAX;
    if (a <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)a;
}

// tokenCount of (rule, value): the hot item's threshold, else (long) rule.count (ParamFlowChecker.java:137-141)
__device__ __forceinline__ int64_t param_token_count(const PArgs& p, const PRule& r, uint64_t v) {
    uint32_t lo = r.hot_begin, hi = r.hot_begin + r.hot_count;  // hot items sorted by value
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t hv = p.hot[mid].value;
        if (hv == v) return p.hot[mid].threshold;
        if (hv < v) lo = mid + 1;
        else hi = mid;
    }
    return r.token_count;
}

// find-or-insert (rule, value) → global slot index
__device__ __forceinline__ uint64_t param_slot(const PArgs& p, const PRule& r, uint64_t v) {
    if (v == kEmptyValue) return r.table_base + r.table_mask + 1;  // side slot
    uint64_t h = v + 0x9E3779B97F4A7C15ull;
    h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
    h ^= h >> 31;
    uint64_t i = h & r.table_mask;
    for (uint64_t probes = 0; probes <= r.table_mask; ++probes) {
        unsigned long long* vw = (unsigned long long*)&p.table[r.table_base + i].value;
        // a plain (L2-cached) load: a slot only ever goes from empty to its value, so a stale read can only say
        // "empty", and the CAS below then returns the value that is there (an agent-scope atomic load bypassed
        // the XCD's L2 on every probe, also for the hot values that repeat throughout a batch)
        const unsigned long long cur = *vw;
        if (cur == v) return r.table_base + i;
        if (cur == kEmptyValue) {
            const unsigned long long old = atomicCAS(vw, (unsigned long long)kEmptyValue, (unsigned long long)v);
            if (old == kEmptyValue || old == v) return r.table_base + i;
        }
        i = (i + 1) & r.table_mask;
    }
    return ~0ull;  // table full
}

struct PState {
    int64_t time, tokens;
    uint32_t flags;  // bit0 time counter present, bit1 token counter present
};

struct PReqView {
    int64_t t;
    int64_t acq;
};

// One request of passDefaultLocalCheck at time t (ParamFlowChecker.java:147-201); returns pass.
__device__ __forceinline__ bool param_default_step(PState& s, int64_t tc, int64_t maxc, int64_t dur_ms, int64_t t,
                                                   int64_t acq) {
    if (!(s.flags & 1u)) {
        s.flags |= 1u;
        s.time = t;
        if (!(s.flags & 2u)) {
            s.flags |= 2u;
            s.tokens = maxc - acq;
        }
        return true;
    }
    const int64_t pass_time = t - s.time;
    if (pass_time > dur_ms) {
        if (!(s.flags & 2u)) {
            s.flags |= 2u;
            s.tokens = maxc - acq;
            s.time = t;
            return true;
        }
        const int64_t rest = s.tokens;
        const int64_t to_add = (pass_time * tc) / dur_ms;
        const int64_t nq = to_add + rest > maxc ? (maxc - acq) : (rest + to_add - acq);
        if (nq < 0) return false;
        s.tokens = nq;
        s.time = t;
        return true;
    }
    if ((s.flags & 2u) && s.tokens - acq >= 0) {
        s.tokens -= acq;
        return true;
    }
    return false;
}

// One request of passThrottleLocalCheck (:214-253); the wait is a sleep in Java, skipped in replay.
__device__ __forceinline__ bool param_throttle_step(PState& s, int64_t cost, int32_t max_queue, int64_t t) {
    if (!(s.flags & 1u)) {
        s.flags |= 1u;
        s.time = t;
        return true;
    }
    const int64_t expected = s.time + cost;
    if (expected <= t || expected - t < max_queue) {
        s.time = t;
        if (expected - t > 0) s.time = expected;
        return true;
    }
    return false;
}

__device__ __forceinline__ int64_t throttle_cost(const PRule& r, int64_t tc, int64_t acq) {
    return java_math_round(1.0 * 1000 * (double)acq * (double)r.duration_sec / (double)tc);
}

__device__ __forceinline__ uint64_t ps_hash(unsigned long long owner, uint64_t v) {
    uint64_t z = v + 0x9E3779B97F4A7C15ull * (owner + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned long long ps_owner(uint32_t res, int32_t idx) {
    return ((unsigned long long)(res + 1) << 32) | (unsigned long long)(uint32_t)(idx + 1);
}

// threadCountMap lookup; create: insert at 0 when absent (putIfAbsent). Returns the slot or -1.
__device__ inline int64_t ps_tc(const PSArgs& s, uint32_t res, int32_t idx, uint64_t v, bool create) {
    const unsigned long long own = ps_owner(res, idx);
    uint64_t h = ps_hash(own, v) & s.tc_mask;
    for (uint64_t probes = 0; probes <= s.tc_mask; ++probes, h = (h + 1) & s.tc_mask) {
        PSThread& e = s.tc[h];
        const unsigned long long o = __hip_atomic_load(&e.owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o == own && e.value == v) return (int64_t)h;
        if (o == 0) {
            if (!create) return -1;
            // claim the slot; only this resource's walker ever reads entries with this owner word — one lane, or
            // one wave whose lanes run the same step (k_lwalk_cxw): a lane of the same wave that lost the claim to
            // another with the same owner claims it with the same value
            const unsigned long long prev = atomicCAS(&e.owner, 0ull, own);
            if (prev == 0ull || prev == own) {
                e.value = v;
                e.count = 0;
                return (int64_t)h;
            }
        }
    }
    if (create) atomicOr(s.err, kErrTableFull);
    return -1;
}

// passSingleValueCheck (:106-125) for rule ri at time t
__device__ inline bool ps_single(const PSArgs& s, uint32_t ri, uint32_t res, int64_t t, int64_t acq, uint64_t v) {
    const PRule r = s.p.rules[ri];
    const int64_t tc = param_token_count(s.p, r, v);  // the hot item's threshold, else (long) count
    if (s.grade[ri] == 1) {
        if (tc == 0) return false;
        if (r.behavior != 2 && acq > tc + r.burst) return false;
        const uint64_t g = param_slot(s.p, r, v);
        if (g == ~0ull) {
            atomicOr(s.err, kErrTableFull);
            return false;
        }
        PSlot& slot = s.p.table[g];
        PState st{slot.time, slot.tokens, slot.flags};
        const bool ok = r.behavior == 2 ? param_throttle_step(st, throttle_cost(r, tc, acq), r.max_queueing_ms, t)
                                        : param_default_step(st, tc, tc + r.burst, r.duration_sec * 1000, t, acq);
        slot.time = st.time;
        slot.tokens = st.tokens;
        slot.flags = st.flags;
        return ok;
    }
    if (s.grade[ri] == 0) {
        const int64_t e = ps_tc(s, res, s.cur_idx[ri], v, false);
        const int64_t threads = e >= 0 ? s.tc[e].count : 0;
        return threads + 1 <= tc;
    }
    return true;
}

// addThreadCount / decreaseThreadCount (ParameterMetric.java:184-239) over the argument indices that have a thread
// map (a rule of the resource with that paramIdx ran initParamMetricsFor); args[arg_begin .. + arg_count)
__device__ inline void ps_threads(const PSArgs& s, uint32_t res, uint32_t arg_begin, uint32_t arg_count, int d) {
    const uint32_t rb = s.res_begin[res], re = s.res_begin[res + 1];
    for (uint32_t idx = 0; idx < arg_count; ++idx) {
        bool has_map = false;
        for (uint32_t k = rb; k < re && !has_map; ++k) {
            const uint32_t ri = s.res_rules[k];
            has_map = s.inited[ri] && s.cur_idx[ri] == (int32_t)idx;
        }
        if (!has_map) continue;
        const sg_pslot_arg a = s.args[arg_begin + idx];
        if (a.kind == SG_ARG_NULL) continue;
        const uint32_t m = a.kind == SG_ARG_COLLECTION ? a.value_count : 1u;
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t v = s.values[a.value_begin + j];
            if (d > 0) {
                const int64_t x = ps_tc(s, res, (int32_t)idx, v, true);
                if (x >= 0) s.tc[x].count += 1;
            } else {
                const int64_t x = ps_tc(s, res, (int32_t)idx, v, false);
                if (x >= 0) s.tc[x].count = s.tc[x].count > 0 ? s.tc[x].count - 1 : 0;  // <= 0: removed (reads 0)
                else ps_tc(s, res, (int32_t)idx, v, true);                             // putIfAbsent(0)
            }
        }
    }
}

// RequestLimiter.tryPass (RequestLimiter.java:72-87) over the namespace's UnaryLeapArray(10, 1000) at time t.
__device__ inline bool emb_lim_try_pass(LimRing* r, int64_t t, double qps) {
    const int64_t P = t / kLimWindowMs;
    const int I = (int)(P % kLimSamples);
    const int64_t ws = P * kLimWindowMs;
    if (r->start[I] != ws) {  // currentWindow: create or reset (time-ordered: never an older window)
        r->start[I] = ws;
        r->count[I] = 0;
    }
    const int64_t lo = ws - (int64_t)(kLimSamples - 1) * kLimWindowMs;
    int64_t sum = 0;
    for (int j = 0; j < kLimSamples; ++j)
        if (r->start[j] != INT64_MIN && r->start[j] >= lo) sum += r->count[j];
    if (!((double)sum + 1 <= qps)) return false;  // getQps() + 1 <= qpsAllowed (intervalInSecond 1.0)
    r->count[I] += 1;
    return true;
}

// DefaultTokenService.requestParamToken (DefaultTokenService.java:53-64) → ClusterParamFlowChecker.acquireClusterToken
// (ClusterParamFlowChecker.java:42-87) on the embedded token server, for one request of the m values vals at time t: the
// namespace limiter (allowProceed), every value checked on its window (the first failure blocks and adds nothing), then
// the count added to every value (addValue: currentWindow resets a stale bucket). One lane walks all requests that
// share the rule's metric or limiter (key groups), in event order.
__device__ inline int32_t ps_emb_param_token(const PSArgs& s, uint32_t key, int64_t t, int32_t acq, const uint64_t* vals,
                                             uint32_t m) {
    const CPArgs& c = s.cp;
    key &= SG_KEY_INDEX;
    if (key == SG_KEY_BAD || acq <= 0 || m == 0) return SG_STATUS_BAD_REQUEST;  // notValidRequest, params.isEmpty()
    if (key >= c.n_rules) return SG_STATUS_NO_RULE_EXISTS;                      // getParamRuleById == null
    const uint8_t ls = s.cp_rule_lim ? s.cp_rule_lim[key] : (uint8_t)0xFF;
    if (ls != 0xFF && !emb_lim_try_pass(s.lim_ring + ls, t, s.lim_qps[ls])) return SG_STATUS_TOO_MANY_REQUEST;
    const CPRule r = c.rules[key];
    const int64_t P = t / r.wl;
    for (uint32_t j = 0; j < m; ++j) {  // getAvg(value): the value's window sum at t / intervalInSecond
        const uint64_t g = cp_find(c, r, vals[j]);
        int64_t cur = 0;
        const int64_t other = g != ~0ull ? cp_window(c.ring + g * (uint64_t)c.stride, r.S, r.wl, P, &cur) : 0;
        const double rem = cp_threshold(c, r, vals[j]) - avg_div((double)(other + cur), r.isec) - (double)acq;
        if (rem < 0) return SG_STATUS_BLOCKED;
    }
    const int I = (int)(P % r.S);
    const int64_t ws = P * r.wl;
    for (uint32_t j = 0; j < m; ++j) {  // addValue(value, count) on currentWindow
        const uint64_t g = cp_slot(c, r, vals[j]);
        if (g == ~0ull) {
            atomicOr(s.err, kErrTableFull);
            return SG_STATUS_FAIL;
        }
        CPBucket& b = c.ring[g * (uint64_t)c.stride + I];
        if (b.start != ws) {
            b.start = ws;
            b.count = 0;
        }
        b.count += acq;
    }
    return SG_STATUS_OK;
}

// ParamFlowChecker.passLocalCheck (:78-103) of rule ri on argument a: every value in order, the first failing one blocks
__device__ inline bool ps_local(const PSArgs& s, uint32_t ri, uint32_t res, int64_t t, int64_t acq, const sg_pslot_arg& a) {
    const uint32_t m = a.kind == SG_ARG_COLLECTION ? a.value_count : 1u;
    for (uint32_t j = 0; j < m; ++j)
        if (!ps_single(s, ri, res, t, acq, s.values[a.value_begin + j])) return false;
    return true;
}

// ParamFlowSlot.checkFlow (ParamFlowSlot.java:66-93) for one entry of resource res with non-null args: every rule
// of the resource in load order — applyRealParamIdx, initParamMetricsFor, passCheck on args[paramIdx] (a collection /
// array element by element, the state changes before a failing element kept). Returns the index of the rule that
// throws ParamFlowException, or -1 when every rule passes.
__device__ inline int32_t ps_check_entry(const PSArgs& s, uint32_t res, int64_t t, int32_t count, uint32_t arg_begin,
                                         uint32_t arg_count) {
    const uint32_t rb = s.res_begin[res], re = s.res_begin[res + 1];
    for (uint32_t k = rb; k < re; ++k) {
        const uint32_t ri = s.res_rules[k];
        int32_t idx = s.cur_idx[ri];
        if (idx < 0) {  // applyRealParamIdx(rule, args.length)
            idx = (-idx <= (int32_t)arg_count) ? (int32_t)arg_count + idx : -idx;
            s.cur_idx[ri] = idx;
        }
        s.inited[ri] = 1;
        if ((int32_t)arg_count <= idx) continue;
        const sg_pslot_arg a = s.args[arg_begin + (uint32_t)idx];
        if (a.kind == SG_ARG_NULL) continue;
        const int32_t cm = s.cmode ? s.cmode[ri] : SG_CLUSTER_MODE_OFF;
        if (cm != SG_CLUSTER_MODE_OFF && s.grade[ri] == 1) {  // passClusterCheck (:278-303)
            if (s.emb) {
                const uint32_t m = a.kind == SG_ARG_COLLECTION ? a.value_count : 1u;
                const int32_t st = ps_emb_param_token(s, s.ckey[ri], t, count, s.values + a.value_begin, m);
                if (st == SG_STATUS_OK) continue;
                if (st == SG_STATUS_BLOCKED) return (int32_t)ri;
            }
            // no token service, or NO_RULE_EXISTS / BAD_REQUEST / TOO_MANY_REQUEST: fallbackToLocalOrPass (:305-313)
            if (cm == SG_CLUSTER_MODE_NO_FALLBACK) continue;
        }
        if (!ps_local(s, ri, res, t, (int64_t)count, a)) return (int32_t)ri;
    }
    return -1;
}

}  // namespace sg
