// cparam.hip — cluster hot-parameter tokens on the device: TokenService.requestParamToken →
// DefaultTokenService (srv/flow/DefaultTokenService.java:53-64) → ClusterParamFlowChecker.acquireClusterToken
// (srv/flow/ClusterParamFlowChecker.java:42-87) over each flowId's ClusterParamMetric
// (srv/flow/statistic/metric/ClusterParamMetric.java, ClusterParameterLeapArray.java).
//
// The reference keeps one LeapArray per flowId whose buckets are value → count maps, cleared when the
// bucket is reset. A value's window sum is therefore the sum of its own adds over the last sampleCount
// window periods: bucket resets caused by other values' requests only ever clear counts of periods that
// have left the window (a bucket holds the adds of the flow's latest touched period with its index, and
// a value's adds in period p imply the flow was touched in p). So each (rule, value) is an independent
// ring of S {period start, count} — an exact open-addressing sub-table per rule in HBM, as for the local
// hot-parameter path (param.hip) — and single-value requests are independent per (rule, value):
//   k_cp_prep   validation (BAD_REQUEST / NO_RULE_EXISTS), find-or-insert of (rule, value), packed record
//               {slot | request index}; results start as BLOCKED.
//   radix sort by slot (sort.hip), then k_seg (engine.hip) + k_cp_walk: one lane per (rule, value)
//               segment, sequential replay (window sum, threshold - avg - count >= 0, add).
// A request with several values is all-or-nothing across its values: the host driver (api.cpp) cuts the
// batch at such requests and decides each of them alone (k_cp_multi) between the single-value runs.
#include "engine.h"

namespace sg {

namespace {

constexpr uint64_t kCpEmpty = ~0ull;

__device__ __forceinline__ int32_t cp_d2i(double x) {  // JLS §5.1.3
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

__device__ __forceinline__ void cp_store(sg_result* out, uint64_t i, int32_t st, int32_t rem) {
    sg_result r;
    r.status = st;
    r.remaining = rem;
    r.wait_ms = 0;
    out[i] = r;
}

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
        const unsigned long long cur = __hip_atomic_load(vw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    uint32_t lo = 0, hi = c.n_rules;  // rules by table_base
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (c.rules[mid].table_base <= g) lo = mid;
        else hi = mid;
    }
    return lo;
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

}  // namespace

__global__ void __launch_bounds__(256) k_cp_prep(CPArgs c, uint64_t lo, uint64_t hi, uint64_t sentinel) {
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_cparam_req q = c.req[i];
        if (q.ts_ms < 0 || (i == 0 ? q.ts_ms < *c.last_ts : q.ts_ms < c.req[i - 1].ts_ms)) atomicOr(c.err, kErrTime);
        const uint32_t key = q.key & SG_KEY_INDEX;
        uint64_t rec = sentinel;
        if (key == SG_KEY_BAD || q.acquire <= 0 || q.value_count == 0) {
            cp_store(c.out, i, SG_STATUS_BAD_REQUEST, 0);
        } else if (key >= c.n_rules) {
            cp_store(c.out, i, SG_STATUS_NO_RULE_EXISTS, 0);
        } else {
            cp_store(c.out, i, SG_STATUS_BLOCKED, 0);  // the walkers write the passes
            if ((uint64_t)q.value_begin + q.value_count > c.n_values) {
                atomicOr(c.err, kErrBounds);
            } else if (q.value_count == 1) {  // (several values: decided alone by k_cp_multi)
                const uint64_t g = cp_slot(c, c.rules[key], c.values[q.value_begin]);
                if (g == ~0ull) atomicOr(c.err, kErrTableFull);
                else rec = (g << c.ibits) | (i - lo);
            }
        }
        c.rec[i - lo] = rec;
    }
}

// One lane per (rule, value) segment of the sorted records of [lo, hi).
__global__ void __launch_bounds__(256) k_cp_walk(CPArgs c, BatchArgs sg, uint64_t lo) {
    if (*c.err) return;
    const int lane = (int)__lane_id();
    uint32_t cnt[kClasses], grp_end[kClasses];
    uint32_t total = 0;
    for (int k = kClasses - 1; k >= 0; --k) {
        cnt[k] = sg.short_count[k];
        total += (cnt[k] + 63) / 64;
        grp_end[k] = total;
    }
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t gi = wave; gi < total; gi += nwaves) {
        int cl = kClasses - 1;
        uint32_t g0 = 0;
        while (gi >= grp_end[cl]) {
            g0 = grp_end[cl];
            --cl;
        }
        const uint32_t i = (gi - g0) * 64 + (uint32_t)lane;
        if (i >= cnt[cl]) continue;
        uint64_t j = sg.short_list[sg.class_off[cl] + i];
        const uint64_t g = sg.rec_sorted[j] >> c.ibits;
        const CPRule r = c.rules[cp_rule_of_slot(c, g)];
        const double thr = cp_threshold(c, r, c.keys[g]);  // the side slot's key stays ~0, its value
        CPBucket* ring = c.ring + g * (uint64_t)c.stride;
        const int S = r.S;
        const int64_t wl = r.wl;
        int64_t P = INT64_MIN, other = 0, cur = 0;
        for (; j < sg.n; ++j) {
            const uint64_t rec = sg.rec_sorted[j];
            if ((rec >> c.ibits) != g) break;
            const uint64_t idx = lo + (rec & c.imask);
            const sg_cparam_req q = c.req[idx];
            const int64_t Pq = q.ts_ms / wl;
            if (Pq != P) {  // currentWindow(t): close the open period, open this one
                if (P != INT64_MIN) {
                    CPBucket b;
                    b.start = P * wl;
                    b.count = cur;
                    ring[(int)(P % S)] = b;
                }
                P = Pq;
                other = cp_window(ring, S, wl, P, &cur);
            }
            // ClusterParamFlowChecker.java:62-70: threshold - getAvg(value) - count
            const double latest = (double)(other + cur) / r.isec;
            const double rem = thr - latest - (double)q.acquire;
            if (rem >= 0) {
                cur += q.acquire;  // addValue
                cp_store(c.out, idx, SG_STATUS_OK, cp_d2i(rem));
            }
        }
        if (P != INT64_MIN) {
            CPBucket b;
            b.start = P * wl;
            b.count = cur;
            ring[(int)(P % S)] = b;
        }
    }
}

// One request with several values (index m), all-or-nothing (ClusterParamFlowChecker.java:58-80).
__global__ void k_cp_multi(CPArgs c, uint64_t m) {
    if (*c.err) return;
    const sg_cparam_req q = c.req[m];
    if (q.ts_ms < 0 || (m == 0 ? q.ts_ms < *c.last_ts : q.ts_ms < c.req[m - 1].ts_ms)) {
        atomicOr(c.err, kErrTime);
        return;
    }
    const uint32_t key = q.key & SG_KEY_INDEX;
    if (key == SG_KEY_BAD || q.acquire <= 0 || q.value_count == 0) {
        cp_store(c.out, m, SG_STATUS_BAD_REQUEST, 0);
        return;
    }
    if (key >= c.n_rules) {
        cp_store(c.out, m, SG_STATUS_NO_RULE_EXISTS, 0);
        return;
    }
    if ((uint64_t)q.value_begin + q.value_count > c.n_values) {
        atomicOr(c.err, kErrBounds);
        return;
    }
    const CPRule r = c.rules[key];
    const int64_t P = q.ts_ms / r.wl;
    bool passed = true;
    for (uint32_t v = 0; v < q.value_count && passed; ++v) {
        const uint64_t value = c.values[q.value_begin + v];
        const uint64_t g = cp_slot(c, r, value);
        if (g == ~0ull) {
            atomicOr(c.err, kErrTableFull);
            return;
        }
        int64_t cur = 0;
        const int64_t other = cp_window(c.ring + g * (uint64_t)c.stride, r.S, r.wl, P, &cur);
        const double rem = cp_threshold(c, r, value) - (double)(other + cur) / r.isec - (double)q.acquire;
        passed = rem >= 0;
    }
    if (passed) {
        for (uint32_t v = 0; v < q.value_count; ++v) {  // addValue for every value (duplicates add twice)
            const uint64_t g = cp_slot(c, r, c.values[q.value_begin + v]);
            CPBucket* ring = c.ring + g * (uint64_t)c.stride;
            CPBucket& b = ring[(int)(P % r.S)];
            if (b.start != P * r.wl) {
                b.start = P * r.wl;
                b.count = 0;
            }
            b.count += q.acquire;
        }
    }
    cp_store(c.out, m, passed ? SG_STATUS_OK : SG_STATUS_BLOCKED, passed ? -1 : 0);
}

__global__ void k_cp_finish(CPArgs c, uint64_t last) {
    if (*c.err == 0) *c.last_ts = c.req[last].ts_ms;
}

__global__ void __launch_bounds__(256) k_cp_count_multi(CPArgs c, uint32_t* list, uint32_t* count) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x)
        if (c.req[i].value_count > 1 && (c.req[i].key & SG_KEY_INDEX) < c.n_rules) list[atomicAdd(count, 1u)] = (uint32_t)i;
}

__global__ void __launch_bounds__(256) k_cp_clear(uint64_t* keys, CPBucket* ring, uint64_t slots, int stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots * stride; i += (uint64_t)gridDim.x * blockDim.x) {
        CPBucket b;
        b.start = INT64_MIN;
        b.count = 0;
        ring[i] = b;
        if (i % stride == 0) keys[i / stride] = kCpEmpty;
    }
}

// A surviving flowId's sub-table moved into a reloaded table (ClusterParamMetricStatistics keeps its
// metric, putMetricIfAbsent): keys and the first S buckets of every slot.
__global__ void __launch_bounds__(256) k_cp_copy(const uint64_t* okeys, const CPBucket* oring, uint64_t obase, int ostride,
                                                 uint64_t* nkeys, CPBucket* nring, uint64_t nbase, int nstride,
                                                 uint64_t slots, int S) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots * S; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t sl = i / S;
        const int j = (int)(i % S);
        nring[(nbase + sl) * nstride + j] = oring[(obase + sl) * ostride + j];
        if (j == 0) nkeys[nbase + sl] = okeys[obase + sl];
    }
}

// ClusterParamMetric.getSum(value) of a rule at `now`, without the currentWindow side effect.
__global__ void k_cp_read(CPArgs c, uint32_t rule, uint64_t value, int64_t now, int64_t* out) {
    const CPRule r = c.rules[rule];
    uint64_t g = ~0ull;
    if (value == kCpEmpty) {
        g = r.table_base + r.table_mask + 1;
    } else {
        for (uint64_t i = 0; i <= r.table_mask; ++i)
            if (c.keys[r.table_base + i] == value) {
                g = r.table_base + i;
                break;
            }
    }
    int64_t cur = 0, other = 0;
    if (g != ~0ull) other = cp_window(c.ring + g * (uint64_t)c.stride, r.S, r.wl, now / r.wl, &cur);
    *out = other + cur;
}

// ClusterParamMetric.getTopValues: every (rule, value) with a positive window sum at now, appended in any order
// (the host picks each rule's top entries). per = slots per rule (all rules share one table size).
__global__ void __launch_bounds__(256) k_cp_top(CPArgs c, int64_t now, uint64_t per, CPTop* out,
                                                unsigned long long* count) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < c.total_slots;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t rule = (uint32_t)(g / per);
        const CPRule r = c.rules[rule];
        const bool side = g == r.table_base + r.table_mask + 1;  // the slot of the value ~0
        const uint64_t v = side ? kCpEmpty : c.keys[g];
        if (!side && v == kCpEmpty) continue;
        int64_t cur = 0;
        const int64_t sum = cp_window(c.ring + g * (uint64_t)c.stride, r.S, r.wl, now / r.wl, &cur) + cur;
        if (sum <= 0) continue;
        CPTop t;
        t.value = v;
        t.sum = sum;
        t.rule = rule;
        t.pad = 0;
        out[atomicAdd(count, 1ull)] = t;
    }
}

static unsigned cgrid(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

hipError_t launch_cp_clear(uint64_t* keys, CPBucket* ring, uint64_t slots, int stride, hipStream_t stream) {
    if (slots == 0) return hipSuccess;
    hipLaunchKernelGGL(k_cp_clear, dim3(cgrid(slots * stride, 8192)), dim3(256), 0, stream, keys, ring, slots, stride);
    return hipGetLastError();
}

hipError_t launch_cp_copy(const uint64_t* okeys, const CPBucket* oring, uint64_t obase, int ostride, uint64_t* nkeys,
                          CPBucket* nring, uint64_t nbase, int nstride, uint64_t slots, int S, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_copy, dim3(cgrid(slots * S, 8192)), dim3(256), 0, stream, okeys, oring, obase, ostride, nkeys,
                       nring, nbase, nstride, slots, S);
    return hipGetLastError();
}

hipError_t launch_cp_read(const CPArgs& c, uint32_t rule, uint64_t value, int64_t now, int64_t* out_dev, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_read, dim3(1), dim3(1), 0, stream, c, rule, value, now, out_dev);
    return hipGetLastError();
}

hipError_t launch_cp_top(const CPArgs& c, int64_t now, uint64_t per, CPTop* out, unsigned long long* count,
                         hipStream_t stream) {
    if (c.total_slots == 0) return hipSuccess;
    hipLaunchKernelGGL(k_cp_top, dim3(cgrid(c.total_slots, 8192)), dim3(256), 0, stream, c, now, per, out, count);
    return hipGetLastError();
}

hipError_t launch_cp_count_multi(const CPArgs& c, uint32_t* list, uint32_t* count, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_count_multi, dim3(cgrid(c.n, 4096)), dim3(256), 0, stream, c, list, count);
    return hipGetLastError();
}

// Single-value requests of [lo, hi): prep, sort by slot, segments, walk.
hipError_t launch_cp_range(const CPArgs& c, BatchArgs& sg, uint64_t lo, uint64_t hi, uint64_t* a_buf, uint64_t* b_buf,
                           uint32_t* hist, int lo_bit, int hi_bit, hipStream_t stream) {
    const uint64_t n = hi - lo;
    if (n == 0) return hipSuccess;
    const uint64_t sentinel = c.total_slots << c.ibits;
    CPArgs q = c;
    q.rec = a_buf;
    hipLaunchKernelGGL(k_cp_prep, dim3(cgrid(n, 8192)), dim3(256), 0, stream, q, lo, hi, sentinel);
    uint64_t* sorted = nullptr;
    hipError_t e = radix_sort_records(a_buf, b_buf, n, lo_bit, hist, &sorted, stream, hi_bit);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(sg.long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    sg.n = n;
    sg.rec_sorted = sorted;
    e = launch_seg(sg, stream);
    if (e != hipSuccess) return e;
    static unsigned blocks = 0;
    if (blocks == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cp_walk, 256, 0);
        blocks = (unsigned)((cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1));
    }
    hipLaunchKernelGGL(k_cp_walk, dim3(blocks), dim3(256), 0, stream, c, sg, lo);
    hipLaunchKernelGGL(k_cp_finish, dim3(1), dim3(1), 0, stream, c, hi - 1);
    return hipGetLastError();
}

hipError_t launch_cp_multi(const CPArgs& c, uint64_t m, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_multi, dim3(1), dim3(1), 0, stream, c, m);
    hipLaunchKernelGGL(k_cp_finish, dim3(1), dim3(1), 0, stream, c, m);
    return hipGetLastError();
}

}  // namespace sg
