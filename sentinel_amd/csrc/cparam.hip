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
//   k_cp_limprep + launch_limiter (limiter.hip)  allowProceed → GlobalRequestLimiter.tryPass of the rule's
//               namespace (ClusterParamFlowChecker.java:43-45), state shared with the flow-token path;
//   k_cp_prep2  validation (BAD_REQUEST / NO_RULE_EXISTS), find-or-insert of every (rule, value), one packed
//               record {slot | value position} per value;
//   radix sort by slot (sort.hip), k_seg (engine.hip), then k_cp_walk2: one lane per (rule, value) slot,
//               sequential replay (window sum, threshold - avg - count >= 0, add);
//   requests with several values (all-or-nothing over their values) are resolved by the fixed point below.
#include "cparam_dev.h"

namespace sg {

namespace {

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

}  // namespace

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

}  // namespace sg

// ------------------------------------------------------------------- one pipeline, multi-value requests
//
// Every value of every request becomes a record {slot | value position}; value positions increase with the
// request index (sg_cparam_req contract), so a slot's records sorted by position are in arrival order and a
// request's duplicate values are adjacent. A lane walks a slot: single-value requests exactly as k_cp_walk; a
// multi-value request (ClusterParamFlowChecker.java:58-80: every value checked against the pre-request state,
// then all added iff all passed) writes its check for this value and adds its count iff its outcome is assumed to
// be a pass and this check passed (a failing check on the exact state decides the request). k_cp_combine then
// sets each multi-value request's outcome to the AND of its checks and marks for a re-walk only the slots whose
// adds change (those whose check passed). The walk of a slot is exact once the outcomes of the earlier
// multi-value requests touching it are, so re-walking from the saved pre-batch rings until no outcome changes
// converges to the sequential answer (any consistent assignment is it: by induction over the requests in
// arrival order, each one's checks see exact states); with the assumption "passes" most batches need one or two
// rounds, and a saturated hot slot, whose checks fail, is not re-walked for the outcomes it already decided.
// When the rounds run out, the slots linked by multi-value requests are replayed per connected group (k_cpfb_*).

namespace sg {

namespace {

constexpr uint32_t kNoOwner = 0xFFFFFFFFu;

__device__ __forceinline__ bool cp_valid(const CPArgs& c, const sg_cparam_req& q) {
    const uint32_t key = q.key & SG_KEY_INDEX;
    return !(key == SG_KEY_BAD || q.acquire <= 0 || q.value_count == 0) && key < c.n_rules;
}

constexpr uint32_t kCpAesc = 127;  // acquire code: read req[i].acquire

// A value record, decoded (CPBatch::rec): the request, the value position (multi-value requests), the count.
struct CPRec {
    uint32_t i;
    uint64_t p;
    bool multi;
    int64_t acq;
};

__device__ __forceinline__ CPRec cp_dec(const CPArgs& c, const CPBatch& b, uint64_t rec) {
    CPRec d;
    const uint64_t pl = rec & b.pmask;
    d.multi = ((pl >> (b.pbits - 1)) & 1ull) != 0;
    const uint32_t ac = (uint32_t)(pl >> b.idbits) & 127u;
    d.p = pl & b.idmask;
    d.i = d.multi ? b.owner[d.p] : (uint32_t)d.p;
    d.acq = ac == kCpAesc ? (int64_t)c.req[d.i].acquire : (int64_t)ac;
    return d;
}

}  // namespace

// The batch's period tables (first request index of every window period, per distinct window length of the rules)
// staged in LDS when they fit, else read from b.bnd: a value record's window period is a function of its request
// index (requests are time-ordered), so the walkers never read a request's timestamp.
constexpr int kCpLdsBnd = 2048;
__shared__ uint32_t cp_sbnd[kCpLdsBnd];
__shared__ uint32_t cp_boff[kMaxWl];
__shared__ int cp_blds;
__shared__ int64_t cp_p0[kMaxWl];
__shared__ uint32_t cp_np[kMaxWl];

__device__ __forceinline__ void cp_stage_periods(const CPBatch& b) {
    uint32_t tot = 0;
    for (int w = 0; w < b.n_wl; ++w) tot += b.np[w];
    const bool lds = tot <= (uint32_t)kCpLdsBnd;
    uint32_t off = 0;
    for (int w = 0; w < b.n_wl; ++w) {
        const uint32_t npw = b.np[w];
        if (lds) {
            const uint32_t* g = b.bnd + (size_t)w * kMaxPeriods;
            for (uint32_t x = threadIdx.x; x < npw; x += blockDim.x) cp_sbnd[off + x] = g[x];
        }
        if (threadIdx.x == 0) cp_boff[w] = off;
        off += npw;
    }
    if (threadIdx.x == 0) cp_blds = lds ? 1 : 0;
    if (threadIdx.x < (unsigned)b.n_wl) {
        cp_p0[threadIdx.x] = b.p0[threadIdx.x];
        cp_np[threadIdx.x] = b.np[threadIdx.x];
    }
    __syncthreads();
}

// window period (absolute) of request i for window length w: the largest q with table[q] <= i (entry 0 unused)
__device__ __forceinline__ int64_t cp_period(const CPBatch& b, int w, uint32_t i) {
    uint32_t lo = 0, hi = cp_np[w];
    if (cp_blds) {
        const uint32_t* t = cp_sbnd + cp_boff[w];
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (t[mid] <= i) lo = mid;
            else hi = mid;
        }
    } else {
        const uint32_t* t = b.bnd + (size_t)w * kMaxPeriods;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (t[mid] <= i) lo = mid;
            else hi = mid;
        }
    }
    return cp_p0[w] + (int64_t)lo;
}

// The 100 ms limiter periods of the batch (row 0 of the period table) and {cparam rule | request} records of the
// valid requests; runs after k_cp_prep2, and the limiter then overwrites the refused requests' results with
// TOO_MANY_REQUEST (the walkers skip them).
__global__ void __launch_bounds__(256) k_cp_limprep(CPArgs c, BatchArgs a) {
    const int64_t t0 = c.req[0].ts_ms;
    const uint64_t sentinel = (uint64_t)a.K << a.kshift;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_cparam_req q = c.req[i];
        const int64_t t = q.ts_ms;
        if (i == 0) {
            a.p0[0] = t / 100;
        } else {
            const int64_t tp = c.req[i - 1].ts_ms;
            if (t > tp && tp >= 0) {
                for (int64_t p = tp / 100 + 1; p <= t / 100; ++p) {
                    const int64_t qq = p - t0 / 100;
                    if (qq >= (int64_t)kMaxPeriods) {
                        atomicOr(c.err, kErrPeriods);
                        break;
                    }
                    if (qq > 0) a.bnd[qq] = (uint32_t)i;
                }
            }
        }
        if (i == c.n - 1) {
            const int64_t qq = t / 100 - t0 / 100 + 1;
            a.np[0] = qq > (int64_t)kMaxPeriods ? kMaxPeriods : qq < 1 ? 1u : (uint32_t)qq;  // < 1: out of order
        }
        a.rec[i] = cp_valid(c, q) ? (((uint64_t)(q.key & SG_KEY_INDEX) << a.kshift) | i) : sentinel;
    }
}

__global__ void __launch_bounds__(256) k_cp_recinit(CPBatch b, uint64_t n_values, uint64_t sentinel) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_values; p += (uint64_t)gridDim.x * blockDim.x) {
        b.rec[p] = sentinel | p;
        b.owner[p] = kNoOwner;
        b.chk[p] = 0;
    }
}

__global__ void __launch_bounds__(256) k_cp_prep2(CPArgs c, CPBatch b) {
    const int64_t t0 = c.req[0].ts_ms;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_cparam_req q = c.req[i];
        const int64_t t = q.ts_ms;
        // timestamps, and the window-period tables (as k_prep: a new period can only start at a new timestamp)
        if (i == 0) {
            if (t < 0 || t < *c.last_ts) atomicOr(c.err, kErrTime);
            for (int w = 0; w < b.n_wl; ++w) b.p0[w] = t / b.wl[w];
        } else {
            const int64_t tp = c.req[i - 1].ts_ms;
            if (t < tp || t < 0) {
                atomicOr(c.err, kErrTime);
            } else if (t != tp) {
                for (int w = 0; w < b.n_wl; ++w) {
                    const int64_t wl = b.wl[w];
                    const int64_t P0 = t0 / wl;
                    for (int64_t pp = tp / wl + 1; pp <= t / wl; ++pp) {
                        const int64_t qq = pp - P0;
                        if (qq <= 0) continue;
                        if (qq >= (int64_t)kMaxPeriods) {
                            atomicOr(c.err, kErrPeriods);
                            break;
                        }
                        b.bnd[(size_t)w * kMaxPeriods + qq] = (uint32_t)i;
                    }
                }
            }
        }
        if (i == c.n - 1) {
            for (int w = 0; w < b.n_wl; ++w) {
                const int64_t qq = t / b.wl[w] - t0 / b.wl[w] + 1;
                b.np[w] = qq > (int64_t)kMaxPeriods ? kMaxPeriods : qq < 1 ? 1u : (uint32_t)qq;
            }
        }
        const uint32_t key = q.key & SG_KEY_INDEX;
        b.assume[i] = 1;
        if (key == SG_KEY_BAD || q.acquire <= 0 || q.value_count == 0) {
            cp_store(c.out, i, SG_STATUS_BAD_REQUEST, 0);
            continue;
        }
        if (key >= c.n_rules) {
            cp_store(c.out, i, SG_STATUS_NO_RULE_EXISTS, 0);
            continue;
        }
        cp_store(c.out, i, SG_STATUS_BLOCKED, 0);
        if ((uint64_t)q.value_begin + q.value_count > c.n_values) {
            atomicOr(c.err, kErrBounds);
            continue;
        }
        if (q.value_count > 1) {
            *b.changed = 1;    // vector store; the host reads it as "has multi-value requests"
            b.assume[i] = 3;   // assumed to pass, listed by k_cp_mlist
        }
        const CPRule r = c.rules[key];
        for (uint32_t j = 0; j < q.value_count; ++j) {
            const uint64_t p = (uint64_t)q.value_begin + j;
            if (atomicCAS(&b.owner[p], kNoOwner, (uint32_t)i) != kNoOwner) {  // value ranges must not overlap
                atomicOr(c.err, kErrBounds);
                continue;
            }
            const uint64_t g = cp_slot(c, r, c.values[p]);
            if (g == ~0ull) {
                atomicOr(c.err, kErrTableFull);
            } else {
                const uint64_t ac = q.acquire >= (int32_t)kCpAesc ? kCpAesc : (uint64_t)q.acquire;
                const uint64_t pl = q.value_count > 1 ? ((1ull << (b.pbits - 1)) | (ac << b.idbits) | p)
                                                      : ((ac << b.idbits) | i);
                b.rec[p] = (g << b.pbits) | pl;
                b.pslot[p] = (uint32_t)g;
            }
        }
    }
}

// Block-aggregated list appends: each thread holds kAggItems candidates; a block scan of the (two 16-bit packed)
// per-thread counts and one atomic per block and list (one per wave on a single counter serialised at ~10 ns each:
// 2.8 ms for a 16M-request batch).
constexpr int kAggItems = 16;

__device__ __forceinline__ uint32_t cp_block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t off = x - v, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) off += wsum[w];
        tot += wsum[w];
    }
    *total = tot;
    return off;
}

// The valid multi-value requests (k_cp_prep2 flagged them in assume[], bit 1): k_cp_combine's work list (any order).
// A thread reads the flag bytes of kAggItems consecutive requests at once.
__global__ void __launch_bounds__(256) k_cp_mlist(CPArgs c, CPBatch b) {
    __shared__ uint32_t wsum[4], gbase;
    const uint64_t i0 = (uint64_t)blockIdx.x * (256 * kAggItems) + (uint64_t)threadIdx.x * kAggItems;
    static_assert(kAggItems == 16, "one 16-byte load of flags per thread");
    uint32_t m = 0;
    if (i0 + kAggItems <= c.n) {
        const uint4 v = *(const uint4*)(b.assume + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < kAggItems; ++u) m |= ((w[u >> 2] >> (8 * (u & 3) + 1)) & 1u) << u;
    } else {
        for (int u = 0; u < kAggItems && i0 + u < c.n; ++u) m |= ((b.assume[i0 + u] >> 1) & 1u) << u;
    }
    uint32_t tot;
    uint32_t off = cp_block_excl_scan((uint32_t)__builtin_popcount(m), wsum, &tot);
    if (threadIdx.x == 0) gbase = tot ? atomicAdd(b.mcount, tot) : 0u;
    __syncthreads();
    off += gbase;
    while (m) {
        const int u = __builtin_ctz(m);
        m &= m - 1;
        b.mlist[off++] = (uint32_t)(i0 + (uint64_t)u);
    }
}

// Within a slot, value positions (the sort order) must follow the request order: the walk replays them in that
// order. Checked on the sorted records, before anything is charged.
__global__ void __launch_bounds__(256) k_cp_order(CPArgs c, CPBatch b, const uint64_t* sorted, uint64_t n) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r0 = sorted[j - 1], r1 = sorted[j];
        if ((r0 >> b.pbits) != (r1 >> b.pbits) || (r1 >> b.pbits) >= c.total_slots) continue;
        const uint32_t a0 = cp_dec(c, b, r0).i, a1 = cp_dec(c, b, r1).i;
        if (a1 < a0) atomicOr(c.err, kErrBounds);
    }
}

// Slot prologue of a walk: round 0 saves the pre-batch ring (when re-walks may follow); later rounds walk only the
// work items k_cp_combine listed (their flag set) and restore their rings first. `x0`/`dx` spread the bucket copies
// over the caller's lanes.
__device__ __forceinline__ bool cp_prologue(const CPArgs& c, const CPBatch& b, uint64_t g, uint64_t t, int x0, int dx) {
    CPBucket* ring = c.ring + g * (uint64_t)c.stride;
    CPBucket* sv = b.save + t * (uint64_t)c.stride;
    if (b.round > 0) {
        if (!b.dflag[t]) return false;
        for (int x = x0; x < c.stride; x += dx) ring[x] = sv[x];
        if (x0 == 0) b.dflag[t] = 0;
    } else if (b.save) {
        for (int x = x0; x < c.stride; x += dx) sv[x] = ring[x];
    }
    return true;
}

// Sequential replay of the records [j, ...) of slot g (one lane). Single-value requests: window check and add.
// A multi-value request's records in this slot (repeated values) check the state before the request, and add
// its count each iff its outcome is assumed to be a pass and the check passed. Needs cp_stage_periods.
__device__ void cp_walk_serial_mem(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t g, uint64_t j,
                                   const CPRule& r) {
    const double thr = cp_threshold(c, r, c.keys[g]);
    CPBucket* ring = c.ring + g * (uint64_t)c.stride;
    const int S = r.S;
    const int64_t wl = r.wl;
    int64_t P = INT64_MIN, other = 0, cur = 0;
    uint32_t qn = 0xFFFFFFFFu;  // first request index of the period after P (monotone cursor)
    uint32_t mi = kNoOwner;     // the multi-value request of the previous record, and its check here
    bool mok = false;
    uint64_t rec = sg.rec_sorted[j];
    while ((rec >> b.pbits) == g) {
        const uint64_t nrec = j + 1 < sg.n ? sg.rec_sorted[j + 1] : ~0ull;  // issued before this record is decided
        const CPRec d = cp_dec(c, b, rec);
        const uint32_t i = d.i;
        rec = nrec;
        ++j;
        if (b.lim && c.out[i].status == SG_STATUS_TOO_MANY_REQUEST) continue;  // allowProceed refused it
        if (d.multi && i == mi) {  // a repeated value: the check of the request's first record here, and its add
            b.chk[d.p] = mok ? 1 : 0;
            if (b.assume[i] && mok) cur += d.acq;
            continue;
        }
        if (P == INT64_MIN || i >= qn) {  // currentWindow(t): close the open period, open this one
            const int64_t Pq = cp_period(b, r.wl_idx, i);
            if (P != INT64_MIN) {
                CPBucket bk;
                bk.start = P * wl;
                bk.count = cur;
                ring[(int)(P % S)] = bk;
            }
            P = Pq;
            other = cp_window(ring, S, wl, P, &cur);
            const uint32_t q1 = (uint32_t)(P - cp_p0[r.wl_idx]) + 1;
            qn = q1 < cp_np[r.wl_idx] ? (cp_blds ? cp_sbnd[cp_boff[r.wl_idx] + q1]
                                                  : b.bnd[(size_t)r.wl_idx * kMaxPeriods + q1])
                                      : 0xFFFFFFFFu;
        }
        const double rem = thr - avg_div((double)(other + cur), r.isec) - (double)d.acq;
        if (!d.multi) {
            mi = kNoOwner;
            if (rem >= 0) {
                cur += d.acq;
                cp_store(c.out, i, SG_STATUS_OK, cp_d2i(rem));
            } else if (b.round > 0) {  // round 0: BLOCKED is k_cp_prep2's default already
                cp_store(c.out, i, SG_STATUS_BLOCKED, 0);
            }
            continue;
        }
        // a multi-value request's first record here: its check on the pre-request state; it adds (and so do its
        // repeated values after it) iff the request is assumed to pass and the check passed
        mi = i;
        mok = rem >= 0;
        b.chk[d.p] = mok ? 1 : 0;
        if (b.assume[i] && mok) cur += d.acq;
    }
    if (P != INT64_MIN) {
        CPBucket bk;
        bk.start = P * wl;
        bk.count = cur;
        ring[(int)(P % S)] = bk;
    }
}

// cp_walk_serial with the slot's ring in registers (sampleCount <= SM): the ring is read once, with all loads issued
// together, and the changed buckets are written back at the end — the memory version reads S buckets at every
// window-period change, a dependent round trip per period of a slot's records.
//
// save_t >= 0 (round 0 of the lane walker): the pre-batch ring goes to save slot save_t only if the slot holds a
// multi-value record — only such slots are ever restored (re-walks and the fallback groups follow multi-value
// requests) — copied at the end of the walk, before the changed buckets are written back.
template <int SM>
__device__ void cp_walk_serial_reg(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t g, uint64_t j,
                                   const CPRule& r, int64_t save_t = -1) {
    const double thr = cp_threshold(c, r, c.keys[g]);
    CPBucket* ring = c.ring + g * (uint64_t)c.stride;
    const int S = r.S;
    const int64_t wl = r.wl;
    int64_t bs[SM], bc[SM];
#pragma unroll
    for (int x = 0; x < SM; ++x) {
        const CPBucket bk = ring[x < S ? x : 0];
        bs[x] = x < S ? bk.start : INT64_MIN;
        bc[x] = bk.count;
    }
    uint32_t dirty = 0;
    int64_t P = INT64_MIN, other = 0, cur = 0;
    uint32_t qn = 0xFFFFFFFFu;  // first request index of the period after P (monotone cursor)
    uint32_t mi = kNoOwner;     // the multi-value request of the previous record, and its check here
    bool mok = false;
    bool any_multi = false;
    auto close = [&]() {  // the open period's bucket into the register ring
        if (P == INT64_MIN) return;
        const int xo = (int)(P % S);
#pragma unroll
        for (int x = 0; x < SM; ++x) {
            if (x == xo) {
                bs[x] = P * wl;
                bc[x] = cur;
            }
        }
        dirty |= 1u << xo;
    };
    uint64_t rec = sg.rec_sorted[j];
    while ((rec >> b.pbits) == g) {
        const uint64_t nrec = j + 1 < sg.n ? sg.rec_sorted[j + 1] : ~0ull;  // issued before this record is decided
        const CPRec d = cp_dec(c, b, rec);
        const uint32_t i = d.i;
        rec = nrec;
        ++j;
        if (b.lim && c.out[i].status == SG_STATUS_TOO_MANY_REQUEST) continue;  // allowProceed refused it
        any_multi |= d.multi;
        if (d.multi && i == mi) {  // a repeated value: the check of the request's first record here, and its add
            b.chk[d.p] = mok ? 1 : 0;
            if (b.assume[i] && mok) cur += d.acq;
            continue;
        }
        if (P == INT64_MIN || i >= qn) {  // currentWindow(t): close the open period, open this one
            close();
            P = cp_period(b, r.wl_idx, i);
            const int I = (int)(P % S);
            const int64_t ws = P * wl, lo = ws - (int64_t)(S - 1) * wl;
            other = 0;
            cur = 0;
#pragma unroll
            for (int x = 0; x < SM; ++x) {
                const bool v = x < S && x != I && bs[x] != INT64_MIN && bs[x] >= lo;
                other += v ? bc[x] : 0;
                if (x == I) cur = bs[x] == ws ? bc[x] : 0;
            }
            const uint32_t q1 = (uint32_t)(P - cp_p0[r.wl_idx]) + 1;
            qn = q1 < cp_np[r.wl_idx] ? (cp_blds ? cp_sbnd[cp_boff[r.wl_idx] + q1]
                                                  : b.bnd[(size_t)r.wl_idx * kMaxPeriods + q1])
                                      : 0xFFFFFFFFu;
        }
        const double rem = thr - avg_div((double)(other + cur), r.isec) - (double)d.acq;
        if (!d.multi) {
            mi = kNoOwner;
            if (rem >= 0) {
                cur += d.acq;
                cp_store(c.out, i, SG_STATUS_OK, cp_d2i(rem));
            } else if (b.round > 0) {  // round 0: BLOCKED is k_cp_prep2's default already
                cp_store(c.out, i, SG_STATUS_BLOCKED, 0);
            }
            continue;
        }
        mi = i;
        mok = rem >= 0;
        b.chk[d.p] = mok ? 1 : 0;
        if (b.assume[i] && mok) cur += d.acq;
    }
    close();
    if (save_t >= 0 && any_multi) {  // the ring in memory is still the pre-batch one
        CPBucket* sv = b.save + (uint64_t)save_t * (uint64_t)c.stride;
        for (int x = 0; x < c.stride; ++x) sv[x] = ring[x];
    }
#pragma unroll
    for (int x = 0; x < SM; ++x) {
        if ((dirty >> x) & 1u) {
            CPBucket bk;
            bk.start = bs[x];
            bk.count = bc[x];
            ring[x] = bk;
        }
    }
}

__device__ void cp_walk_serial(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t g, uint64_t j) {
    const CPRule r = c.rules[cp_rule_of_slot(c, g)];
    if (r.S <= 10) cp_walk_serial_reg<10>(c, b, sg, g, j, r);
    else cp_walk_serial_mem(c, b, sg, g, j, r);
}

// Round 0 of the lane walker: the register walker saves the ring itself when the slot needs it (see
// cp_walk_serial_reg), the memory walker (sampleCount > 10) through cp_prologue first.
__device__ void cp_walk_serial_r0(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t g, uint64_t j,
                                  uint64_t t) {
    const CPRule r = c.rules[cp_rule_of_slot(c, g)];
    if (r.S <= 10) {
        cp_walk_serial_reg<10>(c, b, sg, g, j, r, b.save ? (int64_t)t : -1);
    } else {
        cp_prologue(c, b, g, t, 0, 1);
        cp_walk_serial_mem(c, b, sg, g, j, r);
    }
}

// One lane per slot of at most short_max records. Work item t: the slot's index in the save area (the long
// list comes first, then the short lists in class order); rounds > 0 walk the re-walk list of short items.
#ifndef SG_CPS_BLOCKS
#define SG_CPS_BLOCKS 1
#endif
__global__ void __launch_bounds__(256, SG_CPS_BLOCKS) k_cp_walk2(CPArgs c, CPBatch b, BatchArgs sg) {
    if (*c.err) return;
    cp_stage_periods(b);
    const uint32_t nlong = *sg.long_count;
    if (b.round > 0) {
        const uint32_t cnt = b.din_count[1];
        for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < cnt; x += gridDim.x * blockDim.x) {
            const uint32_t t = b.din[b.dcap + x];
            const uint64_t j = b.item_start[t];
            const uint64_t g = sg.rec_sorted[j] >> b.pbits;
            if (!cp_prologue(c, b, g, t, 0, 1)) continue;
            cp_walk_serial(c, b, sg, g, j);
        }
        return;
    }
    uint32_t total = 0;
    for (int k = 0; k < kClasses; ++k) total += sg.short_count[k];
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
        uint32_t r0 = u;
        int k = 0;
        while (r0 >= sg.short_count[k]) r0 -= sg.short_count[k++];
        const uint64_t j = sg.short_list[sg.class_off[k] + r0];
        const uint64_t g = sg.rec_sorted[j] >> b.pbits;
        cp_walk_serial_r0(c, b, sg, g, j, (uint64_t)nlong + u);  // round 0: cp_prologue only saves
    }
}

// Work items of the batch (long list, then the short lists in class order): each item's segment start, and each
// touched slot's item (k_cp_combine lists the items of the slots a changed outcome dirties).
__global__ void __launch_bounds__(256) k_cp_items(CPBatch b, BatchArgs sg) {
    const uint32_t nlong = *sg.long_count;
    uint32_t total = nlong;
    for (int k = 0; k < kClasses; ++k) total += sg.short_count[k];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        uint64_t j;
        if (t < nlong) {
            j = sg.long_list[t];
        } else {
            uint32_t r0 = t - nlong;
            int k = 0;
            while (r0 >= sg.short_count[k]) r0 -= sg.short_count[k++];
            j = sg.short_list[sg.class_off[k] + r0];
        }
        const uint64_t g = sg.rec_sorted[j] >> b.pbits;
        b.item_start[t] = (uint32_t)j;
        b.item_slot[t] = (uint32_t)g;
        b.slot_item[g] = t;
        // the segment's end: exponential then binary search (once per batch; every round's walkers reuse it)
        uint64_t lo = j, step = 1, hi = j + 1;
        while (hi < sg.n && (sg.rec_sorted[hi] >> b.pbits) == g) {
            lo = hi;
            step *= 2;
            hi = min(j + step, sg.n);
        }
        while (hi - lo > 1) {  // rec[lo] is g, rec[hi] (or the end) is not
            const uint64_t mid = (lo + hi) >> 1;
            if ((sg.rec_sorted[mid] >> b.pbits) == g) lo = mid;
            else hi = mid;
        }
        b.item_end[t] = (uint32_t)hi;
    }
}

template <class Pred>
__device__ __forceinline__ uint64_t cp_wave_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t q = lo + (uint64_t)lane * step;
        const uint64_t m = __ballot(q >= hi || pred(q));
        if (m == 0) {
            lo = lo + 63 * step + 1;
            continue;
        }
        const int f = __builtin_ctzll(m);
        if (f == 0) return lo;
        const uint64_t nhi = lo + (uint64_t)f * step;
        lo = lo + (uint64_t)(f - 1) * step + 1;
        hi = nhi < hi ? nhi : hi;
    }
    const uint64_t q = lo + (uint64_t)lane;
    const uint64_t m = __ballot(q < hi && pred(q));
    return m ? lo + (uint64_t)__builtin_ctzll(m) : hi;
}

__device__ __forceinline__ int64_t cp_excl_scan(int64_t v, int lane) {
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up((long long)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}

__device__ __forceinline__ int64_t cp_wave_sum(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((long long)v, o, 64);
    return v;
}

enum : int { kCpSkip = 0, kCpSingle = 1, kCpMulti = 2, kCpDup = 3 };
__device__ __forceinline__ uint64_t cp_below(int f) { return f >= 64 ? ~0ull : ((1ull << f) - 1ull); }
#ifndef SG_CPU
#define SG_CPU 2
#endif
constexpr int kCpU = SG_CPU;  // 64-record chunks whose loads are issued together (three dependent round trips per block)
constexpr uint64_t kCpSkipMin = 256;     // shortest saturated tail worth handing to k_cp_skipfill (records)
constexpr uint64_t kCpSkipPiece = 4096;  // skipped ranges go to k_cp_skipfill in pieces of this size

// One wave per slot of more than short_max records (a hot (rule, value)), 64 records per step with the ring in
// registers (lane x < S holds bucket x). Within one window period the state is the running count `cur`; every
// record's check is thr - (other + cur_before) / intervalSec - acquire >= 0, monotone in cur_before. A step
// assumes every unresolved record adds what it would add on passing — a single-value request its count, a
// multi-value request's first record here its count for each of its records in the chunk iff the request is
// assumed to pass — takes the exclusive scan of the adds, and commits the lanes up to the first such record whose
// check fails (that one adds nothing); records that fail even at the committed state are blocked at once (cur only
// grows). A repeated value of a multi-value request (adjacent record, same owner) carries check 1 and adds only
// through its first record (as cp_walk_serial: the request's count per record iff it is assumed to pass and this
// slot's check passed), or, when the chunk starts inside the request's run, iff that first record passed.
// Records, owners and requests of kCpU chunks are loaded together.
//
// Saturated periods: once not even acquireCount = 1 fits the window (every valid request has acquireCount >= 1,
// and cur only grows within the period), every later record of the period fails its check and adds nothing — a
// single-value request is BLOCKED, a multi-value request's first record checks 0. The wave finds where the period
// ends (64-way search on the requests' timestamps), hands the range to k_cp_skipfill and goes on there: a hot
// slot costs a few steps per window period instead of one or two per 64 records.
#ifndef SG_CPL_BLOCKS
#define SG_CPL_BLOCKS 4  // 128 VGPRs: 4 waves per SIMD (6.8 vs 7.1 ms/step at 3)
#endif
__global__ void __launch_bounds__(256, SG_CPL_BLOCKS) k_cp_walk2_long(CPArgs c, CPBatch b, BatchArgs sg) {
    if (*c.err) return;
    cp_stage_periods(b);
    const int lane = (int)__lane_id();
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t cnt = b.round > 0 ? b.din_count[0] : *sg.long_count;
    // the item headers (work item, segment bounds, slot) are loaded one item ahead: a slot's header is otherwise a
    // chain of three dependent round trips before its first record
    if (cnt == 0 || wave >= cnt) return;  // (after the block-wide staging)
    const uint32_t last = cnt - 1;
    uint32_t tq = b.round > 0 ? b.din[min(wave, last)] : min(wave, last);  // rounds > 0: the re-walk list
    uint64_t sq = b.item_start[tq], eq = b.item_end[tq], gq = b.item_slot[tq];
    for (uint32_t x = wave; x < cnt; x += nwaves) {
        const uint32_t t = tq;
        const uint64_t s = sq, e = eq, g = gq;
        {
            const uint32_t xn = min(x + nwaves, last);
            tq = b.round > 0 ? b.din[xn] : xn;
            sq = b.item_start[tq];
            eq = b.item_end[tq];
            gq = b.item_slot[tq];
        }
        const CPRule r = c.rules[cp_rule_of_slot(c, g)];
        // rounds > 0 with checkpoints: resume at the first record of the earliest window period a changed outcome
        // touches, from the ring as that period opened in the latest walk (the records before it saw unchanged
        // inputs); else restore the pre-batch ring and walk the whole segment
        uint64_t s0 = s;
        int64_t ckq = -1;  // checkpoint to start from (batch-relative period), -1: the ring in memory
        if (b.round > 0 && b.ckpt && r.S <= 64) {
            if (!b.dflag[t]) continue;
            const uint32_t q0 = b.dq[t];
            if (q0 != 0 && q0 < b.ck_np) {
                const int64_t P0 = cp_p0[r.wl_idx];
                s0 = gallop_search(s, e, [&](uint64_t q) {
                    return cp_period(b, r.wl_idx, cp_dec(c, b, sg.rec_sorted[q]).i) - P0 >= (int64_t)q0;
                }, lane);
                if (s0 < e) ckq = cp_period(b, r.wl_idx, cp_dec(c, b, sg.rec_sorted[s0]).i) - P0;
                else s0 = s;
            }
            if (ckq < 0) {
                const CPBucket* sv = b.save + t * (uint64_t)c.stride;
                CPBucket* rg = c.ring + g * (uint64_t)c.stride;
                for (int x = lane; x < c.stride; x += 64) rg[x] = sv[x];
            }
            if (lane == 0) {
                b.dflag[t] = 0;
                b.dq[t] = 0xFFFFFFFFu;
            }
        } else if (!cp_prologue(c, b, g, t, lane, 64)) {
            continue;
        }
        if (r.S > 64) {  // the ring does not fit the wave's registers
            if (lane == 0) cp_walk_serial(c, b, sg, g, s);
            continue;
        }
        const double thr = cp_threshold(c, r, c.keys[g]);
        CPBucket* ring = c.ring + g * (uint64_t)c.stride;
        CPBucket* ck = b.ckpt ? b.ckpt + (uint64_t)t * b.ck_np * c.stride : nullptr;
        const int64_t P0 = cp_p0[r.wl_idx];
        const int S = r.S;
        const int64_t wl = r.wl;
        int64_t bst = INT64_MIN, bcnt = 0;
        if (lane < S) {
            const CPBucket bk = ckq >= 0 ? ck[(uint64_t)ckq * c.stride + lane] : ring[lane];
            bst = bk.start;
            bcnt = bk.count;
        }
        int64_t P = INT64_MIN, other = 0, cur = 0;
        uint32_t carry = kNoOwner;  // owner of the record before the current chunk
        bool carry_ok = false;      // that owner is a multi-value request whose first record here passed its check
        uint64_t blk = s0;
        uint64_t pf = s0;        // position of the records in rcn (the next block, loaded a block ahead)
        uint64_t nosearch = s0;  // a search found the saturated period ending before kCpSkipMin records: walk to there
        uint64_t rcn[kCpU];
#pragma unroll
        for (int u = 0; u < kCpU; ++u) rcn[u] = sg.rec_sorted[min(s0 + (uint64_t)u * 64 + lane, e - 1)];
        while (blk < e) {
            // loads of kCpU chunks at once; indices clamped to the segment (unconditional loads)
            uint64_t rc[kCpU];
            uint32_t ow[kCpU];
            int64_t aq[kCpU];
            int32_t st[kCpU];
            uint8_t as[kCpU];
            const bool have = pf == blk;  // wave-uniform: the block was prefetched (no saturated skip since)
#pragma unroll
            for (int u = 0; u < kCpU; ++u) rc[u] = have ? rcn[u] : sg.rec_sorted[min(blk + (uint64_t)u * 64 + lane, e - 1)];
            pf = blk + 64ull * kCpU;
#pragma unroll
            for (int u = 0; u < kCpU; ++u) rcn[u] = sg.rec_sorted[min(pf + (uint64_t)u * 64 + lane, e - 1)];
#pragma unroll
            for (int u = 0; u < kCpU; ++u) {  // the request: in the record (single value), owner[] (multi-value)
                const uint64_t pl = rc[u] & b.pmask;
                const uint64_t id = pl & b.idmask;
                ow[u] = ((pl >> (b.pbits - 1)) & 1ull) ? b.owner[id] : (uint32_t)id;
            }
#pragma unroll
            for (int u = 0; u < kCpU; ++u) {
                const uint64_t pl = rc[u] & b.pmask;
                const uint32_t ac = (uint32_t)(pl >> b.idbits) & 127u;
                const bool mu = ((pl >> (b.pbits - 1)) & 1ull) != 0;
                aq[u] = ac == kCpAesc ? (int64_t)c.req[ow[u]].acquire : (int64_t)ac;
                st[u] = b.lim ? c.out[ow[u]].status : 0;
                as[u] = mu ? b.assume[ow[u]] : (uint8_t)1;
            }
            uint64_t next = blk + 64ull * kCpU;
#pragma unroll
            for (int u = 0; u < kCpU; ++u) {
                const uint64_t base = blk + (uint64_t)u * 64;
                if (base >= e) break;
                const uint64_t j = base + (uint64_t)lane;
                const bool act = j < e;
                const uint32_t i = ow[u];
                const uint64_t p = rc[u] & b.idmask;  // the value position (multi-value records)
                const bool mu = ((rc[u] >> (b.pbits - 1)) & 1ull) != 0;
                uint32_t prev = (uint32_t)__shfl_up((int)i, 1u, 64);
                if (lane == 0) prev = carry;
                carry = (uint32_t)__shfl((int)i, 63, 64);
                int typ = kCpSkip;
                int64_t acq = 0, Pq = 0;
                if (act && !(b.lim && st[u] == SG_STATUS_TOO_MANY_REQUEST)) {
                    acq = aq[u];
                    Pq = cp_period(b, r.wl_idx, i);
                    typ = !mu ? kCpSingle : prev == i ? kCpDup : kCpMulti;
                }
                // a request's records in this slot are adjacent: a repeated value's first record is the nearest
                // non-repeated lane below it, or (none in the chunk) the carried owner's
                const uint64_t nondup = __ballot(typ != kCpDup);
                int64_t add = 0;
                if (typ == kCpSingle) {
                    add = acq;
                } else if (typ == kCpMulti) {
                    const uint64_t after = nondup & ~cp_below(lane + 1);
                    const int nxt = after ? __builtin_ctzll(after) : 64;
                    add = as[u] ? acq * (int64_t)(nxt - lane) : 0;  // this record and its repeats in the chunk
                } else if (typ == kCpDup) {
                    add = ((nondup & cp_below(lane)) == 0 && carry_ok && as[u]) ? acq : 0;
                    b.chk[p] = 1;  // the request's first record here carries the check
                }
                // lanes whose own check decides their add (a failing check adds nothing)
                const bool cut_kind = typ == kCpSingle || (typ == kCpMulti && add != 0);
                uint64_t pending = __ballot(typ != kCpSkip);
                uint64_t failed = 0;
                bool okv = false;  // this lane's check passed (multi-value first records: carry_ok of the next chunk)
                while (pending) {
                    const int f = __builtin_ctzll(pending);
                    const int64_t Pf = __shfl((long long)Pq, f, 64);
                    if (Pf != P) {  // currentWindow: close the open period, open Pf
                        if (P != INT64_MIN && lane == (int)(P % S)) {
                            bst = P * wl;
                            bcnt = cur;
                        }
                        if (ck && lane < S && Pf - P0 < (int64_t)b.ck_np) {  // the ring as Pf opens
                            CPBucket o;
                            o.start = bst;
                            o.count = bcnt;
                            ck[(uint64_t)(Pf - P0) * c.stride + lane] = o;
                        }
                        P = Pf;
                        const int I = (int)(P % S);
                        const int64_t ws = P * wl, lo = ws - (int64_t)(S - 1) * wl;
                        int64_t o = 0, cc = 0;
                        if (lane < S) {
                            if (lane == I) cc = bst == ws ? bcnt : 0;
                            else if (bst != INT64_MIN && bst >= lo) o = bcnt;
                        }
                        other = cp_wave_sum(o);
                        cur = cp_wave_sum(cc);
                    }
                    uint64_t open = pending & __ballot(typ != kCpSkip && Pq == P);
                    pending &= ~open;
                    while (open) {
                        const bool mine = (open >> lane) & 1ull;
                        const bool dead = (failed >> lane) & 1ull;
                        const int64_t a = (mine && !dead) ? add : 0;
                        const int64_t excl = cp_excl_scan(a, lane);
                        const double rem = thr - avg_div((double)(other + cur + excl), r.isec) - (double)acq;
                        const bool ok = rem >= 0 && !dead;
                        // a dead lane adds nothing already: not a cut (else every pass would stop at one)
                        const uint64_t bad = __ballot(mine && cut_kind && !dead && !(rem >= 0));
                        uint64_t done = open;
                        int64_t adv;
                        if (bad) {
                            const int k = __builtin_ctzll(bad);
                            done = open & ((2ull << k) - 1ull);
                            adv = __shfl((long long)excl, k, 64);  // the failing lane k adds nothing
                        } else {
                            adv = cp_wave_sum(a);
                        }
                        if ((done >> lane) & 1ull) {
                            okv = ok;
                            if (typ == kCpSingle) {
                                if (ok) cp_store(c.out, i, SG_STATUS_OK, cp_d2i(rem));
                                else if (b.round > 0) cp_store(c.out, i, SG_STATUS_BLOCKED, 0);
                            } else if (typ == kCpMulti) {
                                b.chk[p] = ok ? 1 : 0;
                            }
                        }
                        cur += adv;
                        open &= ~done;
                        if (bad && open) {  // failing even at the committed state: fails for good
                            const double lb = thr - avg_div((double)(other + cur), r.isec) - (double)acq;
                            failed |= __ballot(((open >> lane) & 1ull) && (cut_kind || typ == kCpMulti) && lb < 0);
                        }
                    }
                }
                // the next chunk's carried request: lane 63's, whose first record is the highest non-repeated lane
                {
                    const int t63 = __shfl(typ, 63, 64);
                    if (t63 == kCpMulti || t63 == kCpDup) {
                        if (nondup) carry_ok = __shfl((int)okv, 63 - __builtin_clzll(nondup), 64) != 0;
                    } else {
                        carry_ok = false;
                    }
                }
                // saturated period: hand the rest of it to k_cp_skipfill (not while a passed multi-value request's
                // repeated values may still follow: they add)
                const uint64_t pos = base + 64;
                if (pos < e && pos >= nosearch && P != INT64_MIN && !carry_ok && b.skips &&
                    thr - avg_div((double)(other + cur), r.isec) - 1.0 < 0) {
                    const int64_t Pc = P;
                    const uint64_t pe = gallop_search(pos, e, [&](uint64_t q) {
                        return cp_period(b, r.wl_idx, cp_dec(c, b, sg.rec_sorted[q]).i) > Pc;
                    }, lane);
                    if (pe - pos >= kCpSkipMin) {
                        const uint32_t np = (uint32_t)((pe - pos + kCpSkipPiece - 1) / kCpSkipPiece);
                        uint32_t slot = 0;
                        if (lane == 0) slot = atomicAdd(b.skip_count, np);
                        slot = (uint32_t)__shfl((int)slot, 0, 64);
                        if (slot + np <= b.skip_cap) {
                            for (uint32_t pi = (uint32_t)lane; pi < np; pi += 64) {
                                const uint64_t b0 = pos + (uint64_t)pi * kCpSkipPiece;
                                b.skips[slot + pi] = make_uint2((uint32_t)b0, (uint32_t)min(pe, b0 + kCpSkipPiece));
                            }
                            carry = cp_dec(c, b, sg.rec_sorted[pe - 1]).i;
                            next = pe;
                            break;
                        }
                    }
                    nosearch = pe;  // too short to hand over (or no room): the chunks walk it, with no search per chunk
                }
            }
            blk = next;
        }
        if (P != INT64_MIN && lane == (int)(P % S)) {
            bst = P * wl;
            bcnt = cur;
        }
        if (lane < S) {
            CPBucket bk;
            bk.start = bst;
            bk.count = bcnt;
            ring[lane] = bk;
        }
    }
}

// The saturated ranges of k_cp_walk2_long (one wave per piece): every record fails its check and adds nothing — a
// single-value request is BLOCKED, a multi-value request's first record in the slot checks 0, a repeated value
// carries check 1. In round 0 the BLOCKED results and the 0 checks are the defaults already (k_cp_prep2,
// k_cp_recinit): only the repeated values are written.
__global__ void __launch_bounds__(256) k_cp_skipfill(CPArgs c, CPBatch b, BatchArgs sg) {
    if (*c.err || (b.changed_prev && *b.changed_prev == 0)) return;
    const uint32_t cnt = min(*b.skip_count, b.skip_cap);
    const int lane = (int)__lane_id();
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t w = wave; w < cnt; w += nwaves) {
        const uint2 pc = b.skips[w];
        for (uint64_t j = (uint64_t)pc.x + lane; j < pc.y; j += 64) {
            const uint64_t rec = sg.rec_sorted[j];
            const bool multi = ((rec >> (b.pbits - 1)) & 1ull) != 0;
            if (b.round == 0 && !multi) continue;
            const CPRec d = cp_dec(c, b, rec);
            if (b.lim && c.out[d.i].status == SG_STATUS_TOO_MANY_REQUEST) continue;
            if (!d.multi) {
                cp_store(c.out, d.i, SG_STATUS_BLOCKED, 0);
            } else {
                const uint32_t prev = cp_dec(c, b, sg.rec_sorted[j - 1]).i;  // j > the segment start
                if (b.round > 0 || prev == d.i) b.chk[d.p] = prev == d.i ? 1 : 0;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_cp_combine(CPArgs c, CPBatch b) {
    if (blockIdx.x == 0 && threadIdx.x < 2) b.dout_count[threadIdx.x] = 0;  // k_cp_relist fills them next
    if (*c.err || (b.changed_prev && *b.changed_prev == 0)) return;
    const uint32_t m = *b.mcount;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < m; x += gridDim.x * blockDim.x) {
        const uint64_t i = b.mlist[x];  // a valid multi-value request (k_cp_prep2)
        const sg_cparam_req q = c.req[i];
        const bool was = b.assume[i] != 0;
        if (b.lim && c.out[i].status == SG_STATUS_TOO_MANY_REQUEST) continue;
        // the checks of the first four values loaded together (value_count >= 2)
        const uint64_t vb = q.value_begin;
        const uint32_t vc = q.value_count;
        const uint8_t c0 = b.chk[vb], c1 = b.chk[vb + 1], c2 = vc > 2 ? b.chk[vb + 2] : (uint8_t)1,
                      c3 = vc > 3 ? b.chk[vb + 3] : (uint8_t)1;
        bool pass = c0 && c1 && c2 && c3;
        for (uint32_t j = 4; j < vc && pass; ++j) pass = b.chk[vb + j] != 0;
        // the result stands from the previous round unless the outcome changed (remaining -1: multi-value)
        if (b.round == 0 || was != pass) cp_store(c.out, i, pass ? SG_STATUS_OK : SG_STATUS_BLOCKED, pass ? -1 : 0);
        if (was != pass) {
            // re-walk the slots whose adds change: a slot adds the request's count iff it is assumed to pass and
            // the slot's check passed (a repeated value's extra records carry check 1), so slots where the check
            // failed add nothing either way
            b.assume[i] = pass ? 1 : 0;
            *b.changed = 1;
            // the slots' re-walks may resume at this request's window period (hot slots' ring checkpoints)
            const CPRule r = c.rules[q.key & SG_KEY_INDEX];
            const uint32_t qrel = (uint32_t)(q.ts_ms / r.wl - b.p0[r.wl_idx]);
            for (uint32_t j = 0; j < q.value_count; ++j) {
                const uint64_t p = (uint64_t)q.value_begin + j;
                if (!b.chk[p]) continue;
                const uint32_t t = b.slot_item[b.pslot[p]];
                b.dflag[t] = 1u;  // listed by k_cp_relist
                if (b.ckpt) atomicMin(&b.dq[t], qrel);
            }
        }
    }
}

// The next round's re-walk lists from the flags k_cp_combine set (long items, short items; block-aggregated).
__global__ void __launch_bounds__(256) k_cp_relist(CPBatch b, BatchArgs sg, uint32_t items) {
    __shared__ uint32_t wsum[4], gbase[2];
    if (blockIdx.x == 0 && threadIdx.x == 0) *b.skip_count = 0;  // the next round's k_cp_walk2_long appends
    if (*b.changed == 0) return;  // no outcome changed: no item is flagged
    const uint32_t nlong = *sg.long_count;
    const uint32_t base = blockIdx.x * (256 * kAggItems);
    bool f[kAggItems];
    uint32_t cnt = 0;  // long count | short count << 16
#pragma unroll
    for (int u = 0; u < kAggItems; ++u) {
        const uint32_t t = base + (uint32_t)u * 256 + threadIdx.x;
        f[u] = t < items && b.dflag[min(t, items - 1)] != 0u;
        cnt += f[u] ? (t < nlong ? 1u : 0x10000u) : 0u;
    }
    uint32_t tot;
    const uint32_t off = cp_block_excl_scan(cnt, wsum, &tot);
    if (threadIdx.x < 2) {
        const uint32_t c2 = threadIdx.x == 0 ? (tot & 0xFFFFu) : (tot >> 16);
        gbase[threadIdx.x] = c2 ? atomicAdd(&b.dout_count[threadIdx.x], c2) : 0u;
    }
    __syncthreads();
    uint32_t o0 = gbase[0] + (off & 0xFFFFu), o1 = gbase[1] + (off >> 16);
#pragma unroll
    for (int u = 0; u < kAggItems; ++u) {
        if (!f[u]) continue;
        const uint32_t t = base + (uint32_t)u * 256 + threadIdx.x;
        if (t < nlong) b.dout[o0++] = t;
        else b.dout[(size_t)b.dcap + o1++] = t;
    }
}

// Save (restore = 0) or restore (1) the first S buckets of every touched slot.
__global__ void __launch_bounds__(256) k_cp_saverings(CPArgs c, CPBatch b, BatchArgs sg, int restore) {
    uint32_t total = *sg.long_count;
    for (int k = 0; k < kClasses; ++k) total += sg.short_count[k];
    const uint64_t work = (uint64_t)total * c.stride;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < work; w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t r0 = (uint32_t)(w / c.stride);
        const int x = (int)(w % c.stride);
        const uint32_t t = r0;
        uint64_t j;
        if (r0 < *sg.long_count) {
            j = sg.long_list[r0];
        } else {
            r0 -= *sg.long_count;
            int k = 0;
            while (r0 >= sg.short_count[k]) r0 -= sg.short_count[k++];
            j = sg.short_list[sg.class_off[k] + r0];
        }
        const uint64_t g = sg.rec_sorted[j] >> b.pbits;
        CPBucket* ring = c.ring + g * (uint64_t)c.stride;
        if (restore) {
            ring[x] = b.save[(uint64_t)t * c.stride + x];
            if (x == 0) b.dflag[t] = 0;
        } else {
            b.save[(uint64_t)t * c.stride + x] = ring[x];
        }
    }
}

// ------------------------------------------------- fallback: groups of linked slots replayed in arrival order
//
// When the rounds run out (a chain of multi-value requests deeper than the round budget), the work items (touched
// slots) linked by multi-value requests are grouped into connected components — min-label hooking with pointer
// jumping, one launch pair per iteration until no label moves (labels only decrease, so a read that misses another
// block's update in the same launch only delays convergence, and the iteration that changes nothing reads settled
// labels) — the groups the last round still changed get their rings restored from the round-0 saves, and each of
// their requests is replayed on one lane per group in arrival order: each value checked against the state before the
// request, all added iff all pass (ClusterParamFlowChecker.java:58-80, as sequential calls). Groups run in parallel;
// settled groups (and slots no multi-value request touches) keep their walks.

__global__ void __launch_bounds__(256) k_cpfb_init(CPGroups g) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < g.items; t += gridDim.x * blockDim.x) {
        g.label[t] = t;
        g.flag[t] = 0;
    }
}

// Every multi-value request pulls its items' labels (and the items those labels name) down to their minimum.
__global__ void __launch_bounds__(256) k_cpfb_hook(CPArgs c, CPBatch b, CPGroups g) {
    const uint32_t m = *b.mcount;
    bool moved = false;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < m; x += gridDim.x * blockDim.x) {
        const sg_cparam_req q = c.req[b.mlist[x]];
        uint32_t lo = 0xFFFFFFFFu;
        for (uint32_t j = 0; j < q.value_count; ++j) lo = min(lo, g.label[b.slot_item[b.pslot[q.value_begin + j]]]);
        for (uint32_t j = 0; j < q.value_count; ++j) {
            const uint32_t t = b.slot_item[b.pslot[q.value_begin + j]];
            const uint32_t old = atomicMin(&g.label[t], lo);
            if (old > lo) {
                atomicMin(&g.label[old], lo);
                moved = true;
            }
        }
    }
    if (__ballot(moved) && __lane_id() == 0) *g.changed = 1;
}

__global__ void __launch_bounds__(256) k_cpfb_jump(CPGroups g) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < g.items; t += gridDim.x * blockDim.x) {
        uint32_t l = g.label[t];
        for (uint32_t ll = g.label[l]; ll < l; ll = g.label[l]) l = ll;
        atomicMin(&g.label[t], l);
    }
}

// The groups still moving — an item listed for a re-walk by the last round (an outcome of the group changed and
// changes an add) — their rings restored, and one entry {group | request} per request in them. A group whose
// outcomes the last round left unchanged holds a consistent assignment, which is the sequential answer (every
// request's checks then see exact states, by induction in arrival order), and keeps its walk.
__global__ void __launch_bounds__(256) k_cpfb_flag(CPBatch b, CPGroups g) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < g.items; t += gridDim.x * blockDim.x)
        if (b.dflag[t]) g.flag[g.label[t]] = 1;
}

__global__ void __launch_bounds__(256) k_cpfb_restore(CPArgs c, CPBatch b, CPGroups g) {
    const uint64_t work = (uint64_t)g.items * c.stride;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < work; w += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t t = (uint32_t)(w / c.stride);
        if (!g.flag[g.label[t]]) continue;
        const int x = (int)(w % c.stride);
        c.ring[(uint64_t)b.item_slot[t] * c.stride + x] = b.save[(uint64_t)t * c.stride + x];
    }
}

__global__ void __launch_bounds__(256) k_cpfb_entries(CPArgs c, CPBatch b, CPGroups g) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_cparam_req q = c.req[i];
        bool in = cp_valid(c, q) && !(b.lim && c.out[i].status == SG_STATUS_TOO_MANY_REQUEST);
        uint32_t lab = 0;
        if (in) {
            lab = g.label[b.slot_item[b.pslot[q.value_begin]]];
            in = g.all || g.flag[lab] != 0;
        }
        const uint64_t mask = __ballot(in);
        if (!mask) continue;
        const int lane = (int)__lane_id();
        uint32_t base = 0;
        if (lane == __builtin_ctzll(mask)) base = atomicAdd(g.ent_count, (uint32_t)__popcll(mask));
        base = (uint32_t)__shfl((int)base, __builtin_ctzll(mask), 64);
        if (in) g.ent[base + __popcll(mask & ((1ull << lane) - 1ull))] = ((uint64_t)lab << g.ibits) | i;
    }
}

__global__ void __launch_bounds__(256) k_cpfb_heads(CPGroups g, uint32_t m) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint64_t k = g.ent_sorted[j] >> g.ibits;
        if (j == 0 || (g.ent_sorted[j - 1] >> g.ibits) != k) g.heads[atomicAdd(g.head_count, 1u)] = j;
    }
}

__global__ void __launch_bounds__(256) k_cpfb_replay(CPArgs c, CPBatch b, CPGroups g, uint32_t m) {
    const uint32_t nh = *g.head_count;
    const uint64_t imask = (1ull << g.ibits) - 1ull;
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x) {
        uint32_t j = g.heads[h];
        const uint64_t key = g.ent_sorted[j] >> g.ibits;
        for (; j < m && (g.ent_sorted[j] >> g.ibits) == key; ++j) {
            const uint64_t i = g.ent_sorted[j] & imask;
            const sg_cparam_req q = c.req[i];
            const CPRule r = c.rules[q.key & SG_KEY_INDEX];
            const int64_t P = q.ts_ms / r.wl;
            bool pass = true;
            double rem = -1;
            for (uint32_t v = 0; v < q.value_count && pass; ++v) {
                const uint64_t gs = b.pslot[q.value_begin + v];
                int64_t cur = 0;
                const int64_t other = cp_window(c.ring + gs * (uint64_t)c.stride, r.S, r.wl, P, &cur);
                rem = cp_threshold(c, r, c.values[q.value_begin + v]) - avg_div((double)(other + cur), r.isec) - (double)q.acquire;
                pass = rem >= 0;
            }
            if (pass) {
                for (uint32_t v = 0; v < q.value_count; ++v) {
                    CPBucket& bk = c.ring[(uint64_t)b.pslot[q.value_begin + v] * c.stride + (int)(P % r.S)];
                    if (bk.start != P * r.wl) {
                        bk.start = P * r.wl;
                        bk.count = 0;
                    }
                    bk.count += q.acquire;
                }
            }
            if (q.value_count > 1) rem = -1;
            cp_store(c.out, i, pass ? SG_STATUS_OK : SG_STATUS_BLOCKED, pass ? cp_d2i(rem) : 0);
        }
    }
}

static unsigned cgrid2(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

hipError_t launch_cp_limprep(const CPArgs& c, BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_limprep, dim3(cgrid2(c.n, 8192)), dim3(256), 0, stream, c, a);
    return hipGetLastError();
}

hipError_t launch_cp_prep2(const CPArgs& c, const CPBatch& b, hipStream_t stream) {
    const uint64_t sentinel = c.total_slots << b.pbits;
    hipLaunchKernelGGL(k_cp_recinit, dim3(cgrid2(c.n_values, 8192)), dim3(256), 0, stream, b, c.n_values, sentinel);
    hipLaunchKernelGGL(k_cp_prep2, dim3(cgrid2(c.n, 8192)), dim3(256), 0, stream, c, b);
    return hipGetLastError();
}

hipError_t launch_cp_order(const CPArgs& c, const CPBatch& b, const uint64_t* sorted, uint64_t n, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_order, dim3(cgrid2(n, 8192)), dim3(256), 0, stream, c, b, sorted, n);
    return hipGetLastError();
}

// The long (hot-slot) walker on `aux` beside the lane walker, then the saturated ranges.
hipError_t launch_cp_walk2(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, hipStream_t stream, hipStream_t aux,
                           hipEvent_t fork, hipEvent_t join) {
    const uint64_t waves = sg.n / ((uint64_t)sg.short_max + 1) + 1;  // bound on the long list's length
#ifdef SG_CP_ONE_STREAM
    aux = stream;
#endif
    hipError_t e = hipEventRecord(fork, stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cp_walk2_long, dim3(cgrid2(waves * 64, 2048)), dim3(256), 0, aux, c, b, sg);
    hipLaunchKernelGGL(k_cp_walk2, dim3(cgrid2(sg.n, 4096)), dim3(256), 0, stream, c, b, sg);
    e = hipEventRecord(join, aux);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, join, 0);
    if (e != hipSuccess) return e;
    if (b.skips) hipLaunchKernelGGL(k_cp_skipfill, dim3(1024), dim3(256), 0, stream, c, b, sg);
    return hipGetLastError();
}

hipError_t launch_cp_items(const CPBatch& b, const BatchArgs& sg, uint64_t items, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_items, dim3(cgrid2(items, 8192)), dim3(256), 0, stream, b, sg);
    return hipGetLastError();
}

hipError_t launch_cp_mlist(const CPArgs& c, const CPBatch& b, hipStream_t stream) {
    if (c.n == 0) return hipSuccess;
    lds_poison(stream);
    hipLaunchKernelGGL(k_cp_mlist, dim3((unsigned)((c.n + 256 * kAggItems - 1) / (256 * kAggItems))), dim3(256), 0, stream,
                       c, b);
    return hipGetLastError();
}

// k_cp_combine over the multi-value requests, then the re-walk lists of the next round (`items` work items)
hipError_t launch_cp_combine(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t items, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_combine, dim3(cgrid2(c.n / 8 + 1, 4096)), dim3(256), 0, stream, c, b);
    lds_poison(stream);
    if (items) hipLaunchKernelGGL(k_cp_relist, dim3((unsigned)((items + 256 * kAggItems - 1) / (256 * kAggItems))),
                                  dim3(256), 0, stream, b, sg, (uint32_t)items);
    return hipGetLastError();
}

hipError_t launch_cp_saverings(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, int restore, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_saverings, dim3(cgrid2(sg.n * (uint64_t)c.stride, 8192)), dim3(256), 0, stream, c, b, sg,
                       restore);
    return hipGetLastError();
}

__global__ void k_cp_finish_batch(CPArgs c) {
    if (*c.err == 0) *c.last_ts = c.req[c.n - 1].ts_ms;
}

hipError_t launch_cp_finish_batch(const CPArgs& c, hipStream_t stream) {
    hipLaunchKernelGGL(k_cp_finish_batch, dim3(1), dim3(1), 0, stream, c);
    return hipGetLastError();
}

hipError_t launch_cpfb(const CPArgs& c, const CPBatch& b, const CPGroups& g, int step, uint32_t m, hipStream_t stream) {
    switch (step) {
        case 0:
            hipLaunchKernelGGL(k_cpfb_init, dim3(cgrid2(g.items, 4096)), dim3(256), 0, stream, g);
            break;
        case 1:
            hipLaunchKernelGGL(k_cpfb_hook, dim3(cgrid2(m, 4096)), dim3(256), 0, stream, c, b, g);
            hipLaunchKernelGGL(k_cpfb_jump, dim3(cgrid2(g.items, 4096)), dim3(256), 0, stream, g);
            break;
        case 2:
            if (!g.all) hipLaunchKernelGGL(k_cpfb_flag, dim3(cgrid2(g.items, 4096)), dim3(256), 0, stream, b, g);
            if (!g.all)
                hipLaunchKernelGGL(k_cpfb_restore, dim3(cgrid2((uint64_t)g.items * c.stride, 8192)), dim3(256), 0,
                                   stream, c, b, g);
            hipLaunchKernelGGL(k_cpfb_entries, dim3(cgrid2(c.n, 8192)), dim3(256), 0, stream, c, b, g);
            break;
        default:
            if (m == 0) break;
            hipLaunchKernelGGL(k_cpfb_heads, dim3(cgrid2(m, 4096)), dim3(256), 0, stream, g, m);
            hipLaunchKernelGGL(k_cpfb_replay, dim3(cgrid2(m, 4096)), dim3(256), 0, stream, c, b, g, m);
    }
    return hipGetLastError();
}

}  // namespace sg
