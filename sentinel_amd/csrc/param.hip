// param.hip — hot-parameter flow control on the device: ParamFlowChecker.passSingleValueCheck for QPS
// rules (sentinel-extension/sentinel-parameter-flow-control/.../slots/block/flow/param/ParamFlowChecker.java:
// passDefaultLocalCheck :127-202, passThrottleLocalCheck :204-254).
//
// The reference keeps per-rule LRU CacheMaps (value → lastAddTokenTime, value → tokens); here each rule
// owns an exact open-addressing sub-table in HBM (2^capacity_log2 slots + one side slot for the value
// 0xFFFF…FFFF, which doubles as the empty marker). A batch:
//   k_pprep    early rejections that never touch the maps (no rule, tokenCount 0, acquire > maxCount),
//              lock-free find-or-insert of (rule, value) by CAS on the slot's value word, packed record
//              {global slot | request index}; outputs start as "blocked".
//   radix sort by slot (sort.hip): every (rule, value)'s requests contiguous, in arrival order.
//   k_pwalk_short / k_pwalk_long  sequential replay per slot; the wave walker decides 64 requests per
//              step (prefix-scan admit, ballot skip) and, once the bucket cannot pay even 1 token before
//              the next refill, jumps to the first request after the refill time by a 64-way search.
#include "pslot_dev.h"

namespace sg {

constexpr uint32_t kPAesc = 255;    // acquire code: read req[i].acquire
constexpr uint32_t kPLdsMs = 4096;  // millisecond table entries staged in LDS (a batch spanning <= 4 s)

__global__ void __launch_bounds__(256) k_pprep(PArgs p, uint64_t sentinel) {
    const int64_t t0 = p.req[0].ts_ms;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_param_req q = p.req[i];
        const int64_t tp = i == 0 ? *p.last_ts : p.req[i - 1].ts_ms;
        if (q.ts_ms < 0 || q.ts_ms < tp) atomicOr(p.err, kErrTime);
        // the millisecond table: request index -> timestamp for the walkers (a new millisecond starts at i)
        if (i == 0) {
            *p.mt0 = q.ts_ms;
        } else if (q.ts_ms > tp) {
            for (int64_t ms = (tp < t0 ? t0 : tp) + 1; ms <= q.ts_ms; ++ms) {
                const int64_t qq = ms - t0;
                if (qq >= (int64_t)kMaxPeriods) break;
                p.msb[qq] = (uint32_t)i;
            }
        }
        if (i == p.n - 1) *p.mnp = (uint32_t)min(q.ts_ms - t0 + 1, (int64_t)kMaxPeriods + 1);
        if ((i & ((1ull << p.bshift) - 1ull)) == 0) p.mbk[i >> p.bshift] = (uint16_t)min(max(q.ts_ms - t0, (int64_t)0), (int64_t)65535);
        if (q.acquire <= 0) atomicOr(p.err, kErrNonPositive);
        uint64_t rec = sentinel;
        int32_t pass = 0;
        if (q.rule >= p.n_rules) {
            pass = 1;  // no rule for this index: nothing to check
        } else {
            const PRule r = p.rules[q.rule];
            const int64_t tc = param_token_count(p, r, q.value);
            const bool early_block = tc == 0 || (r.behavior != 2 && (int64_t)q.acquire > tc + r.burst);
            if (!early_block) {
                const uint64_t g = param_slot(p, r, q.value);
                const uint64_t ac = (q.acquire <= 0 || (uint64_t)q.acquire >= kPAesc) ? kPAesc : (uint64_t)q.acquire;
                if (g == ~0ull) atomicOr(p.err, kErrTableFull);
                else rec = (g << p.gshift) | (ac << p.ibits) | i;
            }
        }
        p.out[i] = pass;
        p.rec[i] = rec;
    }
}

__device__ __forceinline__ uint32_t rule_of_slot(const PArgs& p, uint64_t g) {
    uint32_t lo = 0, hi = p.n_rules;  // rules sorted by table_base; slot g belongs to the last base <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (p.rules[mid].table_base <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The millisecond table in LDS (the hot-parameter walkers): request index -> exact timestamp (requests are
// time-ordered), so a walker reads nothing per request but its sorted record.
__shared__ uint32_t p_sms[kPLdsMs];
__shared__ uint16_t p_sbk[kPcBuckets];  // the millisecond of request b << bshift
__shared__ uint32_t p_nms;   // table entries, 0: read the timestamps
__shared__ uint32_t p_nbk;
__shared__ int64_t p_t0;

__device__ __forceinline__ void p_stage_ms(const PArgs& p) {
    const uint32_t np = *p.mnp;
    const bool lds = np <= kPLdsMs;
    const uint32_t nb = (uint32_t)((p.n - 1) >> p.bshift) + 1;
    for (uint32_t x = threadIdx.x; lds && x < np; x += blockDim.x) p_sms[x] = p.msb[x];
    for (uint32_t x = threadIdx.x; lds && x < nb; x += blockDim.x) p_sbk[x] = p.mbk[x];
    if (threadIdx.x == 0) {
        p_nms = lds ? np : 0u;
        p_nbk = nb;
        p_t0 = *p.mt0;
    }
    __syncthreads();
}

// The request's bucket bounds its millisecond to [first request's, next bucket's first request's]: a step or two
// of binary search instead of twelve (as pace.hip's pc_ts).
__device__ __forceinline__ int64_t p_ts(const PArgs& p, uint32_t idx) {
    const uint32_t np = p_nms;
    if (np == 0) return p.req[idx].ts_ms;
    const uint32_t b = idx >> p.bshift;
    uint32_t lo = p_sbk[b], hi = b + 1 < p_nbk ? (uint32_t)p_sbk[b + 1] + 1u : np;  // table[lo] <= idx (entry 0 unused)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (p_sms[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return p_t0 + (int64_t)lo;
}

struct PDec {
    uint32_t idx;
    int64_t acq;
};

__device__ __forceinline__ PDec p_dec(const PArgs& p, uint64_t rec) {
    PDec d;
    d.idx = (uint32_t)(rec & p.imask);
    const uint32_t ac = (uint32_t)(rec >> p.ibits) & 255u;
    d.acq = ac == kPAesc ? (int64_t)p.req[d.idx].acquire : (int64_t)ac;
    return d;
}

// Sequential replay of slot g's records from position s on (one lane), until the slot changes.
__device__ void pwalk_serial(const PArgs& p, uint64_t g, uint64_t s) {
    const uint32_t ri = rule_of_slot(p, g);
    const PRule r = p.rules[ri];
    PSlot& slot = p.table[g];
    const uint64_t value = slot.value;  // the side slot's word stays ~0, which is its value
    const int64_t tc = param_token_count(p, r, value);
    PState st{slot.time, slot.tokens, slot.flags};
    uint64_t rec = p.rec_sorted[s];
    for (uint64_t j = s; (rec >> p.gshift) == g;) {
        const uint64_t nrec = ++j < p.n ? p.rec_sorted[j] : ~0ull;  // issued before this request is decided
        const PDec d = p_dec(p, rec);
        rec = nrec;
        const int64_t t = p_ts(p, d.idx);
        bool ok;
        if (r.behavior == 2) ok = param_throttle_step(st, throttle_cost(r, tc, d.acq), r.max_queueing_ms, t);
        else ok = param_default_step(st, tc, tc + r.burst, r.duration_sec * 1000, t, d.acq);
        if (ok) p.out[d.idx] = 1;
    }
    slot.time = st.time;
    slot.tokens = st.tokens;
    slot.flags = st.flags;
}

// One lane per segment of at most short_max records, from k_seg's length-class lists (longest class first, so the
// lanes of a wave walk segments of similar length).
__global__ void __launch_bounds__(256) k_pwalk_short(PArgs p, BatchArgs sg) {
    if (*p.err & ~kErrNonPositive) return;
    p_stage_ms(p);
    uint32_t total = 0;
    for (int k = 0; k < kClasses; ++k) total += sg.short_count[k];
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
        uint32_t r0 = u;
        int k = kClasses - 1;
        while (r0 >= sg.short_count[k]) r0 -= sg.short_count[k--];
        const uint64_t j = sg.short_list[sg.class_off[k] + r0];
        pwalk_serial(p, p.rec_sorted[j] >> p.gshift, j);
    }
}

template <class Pred>
__device__ __forceinline__ uint64_t pwave_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
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

__device__ __forceinline__ int64_t pwave_scan(int64_t v, int lane) {
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up((long long)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}

__device__ __forceinline__ int64_t pwave_sum(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((long long)v, o, 64);
    return v;
}

// Token bucket for one hot (rule, value): sequential semantics, 64 requests per step.
//   - first sight and refill attempts (t − time > duration) are resolved one request at a time;
//   - between refills the bucket only pays out: the admit step passes the longest prefix whose running
//     token count stays >= 0, the skip step passes the next request that fits on its own;
//   - when fewer tokens remain than any request asks (all acquireCounts >= 1 in the batch), every request
//     up to the refill time is blocked: jump to the first one after it.
__device__ void pwalk_wave_default(const PArgs& p, const PRule& r, int64_t tc, PState& st, uint64_t s, uint64_t e) {
    const int lane = (int)__lane_id();
    const int64_t maxc = tc + r.burst;
    const int64_t dur_ms = r.duration_sec * 1000;
    const bool all_positive = !(*p.err & kErrNonPositive);
    uint64_t pos = s;
    while (pos < e) {
        // sequential head: first sight / refill zone
        {
            const PDec d = p_dec(p, p.rec_sorted[pos]);
            const int64_t t = p_ts(p, d.idx);
            if (!(st.flags & 1u) || t - st.time > dur_ms) {
                if (param_default_step(st, tc, maxc, dur_ms, t, d.acq) && lane == 0) p.out[d.idx] = 1;
                ++pos;
                continue;
            }
        }
        // no-refill zone: requests with t <= time + duration
        const int64_t zone_end_t = st.time + dur_ms;
        const uint64_t z = gallop_search(pos, e, [&](uint64_t q) {
            return p_ts(p, (uint32_t)(p.rec_sorted[q] & p.imask)) > zone_end_t;
        }, lane);
        while (pos < z) {
            if (all_positive && st.tokens < 1) {  // nothing fits until the refill: all blocked
                pos = z;
                break;
            }
            const uint64_t j = pos + (uint64_t)lane;
            const bool act = j < z;
            PDec d{0, 0};
            if (act) d = p_dec(p, p.rec_sorted[j]);
            const uint32_t idx = d.idx;
            const int64_t acq = d.acq;
            uint64_t pending = __ballot(act);
            while (pending) {
                const bool pl = (pending >> lane) & 1ull;
                const int64_t ex = pwave_scan(pl ? acq : 0, lane);
                const bool fail = pl && !(st.tokens - ex - acq >= 0);
                const uint64_t fails = __ballot(fail);
                const uint64_t pass = fails ? (pending & ((1ull << __builtin_ctzll(fails)) - 1ull)) : pending;
                if (pass) {
                    if ((pass >> lane) & 1ull) p.out[idx] = 1;
                    st.tokens -= pwave_sum(((pass >> lane) & 1ull) ? acq : 0);
                }
                if (!fails) break;
                const int f = __builtin_ctzll(fails);
                pending &= ~((2ull << f) - 1ull);  // f is blocked
                // skip: the next request that fits on its own
                const uint64_t fit = __ballot(((pending >> lane) & 1ull) && st.tokens - acq >= 0);
                if (!fit) break;
                pending &= ~((1ull << __builtin_ctzll(fit)) - 1ull);
            }
            pos += 64;
            if (pos > z) pos = z;
        }
    }
}

// Throttle (leaky bucket) for one hot (rule, value): 64 requests per step, the first request in the
// step that would be admitted advances the recorder, repeated until none in the step is.
__device__ void pwalk_wave_throttle(const PArgs& p, const PRule& r, int64_t tc, PState& st, uint64_t s, uint64_t e) {
    const int lane = (int)__lane_id();
    for (uint64_t base = s; base < e; base += 64) {
        const uint64_t j = base + (uint64_t)lane;
        const bool act = j < e;
        uint32_t idx = 0;
        int64_t t = 0, cost = 0;
        if (act) {
            const PDec d = p_dec(p, p.rec_sorted[j]);
            idx = d.idx;
            t = p_ts(p, idx);
            cost = throttle_cost(r, tc, d.acq);
        }
        uint64_t pending = __ballot(act);
        while (pending) {
            if (!(st.flags & 1u)) {  // first sight: the first pending request passes
                const int f = __builtin_ctzll(pending);
                const int64_t tf = __shfl((long long)t, f, 64);
                st.flags |= 1u;
                st.time = tf;
                if (lane == f) p.out[idx] = 1;
                pending &= ~(1ull << f);
                continue;
            }
            const int64_t expected = st.time + cost;
            const bool ok = ((pending >> lane) & 1ull) && (expected <= t || expected - t < r.max_queueing_ms);
            const uint64_t m = __ballot(ok);
            if (!m) break;
            const int f = __builtin_ctzll(m);
            const int64_t tf = __shfl((long long)t, f, 64);
            const int64_t ef = __shfl((long long)expected, f, 64);
            st.time = tf;
            if (ef - tf > 0) st.time = ef;
            if (lane == f) p.out[idx] = 1;
            pending &= ~((2ull << f) - 1ull);
        }
    }
}

__global__ void __launch_bounds__(256) k_pwalk_long(PArgs p) {
    if (*p.err & ~kErrNonPositive) return;
    p_stage_ms(p);
    const uint32_t cnt = *p.long_count;
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const int lane = (int)__lane_id();
    for (uint32_t w = wave; w < cnt; w += nwaves) {
        const uint64_t s = p.long_list[w];
        const uint64_t g = p.rec_sorted[s] >> p.gshift;
        const uint64_t e = gallop_search(s + (p.short_max ? p.short_max : 1), p.n, [&](uint64_t q) {
            return (p.rec_sorted[q] >> p.gshift) != g;
        }, lane);
        const uint32_t ri = rule_of_slot(p, g);
        const PRule r = p.rules[ri];
        PSlot& slot = p.table[g];
        const uint64_t value = slot.value;
        const int64_t tc = param_token_count(p, r, value);
        PState st{slot.time, slot.tokens, slot.flags};
        if (r.behavior == 2) pwalk_wave_throttle(p, r, tc, st, s, e);
        else pwalk_wave_default(p, r, tc, st, s, e);
        if (lane == 0) {
            slot.time = st.time;
            slot.tokens = st.tokens;
            slot.flags = st.flags;
        }
    }
}

__global__ void k_pfinish(PArgs p) {
    if ((*p.err & ~kErrNonPositive) == 0 && p.n > 0) *p.last_ts = p.req[p.n - 1].ts_ms;
}

__global__ void __launch_bounds__(256) k_ptable_clear(PSlot* table, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        PSlot s;
        s.value = kEmptyValue;
        s.flags = 0;
        s.pad = 0;
        s.time = 0;
        s.tokens = 0;
        table[i] = s;
    }
}

static unsigned pgrid(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

hipError_t launch_param_clear(PSlot* table, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ptable_clear, dim3(pgrid(n, 8192)), dim3(256), 0, stream, table, n);
    return hipGetLastError();
}

hipError_t launch_param_batch(const PArgs& p, const BatchArgs& sg, uint64_t* a_buf, uint64_t* b_buf, uint32_t* hist,
                              int lo_bit, int hi_bit, uint64_t** sorted_out, hipStream_t stream, hipStream_t aux,
                              hipEvent_t fork, hipEvent_t join) {
    const uint64_t sentinel = p.total_slots << p.gshift;
    lds_poison(stream);
    hipLaunchKernelGGL(k_pprep, dim3(pgrid(p.n, 8192)), dim3(256), 0, stream, p, sentinel);
    uint64_t* sorted = nullptr;
    hipError_t e = radix_sort_records(a_buf, b_buf, p.n, lo_bit, hist, &sorted, stream, hi_bit);
    if (e != hipSuccess) return e;
    PArgs q = p;
    q.rec_sorted = sorted;
    *sorted_out = sorted;
    // segments of the sorted records in length-class lists (k_seg; its error word is a zero word: kErrNonPositive
    // is not an error), then the wave walker on aux beside the lane walker
    BatchArgs sgb = sg;
    sgb.n = p.n;
    sgb.rec_sorted = sorted;
    sgb.kshift = p.gshift;
    sgb.K = (uint32_t)p.total_slots;
    sgb.long_list = p.long_list;
    sgb.long_count = p.long_count;
    sgb.short_max = p.short_max;
    e = launch_seg(sgb, stream);
    if (e != hipSuccess) return e;
    const uint64_t max_long = p.n / ((uint64_t)p.short_max + 1) + 1;
    e = hipEventRecord(fork, stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pwalk_long, dim3(pgrid(max_long * 64, 2048)), dim3(256), 0, aux, q);
    hipLaunchKernelGGL(k_pwalk_short, dim3(pgrid(p.n / 4, 8192)), dim3(256), 0, stream, q, sgb);
    e = hipEventRecord(join, aux);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, join, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pfinish, dim3(1), dim3(1), 0, stream, q);
    return hipGetLastError();
}

}  // namespace sg

// ------------------------------------------------------------------------------ ParamFlowSlot chain
//
// SphU.entry(resource, count, args...) through ParamFlowSlot.checkFlow (ParamFlowSlot.java:66-93): every param rule
// of the resource in load order on args[paramIdx] — a collection / array element by element with early exit
// (ParamFlowChecker.passLocalCheck :75-104), QPS rules through the token bucket / throttle steps above, THREAD rules
// against ParameterMetric's thread counts (:114-122), which passed entries raise and their exits lower
// (ParameterMetric.addThreadCount / decreaseThreadCount :125-239). A resource's rules share its ParameterMetric, so
// its events are walked in order on one lane (k_pswalk); different resources are independent.

namespace sg {

__global__ void __launch_bounds__(256) k_psprep(PSArgs s) {
    const uint64_t sentinel = (uint64_t)s.n_res << s.kshift;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < s.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_pslot_event e = s.ev[i];
        if (e.ts_ms < 0 || (i == 0 ? e.ts_ms < *s.last_ts : e.ts_ms < s.ev[i - 1].ts_ms)) atomicOr(s.err, kErrTime);
        if (i == 0 && s.emb && e.ts_ms < *s.cp_last_ts) atomicOr(s.err, kErrTime);  // the embedded server's param tokens
        sg_pslot_result r;
        r.pass = 1;
        r.rule = -1;
        s.out[i] = r;
        uint64_t rec = sentinel | i;
        if (e.resource < s.n_res && !e.args_null) {
            bool ok = (uint64_t)e.arg_begin + e.arg_count <= s.n_args;
            for (uint32_t k = 0; ok && k < e.arg_count; ++k) {
                const sg_pslot_arg a = s.args[e.arg_begin + k];
                const uint64_t m = a.kind == SG_ARG_COLLECTION ? a.value_count : (a.kind == SG_ARG_VALUE ? 1 : 0);
                ok = (uint64_t)a.value_begin + m <= s.n_values;
            }
            if (!ok) atomicOr(s.err, kErrBounds);
            else rec = ((uint64_t)(s.gkey ? s.gkey[e.resource] : e.resource) << s.kshift) | i;
        }
        s.rec[i] = rec;
    }
}

// One lane per resource segment of the sorted records (per key group on an embedded token server: the resources whose
// cluster-mode rules share a cluster param rule or a limiter, walked together in event order).
__global__ void __launch_bounds__(256) k_pswalk(PSArgs s, const uint64_t* sorted) {
    if (*s.err) return;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < s.n; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t key = (uint32_t)(sorted[p] >> s.kshift);
        if (key >= s.n_res || (p > 0 && (uint32_t)(sorted[p - 1] >> s.kshift) == key)) continue;
        for (uint64_t q = p; q < s.n; ++q) {
            const uint64_t rec = sorted[q];
            if ((uint32_t)(rec >> s.kshift) != key) break;
            const uint64_t i = rec & s.imask;
            const sg_pslot_event e = s.ev[i];
            const uint32_t res = e.resource;
            if (e.kind != SG_LOCAL_ENTRY) {  // ParamFlowStatisticExitCallback (passed entries only)
                ps_threads(s, res, e.arg_begin, e.arg_count, -1);
                continue;
            }
            const int32_t failed = ps_check_entry(s, res, e.ts_ms, e.count, e.arg_begin, e.arg_count);
            if (failed < 0) {
                ps_threads(s, res, e.arg_begin, e.arg_count, +1);
            } else {
                sg_pslot_result r;
                r.pass = 0;
                r.rule = failed;
                s.out[i] = r;
            }
        }
    }
}

__global__ void k_psfinish(PSArgs s) {
    if (*s.err == 0 && s.n > 0) {
        *s.last_ts = s.ev[s.n - 1].ts_ms;
        if (s.emb) *s.cp_last_ts = s.ev[s.n - 1].ts_ms;  // the embedded server's param tokens came up to here
    }
}

__global__ void __launch_bounds__(256) k_psclear(PSThread* tc, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        PSThread e;
        e.owner = 0;
        e.value = 0;
        e.count = 0;
        e.pad = 0;
        tc[i] = e;
    }
}

__global__ void k_psread(PSArgs s, uint32_t res, int32_t idx, uint64_t value, int64_t* out) {
    const int64_t x = ps_tc(s, res, idx, value, false);
    *out = x >= 0 ? s.tc[x].count : 0;
}

static unsigned psgrid(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

hipError_t launch_pslot_batch(PSArgs& s, uint64_t* b_buf, uint32_t* hist, hipStream_t stream) {
    hipLaunchKernelGGL(k_psprep, dim3(psgrid(s.n, 8192)), dim3(256), 0, stream, s);
    uint64_t* sorted = nullptr;
    hipError_t e = radix_sort_records(s.rec, b_buf, s.n, s.kshift, hist, &sorted, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pswalk, dim3(psgrid(s.n, 8192)), dim3(256), 0, stream, s, (const uint64_t*)sorted);
    hipLaunchKernelGGL(k_psfinish, dim3(1), dim3(1), 0, stream, s);
    return hipGetLastError();
}

hipError_t launch_pslot_clear(PSThread* tc, uint64_t n, hipStream_t stream) {
    hipLaunchKernelGGL(k_psclear, dim3(psgrid(n, 8192)), dim3(256), 0, stream, tc, n);
    return hipGetLastError();
}

hipError_t launch_pslot_thread_read(const PSArgs& s, uint32_t res, int32_t idx, uint64_t value, int64_t* out,
                                    hipStream_t stream) {
    hipLaunchKernelGGL(k_psread, dim3(1), dim3(1), 0, stream, s, res, idx, value, out);
    return hipGetLastError();
}

}  // namespace sg
