// pace.hip — RateLimiterController on the device: FlowRules with CONTROL_BEHAVIOR_RATE_LIMITER
// (sentinel-core/src/main/java/com/alibaba/csp/sentinel/slots/block/flow/controller/
//  RateLimiterController.java:46-91), a leaky bucket with one latestPassedTime per rule.
//
// Replay semantics: requests are applied in (ts, arrival) order per rule, currentTimeMillis() = the
// request's ts for the whole call (the reference reads the clock up to three times inside one call; a
// single-threaded caller sees them equal to the millisecond it started in). Under that order the
// second queue check after addAndGet (:76-80) can never fail, so one request is:
//   expected = latest + cost                  (Java long arithmetic: wraps)
//   expected <= now      → latest = now, pass with no sleep
//   expected - now > maxQ → block, latest unchanged
//   else                 → latest = expected, pass after sleeping expected - now ms
// A batch:
//   k_pace_prep     decides what never touches latestPassedTime (no rule, acquireCount <= 0 → pass), packs
//                   {rule | acquire code | request index} for the rest, outputs "blocked", writes the batch's
//                   millisecond table (the walkers' timestamps); a rule with count <= 0 blocks in its walker
//   radix sort by rule (sort.hip): each rule's requests contiguous, in arrival order
//   k_pace_seg      segment heads split by length into the lane walker's and the wave walker's lists
//   k_pace_short    one lane per rule with <= short_max requests, serial recurrence in registers
//   k_pace_long     (second stream, beside k_pace_short) one wave per longer rule: 64 requests per step; the first request of the step the
//                   bucket admits advances latestPassedTime, every pending request before it is blocked;
//                   requests before the earliest instant any of them could pass are jumped over by a
//                   64-way search (a saturated rule costs a few searches per admitted request)
#include "engine.h"

namespace sg {

namespace {

__device__ __forceinline__ int64_t pace_java_round(double a) {
    // java.lang.Math.round(double) (JDK 7u+): floor(a + 1/2) on the bits, saturating
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

// costTime = Math.round(1.0 * acquireCount / count * 1000) (:59)
__device__ __forceinline__ int64_t pace_cost(double count, int32_t acq) {
    return pace_java_round(1.0 * (double)acq / count * 1000.0);
}

__device__ __forceinline__ int64_t wrap_add(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);
}

// One canPass under the replay order; returns the sleep in ms or SG_PACE_BLOCKED.
__device__ __forceinline__ int32_t pace_step(int64_t& latest, int64_t cost, int32_t maxq, int64_t t) {
    const int64_t expected = wrap_add(latest, cost);
    if (expected <= t) {
        latest = t;
        return 0;
    }
    const int64_t wait = expected - t;  // > 0, no overflow: expected > t >= 0
    if (wait > (int64_t)maxq) return SG_PACE_BLOCKED;
    latest = expected;
    return (int32_t)wait;
}

// First q in [lo, hi) with pred(q) (pred monotone: false…false true…true), else hi; 64 probes per round.
template <class Pred>
__device__ __forceinline__ uint64_t pace_wave_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
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

// A window start for the wave walker: some q <= a with a - q < 64, a = the first q in [lo, hi) with pred(q)
// (monotone), hi if none. The walker's step takes 64 requests from q, and those before a are blocked anyway, so the
// search stops as soon as the bracket is 64 wide and its last round doubles as the step's load. One round of 64
// probes g + (lane - 32) w (clamped to [lo, hi - 1]) around a guess g brackets a; a guess that misses falls back to
// a gallop past the last probe or a 64-way search before the first.
template <class Pred>
__device__ __forceinline__ uint64_t pace_window(uint64_t lo, uint64_t hi, Pred pred, int lane) {
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
    return lo;
}

template <class Pred>
__device__ __forceinline__ uint64_t pace_guess_window(uint64_t lo, uint64_t hi, uint64_t g, uint64_t w, Pred pred,
                                                      int lane) {
    if (lo >= hi) return hi;
    const int64_t pq = (int64_t)g + ((int64_t)lane - 32) * (int64_t)w;
    const uint64_t q = pq < (int64_t)lo ? lo : (pq >= (int64_t)hi ? hi - 1 : (uint64_t)pq);
    const uint64_t m = __ballot(pred(q));
    if (m == 0) {  // a > every probe: bracket it by doubling steps past the last one
        const uint64_t l2 = (uint64_t)__shfl((long long)q, 63, 64) + 1;
        if (l2 >= hi) return hi;
        const uint64_t span = hi - l2;
        const uint64_t off = lane < 63 ? (1ull << lane) - 1ull : ~0ull;
        const uint64_t m2 = __ballot(off >= span || pred(l2 + off));
        const int f2 = __builtin_ctzll(m2);
        if (f2 == 0) return l2;
        const uint64_t b1 = l2 + ((1ull << f2) - 1ull);
        return pace_window(l2 + (1ull << (f2 - 1)), b1 < hi ? b1 + 1 : hi, pred, lane);
    }
    const int f = __builtin_ctzll(m);
    const uint64_t qf = (uint64_t)__shfl((long long)q, f, 64);
    const uint64_t qp = f == 0 ? lo : (uint64_t)__shfl((long long)q, f - 1, 64) + 1;
    return pace_window(qp, qf + 1, pred, lane);
}

}  // namespace

// Validation and the records. A request reads nothing but itself: its acquireCount rides in the record (8-bit code,
// 255 = read the request) and its timestamp is recovered from the batch's millisecond table (first request index of
// every millisecond), so neither the rule table nor the requests are gathered per request — count <= 0 (:53-55) is
// answered by the walkers once per rule.
constexpr uint32_t kPcAesc = 255;
constexpr uint32_t kPcLdsMs = 4096;  // millisecond table entries staged in LDS (a batch spanning <= 4 s)

__global__ void __launch_bounds__(256) k_pace_prep(PaceArgs p) {
    const uint64_t none = (uint64_t)p.n_rules << p.gshift;
    const int64_t t0 = p.req[0].ts_ms;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_pace_req q = p.req[i];
        const int64_t tp = i == 0 ? *p.last_ts : p.req[i - 1].ts_ms;
        if (q.ts_ms < 0 || q.ts_ms < tp) atomicOr(p.err, kErrTime);
        if (i == 0) {
            *p.mt0 = q.ts_ms;
        } else if (q.ts_ms > tp) {  // a new millisecond starts at i
            for (int64_t ms = (tp < t0 ? t0 : tp) + 1; ms <= q.ts_ms; ++ms) {
                const int64_t qq = ms - t0;
                if (qq >= (int64_t)kMaxPeriods) break;
                p.msb[qq] = (uint32_t)i;
            }
        }
        if (i == p.n - 1) *p.mnp = (uint32_t)min(q.ts_ms - t0 + 1, (int64_t)kMaxPeriods + 1);
        if ((i & ((1ull << p.bshift) - 1ull)) == 0) p.mbk[i >> p.bshift] = (uint16_t)min(max(q.ts_ms - t0, (int64_t)0), (int64_t)65535);
        uint64_t rec = none;
        int32_t out = SG_PACE_BLOCKED;  // a walked request passes by its walker; count <= 0 leaves it blocked
        if (q.rule >= p.n_rules || q.acquire <= 0) {
            out = 0;  // no rule for the resource / acquireCount <= 0 (:48-50)
        } else {
            const uint64_t ac = (uint64_t)q.acquire >= kPcAesc ? kPcAesc : (uint64_t)q.acquire;
            rec = ((uint64_t)q.rule << p.gshift) | (ac << p.ibits) | i;
        }
        p.out[i] = out;
        p.rec[i] = rec;
    }
}

__shared__ uint32_t pc_sms[kPcLdsMs];
__shared__ uint16_t pc_sbk[kPcBuckets];  // the millisecond of request b << bshift
__shared__ uint32_t pc_nms;  // table entries in LDS, 0: read the timestamps
__shared__ uint32_t pc_nbk;
__shared__ int64_t pc_t0;

__device__ __forceinline__ void pc_stage_ms(const PaceArgs& p) {
    const uint32_t np = *p.mnp;
    const bool lds = np <= kPcLdsMs;
    const uint32_t nb = (uint32_t)((p.n - 1) >> p.bshift) + 1;
    for (uint32_t x = threadIdx.x; lds && x < np; x += blockDim.x) pc_sms[x] = p.msb[x];
    for (uint32_t x = threadIdx.x; lds && x < nb; x += blockDim.x) pc_sbk[x] = p.mbk[x];
    if (threadIdx.x == 0) {
        pc_nms = lds ? np : 0u;
        pc_nbk = nb;
        pc_t0 = *p.mt0;
    }
    __syncthreads();
}

// A request's timestamp: the largest millisecond q whose first request index table[q] <= idx. Its bucket's first
// request and the next bucket's bound q to a few milliseconds (a bucket of a 16M batch holds 8192 requests), so the
// binary search takes a step or two instead of twelve.
__device__ __forceinline__ int64_t pc_ts(const PaceArgs& p, uint32_t idx) {
    const uint32_t np = pc_nms;
    if (np == 0) return p.req[idx].ts_ms;
    const uint32_t b = idx >> p.bshift;
    uint32_t lo = pc_sbk[b], hi = b + 1 < pc_nbk ? (uint32_t)pc_sbk[b + 1] + 1u : np;  // table[lo] <= idx (entry 0 unused)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pc_sms[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return pc_t0 + (int64_t)lo;
}

__device__ __forceinline__ int32_t pc_acq(const PaceArgs& p, uint64_t rec, uint32_t idx) {
    const uint32_t ac = (uint32_t)(rec >> p.ibits) & 255u;
    return ac == kPcAesc ? p.req[idx].acquire : (int32_t)ac;
}

// Segment head classes: 0 = not a head; 1 + c = a rule walked by one lane, in length class c (longer than
// kClassMax[c - 1], at most kClassMax[c] requests, class kClasses - 1 unbounded); kPcLong = a rule with more than
// short_max requests, walked by a wave. Segments are contiguous, so one probe per bound decides the length.
constexpr int kPcLong = kClasses + 1;
constexpr int kPcLists = kClasses + 1;  // list l < kClasses: lane-walker class l; kClasses: the wave walker's

__device__ __forceinline__ int pace_head_class(const PaceArgs& p, uint64_t j) {
    const uint64_t g = p.rec_sorted[j] >> p.gshift;
    if (g >= p.n_rules || (j > 0 && (p.rec_sorted[j - 1] >> p.gshift) == g)) return 0;
    auto longer = [&](uint64_t m) {  // the segment holds more than m requests
        const uint64_t e = j + m;
        return e < p.n && (p.rec_sorted[e] >> p.gshift) == g;
    };
    if (longer((uint64_t)p.short_max)) return kPcLong;
    int c = 0;
#pragma unroll
    for (int k = 0; k < kClasses - 1; ++k) c += (kClassMax[k] < p.short_max && longer(kClassMax[k])) ? 1 : 0;
    return 1 + c;
}

// Segment heads by class: the wave walker's list and the lane walker's length classes (a lane walker wave then
// holds rules of similar length: its time is its longest lane's). Each block owns a contiguous chunk: one pass
// classifies its records (classes kept in registers, 3 bits a round for the first 42 rounds) and counts its heads per
// list with LDS atomics, one global atomic per list reserves the block's slices, and the second pass places each head
// with an LDS atomic (the order within a list is free) — no second read of the records.
__global__ void __launch_bounds__(256) k_pace_seg(PaceArgs p, uint64_t chunk) {
    if (*p.err) return;
    __shared__ uint32_t tot[kPcLists], base[kPcLists];
    const int tid = threadIdx.x;
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < p.n ? lo + chunk : p.n;
    if (tid < kPcLists) tot[tid] = 0;
    __syncthreads();
    auto list_of = [](int c) { return c == kPcLong ? kClasses : c - 1; };
    uint64_t cls[2] = {0, 0};
    int r = 0;
    for (uint64_t j = lo + tid; j < hi; j += 256, ++r) {
        const int c = pace_head_class(p, j);
        if (r < 42) cls[r / 21] |= (uint64_t)c << (3 * (r % 21));
        if (c) atomicAdd(&tot[list_of(c)], 1u);
    }
    __syncthreads();
    if (tid < kPcLists) {
        const uint32_t t = tot[tid];
        base[tid] = t ? atomicAdd(&p.long_count[tid < kClasses ? 1 + tid : 0], t) : 0;
        tot[tid] = 0;
    }
    __syncthreads();
    r = 0;
    for (uint64_t j = lo + tid; j < hi; j += 256, ++r) {
        const int c = r < 42 ? (int)((cls[r / 21] >> (3 * (r % 21))) & 7ull) : pace_head_class(p, j);
        if (!c) continue;
        const int l = list_of(c);
        const uint32_t pos = base[l] + atomicAdd(&tot[l], 1u);
        if (l < kClasses) p.short_list[p.class_off[l] + pos] = (uint32_t)j;
        else p.long_list[pos] = (uint32_t)j;
    }
}

// One lane per rule of at most short_max requests, the longest length class first.
__global__ void __launch_bounds__(256) k_pace_short(PaceArgs p) {
    if (*p.err) return;
    pc_stage_ms(p);
    uint32_t cc[kClasses], total = 0;
#pragma unroll
    for (int c = 0; c < kClasses; ++c) {
        cc[c] = p.long_count[1 + c];
        total += cc[c];
    }
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < total; w += gridDim.x * blockDim.x) {
        uint32_t r0 = w;
        int c = kClasses - 1;
        while (c > 0 && r0 >= cc[c]) r0 -= cc[c--];
        const uint64_t j = p.short_list[p.class_off[c] + r0];
        const uint64_t g = p.rec_sorted[j] >> p.gshift;
        const PaceRule r = p.rules[g];
        if (!(r.count > 0.0)) continue;  // count <= 0 (:53-55): every request stays blocked
        int64_t latest = p.latest[g];
        uint64_t rec = p.rec_sorted[j];
        for (uint64_t k = j; (rec >> p.gshift) == g;) {  // the next record is loaded before this one is decided
            const uint64_t cur = rec;
            rec = ++k < p.n ? p.rec_sorted[k] : ~0ull;
            const uint32_t idx = (uint32_t)(cur & p.imask);
            const int32_t w8 = pace_step(latest, pace_cost(r.count, pc_acq(p, cur, idx)), r.max_queueing_ms, pc_ts(p, idx));
            if (w8 != SG_PACE_BLOCKED) p.out[idx] = w8;
        }
        p.latest[g] = latest;
    }
}

__global__ void __launch_bounds__(256) k_pace_long(PaceArgs p) {
    if (*p.err) return;
    pc_stage_ms(p);
    const uint32_t cnt = *p.long_count;
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const int lane = (int)__lane_id();
    for (uint32_t w = wave; w < cnt; w += nwaves) {
        const uint64_t s = p.long_list[w];
        const uint64_t g = p.rec_sorted[s] >> p.gshift;
        const PaceRule r = p.rules[g];
        if (!(r.count > 0.0)) continue;  // count <= 0 (:53-55): every request stays blocked
        // segment end: first record of another rule (records are sorted by rule)
        const uint64_t e = gallop_search(s + (p.short_max ? p.short_max : 1), p.n, [&](uint64_t q) {
            return (p.rec_sorted[q] >> p.gshift) != g;
        }, lane);
        int64_t latest = p.latest[g];
        // Every walked request has acquireCount >= 1 (k_pace_prep decides the rest), so its cost is at
        // least cost(1) and it can only pass at t >= latest + cost(1) - max(maxQ, 0): requests before that
        // instant are blocked without changing latestPassedTime, and the walker jumps over them.
        // The bound needs latest + cost(a) not to wrap for any acquireCount a: a wrapped sum is negative and
        // passes (Java long arithmetic), however early the request. cost is monotone in a, so checking the
        // largest int acquireCount covers them all; otherwise the walker takes every request in turn.
        const int64_t cost1 = pace_cost(r.count, 1);
        const int64_t cost_max = pace_cost(r.count, INT32_MAX);
        const int64_t slack = r.max_queueing_ms > 0 ? (int64_t)r.max_queueing_ms : 0;
        auto ts_at = [&](uint64_t q) { return pc_ts(p, (uint32_t)(p.rec_sorted[q] & p.imask)); };
        // With the millisecond table in LDS the horizon becomes a request index (the first request of its
        // millisecond) and the search compares record indices, no timestamp lookups. Its first probes are
        // guessed: the rule's requests are spread over the batch at density (e - s) / (index span), so the
        // answer lies about (index distance) x density past the last admitted request, within a few sqrt of it.
        const bool tab = pc_nms != 0;
        uint64_t hq = s;
        uint32_t hidx = (uint32_t)(p.rec_sorted[s] & p.imask);
        const double dens = (double)(e - s) / ((double)(uint32_t)(p.rec_sorted[e - 1] & p.imask) - (double)hidx + 1.0);
        bool seek = true;  // latestPassedTime moved since the last search
        uint64_t base = s;
        while (base < e) {
            int64_t horizon, top;
            if (seek && !__builtin_add_overflow(latest, cost_max, &top) && !__builtin_add_overflow(latest, cost1, &horizon)) {
                horizon -= slack;
                seek = false;
                if (tab) {
                    const int64_t x = horizon - pc_t0;
                    if (x >= (int64_t)pc_nms) break;  // past the batch's last millisecond: the rest is blocked
                    if (x >= 1) {
                        const uint32_t ih = pc_sms[x];
                        const double d = ((double)ih - (double)hidx) * dens;
                        const uint64_t gq = hq + (d > 0.0 ? (uint64_t)d : 0ull);
                        const uint64_t w = (uint64_t)(sqrt(d > 0.0 ? d : 0.0) * 0.125) + 1ull;
                        base = pace_guess_window(base, e, gq < base ? base : gq, w, [&](uint64_t q) {
                            return (uint32_t)(p.rec_sorted[q] & p.imask) >= ih;
                        }, lane);
                    }
                } else if (ts_at(base) < horizon) {
                    base = gallop_search(base, e, [&](uint64_t q) { return ts_at(q) >= horizon; }, lane);
                }
                continue;
            }
            const uint64_t j = base + (uint64_t)lane;
            const bool act = j < e;
            uint32_t idx = 0;
            int64_t t = 0, cost = 0;
            if (act) {
                const uint64_t rec = p.rec_sorted[j];
                idx = (uint32_t)(rec & p.imask);
                t = pc_ts(p, idx);
                cost = pace_cost(r.count, pc_acq(p, rec, idx));
            }
            uint64_t pending = __ballot(act);
            int lastf = -1;
            while (pending) {
                const int64_t expected = wrap_add(latest, cost);
                const bool ok = ((pending >> lane) & 1ull) && (expected <= t || expected - t <= (int64_t)r.max_queueing_ms);
                const uint64_t m = __ballot(ok);
                if (!m) break;  // every pending request of this step is blocked
                const int f = __builtin_ctzll(m);
                const int64_t tf = __shfl((long long)t, f, 64);
                const int64_t ef = __shfl((long long)expected, f, 64);
                if (lane == f) p.out[idx] = ef <= tf ? 0 : (int32_t)(ef - tf);
                latest = ef <= tf ? tf : ef;
                pending &= ~((2ull << f) - 1ull);
                lastf = f;
            }
            if (lastf >= 0) {
                seek = true;
                hq = base + (uint64_t)lastf;
                hidx = (uint32_t)__shfl((int)idx, lastf, 64);
            }
            base += 64;
        }
        if (lane == 0) p.latest[g] = latest;
    }
}

__global__ void k_pace_finish(PaceArgs p) {
    if (*p.err == 0 && p.n > 0) *p.last_ts = p.req[p.n - 1].ts_ms;
}

static unsigned pace_grid(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

hipError_t launch_pace_batch(const PaceArgs& p, uint64_t* a_buf, uint64_t* b_buf, uint32_t* hist, int lo_bit, int hi_bit,
                             uint64_t** sorted_out, hipStream_t stream, hipStream_t aux, hipEvent_t fork,
                             hipEvent_t join) {
    hipLaunchKernelGGL(k_pace_prep, dim3(pace_grid(p.n, 8192)), dim3(256), 0, stream, p);
    uint64_t* sorted = nullptr;
    hipError_t e = radix_sort_records(a_buf, b_buf, p.n, lo_bit, hist, &sorted, stream, hi_bit);
    if (e != hipSuccess) return e;
    PaceArgs q = p;
    q.rec_sorted = sorted;
    *sorted_out = sorted;
    const uint64_t chunk = ((p.n + 2047) / 2048 + 255) / 256 * 256;  // <= 2048 blocks, whole rounds of 256
    lds_poison(stream);
    hipLaunchKernelGGL(k_pace_seg, dim3((unsigned)((p.n + chunk - 1) / chunk)), dim3(256), 0, stream, q, chunk);
    if ((e = hipEventRecord(fork, stream)) != hipSuccess || (e = hipStreamWaitEvent(aux, fork, 0)) != hipSuccess) return e;
    const uint64_t max_long = p.n / ((uint64_t)p.short_max + 1) + 1;
    hipLaunchKernelGGL(k_pace_long, dim3(pace_grid(max_long * 64, 2048)), dim3(256), 0, aux, q);
    hipLaunchKernelGGL(k_pace_short, dim3(pace_grid(p.n, 4096)), dim3(256), 0, stream, q);
    if ((e = hipEventRecord(join, aux)) != hipSuccess || (e = hipStreamWaitEvent(stream, join, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pace_finish, dim3(1), dim3(1), 0, stream, q);
    return hipGetLastError();
}

}  // namespace sg
