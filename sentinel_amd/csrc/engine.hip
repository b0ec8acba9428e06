// engine.hip — gfx950 kernels of the batched cluster flow-decision engine.
//
// A batch of token requests (time-ordered) is decided exactly as the Java token server would decide
// them one by one: DefaultTokenService.requestToken → ClusterFlowChecker.acquireClusterToken
// (srv/flow/ClusterFlowChecker.java:55-112) over a per-flowId ClusterMetric sliding window
// (srv/flow/statistic/metric/ClusterMetric.java, ClusterMetricLeapArray.java, core LeapArray.java).
//
// Pipeline (one batch):
//   k_prep        request order → packed 64-bit records {flowId index | request index | acquire,prio},
//                 validation (BAD_REQUEST / NO_RULE_EXISTS written directly), timestamp checks, and the
//                 window-period boundary table (timestamps are only ever needed as window periods).
//   radix sort    stable partition of the records by flowId (sort.hip; time order kept within a flowId).
//   k_walk_short  one lane per flowId segment of <= kShortMax requests: sequential replay.
//   k_walk_long   one wave per longer segment: bucket ring in registers (lane j = slot j), requests
//                 64 at a time with a wave prefix-scan "admit until the first failure" step and a
//                 ballot "skip blocked requests" step; a failure that needs the occupy path is
//                 resolved wave-uniformly.
//   k_finish      advance the handle's last timestamp.
//
// Only PASS and WAITING are ever read back by decisions; every other counter is an accumulator.
// Exactness: all window arithmetic is int64 (wrapping, -fwrapv), the QPS comparisons are IEEE double
// with the reference's operation order and -ffp-contract=off (no FMA contraction).
#include "engine.h"

namespace sg {

// ----------------------------------------------------------------------------------------- helpers

__device__ __forceinline__ int32_t java_d2i(double x) {
    // JLS §5.1.3: NaN → 0, saturate, truncate toward zero.
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ int64_t wave_sum(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((long long)v, o, 64);
    return v;
}

__device__ __forceinline__ int64_t wave_excl_scan(int64_t v, int lane) {
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up((long long)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    return x - v;
}

__device__ __forceinline__ int64_t bcast64(int64_t v, int src) { return __shfl((long long)v, src, 64); }
__device__ __forceinline__ int bcast32(int v, int src) { return __shfl(v, src, 64); }

__device__ __forceinline__ uint64_t below(int f) { return f >= 64 ? ~0ull : ((1ull << f) - 1ull); }

__device__ __forceinline__ void store_result(sg_result* out, uint32_t idx, int32_t st, int32_t rem, int32_t wait) {
    sg_result r;
    r.status = st;
    r.remaining = rem;
    r.wait_ms = wait;
    out[idx] = r;
}

// Window period q (0-based within the batch) of request `idx`: the largest q with bnd[q] <= idx.
__device__ __forceinline__ uint32_t period_of(const uint32_t* bnd, uint32_t np, uint32_t idx) {
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (bnd[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct Decoded {
    uint32_t idx;
    int64_t acq;
    bool prio;
};

__device__ __forceinline__ Decoded decode(const BatchArgs& a, uint64_t rec) {
    Decoded d;
    d.idx = (uint32_t)((rec >> a.abits) & a.imask);
    uint64_t ac = rec & a.amask;
    d.prio = (ac & 1ull) != 0;
    uint64_t q = ac >> 1;
    d.acq = (q == a.aesc) ? (int64_t)a.req[d.idx].acquire : (int64_t)q;
    return d;
}

// ------------------------------------------------------------------------------------------- prep

__global__ void __launch_bounds__(256) k_prep(BatchArgs a) {
    const uint64_t n = a.n;
    const int64_t t0 = a.req[0].ts_ms;
    const uint64_t sentinel = (uint64_t)a.K << a.kshift;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_req r = a.req[i];
        const int64_t t = r.ts_ms;
        if (i == 0) {
            if (t < 0 || t < *a.last_ts) atomicOr(a.err, kErrTime);
            for (int w = 0; w < a.n_wl; ++w) a.p0[w] = t / a.wl[w];
        } else {
            const int64_t tp = a.req[i - 1].ts_ms;
            if (t < tp || t < 0) {
                atomicOr(a.err, kErrTime);
            } else {
                for (int w = 0; w < a.n_wl; ++w) {
                    const int64_t wl = a.wl[w];
                    const int64_t P0 = t0 / wl, Pp = tp / wl, Pi = t / wl;
                    for (int64_t p = Pp + 1; p <= Pi; ++p) {
                        const int64_t q = p - P0;
                        if (q >= (int64_t)kMaxPeriods) {
                            atomicOr(a.err, kErrPeriods);
                            break;
                        }
                        a.bnd[(size_t)w * kMaxPeriods + q] = (uint32_t)i;
                    }
                }
            }
        }
        if (i == n - 1) {
            for (int w = 0; w < a.n_wl; ++w) {
                const int64_t q = t / a.wl[w] - t0 / a.wl[w] + 1;
                a.np[w] = q > (int64_t)kMaxPeriods ? kMaxPeriods : (uint32_t)q;
            }
        }
        // DefaultTokenService.requestToken validation, srv/flow/DefaultTokenService.java:39-47, 87-89
        const uint32_t key = r.key & SG_KEY_INDEX;
        uint64_t rec;
        if (key == SG_KEY_BAD || r.acquire <= 0) {
            store_result(a.out, (uint32_t)i, SG_STATUS_BAD_REQUEST, 0, 0);
            rec = sentinel;
        } else if (key >= a.K) {
            store_result(a.out, (uint32_t)i, SG_STATUS_NO_RULE_EXISTS, 0, 0);
            rec = sentinel;
        } else {
            uint64_t q = (uint64_t)(uint32_t)r.acquire;
            if (q > a.aesc) q = a.aesc;
            const uint64_t ac = (q << 1) | (uint64_t)(r.key >> 31);
            rec = ((uint64_t)key << a.kshift) | ((uint64_t)i << a.abits) | ac;
        }
        a.rec[i] = rec;
    }
}

// ------------------------------------------------------------------------------------ the decision

// State of the current window period of one flowId, shared by both walkers. All fields are
// wave-uniform in the wave walker.
struct PeriodState {
    int64_t cur[SG_NUM_EVENTS];  // the current bucket (slot I) being accumulated
    int64_t wo_pass;             // Σ PASS over the other valid buckets
    int64_t wo_wait;             // Σ WAITING over the other valid buckets
    int64_t head_other;          // PASS of the valid head bucket (slot (P+1) % S) when it is not slot I
    int64_t occ_pass, occ_req;   // ClusterMetricLeapArray.occupyCounter
};

// The failure branch of acquireClusterToken for one request whose normal check failed
// (ClusterFlowChecker.java:83-111 with ClusterMetric.tryOccupyNext/canOccupy :79-98).
// Returns the status and sets *wait.
__device__ __forceinline__ int32_t decide_fail(const Rule& R, double max_occ_ratio, PeriodState& ps,
                                               int64_t acq, bool prio, int32_t* wait) {
    *wait = 0;
    if (prio) {
        const double occupy_avg = (double)(ps.wo_wait + ps.cur[SG_EV_WAITING]) / R.isec;
        if (occupy_avg <= max_occ_ratio * R.thr) {
            const double latest = (double)(ps.wo_pass + ps.cur[SG_EV_PASS]) / R.isec;
            const int64_t head = (R.S == 1) ? ps.cur[SG_EV_PASS] : ps.head_other;
            if (latest + (double)(acq + ps.occ_pass) - (double)head <= R.thr) {
                ps.occ_pass += acq;  // addOccupyPass, ClusterMetricLeapArray.java:73-77
                ps.occ_req += 1;
                ps.cur[SG_EV_WAITING] += acq;
                if (R.wait_ms > 0) {
                    *wait = R.wait_ms;
                    return SG_STATUS_SHOULD_WAIT;
                }
            }
        }
    }
    ps.cur[SG_EV_BLOCK] += acq;
    ps.cur[SG_EV_BLOCK_REQUEST] += 1;
    if (prio) ps.cur[SG_EV_OCCUPIED_BLOCK] += acq;
    return SG_STATUS_BLOCKED;
}

// currentWindow(t) for slot I at the first request of a new period (LeapArray.java:116-202 with
// ClusterMetricLeapArray.resetWindowTo/transferOccupyToBucket :49-71): `start`/`c` = slot I as stored.
__device__ __forceinline__ void open_bucket(PeriodState& ps, int64_t start, const int64_t* c, int64_t ws) {
    if (start == ws) {
#pragma unroll
        for (int e = 0; e < SG_NUM_EVENTS; ++e) ps.cur[e] = c[e];
        return;
    }
#pragma unroll
    for (int e = 0; e < SG_NUM_EVENTS; ++e) ps.cur[e] = 0;
    if (start != INT64_MIN && ps.occ_req > 0) {  // reset (not creation) transfers the occupied quota
        ps.cur[SG_EV_OCCUPIED_PASS] += ps.occ_pass;
        ps.cur[SG_EV_PASS] += ps.occ_pass;
        ps.cur[SG_EV_PASS_REQUEST] += ps.occ_req;
        ps.occ_pass = 0;
        ps.occ_req = 0;
    }
}

// ------------------------------------------------------------------------ serial walker (short)

__device__ void walk_serial(const BatchArgs& a, uint32_t k, uint64_t s, uint64_t e) {
    const Rule R = a.rules[k];
    Bucket* ring = a.ring + (size_t)k * a.stride;
    const uint32_t* bnd = a.bnd + (size_t)R.wl_idx * kMaxPeriods;
    const int64_t P0 = a.p0[R.wl_idx];
    const uint32_t np = a.np[R.wl_idx];
    PeriodState ps;
    {
        const Occ o = a.occ[k];
        ps.occ_pass = o.pass;
        ps.occ_req = o.pass_req;
    }
    int64_t curP = INT64_MIN, ws = 0;
    int I = -1;
    for (uint64_t j = s; j < e; ++j) {
        const Decoded d = decode(a, a.rec_sorted[j]);
        const int64_t P = P0 + (int64_t)period_of(bnd, np, d.idx);
        if (P != curP) {
            if (I >= 0) {
                ring[I].start = ws;
#pragma unroll
                for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[I].c[ev] = ps.cur[ev];
            }
            curP = P;
            I = (int)(P % R.S);
            ws = P * R.wl;
            {
                int64_t c[SG_NUM_EVENTS];
#pragma unroll
                for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ring[I].c[ev];
                open_bucket(ps, ring[I].start, c, ws);
            }
            // values(t): a slot j != I is valid iff its start >= ws - (S-1)*wl (LeapArray.java:270-272
            // with starts on window boundaries; only slot I can sit exactly `interval` behind).
            const int64_t lo = ws - (int64_t)(R.S - 1) * R.wl;
            const int h = (int)((P + 1) % R.S);
            ps.wo_pass = ps.wo_wait = ps.head_other = 0;
            for (int q = 0; q < R.S; ++q) {
                if (q == I) continue;
                const int64_t st = ring[q].start;
                if (st != INT64_MIN && st >= lo) {
                    const int64_t pp = ring[q].c[SG_EV_PASS];
                    ps.wo_pass += pp;
                    ps.wo_wait += ring[q].c[SG_EV_WAITING];
                    if (q == h) ps.head_other = pp;
                }
            }
        }
        // ClusterFlowChecker.acquireClusterToken, :67-81
        const double latest = (double)(ps.wo_pass + ps.cur[SG_EV_PASS]) / R.isec;
        const double next_remaining = R.thr - latest - (double)d.acq;
        if (next_remaining >= 0) {
            ps.cur[SG_EV_PASS] += d.acq;
            ps.cur[SG_EV_PASS_REQUEST] += 1;
            if (d.prio) ps.cur[SG_EV_OCCUPIED_PASS] += d.acq;
            store_result(a.out, d.idx, SG_STATUS_OK, java_d2i(next_remaining), 0);
        } else {
            int32_t wait;
            const int32_t st = decide_fail(R, a.max_occ_ratio, ps, d.acq, d.prio, &wait);
            store_result(a.out, d.idx, st, 0, wait);
        }
    }
    if (I >= 0) {
        ring[I].start = ws;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[I].c[ev] = ps.cur[ev];
    }
    Occ o;
    o.pass = ps.occ_pass;
    o.pass_req = ps.occ_req;
    a.occ[k] = o;
}

__global__ void __launch_bounds__(256) k_walk_short(BatchArgs a) {
    if (*a.err) return;
    const uint64_t n = a.n;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t rec = a.rec_sorted[j];
        const uint32_t k = (uint32_t)(rec >> a.kshift);
        if (k >= a.K) continue;
        if (j > 0 && (uint32_t)(a.rec_sorted[j - 1] >> a.kshift) == k) continue;  // not a segment head
        uint64_t e = j + 1;
        const uint64_t smax = a.short_max;
        while (e < n && e - j <= smax && (uint32_t)(a.rec_sorted[e] >> a.kshift) == k) ++e;
        if (e - j > smax) {
            const uint32_t pos = atomicAdd(a.long_count, 1u);
            a.long_list[pos] = (uint32_t)j;
            continue;
        }
        walk_serial(a, k, j, e);
    }
}

// --------------------------------------------------------------------------- wave walker (long)

__device__ void walk_wave(const BatchArgs& a, uint32_t k, uint64_t s, uint64_t e) {
    const int lane = lane_id();
    const Rule R = a.rules[k];
    const int S = R.S;
    Bucket* ring = a.ring + (size_t)k * a.stride;
    const uint32_t* bnd = a.bnd + (size_t)R.wl_idx * kMaxPeriods;
    const int64_t P0 = a.p0[R.wl_idx];
    const uint32_t np = a.np[R.wl_idx];
    const double max_occ = a.max_occ_ratio;

    // lane q < S holds slot q of the ring
    int64_t st = INT64_MIN;
    int64_t c[SG_NUM_EVENTS];
#pragma unroll
    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = 0;
    if (lane < S) {
        st = ring[lane].start;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ring[lane].c[ev];
    }
    PeriodState ps;
    {
        const Occ o = a.occ[k];
        ps.occ_pass = o.pass;
        ps.occ_req = o.pass_req;
    }
#pragma unroll
    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ps.cur[ev] = 0;
    ps.wo_pass = ps.wo_wait = ps.head_other = 0;
    int64_t curP = INT64_MIN, ws = 0;
    int I = -1;

    for (uint64_t base = s; base < e; base += 64) {
        const uint64_t j = base + (uint64_t)lane;
        const bool act = j < e;
        Decoded d;
        d.idx = 0;
        d.acq = 0;
        d.prio = false;
        int64_t P = INT64_MAX;
        if (act) {
            d = decode(a, a.rec_sorted[j]);
            P = P0 + (int64_t)period_of(bnd, np, d.idx);
        }
        uint64_t todo = __ballot(act);
        while (todo) {
            const int f0 = __builtin_ctzll(todo);
            const int64_t Prun = bcast64(P, f0);
            if (Prun != curP) {
                // close the current bucket into its owner lane, open the bucket of period Prun
                if (I >= 0 && lane == I) {
                    st = ws;
#pragma unroll
                    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ps.cur[ev];
                }
                curP = Prun;
                I = (int)(Prun % S);
                ws = Prun * R.wl;
                {
                    int64_t cI[SG_NUM_EVENTS];
#pragma unroll
                    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = bcast64(c[ev], I);
                    open_bucket(ps, bcast64(st, I), cI, ws);
                }
                const int64_t lo = ws - (int64_t)(S - 1) * R.wl;
                const bool valid = lane < S && lane != I && st != INT64_MIN && st >= lo;
                ps.wo_pass = wave_sum(valid ? c[SG_EV_PASS] : 0);
                ps.wo_wait = wave_sum(valid ? c[SG_EV_WAITING] : 0);
                const int h = (int)((Prun + 1) % S);
                ps.head_other = (h != I) ? bcast64(valid ? c[SG_EV_PASS] : 0, h) : 0;
            }
            const uint64_t run = __ballot(act && P == Prun) & todo;  // contiguous lanes of this period
            todo &= ~run;

            uint64_t pending = run;
            while (pending) {
                // -- admit mode: every pending request passes until the first one that does not fit
                const bool pl = (pending >> lane) & 1ull;
                const int64_t av = pl ? d.acq : 0;
                const int64_t ex = wave_excl_scan(av, lane);
                const int64_t W = ps.wo_pass + ps.cur[SG_EV_PASS];
                const double latest_l = (double)(W + ex) / R.isec;
                const double nr_l = R.thr - latest_l - (double)d.acq;
                const uint64_t fails = __ballot(pl && !(nr_l >= 0));
                const uint64_t pass_mask = fails ? (pending & below(__builtin_ctzll(fails))) : pending;
                if (pass_mask) {
                    const bool pm = (pass_mask >> lane) & 1ull;
                    if (pm) store_result(a.out, d.idx, SG_STATUS_OK, java_d2i(nr_l), 0);
                    ps.cur[SG_EV_PASS] += wave_sum(pm ? d.acq : 0);
                    ps.cur[SG_EV_PASS_REQUEST] += (int64_t)__popcll(pass_mask);
                    ps.cur[SG_EV_OCCUPIED_PASS] += wave_sum((pm && d.prio) ? d.acq : 0);
                }
                if (!fails) break;
                int x = __builtin_ctzll(fails);
                pending &= ~below(x + 1);
                // -- resolve the failing request x (normal check failed), then skip mode
                for (;;) {
                    {
                        const int64_t ax = bcast64(d.acq, x);
                        const bool px = bcast32((int)d.prio, x) != 0;
                        int32_t wait;
                        const int32_t stx = decide_fail(R, max_occ, ps, ax, px, &wait);
                        if (lane == x) store_result(a.out, d.idx, stx, 0, wait);
                    }
                    // -- skip mode: the window is unchanged, so a request passes iff it fits on its own;
                    // prioritized requests that do not fit stop the skip (they may occupy).
                    if (!pending) break;
                    const bool pl2 = (pending >> lane) & 1ull;
                    const double latest = (double)(ps.wo_pass + ps.cur[SG_EV_PASS]) / R.isec;
                    const bool fit = pl2 && (R.thr - latest - (double)d.acq >= 0);
                    const uint64_t fitm = __ballot(fit);
                    const uint64_t stop = fitm | __ballot(pl2 && d.prio);
                    const uint64_t blk = stop ? (pending & below(__builtin_ctzll(stop))) : pending;
                    if (blk) {
                        const bool b = (blk >> lane) & 1ull;
                        if (b) store_result(a.out, d.idx, SG_STATUS_BLOCKED, 0, 0);
                        ps.cur[SG_EV_BLOCK] += wave_sum(b ? d.acq : 0);
                        ps.cur[SG_EV_BLOCK_REQUEST] += (int64_t)__popcll(blk);
                    }
                    if (!stop) {
                        pending = 0;
                        break;
                    }
                    const int g = __builtin_ctzll(stop);
                    pending &= ~below(g);
                    if ((fitm >> g) & 1ull) break;  // back to admit mode starting at g
                    x = g;                          // a prioritized request that does not fit
                    pending &= ~(1ull << g);
                }
            }
        }
    }
    // close the last bucket and write the ring back
    if (I >= 0 && lane == I) {
        st = ws;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ps.cur[ev];
    }
    if (lane < S) {
        ring[lane].start = st;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[lane].c[ev] = c[ev];
    }
    if (lane == 0) {
        Occ o;
        o.pass = ps.occ_pass;
        o.pass_req = ps.occ_req;
        a.occ[k] = o;
    }
}

__global__ void __launch_bounds__(256) k_walk_long(BatchArgs a) {
    if (*a.err) return;
    const uint32_t cnt = *a.long_count;
    const uint32_t waves_per_block = blockDim.x / 64;
    const uint32_t wave = blockIdx.x * waves_per_block + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * waves_per_block;
    for (uint32_t w = wave; w < cnt; w += nwaves) {
        const uint64_t s = a.long_list[w];
        const uint32_t k = (uint32_t)(a.rec_sorted[s] >> a.kshift);
        // segment end: gallop then binary search for the first record with a larger flowId
        uint64_t lo = s + a.short_max, step = 64, hi;
        for (;;) {
            hi = lo + step;
            if (hi >= a.n) {
                hi = a.n;
                break;
            }
            if ((uint32_t)(a.rec_sorted[hi] >> a.kshift) != k) break;
            lo = hi;
            step <<= 1;
        }
        while (hi - lo > 1) {  // invariant: rec[lo] has key k, rec[hi] (or n) does not
            const uint64_t mid = (lo + hi) >> 1;
            if ((uint32_t)(a.rec_sorted[mid] >> a.kshift) == k) lo = mid;
            else hi = mid;
        }
        walk_wave(a, k, s, hi);
    }
}

__global__ void k_finish(BatchArgs a) {
    if (*a.err == 0 && a.n > 0) *a.last_ts = a.req[a.n - 1].ts_ms;
}

// ---------------------------------------------------------------------------- state management

__global__ void __launch_bounds__(256) k_init_state(Bucket* ring, Occ* occ, uint32_t K, int stride,
                                                    const int32_t* src_map, const Bucket* old_ring,
                                                    const Occ* old_occ, int old_stride) {
    const uint64_t total = (uint64_t)K * stride;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = (uint32_t)(i / stride);
        const int q = (int)(i % stride);
        const int32_t src = src_map ? src_map[k] : -1;
        Bucket b;
        if (src >= 0 && q < old_stride) {
            b = old_ring[(size_t)src * old_stride + q];
        } else {
            b.start = INT64_MIN;
#pragma unroll
            for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) b.c[ev] = 0;
        }
        ring[i] = b;
        if (q == 0) {
            Occ o;
            if (src >= 0) o = old_occ[src];
            else o.pass = o.pass_req = 0;
            occ[k] = o;
        }
    }
}

// ClusterMetric.getAvg(PASS) / getAvg(BLOCK) at `now` for every flowId, evaluated as if currentWindow(now)
// had run (the stale slot reads as reset, plus the occupied transfer) without mutating the state
// (ClusterMetricNodeGenerator.java:39-105 reads these per flowId).
__global__ void __launch_bounds__(256) k_snapshot(const Rule* rules, const Bucket* ring, const Occ* occ, uint32_t K,
                                                  int stride, int64_t now, double* out) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
        const Rule R = rules[k];
        const Bucket* rg = ring + (size_t)k * stride;
        const int64_t P = now / R.wl;
        const int I = (int)(P % R.S);
        const int64_t ws = P * R.wl;
        int64_t pass = 0, block = 0;
        for (int q = 0; q < R.S; ++q) {
            const int64_t s0 = rg[q].start;
            if (q == I) {
                if (s0 == ws) {
                    pass += rg[q].c[SG_EV_PASS];
                    block += rg[q].c[SG_EV_BLOCK];
                } else if (s0 != INT64_MIN && s0 < ws && occ[k].pass_req > 0) {
                    pass += occ[k].pass;
                }
                continue;
            }
            if (s0 != INT64_MIN && now - s0 <= (int64_t)R.S * R.wl) {
                pass += rg[q].c[SG_EV_PASS];
                block += rg[q].c[SG_EV_BLOCK];
            }
        }
        out[2 * (size_t)k] = (double)pass / R.isec;
        out[2 * (size_t)k + 1] = (double)block / R.isec;
    }
}

// ------------------------------------------------------------------------------------ launchers

static unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

hipError_t launch_prep(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_prep, dim3(grid_for(a.n, 256, 8192)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_walk_short(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_walk_short, dim3(grid_for(a.n, 256, 16384)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_walk_long(const BatchArgs& a, hipStream_t stream) {
    // upper bound of long segments = n / (short_max + 1); waves loop over the list
    const uint64_t max_long = a.n / ((uint64_t)a.short_max + 1) + 1;
    const unsigned blocks = grid_for(max_long * 64, 256, 2048);
    hipLaunchKernelGGL(k_walk_long, dim3(blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_finish(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(1), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_init_state(Bucket* ring, Occ* occ, uint32_t K, int stride, const int32_t* src_map,
                             const Bucket* old_ring, const Occ* old_occ, int old_stride, hipStream_t stream) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_init_state, dim3(grid_for((uint64_t)K * stride, 256, 8192)), dim3(256), 0, stream, ring, occ,
                       K, stride, src_map, old_ring, old_occ, old_stride);
    return hipGetLastError();
}

hipError_t launch_snapshot(const Rule* rules, const Bucket* ring, const Occ* occ, uint32_t K, int stride,
                           int64_t now, double* out, hipStream_t stream) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_snapshot, dim3(grid_for(K, 256, 4096)), dim3(256), 0, stream, rules, ring, occ, K, stride,
                       now, out);
    return hipGetLastError();
}

}  // namespace sg
