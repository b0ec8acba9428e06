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

#include <algorithm>
#include <cstdlib>
#include <mutex>

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

// LeapArray sum / intervalInSecond (ClusterMetric.getAvg, ClusterMetric.java:70-72)
__device__ __forceinline__ double qps_of(int64_t sum, double isec) { return avg_div((double)sum, isec); }

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

// The compact record (low 32 bits of a record when abits == 8 and ibits <= 24): {idx : 24, acquire : 7, prio : 1}.
__device__ __forceinline__ Decoded decode_c(const BatchArgs& a, uint32_t c) {
    Decoded d;
    d.idx = c >> 8;
    d.prio = (c & 1u) != 0;
    const uint32_t q = (c >> 1) & 127u;
    d.acq = (q == 127u) ? (int64_t)a.req[d.idx].acquire : (int64_t)q;
    return d;
}

// ------------------------------------------------------------------------------------------- prep

// One block per 4096-request tile (the radix sort's tile). With a.hist0 set the block also counts the
// first sort pass's digits of its records (the sort then skips that histogram read).
constexpr int kPrepItems = kSortRounds;  // k_prep's tile is the sort's (its first-pass histogram rows)
constexpr uint32_t kPrepTile = 256 * kPrepItems;

// BIN (the binned front half): each record also gets its bin digit (a.bin_on, see k_bin_sort): the flowId's hot slot
// from the hot-flowId table, staged in LDS once per block (a block takes kPrepBinTiles tiles), else its key range.
template <bool BIN>
__global__ void __launch_bounds__(256) k_prep(BatchArgs a) {
    __shared__ uint32_t dcnt[1024];
    __shared__ uint16_t ldig[kPrepItems * 256];  // each request's first sort digit (the histogram after the loop)
    __shared__ alignas(16) uint2 htab[BIN ? kHotTab : 1];  // the hot flowIds: two 16-B LDS reads per request
    if constexpr (BIN)
        for (uint32_t x = threadIdx.x; x < kHotTab; x += 256) htab[x] = a.hot_tab[x];
    const uint64_t n = a.n;
    const int64_t t0 = a.req[0].ts_ms;
    const uint64_t sentinel = (uint64_t)a.K << a.kshift;
    const uint32_t dmask = (1u << a.hist0_bits) - 1u;
    const uint32_t kTiles = BIN ? (uint32_t)a.prep_tiles : 1u;
#pragma unroll 1
    for (uint32_t tt = 0; tt < kTiles; ++tt) {
    const uint32_t tile = blockIdx.x * kTiles + tt;
    if ((uint64_t)tile * kPrepTile >= n) break;
    if (tt) __syncthreads();  // the previous tile's histogram row is written
    if (a.hist0)
        for (uint32_t d = threadIdx.x; d <= dmask; d += 256) dcnt[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)tile * kPrepTile;
#pragma unroll 4
    for (int it = 0; it < kPrepItems; ++it) {
        const uint64_t i = base + (uint64_t)it * 256 + threadIdx.x;
        if (i >= n) break;
        const sg_req r = a.req[i];
        const int64_t t = r.ts_ms;
        if (i == 0) {
            if (t < 0 || (a.check_last && (t < *a.last_ts || (a.front_ts && t < *a.front_ts)))) atomicOr(a.err, kErrTime);
            for (int w = 0; w < a.n_wl; ++w) a.p0[w] = t / a.wl[w];
        } else {
            const int64_t tp = a.req[i - 1].ts_ms;
            if (t < tp || t < 0) {
                atomicOr(a.err, kErrTime);
            } else if (t != tp) {  // a new period can only start at a new timestamp (skips the int64 divisions)
                for (int w = 0; w < a.n_wl; ++w) {
                    const int64_t wl = a.wl[w];
                    const int64_t P0 = t0 / wl, Pp = tp / wl, Pi = t / wl;
                    for (int64_t p = Pp + 1; p <= Pi; ++p) {
                        const int64_t q = p - P0;
                        if (q <= 0) continue;  // an out-of-order batch (kErrTime already set by an earlier index)
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
                a.np[w] = q > (int64_t)kMaxPeriods ? kMaxPeriods : q < 1 ? 1u : (uint32_t)q;  // < 1: out of order
            }
        }
        // DefaultTokenService.requestToken validation, srv/flow/DefaultTokenService.java:39-47, 87-89
        const uint32_t key = r.key & SG_KEY_INDEX;
        uint64_t rec;
        int32_t st;
        uint32_t d = kBinDrop;  // BIN: a rejected request's bin
        if (key == SG_KEY_BAD || r.acquire <= 0) {
            st = SG_STATUS_BAD_REQUEST;
            rec = sentinel;
        } else if (key >= a.K) {
            st = SG_STATUS_NO_RULE_EXISTS;
            rec = sentinel;
        } else {
            uint64_t q = (uint64_t)(uint32_t)r.acquire;
            if (q > a.aesc) q = a.aesc;
            const uint64_t ac = (q << 1) | (uint64_t)(r.key >> 31);
            rec = ((uint64_t)key << a.kshift) | ((uint64_t)i << a.abits) | ac;
            st = SG_STATUS_BLOCKED;  // walkers write only non-BLOCKED
            if constexpr (BIN) {  // the flowId's hot slot, else its key range
                d = key >> a.bin_bsh;
                if (!(a.dbg & 131072)) {  // (timing experiment: no hot lookup, every flowId regular)
                    const uint4* hb = reinterpret_cast<const uint4*>(htab + hot_hash(key) * kHotWays);
                    const uint4 e0 = hb[0], e1 = hb[1];
                    d = e0.x == key ? a.bin_R + e0.y : d;
                    d = e0.z == key ? a.bin_R + e0.w : d;
                    d = e1.x == key ? a.bin_R + e1.y : d;
                    d = e1.z == key ? a.bin_R + e1.w : d;
                }
            }
        }
        if constexpr (BIN) rec |= (uint64_t)d << a.bin_dshift;
        if (!(a.dbg & 16384)) {
            int32_t* o = &a.out[i].status;  // the default result {st, 0, 0}
            st_stream(o, st);
            st_stream(o + 1, 0);
            st_stream(o + 2, 0);
        }
        st_stream(a.rec + i, rec);
        if (a.hist0) ldig[it * 256 + threadIdx.x] = (uint16_t)(BIN ? d : (uint32_t)(rec >> a.hist0_shift) & dmask);
    }
    if (a.hist0) {
        // the histogram's LDS atomics after the tile's loads: inside the loop they kept the compiler from overlapping
        // one item's request load with the previous item's work
        for (int it = 0; it < kPrepItems; ++it) {
            if (base + (uint64_t)it * 256 + threadIdx.x >= n) break;
            atomicAdd(&dcnt[ldig[it * 256 + threadIdx.x]], 1u);
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d <= dmask; d += 256) a.hist0[(size_t)tile * (dmask + 1) + d] = dcnt[d];
        if (a.csum0) {  // the chunk's column sums (zeroed before the launch): no k_colsum pass for the first digit
            uint32_t* cs = a.csum0 + (size_t)(tile / kChunkTiles) * (dmask + 1);
            for (uint32_t d = threadIdx.x; d <= dmask; d += 256)
                if (dcnt[d]) atomicAdd(cs + d, dcnt[d]);
        }
    }
    }  // tiles
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
        const double occupy_avg = qps_of(ps.wo_wait + ps.cur[SG_EV_WAITING], R.isec);
        if (occupy_avg <= max_occ_ratio * R.thr) {
            const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
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

// The batch's period tables (first request index of every window period, per distinct window length),
// staged in LDS by stage_periods when they fit, else read from a.bnd. File-scope LDS keeps every access a
// ds_read: a table pointer that may point at LDS or HBM compiles to flat loads, and each of those waits
// for every outstanding global load and store of the wave (s_waitcnt vmcnt(0) lgkmcnt(0)).
__shared__ uint32_t g_sbnd[kLdsBndFlow];
__shared__ uint32_t g_boff[kMaxWl];  // offset of window length w's table in g_sbnd
__shared__ int g_blds;               // 1: tables in g_sbnd, 0: read from a.bnd
__shared__ int64_t g_p0[kMaxWl];     // a.p0 / a.np staged by stage_periods: per-lane reads of these tiny tables
__shared__ uint32_t g_np[kMaxWl];    // (indexed by the rule's window length) were each a memory round trip
constexpr int kModS = 64;
__shared__ uint8_t g_p0mod[kMaxWl][kModS + 1];  // g_p0[w] mod s (s = 1..kModS), staged by stage_periods

// Ring slot of the batch's window period q (period P0 + q of window length w) for sampleCount S: (P0 + q) % S in
// 32 bits from the staged residue (a 64-bit modulo of the absolute period is ~120 instructions).
__device__ __forceinline__ int period_slot(int w, uint32_t q, int S) {
#ifdef SG_NO_PSLOT
    return (int)((g_p0[w] + (int64_t)q) % S);
#endif
    if (S <= kModS) return (int)(((uint32_t)g_p0mod[w][S] + q) % (uint32_t)S);
    return (int)((g_p0[w] + (int64_t)q) % S);
}

// Period tracking shared by the walkers: requests of one flowId arrive in index order, so the
// window period only moves forward; the cached boundary of the next period answers most lookups.
// L: the tables are staged in g_sbnd (a compile-time choice: a run-time one is if-converted into a
// select of two pointers and one flat load). Kernels branch once on g_blds into the two instantiations.
template <bool L>
struct PeriodCursor {
    const uint32_t* gbnd;  // this window length's table in HBM (!L)
    uint32_t base;         // its offset in g_sbnd (L)
    uint32_t np;
    uint32_t q;       // current period (0-based within the batch), 0xFFFFFFFF before the first
    uint32_t next_b;  // first request index of period q + 1 (UINT32_MAX past the last)

    __device__ __forceinline__ void init(const BatchArgs& a, int w) {
        gbnd = a.bnd + (size_t)w * kMaxPeriods;
        base = g_boff[w];
        np = g_np[w];
        q = 0xFFFFFFFFu;
        next_b = 0;
    }
    __device__ __forceinline__ uint32_t at(uint32_t i) const {
        if constexpr (L) return g_sbnd[base + i];
        else return gbnd[i];
    }
    __device__ __forceinline__ void seek(uint32_t qq) {
        q = qq;
        next_b = (qq + 1 < np) ? at(qq + 1) : 0xFFFFFFFFu;
    }
    // period of a request index >= every index seen so far: the largest p with table[p] <= idx
    __device__ __forceinline__ uint32_t of(uint32_t idx) const {
        if (q != 0xFFFFFFFFu && idx < next_b) return q;
        uint32_t lo = 0, hi = np;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (at(mid) <= idx) lo = mid;
            else hi = mid;
        }
        return lo;
    }
};

// Open the bucket of period P (slot I = P % S) from the ring in memory and sum the other valid buckets
// (values(t): a slot j != I is valid iff its start >= ws - (S-1)*wl, LeapArray.java:270-272 with starts on
// window boundaries; only slot I can sit exactly `interval` behind and currentWindow resets it first).
// All loads are issued before any is used.
__device__ __forceinline__ void open_period_serial(PeriodState& ps, const Bucket* ring, const Rule& R, int64_t P,
                                                   int* I_out, int64_t* ws_out) {
    const int S = R.S;
    const int I = (int)(P % S);
    const int64_t ws = P * R.wl;
    const int64_t lo = ws - (int64_t)(S - 1) * R.wl;
    const int h = (int)((P + 1) % S);
    ps.wo_pass = ps.wo_wait = ps.head_other = 0;
    int64_t cI[SG_NUM_EVENTS];
    int64_t stI = INT64_MIN;
#pragma unroll 4
    for (int q = 0; q < S; ++q) {
        const int64_t st = ring[q].start;
        const int64_t pp = ring[q].c[SG_EV_PASS];
        const int64_t ww = ring[q].c[SG_EV_WAITING];
        const bool v = (q != I) && st != INT64_MIN && st >= lo;
        ps.wo_pass += v ? pp : 0;
        ps.wo_wait += v ? ww : 0;
        if (q == h && v) ps.head_other = pp;
        if (q == I) stI = st;
    }
    if (stI == ws) {
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = ring[I].c[ev];
    }
    open_bucket(ps, stI, cI, ws);
    *I_out = I;
    *ws_out = ws;
}

// ------------------------------------------------------------------------ serial walker (short)

// Outputs start as BLOCKED (k_prep), so only OK / SHOULD_WAIT results are written here.
template <bool L>
__device__ uint32_t walk_serial(const BatchArgs& a, uint32_t k, uint64_t s, uint64_t e) {
    uint32_t opened = 0;
    const Rule R = a.rules[k];
    Bucket* ring = a.ring + (size_t)k * a.stride;
    BucketHot* hot = a.hot + (size_t)k * a.stride;
    PeriodCursor<L> pc;
    pc.init(a, R.wl_idx);
    const int64_t P0 = g_p0[R.wl_idx];
    PeriodState ps;
    {
        const Occ o = a.occ[k];
        ps.occ_pass = o.pass;
        ps.occ_req = o.pass_req;
    }
    int64_t ws = 0;
    int I = -1;
    uint64_t nxt = a.rec_sorted[s];
    for (uint64_t j = s; j < e; ++j) {
        const uint64_t cur = nxt;
        if (j + 1 < e) nxt = a.rec_sorted[j + 1];  // issue the next record's load before deciding this one
        const Decoded d = decode(a, cur);
        const uint32_t q = pc.of(d.idx);
        if (q != pc.q) {
            if (I >= 0) {
                ring[I].start = ws;
#pragma unroll
                for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[I].c[ev] = ps.cur[ev];
                store_hot(hot + I, ws, ps.cur[SG_EV_PASS], ps.cur[SG_EV_WAITING]);
            }
            pc.seek(q);
            open_period_serial(ps, ring, R, P0 + (int64_t)q, &I, &ws);
            ++opened;
        }
        // ClusterFlowChecker.acquireClusterToken, :67-81
        const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
        const double next_remaining = R.thr - latest - (double)d.acq;
        if (next_remaining >= 0) {
            ps.cur[SG_EV_PASS] += d.acq;
            ps.cur[SG_EV_PASS_REQUEST] += 1;
            if (d.prio) ps.cur[SG_EV_OCCUPIED_PASS] += d.acq;
            store_result(a.out, d.idx, SG_STATUS_OK, java_d2i(next_remaining), 0);
        } else {
            int32_t wait;
            const int32_t st = decide_fail(R, a.max_occ_ratio, ps, d.acq, d.prio, &wait);
            if (st != SG_STATUS_BLOCKED) store_result(a.out, d.idx, st, 0, wait);
        }
    }
    if (I >= 0) {
        ring[I].start = ws;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[I].c[ev] = ps.cur[ev];
        store_hot(hot + I, ws, ps.cur[SG_EV_PASS], ps.cur[SG_EV_WAITING]);
    }
    Occ o;
    o.pass = ps.occ_pass;
    o.pass_req = ps.occ_req;
    a.occ[k] = o;
    return opened;
}

// --------------------------------------------------------------------------- wave walker (long)

#ifndef SG_WAVE_UNROLL
#define SG_WAVE_UNROLL 4  // 255 VGPRs with no spill once inlined (8: 21 spills; 0.89 vs 0.92 ms/step)
#endif
constexpr int kWaveUnroll = SG_WAVE_UNROLL;  // 64-record chunks kept in flight per wave (register double buffer)

template <bool L>
struct WaveWalker {
    const BatchArgs& a;
    const Rule R;
    const int lane;
    Bucket* ring;
    BucketHot* hot;
    PeriodCursor<L> pc;
    int64_t P0;
    // lane q < S holds slot q of the ring
    int64_t st;
    int64_t c[SG_NUM_EVENTS];
    PeriodState ps;  // wave-uniform
    int64_t ws;
    int I;
    // deferred per-lane BLOCK / BLOCK_REQUEST / OCCUPIED_BLOCK of the current period
    int64_t d_blk, d_blkn, d_oblk;
    // the current period can admit nothing more: not even acquireCount = 1 fits and no prioritized
    // request can occupy (both only get harder within a period), so its remaining requests are BLOCKED
    bool dead;

    __device__ WaveWalker(const BatchArgs& a_, uint32_t k)
        : a(a_), R(a_.rules[k]), lane(lane_id()) {
        ring = a.ring + (size_t)k * a.stride;
        hot = a.hot + (size_t)k * a.stride;
        pc.init(a, R.wl_idx);
        P0 = g_p0[R.wl_idx];
        st = INT64_MIN;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = 0;
        if (lane < R.S) {
            st = ring[lane].start;
#pragma unroll
            for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ring[lane].c[ev];
        }
        const Occ o = a.occ[k];
        ps.occ_pass = o.pass;
        ps.occ_req = o.pass_req;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ps.cur[ev] = 0;
        ps.wo_pass = ps.wo_wait = ps.head_other = 0;
        ws = 0;
        I = -1;
        d_blk = d_blkn = d_oblk = 0;
        dead = false;
    }

    // close the current bucket (flush deferred counts) into its owner lane
    __device__ void close_period() {
        if (I < 0) return;
        ps.cur[SG_EV_BLOCK] += wave_sum(d_blk);
        ps.cur[SG_EV_BLOCK_REQUEST] += wave_sum(d_blkn);
        ps.cur[SG_EV_OCCUPIED_BLOCK] += wave_sum(d_oblk);
        d_blk = d_blkn = d_oblk = 0;
        if (lane == I) {
            st = ws;
#pragma unroll
            for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) c[ev] = ps.cur[ev];
        }
    }

    __device__ void open_period(uint32_t q) {
        close_period();
        dead = false;
        pc.seek(q);
        const int64_t P = P0 + (int64_t)q;
        const int S = R.S;
        I = period_slot(R.wl_idx, q, S);
        ws = P * R.wl;
        int64_t cI[SG_NUM_EVENTS];
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = bcast64(c[ev], I);
        open_bucket(ps, bcast64(st, I), cI, ws);
        const int64_t lo = ws - (int64_t)(S - 1) * R.wl;
        const bool valid = lane < S && lane != I && st != INT64_MIN && st >= lo;
        ps.wo_pass = wave_sum(valid ? c[SG_EV_PASS] : 0);
        ps.wo_wait = wave_sum(valid ? c[SG_EV_WAITING] : 0);
        const int h = I + 1 == S ? 0 : I + 1;
        ps.head_other = (h != I) ? bcast64(valid ? c[SG_EV_PASS] : 0, h) : 0;
    }

    // Can any prioritized request still occupy in this period? (wave-uniform; the window is fixed.)
    __device__ __forceinline__ bool occupy_possible(double latest) const {
        const double occupy_avg = qps_of(ps.wo_wait + ps.cur[SG_EV_WAITING], R.isec);
        if (!(occupy_avg <= a.max_occ_ratio * R.thr)) return false;
        const int64_t head = (R.S == 1) ? ps.cur[SG_EV_PASS] : ps.head_other;
        return latest + (double)(1 + ps.occ_pass) - (double)head <= R.thr;
    }

    // Decide the lanes in `run` (contiguous, same period, in order).
    __device__ void run(uint64_t run_mask, const Decoded& d) {
        const double latest0 = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
        if (!(R.thr - latest0 - 1.0 >= 0)) {
            // Saturated: not even acquireCount = 1 fits, and nothing below can add PASS in this period,
            // so every non-prioritized request blocks; prioritized ones try to occupy one by one until
            // occupying is impossible too.
            const bool in = (run_mask >> lane) & 1ull;
            uint64_t pm = __ballot(in && d.prio);
            bool occ_ok = pm != 0 && occupy_possible(latest0);
            while (pm && occ_ok) {
                const int x = __builtin_ctzll(pm);
                pm &= pm - 1;
                const int64_t ax = bcast64(d.acq, x);
                int32_t wait;
                const int32_t stx = decide_fail(R, a.max_occ_ratio, ps, ax, true, &wait);
                if (lane == x && stx != SG_STATUS_BLOCKED) store_result(a.out, d.idx, stx, 0, wait);
                occ_ok = occupy_possible(latest0);
            }
            const bool rest = in && (!d.prio || ((pm >> lane) & 1ull));
            d_blk += rest ? d.acq : 0;
            d_blkn += rest ? 1 : 0;
            d_oblk += (rest && d.prio) ? d.acq : 0;
            dead = !occupy_possible(latest0);
            return;
        }
        uint64_t pending = run_mask;
        int guard = 0;
        while (pending) {
            if (++guard > 64) {  // every pass removes >= 1 pending lane
                atomicOr(a.err, kErrInternal);
                break;
            }
            // -- admit mode: every pending request passes until the first one that does not fit
            const bool pl = (pending >> lane) & 1ull;
            const int64_t av = pl ? d.acq : 0;
            const int64_t ex = wave_excl_scan(av, lane);
            const int64_t W = ps.wo_pass + ps.cur[SG_EV_PASS];
            const double latest_l = qps_of(W + ex, R.isec);
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
            for (;;) {
                {  // the request x failed the normal check: occupy branch or block
                    const int64_t ax = bcast64(d.acq, x);
                    const bool px = bcast32((int)d.prio, x) != 0;
                    int32_t wait;
                    const int32_t stx = decide_fail(R, a.max_occ_ratio, ps, ax, px, &wait);
                    if (lane == x && stx != SG_STATUS_BLOCKED) store_result(a.out, d.idx, stx, 0, wait);
                }
                // -- skip mode: the window is unchanged, so a request passes iff it fits on its own;
                // prioritized requests that do not fit stop the skip (they may occupy).
                if (!pending) break;
                const bool pl2 = (pending >> lane) & 1ull;
                const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
                const bool fit = pl2 && (R.thr - latest - (double)d.acq >= 0);
                const uint64_t fitm = __ballot(fit);
                const uint64_t stop = fitm | __ballot(pl2 && d.prio);
                const uint64_t blk = stop ? (pending & below(__builtin_ctzll(stop))) : pending;
                const bool b = (blk >> lane) & 1ull;
                d_blk += b ? d.acq : 0;  // non-prioritized, not fitting: BLOCKED (output already BLOCKED)
                d_blkn += b ? 1 : 0;
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

    __device__ void chunk(uint64_t rec, bool act) {
        Decoded d;
        d.idx = 0;
        d.acq = 0;
        d.prio = false;
        uint32_t q = 0xFFFFFFFFu;
        if (act) {
            d = decode(a, rec);
            q = pc.of(d.idx);
        }
        uint64_t todo = __ballot(act);
        int guard = 0;
        while (todo) {
            if (++guard > 64) {  // at most one run per lane; anything else is an internal error
                atomicOr(a.err, kErrInternal);
                break;
            }
            const uint32_t qrun = (uint32_t)bcast32((int)q, __builtin_ctzll(todo));
            if (qrun != pc.q) open_period(qrun);
            const uint64_t rm = __ballot(act && q == qrun) & todo;  // contiguous lanes of this period
            todo &= ~rm;
            run(rm, d);
        }
    }

    __device__ void finish(uint32_t k) {
        close_period();
        if (lane < R.S) {
            ring[lane].start = st;
#pragma unroll
            for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ring[lane].c[ev] = c[ev];
            store_hot(hot + lane, st, c[SG_EV_PASS], c[SG_EV_WAITING]);
        }
        if (lane == 0) {
            Occ o;
            o.pass = ps.occ_pass;
            o.pass_req = ps.occ_req;
            a.occ[k] = o;
        }
    }
};

// First position p in [lo, hi) with pred(p) (pred monotone false→true), hi if none. 64-way wave search:
// every step probes 64 evenly spaced positions, so a million-record range takes 4 dependent loads.
template <class Pred>
__device__ __forceinline__ uint64_t wave_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t p = lo + (uint64_t)lane * step;
        const uint64_t m = __ballot(p >= hi || pred(p));
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
    const uint64_t p = lo + (uint64_t)lane;
    const uint64_t m = __ballot(p < hi && pred(p));
    return m ? lo + (uint64_t)__builtin_ctzll(m) : hi;
}

// Inlined into k_walk_long (SG_WAVE_INLINE=0: a called function, as in round 3): one register allocation for the
// kernel instead of a call frame per segment — 0.90 vs 0.96 ms/step pipelined, same box.
#ifndef SG_WAVE_INLINE
#define SG_WAVE_INLINE 1
#endif
#if SG_WAVE_INLINE
#define SG_WAVE_ATTR __device__ __forceinline__
#else
#define SG_WAVE_ATTR __device__ __noinline__
#endif
template <bool L>
SG_WAVE_ATTR void walk_wave(const BatchArgs& a, uint32_t k, uint64_t s, uint64_t e, uint32_t item) {
    WaveWalker<L> w(a, k);
    const int lane = w.lane;
    // period ends of this segment from k_long_bounds: lane q holds the first position of period q + 1
    const bool tab = a.long_pend != nullptr && item < kLongTab && w.pc.np <= (uint32_t)kLongPeriods;
    uint32_t pend_l = 0;
    if (tab && lane < kLongPeriods) pend_l = a.long_pend[(size_t)item * kLongPeriods + lane];
    const uint64_t* rec = a.rec_sorted;
    constexpr uint64_t kBlock = 64ull * kWaveUnroll;
    uint64_t cur[kWaveUnroll];
#pragma unroll
    for (int u = 0; u < kWaveUnroll; ++u) {
        const uint64_t j = s + (uint64_t)u * 64 + lane;
        cur[u] = j < e ? rec[j] : 0ull;
    }
    uint32_t skip_tried_q = 0xFFFFFFFFu;
    uint64_t pos = s;
    while (pos < e) {
        uint64_t npos = pos + kBlock;
        uint64_t nxt[kWaveUnroll];
#pragma unroll
        for (int u = 0; u < kWaveUnroll; ++u) {  // prefetch the next block before deciding this one
            const uint64_t j = npos + (uint64_t)u * 64 + lane;
            nxt[u] = j < e ? rec[j] : 0ull;
        }
        bool skipped = false;
#pragma unroll
        for (int u = 0; u < kWaveUnroll; ++u) {
            const uint64_t cb = pos + (uint64_t)u * 64;
            if (skipped || cb >= e) continue;
            w.chunk(cur[u], cb + lane < e);
            const uint64_t after = cb + 64;
            if (w.dead && after < e && w.pc.q != skip_tried_q) {
                // The rest of this window period is BLOCKED: find where the period ends in the segment
                // and hand the skipped range to k_skip_apply (its BLOCK counts only).
                skip_tried_q = w.pc.q;
                const uint32_t nb = w.pc.next_b;
                uint64_t pe;
                if (tab) {
                    pe = w.pc.q + 1 >= w.pc.np ? e : (uint64_t)(uint32_t)bcast32((int)pend_l, (int)w.pc.q);
                    pe = pe < after ? after : pe;
                } else {
                    pe = gallop_search(after, e, [&](uint64_t p) {
                        return (uint32_t)((rec[p] >> a.abits) & a.imask) >= nb;
                    }, lane);
                }
                if (pe - after >= kSkipMin) {
                    // hand the range over in pieces of <= kSkipPiece records (one k_skip_apply wave each); the
                    // records after the range are loaded together with the slot reservation (one round trip)
                    const uint32_t np = (uint32_t)((pe - after + kSkipPiece - 1) / kSkipPiece);
                    uint32_t slot = 0;
                    if (lane == 0) slot = atomicAdd(a.skip_count, np);
#pragma unroll
                    for (int v = 0; v < kWaveUnroll; ++v) {
                        const uint64_t j = pe + (uint64_t)v * 64 + lane;
                        nxt[v] = j < e ? rec[j] : 0ull;
                    }
                    slot = (uint32_t)bcast32((int)slot, 0);
                    if (slot + np <= a.skip_cap) {
                        for (uint32_t pi = lane; pi < np; pi += 64) {
                            const uint64_t b0 = after + (uint64_t)pi * kSkipPiece;
                            const uint64_t b1 = min(pe, b0 + kSkipPiece);
                            a.skips[slot + pi] = make_uint4(k, w.pc.q, (uint32_t)b0, (uint32_t)b1);
                        }
                        npos = pe;
                        skipped = true;
                    } else {  // no room: walk on (the next block again)
#pragma unroll
                        for (int v = 0; v < kWaveUnroll; ++v) {
                            const uint64_t j = npos + (uint64_t)v * 64 + lane;
                            nxt[v] = j < e ? rec[j] : 0ull;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kWaveUnroll; ++u) cur[u] = nxt[u];
        pos = npos;
    }
    w.finish(k);
}

// ------------------------------------------------------------------- segments and the walk kernel

// Segment heads of the sorted records (first record of each flowId), compacted into two work lists:
// segments of more than short_max records (one wave each) and the rest (one lane each). One block per
// tile of kSegTile records; appends are block-aggregated (one atomic per block and list), since
// same-address atomics from every wave serialise at the L2.
constexpr int kSegThreads = 256;
constexpr int kSegItems = 16;
constexpr uint32_t kSegTile = kSegThreads * kSegItems;

__global__ void __launch_bounds__(kSegThreads) k_seg(BatchArgs a) {
    constexpr int kL = kClasses + 1;  // list 0..kClasses-1: short length classes, kClasses: long
    __shared__ uint32_t cnt[kL];
    __shared__ uint32_t base[kL];
    __shared__ uint32_t nheads;
    __shared__ uint32_t hpos[kSegTile];  // heads of this tile (tile offsets), in any order
    if (*a.err) return;
    const uint64_t n = a.n;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kSegTile; t0 < n; t0 += (uint64_t)gridDim.x * kSegTile) {
        if (tid < kL) cnt[tid] = 0;
        if (tid == 0) nheads = 0;
        __syncthreads();
        // 1. heads: item u of wave w covers records t0 + (w*kSegItems + u)*64 + lane (wave-contiguous rows)
        uint32_t key[kSegItems];
#pragma unroll
        for (int u = 0; u < kSegItems; ++u) {
            const uint64_t j = t0 + ((uint64_t)(wave * kSegItems + u) << 6) + lane;
            const uint64_t r = j < n ? a.rec_sorted[j] : ~0ull;
            key[u] = j < n ? (uint32_t)(r >> a.kshift) : 0xFFFFFFFFu;
            if (a.exit_cnt) {  // the local chain's exit records of this 64-record row (one exit tile holds the row)
                const uint64_t xm = __ballot(key[u] < a.K && ((r & a.exit_amask) >> 1 & 3ull) != 0);
                const uint64_t j0 = t0 + ((uint64_t)(wave * kSegItems + u) << 6);
                if (xm && lane == 0) atomicAdd(a.exit_cnt + 1 + j0 / kLTile, (uint32_t)__popcll(xm));
            }
        }
        const uint64_t jw = t0 + ((uint64_t)(wave * kSegItems) << 6);  // the wave's first record
        const uint32_t before = (jw > 0 && jw < n) ? (uint32_t)(a.rec_sorted[jw - 1] >> a.kshift) : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < kSegItems; ++u) {
            const uint32_t j_off = (uint32_t)((wave * kSegItems + u) << 6) + (uint32_t)lane;
            uint32_t kp = (uint32_t)__shfl_up((int)key[u], 1u, 64);
            if (lane == 0) kp = u == 0 ? before : (uint32_t)__shfl((int)key[u - 1], 63, 64);
            if (t0 + j_off < n && key[u] != kp) {
                if (key[u] < a.K) hpos[atomicAdd(&nheads, 1u)] = j_off;
                if (a.seg_end && kp < a.K) a.seg_end[kp] = (uint32_t)(t0 + j_off);  // the previous key ends here
            }
            if (a.seg_end && t0 + j_off == n - 1 && key[u] < a.K) a.seg_end[key[u]] = (uint32_t)n;
        }
        __syncthreads();
        // 2. classify the heads, one per thread: all length probes issued at once (the segment is longer
        // than m iff record j + m has the same key; the class is the number of bounds it exceeds)
        const uint32_t nh = nheads;
        uint32_t slot[kSegTile / kSegThreads], hkey[kSegTile / kSegThreads];
#pragma unroll
        for (int r = 0; r < (int)(kSegTile / kSegThreads); ++r) {
            const uint32_t h = (uint32_t)r * kSegThreads + (uint32_t)tid;
            slot[r] = 0xFFFFFFFFu;
            if (h >= nh) continue;
            const uint64_t j = t0 + hpos[h];
            const uint32_t k = (uint32_t)(a.rec_sorted[j] >> a.kshift);
            hkey[r] = k;
            uint32_t pk[kClasses];
#pragma unroll
            for (int c = 0; c < kClasses; ++c) {
                const uint64_t m = c < kClasses - 1 ? (uint64_t)kClassMax[c] : (uint64_t)a.short_max;
                pk[c] = (j + m < n) ? (uint32_t)(a.rec_sorted[j + m] >> a.kshift) : 0xFFFFFFFFu;
            }
            uint32_t l = 0;
#pragma unroll
            for (int c = 0; c < kClasses - 1; ++c) l += pk[c] == k ? 1u : 0u;
            if (pk[kClasses - 1] == k) l = kClasses;  // longer than short_max: the wave walker
            slot[r] = (l << 24) | atomicAdd(&cnt[l], 1u);  // order within a list is irrelevant
        }
        __syncthreads();
        if (tid < kL) {
            const uint32_t t = cnt[tid];
            uint32_t* ctr = tid == kClasses ? a.long_count : a.short_count + tid;
            base[tid] = t ? atomicAdd(ctr, t) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < (int)(kSegTile / kSegThreads); ++r) {
            if (slot[r] == 0xFFFFFFFFu) continue;
            const uint32_t j = (uint32_t)(t0 + hpos[(uint32_t)r * kSegThreads + (uint32_t)tid]);
            const uint32_t l = slot[r] >> 24, pos = base[l] + (slot[r] & 0xFFFFFFu);
            if (l == (uint32_t)kClasses) {
                a.long_list[pos] = j;
                if (a.long_key) a.long_key[pos] = hkey[r];
            } else {
                a.short_list[a.class_off[l] + pos] = j;
                if (a.short_key) a.short_key[a.class_off[l] + pos] = hkey[r];
            }
        }
        __syncthreads();  // cnt / base / hpos are reused by the next tile
    }
}

// Cluster flow segments in two passes without length probes: k_seg_mark finds every flowId's first and last
// record in the sorted batch (one coalesced read; a head writes seg_start of its key and seg_end of the key before
// it), k_seg_classify walks the flowId range in order, turns each marked key into a list entry {start, end, key}
// of its length class (or the long list) and clears the mark for the next batch. Both run whatever the batch's
// error flags (the marks must be consumed); the walkers check them.
constexpr int kMarkItems = 16;  // 64-record rows per wave of k_seg_mark, all loaded at once

__global__ void __launch_bounds__(256) k_seg_mark(BatchArgs a) {
    const uint64_t n = a.n;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    // row u of wave w covers records t0 + (w*kMarkItems + u)*64 + lane: one load round trip per thread (this runs at
    // the end of the front half, on the pipeline's critical path)
    const uint64_t t0 = (uint64_t)blockIdx.x * (256 * kMarkItems);
    const uint64_t jw = t0 + ((uint64_t)(wave * kMarkItems) << 6);  // the wave's first record
    uint32_t key[kMarkItems];
#pragma unroll
    for (int u = 0; u < kMarkItems; ++u) {
        const uint64_t j = jw + ((uint64_t)u << 6) + lane;
        key[u] = j < n ? (uint32_t)(a.rec_sorted[j] >> a.kshift) : 0xFFFFFFFFu;
    }
    const uint32_t before = (jw > 0 && jw < n) ? (uint32_t)(a.rec_sorted[jw - 1] >> a.kshift) : 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < kMarkItems; ++u) {
        const uint64_t j = jw + ((uint64_t)u << 6) + lane;
        const uint32_t row_prev = u == 0 ? before : (uint32_t)__shfl((int)key[u - 1], 63, 64);  // all lanes active
        uint32_t kp = (uint32_t)__shfl_up((int)key[u], 1u, 64);
        if (lane == 0) kp = row_prev;
        if (j < n && key[u] != kp) {
            if (key[u] < a.K) a.seg_start[key[u]] = (uint32_t)j;
            if (kp < a.K) a.seg_end[kp] = (uint32_t)j;
        }
        if (j == n - 1 && key[u] < a.K) a.seg_end[key[u]] = (uint32_t)n;
    }
}

constexpr int kClsItems = 16;  // flowIds per thread of k_seg_classify

__global__ void __launch_bounds__(256) k_seg_classify(BatchArgs a) {
    constexpr int kL = kClasses + 1;  // lists 0..kClasses-1: short length classes, kClasses: long
    __shared__ uint32_t cnt[kL], base[kL];
    const int tid = threadIdx.x;
    for (uint64_t k0 = (uint64_t)blockIdx.x * 256 * kClsItems; k0 < a.K; k0 += (uint64_t)gridDim.x * 256 * kClsItems) {
        if (tid < kL) cnt[tid] = 0;
        __syncthreads();
        uint32_t st[kClsItems], en[kClsItems], slot[kClsItems];
#pragma unroll
        for (int u = 0; u < kClsItems; ++u) {
            const uint64_t k = k0 + (uint64_t)u * 256 + tid;
            st[u] = k < a.K ? a.seg_start[k] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < kClsItems; ++u) {
            const uint64_t k = k0 + (uint64_t)u * 256 + tid;
            slot[u] = 0xFFFFFFFFu;
            if (st[u] == 0xFFFFFFFFu) continue;
            a.seg_start[k] = 0xFFFFFFFFu;  // both marks cleared for the next batch (the sort's last pass
            en[u] = a.seg_end[k];          // takes atomicMin / atomicMax of them)
            a.seg_end[k] = 0;
            const uint32_t len = en[u] - st[u];
            uint32_t l = 0;
#pragma unroll
            for (int c = 0; c < kClasses - 1; ++c) l += len > kClassMax[c] ? 1u : 0u;
            if (len > a.short_max) l = kClasses;
            slot[u] = (l << 24) | atomicAdd(&cnt[l], 1u);
        }
        __syncthreads();
        if (tid < kL) {
            const uint32_t t = cnt[tid];
            uint32_t* ctr = tid == kClasses ? a.long_count : a.short_count + tid;
            base[tid] = t ? atomicAdd(ctr, t) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kClsItems; ++u) {
            if (slot[u] == 0xFFFFFFFFu) continue;
            const uint32_t k = (uint32_t)(k0 + (uint64_t)u * 256 + tid);
            const uint32_t l = slot[u] >> 24, pos = base[l] + (slot[u] & 0xFFFFFFu);
            if (l == (uint32_t)kClasses) {
                a.long_list[pos] = st[u];
                a.long_key[pos] = k;
                a.long_end[pos] = en[u];
            } else {
                const uint64_t q = a.class_off[l] + pos;
                a.short_list[q] = st[u];
                a.short_key[q] = k;
                a.short_end[q] = en[u];
            }
        }
        __syncthreads();  // cnt / base are reused by the next range
    }
}

constexpr uint32_t kPoisonBytes = 65536;

// ------------------------------------------------------------------------------ binned front half
//
// One global pass instead of two: k_prep writes each valid record's bin digit into its free middle bits — the hot slot
// of a flowId among the previous batch's longest segments (a bin of its own: after the stable scatter its records
// are already its segment, in arrival order), else the flowId's key range key >> bin_bsh (a regular bin of at most
// 2^kBinMaxBsh flowIds) — and the one radix pass by that digit leaves the regular bins in a.bin_buf. k_bin_sort then
// sorts each regular bin by flowId with a counting sort in LDS (no second global pass, no segment-marking read) and
// lists every segment by length class as k_seg_classify would; k_hot_update picks the next batch's hot flowIds. The
// sorted array is rec_sorted: regular bins in flowId order, then one segment per hot flowId; the walkers need only
// each flowId's records contiguous and in arrival order, which both kinds of bin give. The hot set is a speed hint:
// a flowId outside it (or a stale one) is sorted by its regular bin, whatever its length.

// Block-aggregated list appends (k_seg_classify's scheme): class of a segment of `len` records.
__device__ __forceinline__ uint32_t seg_class(const BatchArgs& a, uint32_t len) {
    uint32_t l = 0;
#pragma unroll
    for (int c = 0; c < kClasses - 1; ++c) l += len > kClassMax[c] ? 1u : 0u;
    return len > a.short_max ? (uint32_t)kClasses : l;
}

__device__ __forceinline__ void seg_emit(const BatchArgs& a, uint32_t l, uint32_t pos, uint32_t st, uint32_t en,
                                         uint32_t k) {
    if (l == (uint32_t)kClasses) {
        a.long_list[pos] = st;
        a.long_key[pos] = k;
        a.long_end[pos] = en;
    } else {
        const uint64_t q = a.class_off[l] + pos;
        a.short_list[q] = st;
        a.short_key[q] = k;
        a.short_end[q] = en;
    }
}

constexpr uint32_t kBinKeys = 1u << kBinMaxBsh;
constexpr int kBinThreads = 512;
constexpr int kBinWaves = kBinThreads / 64;
constexpr int kBinPer = kBinKeys / kBinThreads;  // keys per thread in the scan (contiguous)
constexpr int kBinRows = 48;                     // 64-record rows a lane holds in registers
constexpr uint32_t kBinRegCap = kBinWaves * 64 * kBinRows;  // bins up to this size take the LDS path (24576)
constexpr uint32_t kBinStage = 14336;            // records of one output window staged in LDS (112 KB)
constexpr uint32_t kBinLdsWords = (kBinWaves * kBinKeys * 2 + kBinStage * 8) / 8;  // u16 counters + stage, in u64
static_assert(kBinWaves * kBinKeys * 4 <= kBinLdsWords * 8, "the big path's u32 counters fit the same LDS");

// Exclusive scan of the 1024 digit totals into dbase (every block: 4 KB, L2-resident).
__device__ __forceinline__ void bin_digit_bases(const BatchArgs& a, uint32_t* dbase, uint32_t* wsum) {
    constexpr int kD = 1 << kBinDigit, kPerT = kD / kBinThreads;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    uint32_t v[kPerT], sum = 0;
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
        v[i] = a.bin_tot[tid * kPerT + i];
        sum += v[i];
    }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
        dbase[tid * kPerT + i] = run;
        run += v[i];
    }
    __syncthreads();
}

// Lanes of this wave whose local key (< 2^kBinMaxBsh) equals this lane's: kBinMaxBsh ballots, branch-free (the
// bits above the bin's bsh are 0 in every lane and change nothing).
__device__ __forceinline__ uint64_t match_key(uint32_t d) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < kBinMaxBsh; ++b) {
        const uint64_t m = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? m : ~m;
    }
    return peers;
}

// Counters of the LDS path: u16 per (wave, flowId). Counted by 32-bit LDS atomics on the word holding two of them
// (1 << 16 for an odd index; a bin of <= kBinRegCap records keeps every count below 2^16, so no carry crosses), read
// and written as u16 only after a barrier: every access of the scan and of the placement has the same type, so the
// compiler keeps a wave's read of a counter after its earlier write (type-based alias analysis would let a u32 read
// pass a u16 store, and the placement's ranks depend on that order).
struct Cnt16 {
    uint32_t* w;
    __device__ __forceinline__ uint32_t get(uint32_t i) const { return reinterpret_cast<const uint16_t*>(w)[i]; }
    __device__ __forceinline__ void inc(uint32_t i) const { atomicAdd(&w[i >> 1], 1u << ((i & 1) * 16)); }
    __device__ __forceinline__ void set(uint32_t i, uint32_t v) const {
        reinterpret_cast<uint16_t*>(w)[i] = (uint16_t)v;
    }
};

// The per-flowId exclusive scan of a regular bin (thread tid's kBinPer contiguous flowIds), each flowId's per-wave
// bases written over its counters, and each segment's list slot within the block (wave ballots per class, lcnt).
template <class CNT>
__device__ __forceinline__ void bin_scan_lists(const BatchArgs& a, CNT cnt, uint32_t nk, uint32_t* wsum, uint32_t* lcnt,
                                               uint32_t* tk, uint32_t* sst, uint32_t* slot) {
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < kBinPer; ++i) {
        const uint32_t j = (uint32_t)tid * kBinPer + i;
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kBinWaves; ++w) t += cnt.get((uint32_t)w * kBinKeys + j);
        tk[i] = t;
        sum += t;
    }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();  // (wsum: the digit bases' scan is done with it)
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < kBinPer; ++i) {
        const uint32_t j = (uint32_t)tid * kBinPer + i;
        sst[i] = run;
        uint32_t pre = run;
#pragma unroll
        for (int w = 0; w < kBinWaves; ++w) {
            const uint32_t c = cnt.get((uint32_t)w * kBinKeys + j);
            cnt.set((uint32_t)w * kBinKeys + j, pre);
            pre += c;
        }
        run += tk[i];
        const uint32_t l = (tk[i] && j < nk) ? seg_class(a, tk[i]) : 0xFFu;
        slot[i] = 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c <= kClasses; ++c) {  // wave-aggregated slots per class
            const uint64_t m = __ballot(l == (uint32_t)c);
            if (!m) continue;
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&lcnt[c], (uint32_t)__popcll(m));
            b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
            if (l == (uint32_t)c) slot[i] = ((uint32_t)c << 24) | (b + (uint32_t)__popcll(m & lt));
        }
    }
}

__device__ __forceinline__ void bin_emit(const BatchArgs& a, const uint32_t* lbase, uint32_t s0, uint32_t kb0,
                                         const uint32_t* tk, const uint32_t* sst, const uint32_t* slot) {
#pragma unroll
    for (int i = 0; i < kBinPer; ++i) {
        if (slot[i] == 0xFFFFFFFFu) continue;
        const uint32_t l = slot[i] >> 24;
        seg_emit(a, l, lbase[l] + (slot[i] & 0xFFFFFFu), s0 + sst[i], s0 + sst[i] + tk[i],
                 kb0 + (uint32_t)threadIdx.x * kBinPer + i);
    }
}

// Blocks [0, R): regular bin b — a stable counting sort by flowId: wave w takes the w-th eighth of the bin in order and
// keeps its own counters, so its records of a flowId follow the earlier waves' ones. A bin of <= kBinRegCap records
// (the usual case) is read once into registers, all rows at once; every record's position is found there (ballot
// ranks, the wave's running counters), and the sorted bin leaves through LDS in windows of kBinStage records, one
// coalesced stream. A larger bin (a flowId that outgrew the hot set) counts in u32, reads its rows twice in groups and
// stores each record straight to its position. The list slots' global atomics (one per class per block) are issued
// before the placement and waited for after it. Block R: the hot bins' segments (one flowId each, in order already).
__global__ void __launch_bounds__(kBinThreads, 1) k_bin_sort(BatchArgs a) {
    constexpr int kL = kClasses + 1;
    __shared__ uint64_t lds[kBinLdsWords];
    __shared__ uint32_t dbase[1 << kBinDigit];
    __shared__ uint32_t wsum[kBinWaves];
    __shared__ uint32_t lcnt[kL], lbase[kL];
    if (*a.err) return;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    if (tid < kL) lcnt[tid] = 0;
    bin_digit_bases(a, dbase, wsum);
    const uint32_t b = blockIdx.x;
    if (b >= a.bin_R) {  // the hot bins
        constexpr int kHR = (kBinHot + kBinThreads - 1) / kBinThreads;
        uint32_t slot[kHR];
#pragma unroll
        for (int r = 0; r < kHR; ++r) {
            const uint32_t hs = (uint32_t)r * kBinThreads + tid;
            slot[r] = 0xFFFFFFFFu;
            if (hs >= kBinHot) continue;
            const uint32_t len = a.bin_tot[a.bin_R + hs];
            if (len == 0) continue;
            const uint32_t l = seg_class(a, len);
            slot[r] = (l << 24) | atomicAdd(&lcnt[l], 1u);
        }
        __syncthreads();
        if (tid < kL) {
            const uint32_t t = lcnt[tid];
            uint32_t* ctr = tid == kClasses ? a.long_count : a.short_count + tid;
            lbase[tid] = t ? atomicAdd(ctr, t) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kHR; ++r) {
            if (slot[r] == 0xFFFFFFFFu) continue;
            const uint32_t hs = (uint32_t)r * kBinThreads + tid;
            const uint32_t st = dbase[a.bin_R + hs], l = slot[r] >> 24;
            seg_emit(a, l, lbase[l] + (slot[r] & 0xFFFFFFu), st, st + a.bin_tot[a.bin_R + hs], a.hot_key[hs]);
        }
        return;
    }
    const uint32_t s0 = dbase[b], len = a.bin_tot[b];
    if (len == 0) return;
    const bool diag = (a.dbg & 65536) != 0;  // per-phase wall clock of the regular bins (dbg_ctr[40..47])
    uint64_t tk0 = diag ? __builtin_amdgcn_s_memrealtime() : 0, tk1 = 0, tk2 = 0, tk3 = 0, tp4 = 0, tp5 = 0, tp6 = 0;
    const int bsh = a.bin_bsh;
    const uint32_t kb0 = b << bsh;
    const uint32_t nk = min(1u << bsh, a.K - kb0);
    const uint32_t C = (len + kBinWaves - 1) / kBinWaves;
    const uint32_t c0 = s0 + min((uint32_t)wave * C, len), c1 = s0 + min((uint32_t)(wave + 1) * C, len);
    const bool small = len <= kBinRegCap;
    const uint32_t last = s0 + len - 1;  // loads are clamped into the bin (unconditional: no phi waits)
    const uint64_t* src = a.bin_buf;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t* lw = reinterpret_cast<uint32_t*>(lds);
    uint64_t v[kBinRows];
#pragma unroll
    for (int u = 0; u < kBinRows; ++u) v[u] = src[min(c0 + (uint32_t)u * 64 + (uint32_t)lane, last)];
    const uint32_t zw = small ? kBinWaves * kBinKeys / 2 : kBinWaves * kBinKeys;  // counter words
    for (uint32_t j = tid; j < zw; j += kBinThreads) lw[j] = 0;
    __syncthreads();
    if (diag) tk1 = __builtin_amdgcn_s_memrealtime();
    uint32_t tk[kBinPer], sst[kBinPer], slot[kBinPer], gb = 0;
    if (small) {
        const Cnt16 cnt{lw};
        // 1. counts per (wave, flowId)
#pragma unroll
        for (int u = 0; u < kBinRows; ++u) {
            const uint32_t j = c0 + (uint32_t)u * 64 + (uint32_t)lane;
            if (j < c1) cnt.inc((uint32_t)wave * kBinKeys + (uint32_t)(v[u] >> a.kshift) - kb0);
        }
        __syncthreads();
        if (diag) tk2 = __builtin_amdgcn_s_memrealtime();
        // 2. segment starts and list slots; the list atomics issued now, waited for after the placement
        bin_scan_lists(a, cnt, nk, wsum, lcnt, tk, sst, slot);
        __syncthreads();
        if (tid < kL && lcnt[tid]) gb = atomicAdd(tid == kClasses ? a.long_count : a.short_count + tid, lcnt[tid]);
        if (diag) tk3 = __builtin_amdgcn_s_memrealtime();
        // 3. positions (ballot ranks, the wave's running counters: LDS ops of one wave execute in order)
        uint32_t pos[kBinRows / 2];  // two u16 positions per register (< kBinRegCap; 0xFFFF: no record)
#pragma unroll
        for (int u = 0; u < kBinRows; ++u) {
            const uint32_t j = c0 + (uint32_t)u * 64 + (uint32_t)lane;
            const bool valid = j < c1;
            const uint32_t d = valid ? (uint32_t)(v[u] >> a.kshift) - kb0 : 0u;
            const uint64_t peers = match_key(d) & __ballot(valid);
            const uint32_t ci = (uint32_t)wave * kBinKeys + d;
            const uint32_t c = cnt.get(ci);
            const uint32_t p16 = valid ? c + (uint32_t)__popcll(peers & lt) : 0xFFFFu;
            pos[u / 2] = (u & 1) ? (pos[u / 2] | (p16 << 16)) : p16;
            // every lane writes its key's new count: peers write the same value, and an invalid lane (d = 0) writes
            // the count of the valid key-0 lanes or, without any, the count it read
            cnt.set(ci, c + (uint32_t)__popcll(peers));
            __builtin_amdgcn_sched_barrier(0);  // row by row: hoisting every row's ballots spilled them
        }
        if (diag) tp4 = __builtin_amdgcn_s_memrealtime();
        // 4. the sorted bin through LDS, kBinStage records at a time (the stage lies past the counters)
        uint64_t* stage = lds + (kBinWaves * kBinKeys * 2) / 8;
        uint64_t* dst = a.rec_sorted + s0;
        for (uint32_t w0 = 0; w0 < len; w0 += kBinStage) {
#pragma unroll
            for (int u = 0; u < kBinRows; ++u) {
                const uint32_t p = (pos[u / 2] >> ((u & 1) * 16)) & 0xFFFFu;
                if (p != 0xFFFFu && p - w0 < kBinStage) stage[p - w0] = v[u];
            }
            __syncthreads();
            const uint32_t m = min(kBinStage, len - w0);
            for (uint32_t p = tid; p < m; p += kBinThreads) dst[w0 + p] = stage[p];
            __syncthreads();
        }
    } else {
        uint32_t(*cnt)[kBinKeys] = reinterpret_cast<uint32_t(*)[kBinKeys]>(lw);
        struct Cnt32 {
            uint32_t* w;
            __device__ __forceinline__ uint32_t get(uint32_t i) const { return w[i]; }
            __device__ __forceinline__ void set(uint32_t i, uint32_t x) const { w[i] = x; }
        } c32{lw};
        for (uint32_t r0 = c0; r0 < c1; r0 += 64u * kBinRows) {
            if (r0 != c0) {
#pragma unroll
                for (int u = 0; u < kBinRows; ++u) v[u] = src[min(r0 + (uint32_t)u * 64 + (uint32_t)lane, last)];
            }
#pragma unroll
            for (int u = 0; u < kBinRows; ++u) {
                const uint32_t j = r0 + (uint32_t)u * 64 + (uint32_t)lane;
                if (j < c1) atomicAdd(&cnt[wave][(uint32_t)(v[u] >> a.kshift) - kb0], 1u);
            }
        }
        __syncthreads();
        if (diag) tk2 = __builtin_amdgcn_s_memrealtime();
        bin_scan_lists(a, c32, nk, wsum, lcnt, tk, sst, slot);
        __syncthreads();
        if (tid < kL && lcnt[tid]) gb = atomicAdd(tid == kClasses ? a.long_count : a.short_count + tid, lcnt[tid]);
        if (diag) tk3 = __builtin_amdgcn_s_memrealtime();
        uint64_t* dst = a.rec_sorted + s0;
        for (uint32_t r0 = c0; r0 < c1; r0 += 64u * kBinRows) {
#pragma unroll
            for (int u = 0; u < kBinRows; ++u) v[u] = src[min(r0 + (uint32_t)u * 64 + (uint32_t)lane, last)];
#pragma unroll
            for (int u = 0; u < kBinRows; ++u) {
                const uint32_t j = r0 + (uint32_t)u * 64 + (uint32_t)lane;
                const bool valid = j < c1;
                const uint32_t d = valid ? (uint32_t)(v[u] >> a.kshift) - kb0 : 0u;
                const uint64_t peers = match_key(d) & __ballot(valid);
                const uint32_t c = cnt[wave][d];
                if (valid) {
                    dst[c + (uint32_t)__popcll(peers & lt)] = v[u];
                    if (lane == __builtin_ctzll(peers)) cnt[wave][d] = c + (uint32_t)__popcll(peers);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (diag) tp5 = __builtin_amdgcn_s_memrealtime();
    if (tid < kL) lbase[tid] = gb;
    __syncthreads();
    if (diag) tp6 = __builtin_amdgcn_s_memrealtime();
    bin_emit(a, lbase, s0, kb0, tk, sst, slot);
    if (diag) {
        __syncthreads();
        if (tid == 0) {
            const uint64_t tk4 = __builtin_amdgcn_s_memrealtime();
            if (small) {
                atomicAdd(&a.dbg_ctr[48], (unsigned long long)(tp4 - tk3));
                atomicAdd(&a.dbg_ctr[49], (unsigned long long)(tp5 - tp4));
                atomicAdd(&a.dbg_ctr[50], (unsigned long long)(tp6 - tp5));
                atomicAdd(&a.dbg_ctr[51], (unsigned long long)(tk4 - tp6));
            }
            atomicAdd(&a.dbg_ctr[40], (unsigned long long)(tk1 - tk0));
            atomicAdd(&a.dbg_ctr[41], (unsigned long long)(tk2 - tk1));
            atomicAdd(&a.dbg_ctr[42], (unsigned long long)(tk3 - tk2));
            atomicAdd(&a.dbg_ctr[43], (unsigned long long)(tk4 - tk3));
            atomicAdd(&a.dbg_ctr[44], 1ull);
            atomicAdd(&a.dbg_ctr[45], small ? 0ull : 1ull);
            atomicAdd(&a.dbg_ctr[47], (unsigned long long)len);
        }
    }
}

// The next batch's hot flowIds: the segments of more than short_max records, the longest first (a histogram of
// floor(log2 len) picks the length class that fills kBinHot slots), as an open-addressing table {flowId, slot} built in
// LDS and written whole. One block; runs after k_bin_sort on the front stream, so the next k_prep reads the new table.
__global__ void __launch_bounds__(1024) k_hot_update(BatchArgs a) {
    __shared__ uint32_t hcnt[32];
    __shared__ uint32_t thr, nslot;
    __shared__ uint32_t tkey[kHotTab], tslot[kHotTab], bfill[kHotTab / kHotWays];
    const uint32_t tid = threadIdx.x;
    if (tid < 32) hcnt[tid] = 0;
    if (tid == 0) nslot = 0;
    for (uint32_t x = tid; x < kHotTab; x += 1024) {
        tkey[x] = kHotEmpty;
        tslot[x] = 0;
    }
    for (uint32_t x = tid; x < kHotTab / kHotWays; x += 1024) bfill[x] = 0;
    __syncthreads();
    const uint32_t nl = *a.err ? 0u : *a.long_count;  // a refused batch listed nothing: no hot flowIds next
    for (uint32_t i = tid; i < nl; i += 1024) {
        const uint32_t len = a.long_end[i] - a.long_list[i];
        atomicAdd(&hcnt[31 - __clz(len)], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // the lowest length class whose longer segments still fit the slots
        uint32_t cum = 0, t = 0;
        for (int c = 31; c >= 0; --c) {
            cum += hcnt[c];
            if (cum >= kBinHot) {
                t = (uint32_t)c;
                break;
            }
        }
        thr = t;
    }
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {  // the classes above thr first (they fit), then thr's own in any order
        for (uint32_t i = tid; i < nl; i += 1024) {
            const uint32_t len = a.long_end[i] - a.long_list[i];
            const uint32_t c = 31 - __clz(len);
            if (pass == 0 ? c <= thr : c != thr) continue;
            if (nslot >= kBinHot) continue;  // (a stale read only costs a wasted attempt)
            const uint32_t k = a.long_key[i];
            const uint32_t bk = hot_hash(k);
            const uint32_t w = atomicAdd(&bfill[bk], 1u);
            if (w >= kHotWays) continue;  // home bucket full: the flowId stays in its regular bin
            const uint32_t s = atomicAdd(&nslot, 1u);
            if (s >= kBinHot) {
                tkey[bk * kHotWays + w] = kHotEmpty;  // (this way stays empty)
                continue;
            }
            a.hot_key[s] = k;
            tkey[bk * kHotWays + w] = k;
            tslot[bk * kHotWays + w] = s;
        }
        __syncthreads();
    }
    for (uint32_t x = tid; x < kHotTab; x += 1024) a.hot_tab[x] = make_uint2(tkey[x], tslot[x]);
}

__global__ void __launch_bounds__(256) k_hot_reset(uint2* hot_tab) {
    for (uint32_t x = threadIdx.x; x < kHotTab; x += 256) hot_tab[x] = make_uint2(kHotEmpty, 0u);
}

// Stage the batch's period tables in g_sbnd when they fit (else the cursors read a.bnd).
__device__ __forceinline__ void stage_periods(const BatchArgs& a) {
    uint32_t tot = 0;
    for (int w = 0; w < a.n_wl; ++w) tot += a.np[w];
    const bool lds = tot <= (uint32_t)kLdsBndFlow && !(a.dbg & 1);
    uint32_t off = 0;
    for (int w = 0; w < a.n_wl; ++w) {
        const uint32_t npw = a.np[w];
        if (lds) {
            const uint32_t* g = a.bnd + (size_t)w * kMaxPeriods;
            for (uint32_t i = threadIdx.x; i < npw; i += blockDim.x) g_sbnd[off + i] = g[i];
        }
        if (threadIdx.x == 0) g_boff[w] = off;
        off += npw;
    }
    if (threadIdx.x == 0) g_blds = lds ? 1 : 0;
    if (threadIdx.x < (unsigned)a.n_wl) {
        g_p0[threadIdx.x] = a.p0[threadIdx.x];
        g_np[threadIdx.x] = a.np[threadIdx.x];
    }
    for (uint32_t x = threadIdx.x; x < (uint32_t)a.n_wl * (kModS + 1); x += blockDim.x) {
        const uint32_t w = x / (kModS + 1), m = x % (kModS + 1);
        g_p0mod[w][m] = m ? (uint8_t)(a.p0[w] % (int64_t)m) : (uint8_t)0;  // p0 >= 0: timestamps are
    }
    __syncthreads();
}

// Long-segment walker: one wave per segment of more than short_max records (grid-stride over the list,
// grid sized to what is resident at once). Runs concurrently with k_walk_short (separate stream).
template <bool L>
__device__ __forceinline__ void walk_long_body(const BatchArgs& a) {
    const int lane = lane_id();
    const uint32_t n_long = *a.long_count;
    // static wave → item assignment (wave-uniform loop control; a dynamic atomic work queue here
    // miscompiled: lanes of a wave lost convergence after the first walk)
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t item = wave; item < n_long; item += nwaves) {
        const uint64_t s = a.long_list[item];
        uint32_t k;
        uint64_t e;
        if (a.long_key && a.seg_end) {  // segment key and end from k_seg / k_seg_classify
            k = a.long_key[item];
            e = a.long_end ? a.long_end[item] : a.seg_end[k];
        } else {  // segment end: the first record with another flowId
            k = (uint32_t)(a.rec_sorted[s] >> a.kshift);
            e = gallop_search(s + (a.short_max ? a.short_max : 1), a.n, [&](uint64_t p) {
                return (uint32_t)(a.rec_sorted[p] >> a.kshift) != k;
            }, lane);
        }
        const uint64_t t0 = (a.dbg & 64) ? __builtin_amdgcn_s_memrealtime() : 0;
        walk_wave<L>(a, k, s, e, item);
        if (a.dbg & 64) {
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            const uint64_t len = e - s;
            const int b = len <= 64 ? 0 : len <= 256 ? 1 : len <= 1024 ? 2 : 3;
            if (lane == 0) {
                atomicAdd(&a.dbg_ctr[16 + 2 * b], 1ull);
                atomicAdd(&a.dbg_ctr[17 + 2 * b], (unsigned long long)(t1 - t0));
                atomicMax(&a.dbg_ctr[24 + b], (unsigned long long)(t1 - t0));
            }
        }
    }
}

// Period ends of the long segments (one thread per segment and period): the wave walker jumps over a
// window period that can admit nothing more without searching for where it ends (that search was a
// chain of dependent loads per period). Runs on the wave walker's stream just before it.
__global__ void __launch_bounds__(256) k_long_bounds(BatchArgs a) {
    if (*a.err) return;
    const uint32_t n_long = min(*a.long_count, kLongTab);
    const uint32_t total = n_long * (uint32_t)kLongPeriods;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const uint32_t item = t / kLongPeriods, q = t % kLongPeriods;
        const uint32_t k = a.long_key[item];
        const int w = a.rules[k].wl_idx;
        const uint32_t npw = a.np[w];
        if (npw > (uint32_t)kLongPeriods || q + 1 >= npw) continue;
        const uint32_t nb = a.bnd[(size_t)w * kMaxPeriods + q + 1];
        uint64_t lo = a.long_list[item], hi = a.long_end ? a.long_end[item] : a.seg_end[k];
        while (lo < hi) {  // first record of the segment in period q + 1 or later
            const uint64_t mid = (lo + hi) >> 1;
            if ((uint32_t)((a.rec_sorted[mid] >> a.abits) & a.imask) >= nb) hi = mid;
            else lo = mid + 1;
        }
        a.long_pend[t] = (uint32_t)lo;
    }
}

#ifndef SG_WLONG_BLOCKS
#define SG_WLONG_BLOCKS 2
#endif
__global__ void __launch_bounds__(256, SG_WLONG_BLOCKS) k_walk_long(BatchArgs a) {
    if (*a.err || (a.dbg & 4096)) return;
    stage_periods(a);
    if (g_blds) walk_long_body<true>(a);
    else walk_long_body<false>(a);
}

// Serial walk of one flowId segment with the ring's {period, PASS, WAITING} of all SM >= S slots held in
// registers: the ring is read from HBM once (and slot I's full bucket only when the batch continues the
// stored period), each closed bucket is written back, nothing is re-read. Same decisions as walk_serial,
// which re-reads the ring at every new period (the working set of all lanes does not fit L2).

// {start, PASS, WAITING} of one ring slot, staged in LDS by a wave's cooperative ring gather: 12 B, so that
// four 256-thread blocks of the short walker fit a CU's LDS. `st` is the window start relative to the batch's
// base time T0 (INT32_MIN: never created; starts older than T0 - 2^30 clamp to -2^30, which every validity
// test treats as deprecated). PASS and WAITING are exact in int32 when BatchArgs::narrow holds (the host's
// bound on every rule's threshold, see upload_rule_table); the walker runs only then, and when the batch's
// periods lie within 2^29 ms of T0 (narrow_span).
struct SlotSnap {
    int32_t st, pass, wait;
};
constexpr int32_t kSnapOld = -(1 << 30);

// A relative bound clamped to 32 bits: compares with snapshot starts as the 64-bit one (an empty slot, INT32_MIN,
// holds no counts either way).
__device__ __forceinline__ int32_t rel32(int64_t x) {
    return x > (int64_t)INT32_MAX ? INT32_MAX : x < (int64_t)INT32_MIN ? INT32_MIN : (int32_t)x;
}

__device__ __forceinline__ int32_t snap_rel(int64_t start, int64_t T0) {
    if (start == INT64_MIN) return INT32_MIN;
    const int64_t d = start - T0;
    return d < (int64_t)kSnapOld ? kSnapOld : d > (int64_t)(1 << 30) ? (1 << 30) : (int32_t)d;
}

// All of the batch's window periods, and S + 1 periods before them, lie within 2^29 ms of T0 (wave-uniform).
__device__ __forceinline__ bool narrow_span(const BatchArgs& a, int64_t T0) {
    bool ok = true;
    for (int w = 0; w < a.n_wl; ++w) {
        const int64_t wl = a.wl[w];
        const int64_t b = a.p0[w] * wl;
        ok = ok && (b + ((int64_t)a.np[w] + 1) * wl - T0 < (1ll << 29)) &&
             (b - ((int64_t)a.stride + 1) * wl - T0 > -(1ll << 29));
    }
    return ok;
}

// k_walk_tiny takes length class 0 (same answer in every kernel of the batch: batch constants only)
__device__ __forceinline__ bool tiny_active(const BatchArgs& a) {
    return a.tiny && a.narrow && narrow_span(a, a.p0[0] * (int64_t)a.wl[0]);
}

__device__ __forceinline__ void store_bucket(Bucket* b, BucketHot* h, int64_t start, const int64_t* c) {
    ulonglong2* p = reinterpret_cast<ulonglong2*>(b);
    p[0] = make_ulonglong2((unsigned long long)start, (unsigned long long)c[0]);
    p[1] = make_ulonglong2((unsigned long long)c[1], (unsigned long long)c[2]);
    p[2] = make_ulonglong2((unsigned long long)c[3], (unsigned long long)c[4]);
    p[3] = make_ulonglong2((unsigned long long)c[5], (unsigned long long)c[6]);
    store_hot(h, start, c[SG_EV_PASS], c[SG_EV_WAITING]);
}

constexpr int kBlk = 4;  // records per block of the short walker's double-buffered record stream

// Walk of one flowId segment per lane, all 64 lanes of the wave together (inactive lanes pass act =
// false). `snap` holds the lane's ring snapshot {start, PASS, WAITING} of its S <= SM slots (gathered
// by the wave into LDS, kept up to date as buckets close) and `buf` its first kBlk records (loaded by the
// caller, so that every load of the wave's group is in flight at once). Same decisions as walk_serial.
//
// Phased for SIMT: a lane whose next record starts a new window period parks; the wave runs the cheap
// per-record step (one decision) while any lane can take it, then opens the parked lanes' periods in one
// pass. The period-open code (ring sums over S slots, bucket close) thus runs ~once per period of the
// wave instead of in almost every record step (64 lanes each change period every few records).
template <int SM, bool L>
__device__ __forceinline__ void walk_reg(const BatchArgs& a, bool act, uint32_t k, uint64_t s, uint64_t e,
                                         const Rule& R, const Occ& occ, SlotSnap* snap, uint64_t* buf, int64_t T0) {
    Bucket* ring = a.ring + (size_t)k * a.stride;
    BucketHot* hot = a.hot + (size_t)k * a.stride;
    const int S = R.S;
    const int64_t wl = R.wl;
    PeriodCursor<L> pc;
    pc.init(a, act ? R.wl_idx : 0);
    const int64_t P0 = g_p0[act ? R.wl_idx : 0];
    PeriodState ps;
    ps.occ_pass = occ.pass;
    ps.occ_req = occ.pass_req;
#pragma unroll
    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ps.cur[ev] = 0;
    ps.wo_pass = ps.wo_wait = ps.head_other = 0;
    int I = -1;      // slot of the open period
    int64_t ws = 0;  // its window start
    // Record loads are unconditional (indices clamped to n - 1; the segment end is tested by position): a
    // conditional load's value meets a constant in a phi, and that copy waits for the load at once, which
    // turned the prefetch into a full memory round trip every kBlk records.
    const uint64_t n1 = a.n - 1;
    uint64_t nb[kBlk];
    uint64_t p = s;  // position of buf[0]'s block
    int left = kBlk; // records of the current block not yet consumed (buf[0] is the next one)
    bool more = act && p + kBlk < e;  // the segment continues past this block
#pragma unroll
    for (int u = 0; u < kBlk; ++u) nb[u] = a.rec_sorted[min(p + kBlk + u, n1)];
    bool live = act;  // records left
    uint32_t qn = 0;  // period of the next record (valid when live)
    Decoded dn;       // the next record, decoded
    auto peek = [&]() {  // look at buf[0]: end of segment, or decode it and find its period
        if (p + (uint64_t)(kBlk - left) >= e) {
            live = false;
            return;
        }
        dn = decode(a, buf[0]);
        qn = pc.of(dn.idx);
    };
    auto advance = [&]() {  // consume buf[0]
#pragma unroll
        for (int v = 0; v < kBlk - 1; ++v) buf[v] = buf[v + 1];  // resident values: plain moves
        buf[kBlk - 1] = ~0ull;
        if (--left == 0) {
            if (!more) {
                live = false;
                return;
            }
#pragma unroll
            for (int u = 0; u < kBlk; ++u) buf[u] = nb[u];
            p += kBlk;
            left = kBlk;
            more = p + kBlk < e;
#pragma unroll
            for (int u = 0; u < kBlk; ++u) nb[u] = a.rec_sorted[min(p + kBlk + u, n1)];
        }
    };
    if (live) peek();
    while (__ballot(live)) {
        // 1. open the period of every lane whose next record starts one (the first record included)
        if (live && qn != pc.q) {
            if (I >= 0) {  // close the open bucket: memory and the snapshot
                if (!(a.dbg & 512)) store_bucket(ring + I, hot + I, ws, ps.cur);
                snap[I].st = (int32_t)(ws - T0);
                snap[I].pass = (int32_t)ps.cur[SG_EV_PASS];
                snap[I].wait = (int32_t)ps.cur[SG_EV_WAITING];
            }
            const uint32_t qprev = pc.q;
            pc.seek(qn);
            const int64_t P = P0 + (int64_t)qn;
            I = I < 0 ? period_slot(R.wl_idx, qn, S) : (int)((uint32_t)(I + (int)(qn - qprev)) % (uint32_t)S);
            ws = P * wl;
            // LeapArray.isWindowDeprecated: valid iff start > ws - S*wl (compared relative to T0)
            const int64_t lo_rel = ws - (int64_t)S * wl - T0;
            const int32_t lo32 = rel32(lo_rel);  // snapshot starts are 32-bit (snap_rel)
            const int h = I + 1 == S ? 0 : I + 1;
            // all slots read at once, then summed branch-free; sums of valid buckets are window sums, < 2^30
            // under BatchArgs::narrow, so 32-bit accumulation is exact
            int32_t sx[SM], px[SM], wx[SM];
#pragma unroll
            for (int x = 0; x < SM; ++x) {
                sx[x] = snap[x].st;
                px[x] = snap[x].pass;
                wx[x] = snap[x].wait;
            }
            uint32_t wp = 0, ww = 0, ho = 0;
#pragma unroll
            for (int x = 0; x < SM; ++x) {
                const bool v = (x < S) & (x != I) & (sx[x] > lo32);
                const uint32_t m = v ? 0xFFFFFFFFu : 0u;
                wp += (uint32_t)px[x] & m;
                ww += (uint32_t)wx[x] & m;
                ho = (x == h) ? ((uint32_t)px[x] & m) : ho;
            }
            ps.wo_pass = (int64_t)wp;
            ps.wo_wait = (int64_t)ww;
            ps.head_other = (int64_t)ho;
            // currentWindow on slot I: continue (only possible at the batch's first period), create or reset
            const int32_t stI_rel = snap[I].st;
            const int64_t stI = stI_rel == INT32_MIN ? INT64_MIN : T0 + (int64_t)stI_rel;
            int64_t cI[SG_NUM_EVENTS];
            if (stI == ws) {
#pragma unroll
                for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = ring[I].c[ev];
            }
            open_bucket(ps, stI, cI, ws);
        }
        // 2. decide records while they stay in the open period (ClusterFlowChecker.acquireClusterToken :67-111)
        while (live && qn == pc.q) {
            const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
            const double next_remaining = R.thr - latest - (double)dn.acq;
            if (next_remaining >= 0) {
                ps.cur[SG_EV_PASS] += dn.acq;
                ps.cur[SG_EV_PASS_REQUEST] += 1;
                if (dn.prio) ps.cur[SG_EV_OCCUPIED_PASS] += dn.acq;
                if (!(a.dbg & 256)) store_result(a.out, dn.idx, SG_STATUS_OK, java_d2i(next_remaining), 0);
            } else {
                int32_t wait;
                const int32_t stt = decide_fail(R, a.max_occ_ratio, ps, dn.acq, dn.prio, &wait);
                if (stt != SG_STATUS_BLOCKED && !(a.dbg & 256)) store_result(a.out, dn.idx, stt, 0, wait);
            }
            advance();
            if (live) peek();
        }
    }

    if (act) {
        if (I >= 0) store_bucket(ring + I, hot + I, ws, ps.cur);
        if (ps.occ_pass != occ.pass || ps.occ_req != occ.pass_req) {  // rarely changes: no partial-line store
            Occ o;
            o.pass = ps.occ_pass;
            o.pass_req = ps.occ_req;
            a.occ[k] = o;
        }
    }
}

// LDS-DMA of the compact records at positions p .. p + R - 1 of every active lane
// into its column of `wrecs` ([kRecW][64] words: row r, lane j). No VGPR holds a record in flight, so nothing
// waits for these loads until the walk reads them (one vmcnt wait per window instead of one per few records).
// p < n: the record buffers have kRecW records of slack past max_batch, so the window needs no clamping.
// s_waitcnt vmcnt(0) as a builtin (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15), not inline asm: the compiler's
// wait-count pass sees it and knows the LDS-DMA writes have landed. After an inline-asm wait it still counted them
// as pending and put a vmcnt(0) before every later LDS read of the loop — each one also waiting for the stores
// issued since (a store round trip per period open).
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int R>
__device__ __forceinline__ void glds_rows(const uint32_t* src, uint32_t* wrecs) {
    if constexpr (R > 0) {
        // row R - 1: the low word of record R - 1. The immediate offset (8 (R - 1) bytes) is added to the LDS
        // address too, so the LDS base is moved back by as much.
        glds_rows<R - 1>(src, wrecs);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(wrecs + (R - 1) * 64 - 2 * (R - 1)),
                                         4, 8 * (R - 1), 0);
    }
}

template <int R>
__device__ __forceinline__ void stage_records(const BatchArgs& a, uint32_t* wrecs, uint64_t p) {
    glds_rows<R>(reinterpret_cast<const uint32_t*>(a.rec_sorted + p), wrecs);
}

// walk_reg with the records read from LDS: the group staged each lane's first kRecW compact records (with the
// ring gather, one wait for both); a lane that has used its window parks, and when no lane can go on the wave
// stages the parked lanes' next windows at once. Same decisions as walk_serial.
template <int SM, bool L>
__device__ __forceinline__ void walk_lds(const BatchArgs& a, bool act, uint32_t k, uint64_t s, uint64_t e,
                                         const Rule& R, const Occ& occ, SlotSnap* snap, uint32_t* wrecs, int lane,
                                         int64_t T0, int rows) {
    Bucket* ring = a.ring + (size_t)k * a.stride;
    BucketHot* hot = a.hot + (size_t)k * a.stride;
    const int S = R.S;
    const int64_t wl = R.wl;
    PeriodCursor<L> pc;
    pc.init(a, act ? R.wl_idx : 0);
    const int64_t P0 = g_p0[act ? R.wl_idx : 0];
    PeriodState ps;
    ps.occ_pass = occ.pass;
    ps.occ_req = occ.pass_req;
#pragma unroll
    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ps.cur[ev] = 0;
    ps.wo_pass = ps.wo_wait = ps.head_other = 0;
    int I = -1;      // slot of the open period
    int64_t ws = 0;  // its window start
    uint64_t wb = s;  // position of the lane's LDS window row 0
    uint64_t p = s;   // position of the next record
    bool live = act && p < e;
    bool park = false;  // window used up, records left
    uint32_t win = (uint32_t)rows;  // records in the lane's window (the first window may be shorter than kRecW)
    uint32_t qn = 0;    // period of the next record (valid when live && !park)
    Decoded dn;
    auto peek = [&]() {
        if (p >= e) {
            live = false;
            return;
        }
        if (p - wb >= (uint64_t)win) {
            park = true;
            return;
        }
        dn = decode_c(a, wrecs[(uint32_t)(p - wb) * 64 + lane]);
        qn = pc.of(dn.idx);
    };
    if (live) peek();
    for (;;) {
        if (!__ballot(live && !park)) {
            if (!__ballot(live)) break;
            // every live lane waits for its next window: stage them all, one wait
            if (park) {
                stage_records<kRecW>(a, wrecs, p);
                wb = p;
                win = kRecW;
            }
            wait_vm0();
            __builtin_amdgcn_wave_barrier();
            if (park) {
                park = false;
                peek();
            }
            continue;
        }
        // 1. open the period of every lane whose next record starts one (the first record included)
        if (live && !park && qn != pc.q) {
            if (I >= 0) {  // close the open bucket: memory and the snapshot
                store_bucket(ring + I, hot + I, ws, ps.cur);
                snap[I].st = (int32_t)(ws - T0);
                snap[I].pass = (int32_t)ps.cur[SG_EV_PASS];
                snap[I].wait = (int32_t)ps.cur[SG_EV_WAITING];
            }
            const uint32_t qprev = pc.q;
            pc.seek(qn);
            const int64_t P = P0 + (int64_t)qn;
            I = I < 0 ? period_slot(R.wl_idx, qn, S) : (int)((uint32_t)(I + (int)(qn - qprev)) % (uint32_t)S);
            ws = P * wl;
            const int64_t lo_rel = ws - (int64_t)S * wl - T0;
            const int32_t lo32 = rel32(lo_rel);  // snapshot starts are 32-bit (snap_rel)
            const int h = I + 1 == S ? 0 : I + 1;
            int32_t sx[SM], px[SM], wx[SM];
#pragma unroll
            for (int x = 0; x < SM; ++x) {
                sx[x] = snap[x].st;
                px[x] = snap[x].pass;
                wx[x] = snap[x].wait;
            }
            uint32_t wp = 0, ww = 0, ho = 0;
#pragma unroll
            for (int x = 0; x < SM; ++x) {
                const bool v = (x < S) & (x != I) & (sx[x] > lo32);
                const uint32_t m = v ? 0xFFFFFFFFu : 0u;
                wp += (uint32_t)px[x] & m;
                ww += (uint32_t)wx[x] & m;
                ho = (x == h) ? ((uint32_t)px[x] & m) : ho;
            }
            ps.wo_pass = (int64_t)wp;
            ps.wo_wait = (int64_t)ww;
            ps.head_other = (int64_t)ho;
            const int32_t stI_rel = snap[I].st;
            const int64_t stI = stI_rel == INT32_MIN ? INT64_MIN : T0 + (int64_t)stI_rel;
            int64_t cI[SG_NUM_EVENTS];
            if (stI == ws) {
#pragma unroll
                for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = ring[I].c[ev];
            }
            open_bucket(ps, stI, cI, ws);
        }
        // 2. decide records while they stay in the open period (ClusterFlowChecker.acquireClusterToken :67-111)
        while (live && !park && qn == pc.q) {
            const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
            const double next_remaining = R.thr - latest - (double)dn.acq;
            if (next_remaining >= 0) {
                ps.cur[SG_EV_PASS] += dn.acq;
                ps.cur[SG_EV_PASS_REQUEST] += 1;
                if (dn.prio) ps.cur[SG_EV_OCCUPIED_PASS] += dn.acq;
                store_result(a.out, dn.idx, SG_STATUS_OK, java_d2i(next_remaining), 0);
            } else {
                int32_t wait;
                const int32_t stt = decide_fail(R, a.max_occ_ratio, ps, dn.acq, dn.prio, &wait);
                if (stt != SG_STATUS_BLOCKED) store_result(a.out, dn.idx, stt, 0, wait);
            }
            ++p;
            peek();
        }
    }
    if (act) {
        if (I >= 0) store_bucket(ring + I, hot + I, ws, ps.cur);
        if (ps.occ_pass != occ.pass || ps.occ_req != occ.pass_req) {  // rarely changes: no partial-line store
            Occ o;
            o.pass = ps.occ_pass;
            o.pass_req = ps.occ_req;
            a.occ[k] = o;
        }
    }
}

// Short-segment walker: each wave takes 64 segments of <= short_max records of one length class and
// walks one per lane; the classes of longer segments go first. SM > 0: ring snapshot in LDS (every flow
// has sampleCount <= SM <= kGatherMaxS); SM == 0: generic walker re-reading the ring.
//
// SM > 0, one group of 64 segments: every load the group needs is issued before any is waited for
// (k_seg hands over each segment's flowId with its start): the rules, occupy counters, first record
// blocks, and the rings. Rings of up to kGatherMaxS slots are gathered cooperatively into LDS — a
// wave-instruction loads 16-B pieces of ~3 consecutive rings ({start, PASS} at byte 0 and
// {OCCUPIED_BLOCK, WAITING} at byte 48 of each bucket), row-shaped instead of 64 lanes in 64 rows.
constexpr int kGatherMaxS = 10;
#ifndef SG_SHORT_BLOCKS
#define SG_SHORT_BLOCKS 3
#endif
constexpr int kShortBlocksPerCu = SG_SHORT_BLOCKS;  // occupancy target (VGPR budget) of the short walker

// Short walker over compact LDS records (C): as walk_short_body, with each group's segment descriptors loaded
// one group ahead (they ride along with the previous group's loads, so a group costs one memory round trip
// before its walk: ring, rule, occupy counters, segment end and records together) and first record windows
// sized to the length class.
template <int SM, bool L>
__device__ __forceinline__ void walk_short_lds(const BatchArgs& a, SlotSnap* snap_all, uint32_t* recs_all) {
    static_assert(SM > 0, "LDS ring snapshot");
    const int lane = lane_id();
    const bool tiny = tiny_active(a);
    SlotSnap* snap = snap_all + (threadIdx.x / 64) * (64 * SM);
    uint32_t* wrecs = recs_all + (threadIdx.x / 64) * (kRecW * 64);
    uint32_t cnt[kClasses], grp_end[kClasses];
    uint32_t total = 0;
#pragma unroll
    for (int c = kClasses - 1; c >= 0; --c) {  // group order: longest class first
        cnt[c] = (c == 0 && tiny) ? 0u : a.short_count[c];  // class 0: k_walk_tiny
        total += (cnt[c] + 63) / 64;
        grp_end[c] = total;
    }
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    if (wave >= total) return;
    const int64_t T0 = a.p0[0] * (int64_t)a.wl[0];
    // group g: class (wave-uniform), this lane's list entry; inactive lanes of a class's last group repeat
    // the class's entry 0 (valid addresses)
    auto desc = [&](uint32_t g, int& c, bool& act, uint32_t& s, uint32_t& k, uint32_t& e) {
        c = kClasses - 1;
        uint32_t g0 = 0;
        while (g >= grp_end[c]) {
            g0 = grp_end[c];
            --c;
        }
        c = __builtin_amdgcn_readfirstlane(c);
        const uint32_t i = (g - g0) * 64 + (uint32_t)lane;
        act = i < cnt[c];
        const uint64_t li = a.class_off[c] + (act ? i : 0u);
        s = a.short_list[li];
        k = a.short_key[li];
        e = a.short_end[li];
    };
    int c_n;
    bool act_n;
    uint32_t s_n, k_n, e_n;
    desc(wave, c_n, act_n, s_n, k_n, e_n);
    for (uint32_t g = wave; g < total; g += nwaves) {
        const uint64_t tw0 = (a.dbg & 64) ? __builtin_amdgcn_s_memrealtime() : 0;
        const int c = c_n;
        const bool act = act_n;
        const uint64_t s = s_n;
        const uint32_t k = k_n;
        const uint64_t e = e_n;
        const Rule R = a.rules[k];
        const Occ occ = a.occ[k];
        // first window: the class's longest segment (<= 4, <= 16 records) or kRecW
        static_assert(kRecW >= (int)kClassMax[1], "the first window of class 1 must fit the lane's LDS rows");
        const int rows = c == 0 ? (int)kClassMax[0] : c == 1 ? (int)kClassMax[1] : kRecW;
        if (c == 0) stage_records<kClassMax[0]>(a, wrecs, s);
        else if (c == 1) stage_records<kClassMax[1]>(a, wrecs, s);
        else stage_records<kRecW>(a, wrecs, s);
        // the next group's descriptors (unconditional: a conditional load would be copied, and wait, at the merge)
        desc(min(g + nwaves, total - 1), c_n, act_n, s_n, k_n, e_n);
        {
            // ring gather from the hot mirror: piece t*64 + lane = bucket q of the ring of lane j = piece / SM,
            // {start, PASS | WAITING << 32} (16 B: a flowId's ten buckets are 160 contiguous bytes); slots past the
            // handle's stride read slot 0 again (ignored: q >= S). Every piece is loaded before any is used (the
            // scheduling barrier keeps the compiler from interleaving the loads with their LDS writes, which
            // serialised the gather into round trips)
            constexpr int kT = SM;
            int gl = lane;
            asm volatile("" : "+v"(gl));
            ulonglong2 v[kT];
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                const int pc = t * 64 + gl;
                const int j = pc / kT;
                const int q = pc % kT;
                const uint32_t kj = (uint32_t)__shfl((int)k, j, 64);
                const int qq = q < a.stride ? q : 0;
                v[t] = *reinterpret_cast<const ulonglong2*>(a.hot + (size_t)kj * a.stride + qq);
            }
            __builtin_amdgcn_sched_barrier(0);
            // every dword of every piece stays live until here: the allocator would otherwise reuse the unused
            // halves as temporaries, and overwriting a register a load is still filling waits for that load
#pragma unroll
            for (int t = 0; t < kT; ++t) asm volatile("" ::"v"(v[t].x), "v"(v[t].y));
#pragma unroll
            for (int t = 0; t < kT; ++t) {
                const int pc = t * 64 + gl;
                SlotSnap& d = snap[pc];  // (pc / SM) * SM + pc % SM
                d.st = snap_rel((int64_t)v[t].x, T0);
                d.pass = (int32_t)(uint32_t)v[t].y;
                d.wait = (int32_t)(uint32_t)(v[t].y >> 32);
            }
        }
        wait_vm0();  // the staged records have landed
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t tw1 = (a.dbg & 64) ? __builtin_amdgcn_s_memrealtime() : 0;
        walk_lds<SM, L>(a, act, k, s, e, R, occ, snap + lane * SM, wrecs, lane, T0, rows);
        if (a.dbg & 64) {  // per class: groups, gather time, walk time (100 MHz ticks)
            const uint64_t tw2 = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) {
                atomicAdd(&a.dbg_ctr[0], (unsigned long long)(tw2 - tw0));
                atomicAdd(&a.dbg_ctr[1 + c], 1ull);
                atomicAdd(&a.dbg_ctr[7 + c], (unsigned long long)(tw1 - tw0));
                atomicAdd(&a.dbg_ctr[7 + c], (unsigned long long)(tw2 - tw1) << 32);
            }
        }
    }
}

template <int SM, bool L, bool C>
__device__ __forceinline__ void walk_short_body(const BatchArgs& a, SlotSnap* snap_all, uint32_t* recs_all) {
    if constexpr (SM > 0 && C) {
        const int64_t T0 = a.p0[0] * (int64_t)a.wl[0];
        if (a.narrow && narrow_span(a, T0)) {
            walk_short_lds<SM, L>(a, snap_all, recs_all);
            return;
        }
    }
    constexpr int kSnapPerWave = SM > 0 ? 64 * SM : 1;
    const int lane = lane_id();
    const bool tiny = tiny_active(a);
    SlotSnap* snap = snap_all + (threadIdx.x / 64) * kSnapPerWave;
    uint32_t cnt[kClasses], grp_end[kClasses];
    uint32_t total = 0;
#pragma unroll
    for (int c = kClasses - 1; c >= 0; --c) {  // group order: longest class first
        cnt[c] = (c == 0 && tiny) ? 0u : a.short_count[c];  // class 0: k_walk_tiny
        total += (cnt[c] + 63) / 64;
        grp_end[c] = total;
    }
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    // the LDS-snapshot walker needs the narrow encoding (else every lane re-reads its ring: walk_serial)
    const int64_t T0 = a.p0[0] * (int64_t)a.wl[0];
    const bool snap_ok = SM > 0 && a.narrow && narrow_span(a, T0);
    for (uint32_t g = wave; g < total; g += nwaves) {
        int c = kClasses - 1;
        uint32_t g0 = 0;
        while (g >= grp_end[c]) {
            g0 = grp_end[c];
            --c;
        }
        c = __builtin_amdgcn_readfirstlane(c);
        const uint32_t i = (g - g0) * 64 + (uint32_t)lane;
        const bool act = i < cnt[c];
        if constexpr (SM > 0 && !C) if (snap_ok) {
            const uint64_t tw0 = (a.dbg & 64) ? __builtin_amdgcn_s_memrealtime() : 0;
            // 1. segment descriptors (inactive lanes of the last group repeat entry 0: valid addresses)
            const uint64_t li = a.class_off[c] + (act ? i : 0u);
            const uint64_t s = a.short_list[li];
            const uint32_t k = a.short_key[li];
            // 2. everything that depends on (s, k) only
            const uint64_t e = a.short_end ? a.short_end[li] : a.seg_end[k];
            const Rule R = a.rules[k];
            const Occ occ = a.occ[k];
            uint64_t buf[kBlk];
#pragma unroll
            for (int u = 0; u < kBlk; ++u) buf[u] = a.rec_sorted[min(s + u, a.n - 1)];
            {
                // piece t*64 + lane: bucket q = piece % SM of the ring of lane j = piece / SM, from the hot mirror
                // ({start, PASS | WAITING << 32}); slots past the handle's stride read slot 0 again (ignored: q >= S)
                constexpr int kT = SM;  // pieces per lane
                // the piece addresses depend on the lane only: an opaque copy of it keeps the compiler from
                // hoisting ~3 * kT of them out of the group loop (they held 60+ VGPRs for the whole walk)
                int gl = lane;
                asm volatile("" : "+v"(gl));
                {
                    ulonglong2 v[SM];
#pragma unroll
                    for (int t = 0; t < SM; ++t) {
                        const int pc = t * 64 + gl;
                        const int j = pc / kT;
                        const int q = pc % kT;
                        const uint32_t kj = (uint32_t)__shfl((int)k, j, 64);
                        const int qq = q < a.stride ? q : 0;
                        v[t] = *reinterpret_cast<const ulonglong2*>(a.hot + (size_t)kj * a.stride + qq);
                    }
#pragma unroll
                    for (int t = 0; t < SM; ++t) {
                        SlotSnap& d = snap[t * 64 + gl];
                        d.st = snap_rel((int64_t)v[t].x, T0);
                        d.pass = (int32_t)(uint32_t)v[t].y;
                        d.wait = (int32_t)(uint32_t)(v[t].y >> 32);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const uint64_t tw1 = (a.dbg & 64) ? __builtin_amdgcn_s_memrealtime() : 0;
            walk_reg<SM, L>(a, act, k, s, e, R, occ, snap + lane * SM, buf, T0);
            if (a.dbg & 64) {  // per class: groups, gather time, walk time (100 MHz ticks)
                const uint64_t tw2 = __builtin_amdgcn_s_memrealtime();
                if (lane == 0) {
                    atomicAdd(&a.dbg_ctr[0], (unsigned long long)(tw2 - tw0));
                    atomicAdd(&a.dbg_ctr[1 + c], 1ull);
                    atomicAdd(&a.dbg_ctr[7 + c], (unsigned long long)(tw1 - tw0));
                    atomicAdd(&a.dbg_ctr[7 + c], (unsigned long long)(tw2 - tw1) << 32);
                }
            }
            continue;
        }
        if (!act) continue;
        const uint64_t s = a.short_list[a.class_off[c] + i];
        const uint32_t k = (uint32_t)(a.rec_sorted[s] >> a.kshift);
        const uint64_t lim = s + (uint64_t)min(a.short_max, c < kClasses - 1 ? kClassMax[c] : 0xFFFFFFFFu) + 1;
        uint64_t e = s + 1;
        while (e < a.n && e < lim && (uint32_t)(a.rec_sorted[e] >> a.kshift) == k) ++e;
        walk_serial<L>(a, k, s, e);
    }
}

template <int SM, bool C>
#ifndef SG_SHORT_C_BLOCKS
#define SG_SHORT_C_BLOCKS 2
#endif
__global__ void __launch_bounds__(256, C ? SG_SHORT_C_BLOCKS : kShortBlocksPerCu) k_walk_short(BatchArgs a) {
    static_assert(SM <= kGatherMaxS, "LDS budget of the ring snapshot");
    __shared__ SlotSnap snap_all[4 * (SM > 0 ? 64 * SM : 1)];
    __shared__ uint32_t recs_all[SM > 0 && C ? 4 * kRecW * 64 : 1];
    if (*a.err || (a.dbg & 8192)) return;
    stage_periods(a);
    if (g_blds) walk_short_body<SM, true, C>(a, snap_all, recs_all);
    else walk_short_body<SM, false, C>(a, snap_all, recs_all);
}

// Tiny-segment walker: one thread per flowId of length class 0 (<= kClassMax[0] records, most touched flowIds of a
// Zipf batch), everything in registers — the ring's {start, PASS, WAITING} (S <= SM slots, the 32-bit encoding of
// SlotSnap: exact under BatchArgs::narrow and narrow_span), the records, the open bucket — so the kernel needs no
// LDS beyond the period tables and runs at more waves per SIMD: a group of 64 such segments in the lane-per-segment
// walker paid two memory round trips and a wave-wide period phase for a handful of decisions. Same decisions as
// walk_serial (ClusterFlowChecker.acquireClusterToken :67-111).
template <int SM, bool L>
__device__ __forceinline__ void walk_tiny_body(const BatchArgs& a) {
    constexpr int kR = (int)kClassMax[0];
    const uint32_t cnt = a.short_count[0];
    const uint64_t base = a.class_off[0];
    const int64_t T0 = a.p0[0] * (int64_t)a.wl[0];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += gridDim.x * blockDim.x) {
        const uint64_t s = a.short_list[base + t];
        const uint32_t k = a.short_key[base + t];
        const uint32_t e = a.short_end[base + t];
        const Rule R = a.rules[k];
        const Occ occ = a.occ[k];
        uint64_t r0 = a.rec_sorted[s], r1 = a.rec_sorted[min(s + 1, a.n - 1)];
        uint64_t r2 = a.rec_sorted[min(s + 2, a.n - 1)], r3 = a.rec_sorted[min(s + 3, a.n - 1)];
        static_assert(kR == 4, "four record registers");
        Bucket* ring = a.ring + (size_t)k * a.stride;
        BucketHot* hot = a.hot + (size_t)k * a.stride;
        int32_t st[SM], pa[SM], wa[SM];
#pragma unroll
        for (int x = 0; x < SM; ++x) {
            const int xx = x < R.S ? x : 0;
            const ulonglong2 hv = *reinterpret_cast<const ulonglong2*>(hot + xx);  // {start, PASS | WAITING << 32}
            st[x] = snap_rel((int64_t)hv.x, T0);
            pa[x] = (int32_t)(uint32_t)hv.y;
            wa[x] = (int32_t)(uint32_t)(hv.y >> 32);
        }
        PeriodCursor<L> pc;
        pc.init(a, R.wl_idx);
        const int64_t P0 = g_p0[R.wl_idx];
        const int S = R.S;
        PeriodState ps;
        ps.occ_pass = occ.pass;
        ps.occ_req = occ.pass_req;
#pragma unroll
        for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) ps.cur[ev] = 0;
        ps.wo_pass = ps.wo_wait = ps.head_other = 0;
        int I = -1;
        int64_t ws = 0;
        const uint32_t m = e - (uint32_t)s;
        for (uint32_t u = 0; u < m; ++u) {
            const Decoded d = decode(a, r0);
            r0 = r1;
            r1 = r2;
            r2 = r3;
            const uint32_t q = pc.of(d.idx);
            if (q != pc.q) {
                if (I >= 0) {  // close the open bucket: memory and the register ring
                    store_bucket(ring + I, hot + I, ws, ps.cur);
#pragma unroll
                    for (int x = 0; x < SM; ++x) {
                        st[x] = x == I ? (int32_t)(ws - T0) : st[x];
                        pa[x] = x == I ? (int32_t)ps.cur[SG_EV_PASS] : pa[x];
                        wa[x] = x == I ? (int32_t)ps.cur[SG_EV_WAITING] : wa[x];
                    }
                }
                const uint32_t qprev = pc.q;
                pc.seek(q);
                const int64_t P = P0 + (int64_t)q;
                I = I < 0 ? period_slot(R.wl_idx, q, S) : (int)((uint32_t)(I + (int)(q - qprev)) % (uint32_t)S);
                ws = P * R.wl;
                const int64_t lo_rel = ws - (int64_t)S * R.wl - T0;  // valid iff start > ws - S * wl
                const int32_t lo32 = rel32(lo_rel);  // snapshot starts are 32-bit (snap_rel)
                const int h = I + 1 == S ? 0 : I + 1;
                uint32_t wp = 0, ww = 0, ho = 0;
                int32_t stI_rel = INT32_MIN;
#pragma unroll
                for (int x = 0; x < SM; ++x) {
                    const bool v = (x < S) & (x != I) & (st[x] > lo32);
                    const uint32_t mk = v ? 0xFFFFFFFFu : 0u;
                    wp += (uint32_t)pa[x] & mk;
                    ww += (uint32_t)wa[x] & mk;
                    ho = (x == h) ? ((uint32_t)pa[x] & mk) : ho;
                    stI_rel = x == I ? st[x] : stI_rel;
                }
                ps.wo_pass = (int64_t)wp;
                ps.wo_wait = (int64_t)ww;
                ps.head_other = (int64_t)ho;
                const int64_t stI = stI_rel == INT32_MIN ? INT64_MIN : T0 + (int64_t)stI_rel;
                int64_t cI[SG_NUM_EVENTS];
                if (stI == ws) {  // the batch continues the stored period
#pragma unroll
                    for (int ev = 0; ev < SG_NUM_EVENTS; ++ev) cI[ev] = ring[I].c[ev];
                }
                open_bucket(ps, stI, cI, ws);
            }
            const double latest = qps_of(ps.wo_pass + ps.cur[SG_EV_PASS], R.isec);
            const double next_remaining = R.thr - latest - (double)d.acq;
            if (next_remaining >= 0) {
                ps.cur[SG_EV_PASS] += d.acq;
                ps.cur[SG_EV_PASS_REQUEST] += 1;
                if (d.prio) ps.cur[SG_EV_OCCUPIED_PASS] += d.acq;
                store_result(a.out, d.idx, SG_STATUS_OK, java_d2i(next_remaining), 0);
            } else {
                int32_t wait;
                const int32_t stt = decide_fail(R, a.max_occ_ratio, ps, d.acq, d.prio, &wait);
                if (stt != SG_STATUS_BLOCKED) store_result(a.out, d.idx, stt, 0, wait);
            }
        }
        if (I >= 0) store_bucket(ring + I, hot + I, ws, ps.cur);
        if (ps.occ_pass != occ.pass || ps.occ_req != occ.pass_req) {  // rarely changes: no partial-line store
            Occ o;
            o.pass = ps.occ_pass;
            o.pass_req = ps.occ_req;
            a.occ[k] = o;
        }
    }
}

template <int SM>
#ifndef SG_TINY_BLOCKS
#define SG_TINY_BLOCKS 4
#endif
__global__ void __launch_bounds__(256, SG_TINY_BLOCKS) k_walk_tiny(BatchArgs a) {
    if (*a.err || !tiny_active(a)) return;
    stage_periods(a);
    if (g_blds) walk_tiny_body<SM, true>(a);
    else walk_tiny_body<SM, false>(a);
}

// One wave per skipped piece: Σ acquire and Σ prioritized acquire over its records, added with 64-bit
// atomics (pieces of one range share a bucket).
constexpr int kSkipU = 8;
__global__ void __launch_bounds__(256) k_skip_apply(BatchArgs a) {
    if (*a.err) return;
    const uint32_t cnt = min(*a.skip_count, a.skip_cap);
    const int lane = lane_id();
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t i = wave; i < cnt; i += nwaves) {
        const uint4 sk = a.skips[i];
        int64_t sa = 0, spa = 0;
        // kSkipU rows of 64 records loaded together (one row per round trip left the wave latency-bound: a 4096-record
        // piece took 64 of them)
        for (uint64_t j0 = (uint64_t)sk.z; j0 < sk.w; j0 += 64ull * kSkipU) {
            uint64_t r[kSkipU];
#pragma unroll
            for (int u = 0; u < kSkipU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * 64 + lane;
                r[u] = j < sk.w ? a.rec_sorted[j] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < kSkipU; ++u) {
                if (j0 + (uint64_t)u * 64 + lane >= sk.w) continue;
                const Decoded d = decode(a, r[u]);
                sa += d.acq;
                spa += d.prio ? d.acq : 0;
            }
        }
        sa = wave_sum(sa);
        spa = wave_sum(spa);
        if (lane == 0) {
            const Rule R = a.rules[sk.x];
            const int64_t P = a.p0[R.wl_idx] + (int64_t)sk.y;
            Bucket& bk = a.ring[(size_t)sk.x * a.stride + (int)(P % R.S)];
            if (bk.start == P * R.wl) {
                atomicAdd((unsigned long long*)&bk.c[SG_EV_BLOCK], (unsigned long long)sa);
                atomicAdd((unsigned long long*)&bk.c[SG_EV_BLOCK_REQUEST], (unsigned long long)(sk.w - sk.z));
                atomicAdd((unsigned long long*)&bk.c[SG_EV_OCCUPIED_BLOCK], (unsigned long long)spa);
            }
        }
    }
}

// The cross-batch half of k_prep's time check, for a batch whose front half ran before the previous batch
// finished (pipelined): the first timestamp may not precede the last one of every earlier accepted batch.
__global__ void k_check_last(BatchArgs a) {
    if (a.n > 0 && a.req[0].ts_ms < *a.last_ts) atomicOr(a.err, kErrTime);
}

__global__ void k_finish(BatchArgs a) {
    if (*a.err == 0 && a.n > 0) *a.last_ts = a.req[a.n - 1].ts_ms;
}

// The front half's own time order (pipelined batches with namespace limiters): once a batch has passed validation
// and the limiter pre-pass, the next front half may start, checked against this batch's last timestamp, without
// waiting for this batch's walkers to advance last_ts.
__global__ void k_front_ts(BatchArgs a) {
    if (*a.err == 0 && a.n > 0) *a.front_ts = a.req[a.n - 1].ts_ms;
}

// ---------------------------------------------------------------------------- state management

// The hot mirror of every bucket, rebuilt from the ring (after rule loads and state imports).
__global__ void __launch_bounds__(256) k_hot_sync(const Bucket* ring, BucketHot* hot, uint64_t buckets) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < buckets; i += (uint64_t)gridDim.x * blockDim.x)
        store_hot(hot + i, ring[i].start, ring[i].c[SG_EV_PASS], ring[i].c[SG_EV_WAITING]);
}

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
    lds_poison(stream);
    if (a.bin_on) {
        const uint64_t tiles = (a.n + kPrepTile - 1) / kPrepTile;
        hipLaunchKernelGGL(k_prep<true>, dim3((unsigned)((tiles + a.prep_tiles - 1) / a.prep_tiles)), dim3(256), 0,
                           stream, a);
    }
    else hipLaunchKernelGGL(k_prep<false>, dim3((unsigned)((a.n + kPrepTile - 1) / kPrepTile)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_seg(const BatchArgs& a, hipStream_t stream) {
    lds_poison(stream);
    hipLaunchKernelGGL(k_seg, dim3(grid_for(a.n, kSegTile, 8192)), dim3(kSegThreads), 0, stream, a);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_lds_poison() {
    extern __shared__ uint32_t lds_all[];
    volatile uint32_t* p = lds_all;  // stores no later read needs: volatile keeps them
    for (uint32_t i = threadIdx.x; i < kPoisonBytes / 4; i += 256) p[i] = 0xA5A5A5A5u;
}

void lds_poison(hipStream_t stream) {
    struct Cfg {
        int mode;
        unsigned blocks;
    };
    static const Cfg cfg = [] {  // once, thread-safe (node shards decide from several host threads)
        const char* e = std::getenv("SG_LDS_POISON");
        Cfg c{e ? std::atoi(e) : 0, 0u};
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        c.blocks = 2u * (unsigned)(cus > 0 ? cus : 256);  // two 64 KB blocks per CU: 128 of its 160 KB
        if (c.mode) (void)hipFuncSetAttribute((const void*)k_lds_poison, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)kPoisonBytes);
        return c;
    }();
    if (cfg.mode) hipLaunchKernelGGL(k_lds_poison, dim3(cfg.blocks), dim3(256), kPoisonBytes, stream);
}

hipError_t launch_bin_front(const BatchArgs& a, uint32_t* hist_ws, bool hist_ready, bool csum_ready, hipStream_t stream) {
    hipError_t e = radix_bin_pass(a.rec, a.rec_sorted, a.bin_buf, a.bin_R, a.n, a.bin_dshift, hist_ws, hist_ready,
                                  csum_ready, stream);
    if (e != hipSuccess) return e;
    BatchArgs b = a;
    b.bin_tot = radix_tot(hist_ws, a.n, kBinDigit);
    lds_poison(stream);
    hipLaunchKernelGGL(k_bin_sort, dim3(a.bin_R + 1), dim3(kBinThreads), 0, stream, b);
    lds_poison(stream);
    hipLaunchKernelGGL(k_hot_update, dim3(1), dim3(1024), 0, stream, b);
    return hipGetLastError();
}

hipError_t launch_hot_reset(uint2* hot_tab, hipStream_t stream) {
    hipLaunchKernelGGL(k_hot_reset, dim3(1), dim3(256), 0, stream, hot_tab);
    return hipGetLastError();
}

hipError_t launch_seg_flow(const BatchArgs& a, hipStream_t stream) {
    if (!a.seg_marked)
        hipLaunchKernelGGL(k_seg_mark, dim3((unsigned)((a.n + 256 * kMarkItems - 1) / (256 * kMarkItems))), dim3(256), 0,
                       stream, a);
    lds_poison(stream);
    if (a.K) hipLaunchKernelGGL(k_seg_classify, dim3(grid_for(a.K, 256 * kClsItems, 4096)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

// Blocks of `kernel` resident at once on `cus` CUs (0: all of the device's).
static unsigned resident_blocks(const void* kernel, int block, int cus_used) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0);
    const bool all = !(cus_used > 0 && cus_used < cus);
    if (!all) cus = cus_used;
    unsigned b = (unsigned)((cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1));
    // on the whole chip (synchronous batches) twice that: the waves stride over the segments statically, and blocks
    // that start as others finish even out the lanes' uneven work (r04: one batch 0.965 -> 0.91 ms); on the pipeline's
    // walker CUs, beside the next batch's front half, exactly what fits (oversubscribed there: +1-2 %)
    if (all) b *= 2;
    // env SG_WALK_PCT (tuning): persistent walker grids at this percentage of what is resident at once
    if (const char* e = std::getenv("SG_WALK_PCT")) {
        const long pct = std::strtol(e, nullptr, 10);
        if (pct > 0 && pct <= 400) b = std::max(1u, (unsigned)(b * pct / 100));
    }
    return b;
}

// A persistent walker's grid for `walk_cus` CUs (0: the whole chip; the pipeline's walker CUs; a same-device node
// shard's share of either), cached per (kernel, CU count).
static unsigned walker_grid(const void* kern, int walk_cus) {
    struct Entry {
        const void* k;
        int cus;
        unsigned blocks;
    };
    static std::mutex mu;
    static Entry cache[64];
    static int used = 0;
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < used; ++i)
        if (cache[i].k == kern && cache[i].cus == walk_cus) return cache[i].blocks;
    const unsigned b = resident_blocks(kern, 256, walk_cus);
    if (used < 64) cache[used++] = Entry{kern, walk_cus, b};
    return b;
}

// Persistent walkers: at most as many blocks as fit on the chip at once (each wave loops over its queue).
hipError_t launch_walk_long(const BatchArgs& a, hipStream_t stream) {
    if (a.long_pend && a.long_key && a.seg_end) hipLaunchKernelGGL(k_long_bounds, dim3(1024), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(k_walk_long, dim3(walker_grid((const void*)k_walk_long, a.walk_cus)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

// Compact LDS records for the short walker: {idx, acode} fill the low 32 bits (abits == 8, ibits <= 24).
static bool short_compact(const BatchArgs& a) { return a.abits == 8 && a.imask <= 0xFFFFFFull && !(a.dbg & 4); }

template <int SM>
static hipError_t launch_short_sm(const BatchArgs& a, hipStream_t stream) {
    const bool c = SM > 0 && short_compact(a);
    const void* kern = c ? (const void*)k_walk_short<SM, true> : (const void*)k_walk_short<SM, false>;
    const unsigned blocks = walker_grid(kern, a.walk_cus);
    if (c) hipLaunchKernelGGL((k_walk_short<SM, true>), dim3(blocks), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_walk_short<SM, false>), dim3(blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

template <int SM>
static hipError_t launch_tiny_sm(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL((k_walk_tiny<SM>), dim3(walker_grid((const void*)k_walk_tiny<SM>, a.walk_cus)), dim3(256), 0,
                       stream, a);
    return hipGetLastError();
}

// Whether k_walk_tiny takes length class 0 (the host sets BatchArgs::tiny from the same answer).
bool tiny_walker_enabled(const BatchArgs& a) {
    // opt-in (SG_DEBUG & 128): measured 11 % slower per C3 step than class 0 inside k_walk_short (r03 A/B:
    // 0.999 vs 0.897 ms), the extra launch serialises behind the short walker on the same stream
    return !a.generic_walker && a.stride <= 10 && a.short_max >= kClassMax[0] && (a.dbg & 128);
}

hipError_t launch_walk_tiny(const BatchArgs& a, hipStream_t stream) {
    if (!a.tiny) return hipSuccess;
    if (a.stride <= 2) return launch_tiny_sm<2>(a, stream);
    if (a.stride <= 4) return launch_tiny_sm<4>(a, stream);
    if (a.stride <= 8) return launch_tiny_sm<8>(a, stream);
    return launch_tiny_sm<10>(a, stream);
}

hipError_t launch_walk_short(const BatchArgs& a, hipStream_t stream) {
    // the register-snapshot walker for the handle's largest sampleCount (a.stride)
    if (a.generic_walker) return launch_short_sm<0>(a, stream);
    if (a.stride <= 2) return launch_short_sm<2>(a, stream);
    if (a.stride <= 4) return launch_short_sm<4>(a, stream);
    if (a.stride <= 8) return launch_short_sm<8>(a, stream);
    if (a.stride <= 10) return launch_short_sm<10>(a, stream);  // ClusterFlowConfig default sampleCount
    return launch_short_sm<0>(a, stream);
}

hipError_t launch_skip_apply(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_skip_apply, dim3(2048), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_check_last(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_check_last, dim3(1), dim3(1), 0, stream, a);
    return hipGetLastError();
}

// Result copy to host memory by the shader (sg_flow_submit with a device-accessible host buffer): 16-B stores in
// order over the PCIe link, so the results of batch i travel while the copy engine brings batch i + 1's requests
// in (the two directions of the link in use at once, whatever the SDMA engine assignment). `dst` is the buffer's
// device alias; bytes % 16 == 0 or the tail is copied by 4-B words.
__global__ void __launch_bounds__(256) k_copy_out(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16,
                                                  const uint32_t* __restrict__ src_tail, uint32_t* __restrict__ dst_tail,
                                                  uint32_t tail_words) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {  // four loads in flight per thread
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < tail_words) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

hipError_t launch_copy_out(const void* src, void* dst_dev, uint64_t bytes, int blocks, hipStream_t stream) {
    const uint64_t n16 = bytes / 16;
    const uint32_t tail = (uint32_t)((bytes % 16) / 4);
    hipLaunchKernelGGL(k_copy_out, dim3(blocks), dim3(256), 0, stream, (const uint4*)src, (uint4*)dst_dev, n16,
                       (const uint32_t*)src + n16 * 4, (uint32_t*)dst_dev + n16 * 4, tail);
    return hipGetLastError();
}

hipError_t launch_front_ts(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_front_ts, dim3(1), dim3(1), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_finish(const BatchArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(1), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_hot_sync(const Bucket* ring, BucketHot* hot, uint64_t buckets, hipStream_t stream) {
    if (buckets == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hot_sync, dim3(grid_for(buckets, 256, 8192)), dim3(256), 0, stream, ring, hot, buckets);
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
