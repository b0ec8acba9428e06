// local.hip — gfx950 kernels of the local slot chain for a time-ordered batch of entry/exit events:
// StatisticSlot (core/slots/statistic/StatisticSlot.java:55-165) around FlowSlot's DefaultController
// (core/slots/block/flow/controller/DefaultController.java:49-76) and DegradeSlot's circuit breakers
// (core/slots/block/degrade/DegradeSlot.java:43-81, circuitbreaker/*), over each resource's
// StatisticNode (core/node/StatisticNode.java): the occupiable second window with its borrow array
// (OccupiableBucketLeapArray / FutureBucketLeapArray), the 60-bucket minute window and curThreadNum.
//
// Pipeline: k_local_prep (records + period tables) → radix sort by resource (sort.hip) → k_seg (segment
// heads by length class, engine.hip) → k_lwalk_long (one wave per hot resource) beside k_lwalk_short (one
// lane per resource).
//
// Every event of a resource opens the second- and minute-window buckets of its time (passQps / addPass /
// increaseBlockQps / addRtAndSuccess all call currentWindow first), so both walkers keep the two current
// buckets in registers and touch the rings in memory only when a window period changes. The rarely used
// paths (prioritized occupy through the borrow array, thread-grade rules, breaker state changes) run one
// event at a time ("serial step"); the wave walker decides everything else 64 events at a time.
#include "pslot_dev.h"

namespace sg {

namespace {

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ int32_t java_d2i(double x) {  // JLS §5.1.3
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

__device__ __forceinline__ double qps_of(int64_t sum, double isec) { return avg_div((double)sum, isec); }

__device__ __forceinline__ int64_t wave_sum(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((long long)v, o, 64);
    return v;
}

__device__ __forceinline__ int64_t wave_min(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, o, 64));
    return v;
}

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up((long long)v, (unsigned)o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

// v of lane src (wave-uniform src): v_readlane, not an LDS permute round trip
__device__ __forceinline__ int bcast32(int v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ int64_t bcast64(int64_t v, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t below(int f) { return f >= 64 ? ~0ull : ((1ull << f) - 1ull); }

// Loads / stores through a pointer known to address global memory: global_load / global_store, counted by vmcnt
// alone — a flat access (what a generic pointer reached through a non-kernel function's arguments gets) also counts
// in lgkmcnt, so every LDS / cross-lane wait after it would wait for it too.
template <typename T>
__device__ __forceinline__ T gload(const T* p) {
    static_assert(sizeof(T) % 4 == 0 && sizeof(T) <= 32, "gload: 4-byte words, at most 32 bytes");
    typedef unsigned int W __attribute__((ext_vector_type(sizeof(T) / 4)));
    typedef const __attribute__((address_space(1))) W GW;
    const W w = *(GW*)p;
    T v;
    __builtin_memcpy(&v, &w, sizeof(T));
    return v;
}
template <typename T>
__device__ __forceinline__ void gstore(T* p, const T& v) {
    static_assert(sizeof(T) % 4 == 0 && sizeof(T) <= 32, "gstore: 4-byte words, at most 32 bytes");
    typedef unsigned int W __attribute__((ext_vector_type(sizeof(T) / 4)));
    typedef __attribute__((address_space(1))) W GW;
    W w;
    __builtin_memcpy(&w, &v, sizeof(T));
    *(GW*)p = w;
}

__device__ __forceinline__ uint32_t period_of(const uint32_t* bnd, uint32_t np, uint32_t idx) {
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bnd[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct Cursor {  // window period of monotonically increasing request indices (see PeriodCursor)
    const uint32_t* bnd;
    uint32_t np, q, next_b;
    __device__ __forceinline__ void seek(uint32_t qq) {
        q = qq;
        next_b = (qq + 1 < np) ? bnd[qq + 1] : 0xFFFFFFFFu;
    }
    __device__ __forceinline__ uint32_t of(uint32_t idx) const {
        if (q != 0xFFFFFFFFu && idx < next_b) return q;
        return period_of(bnd, np, idx);
    }
};

struct LEvent {  // one decoded event
    uint32_t idx;
    int32_t count;
    int kind;    // SG_LOCAL_ENTRY / EXIT / EXIT_ERROR
    bool prio;
};

__device__ __forceinline__ LEvent ldecode(const LArgs& a, uint64_t rec) {
    LEvent e;
    e.idx = (uint32_t)((rec >> a.abits) & a.imask);
    const uint64_t ac = rec & a.amask;
    e.prio = (ac & 1ull) != 0;
    e.kind = (int)((ac >> 1) & 3ull);
    const uint64_t c = ac >> 3;
    e.count = (c == a.aesc) ? a.ev[e.idx].count : (int32_t)c;
    return e;
}

__device__ __forceinline__ void lstore(const LArgs& a, uint32_t idx, int32_t st, int32_t wait) {
    sg_local_result r;
    r.status = st;
    r.wait_ms = wait;
    gstore(a.out + idx, r);
}

}  // namespace

// ------------------------------------------------------------------------------------------ prep

// One block per 4096-event tile (the radix sort's): with a.hist0 the block also counts its records' first sort
// digit, so the sort skips that histogram pass (as k_prep does for the cluster flow batch).
constexpr int kLPrepItems = 16;
__global__ void __launch_bounds__(256) k_local_prep(LArgs a) {
    __shared__ uint32_t dcnt[1024];
    __shared__ uint16_t ldig[kLPrepItems * 256];  // each item's first sort digit (the histogram after the loop)
    const uint64_t n = a.n;
    const int64_t t0 = a.ev[0].ts_ms;
    const uint64_t sentinel = (uint64_t)a.K << a.kshift;
    const uint32_t dmask = (1u << a.hist0_bits) - 1u;
    if (a.hist0)
        for (uint32_t d = threadIdx.x; d <= dmask; d += 256) dcnt[d] = 0;
    __syncthreads();
    const uint64_t tile = (uint64_t)blockIdx.x * (256 * kLPrepItems);
#pragma unroll 4
    for (int it = 0; it < kLPrepItems; ++it) {
        const uint64_t i = tile + (uint64_t)it * 256 + threadIdx.x;
        if (i >= n) break;
        const sg_local_event e = a.ev[i];
        const int64_t t = e.ts_ms;
        if (i == 0) {
            if (t < 0 || (!a.defer_last && t < *a.last_ts) || (a.c3_last_ts && t < *a.c3_last_ts) ||
                (a.has_ps && a.ps.emb && t < *a.ps.cp_last_ts))  // the embedded server's flow / param tokens
                atomicOr(a.err, kErrTime);
            for (int w = 0; w < a.n_wl; ++w) a.p0[w] = t / a.wl[w];
        } else {
            const int64_t tp = a.ev[i - 1].ts_ms;
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
        const uint32_t res = e.resource & SG_KEY_INDEX;
        if (e.origin < 0 || e.origin > a.n_origins) atomicOr(a.err, kErrBounds);
        if (a.ext) {  // the event's context and argument records (ParamFlowSlot reads them)
            const sg_slot_ext x = a.ext[i];
            if ((int64_t)x.context >= (int64_t)(a.n_contexts > 0 ? a.n_contexts : 1)) atomicOr(a.err, kErrBounds);
            if (a.has_ps && !x.args_null && res < a.K) {
                bool ok = (uint64_t)x.arg_begin + x.arg_count <= a.ps.n_args;
                for (uint32_t k = 0; ok && k < x.arg_count; ++k) {
                    const sg_pslot_arg g = a.ps.args[x.arg_begin + k];
                    const uint64_t m = g.kind == SG_ARG_COLLECTION ? g.value_count : (g.kind == SG_ARG_VALUE ? 1 : 0);
                    ok = (uint64_t)g.value_begin + m <= a.ps.n_values;
                }
                if (!ok) atomicOr(a.err, kErrBounds);
            }
        }
        uint64_t rec = sentinel;
        if (res < a.K) {
            const uint32_t key = a.gkey ? a.gkey[res] : res;  // a RELATE group sorts as one key
            uint64_t c = (e.count < 0) ? a.aesc : (uint64_t)(uint32_t)e.count;
            if (c > a.aesc) c = a.aesc;
            // kind: 0 entry, 2 exit after a business error, anything else a plain exit
            const uint64_t kind = e.kind == SG_LOCAL_ENTRY ? 0 : (e.kind == SG_LOCAL_EXIT_ERROR ? 2 : 1);
            const uint64_t ac = (c << 3) | (kind << 1) | (uint64_t)(e.resource >> 31);
            rec = ((uint64_t)key << a.kshift) | ((uint64_t)i << a.abits) | ac;
            if (kind == 0 && (e.resource >> 31)) atomicOr(a.flags, kLFlagPrio);
            if (kind == 0 && e.count <= 0) atomicOr(a.flags, kLFlagNonPos);
        }
        // ParamFlowSlot lookup of an entry of a resource with one QPS param rule (resolved paramIdx, local): the
        // walkers' dead periods read the (rule, value) slot instead of the arguments (ParamFlowChecker.passSingleValue
        // Check's early exits and the CacheMap putIfAbsent happen at the check: every such entry reaches it first)
        if (a.pslot) {
            uint64_t code = kPsUnknown;
            if (res < a.K && e.kind == SG_LOCAL_ENTRY && a.rules[res].ps && a.has_ps) {
                const uint32_t rb = a.ps.res_begin[res];
                if (a.ps.res_begin[res + 1] == rb + 1) {
                    const uint32_t ri = a.ps.res_rules[rb];
                    const int32_t idx = a.ps.cur_idx[ri];
                    const int32_t cm = a.ps.cmode ? a.ps.cmode[ri] : SG_CLUSTER_MODE_OFF;
                    if (a.ps.grade[ri] == 1 && cm == SG_CLUSTER_MODE_OFF && idx >= 0) {
                        const sg_slot_ext x = a.ext ? a.ext[i] : sg_slot_ext{0, 0, 0, 1};
                        code = x.args_null ? kPsNoCheck : kPsNoCheckInit;
                        // out-of-range argument records (kErrBounds above: the batch is refused) are not read
                        const bool in_range = (uint64_t)x.arg_begin + x.arg_count <= a.ps.n_args;
                        if (!x.args_null && (int32_t)x.arg_count > idx && in_range) {
                            const sg_pslot_arg g = a.ps.args[x.arg_begin + (uint32_t)idx];
                            if (g.kind != SG_ARG_NULL && (uint64_t)g.value_begin + 1 > a.ps.n_values) {
                                code = kPsUnknown;
                            } else if (g.kind == SG_ARG_COLLECTION) {
                                code = kPsUnknown;
                            } else if (g.kind == SG_ARG_VALUE) {
                                const PRule pr = a.ps.p.rules[ri];
                                const uint64_t v = a.ps.values[g.value_begin];
                                const int64_t tc = param_token_count(a.ps.p, pr, v);
                                if (tc == 0 || (pr.behavior != 2 && (int64_t)e.count > tc + pr.burst)) {
                                    code = kPsEarlyFail;
                                } else {
                                    code = param_slot(a.ps.p, pr, v);
                                    if (code == ~0ull) atomicOr(a.err, kErrTableFull);
                                }
                            }
                        }
                    }
                }
            }
            a.pslot[i] = code;
        }
        // default result: FlowException for entries (the common outcome of a saturated resource; the walkers
        // write every other outcome), plain 0 for exits and events of unknown resources
        const uint32_t dst = (res < a.K && e.kind == SG_LOCAL_ENTRY) ? SG_LOCAL_BLOCK_FLOW : SG_LOCAL_PASS;
        st_stream(reinterpret_cast<uint64_t*>(a.out + i), (uint64_t)dst);  // {status, wait_ms 0}
        st_stream(a.rec + i, rec);
        if (a.hist0) ldig[it * 256 + threadIdx.x] = (uint16_t)((uint32_t)(rec >> a.kshift) & dmask);
    }
    if (a.hist0) {
        // the histogram's LDS atomics after the tile's loads: inside the loop they kept the compiler from
        // overlapping one item's event load with the previous item's work (k_local_prep 285 → ~200 µs at C5 without them)
        for (int it = 0; it < kLPrepItems; ++it) {
            const uint64_t i = tile + (uint64_t)it * 256 + threadIdx.x;
            if (i >= n) break;
            atomicAdd(&dcnt[ldig[it * 256 + threadIdx.x]], 1u);
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d <= dmask; d += 256) a.hist0[(size_t)blockIdx.x * (dmask + 1) + d] = dcnt[d];
        if (a.csum0) {
            uint32_t* cs = a.csum0 + (size_t)(blockIdx.x / kChunkTiles) * (dmask + 1);
            for (uint32_t d = threadIdx.x; d <= dmask; d += 256)
                if (dcnt[d]) atomicAdd(cs + d, dcnt[d]);
        }
    }
}

// Empty nodes [lo, hi) (one thread per minute slot of a node).
__global__ void __launch_bounds__(256) k_local_init(LArgs a, uint64_t lo, uint64_t hi) {
    const uint64_t total = (hi - lo) * kMinuteS;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        LBucket b;
        b.start = INT64_MIN;
        for (int e = 0; e < kLEv; ++e) b.c[e] = 0;
        b.min_rt = kStatMaxRt;
        const uint64_t k = lo + i / kMinuteS;
        const int q = (int)(i % kMinuteS);
        a.minute[k * kMinuteS + q] = b;
        if (q < a.S) {
            a.sec[k * a.S + q] = b;
            LFuture f;
            f.start = INT64_MIN;
            f.pass = 0;
            a.bor[k * a.S + q] = f;
        }
        if (q == 0) {
            LHead h;
            h.threads = 0;
            h.created = 0;
            for (int j = 0; j < 2; ++j) {
                h.cb[j].next_retry = 0;
                h.cb[j].stat_start = INT64_MIN;
                h.cb[j].bad = h.cb[j].total = 0;
                h.cb[j].state = kCbClosed;
                h.cb[j].pad = 0;
            }
            h.pad2[0] = h.pad2[1] = 0;
            a.head[k] = h;
        }
    }
}

// ------------------------------------------------------------------------------------ node pool

namespace {

// Find or insert key; returns its map slot. A new key takes the next pool node (a.node_base + creation order).
// Lanes never wait on one another: the node index is written by the inserting lane and read only by later kernels.
__device__ uint32_t lnode_slot(const LArgs& a, uint64_t key) {
    uint64_t s = lnode_hash(key) & a.nmask;
    for (;;) {
        const uint64_t cur = a.nkeys[s];
        if (cur == key) return (uint32_t)s;
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long*)&a.nkeys[s], 0ull, (unsigned long long)key);
            if (prev == 0) {
                a.nvals[s] = a.node_base + atomicAdd(a.node_new, 1u);
                return (uint32_t)s;
            }
            if (prev == key) return (uint32_t)s;
        }
        s = (s + 1) & a.nmask;
    }
}

}  // namespace

// ClusterBuilderSlot's origin node (an event with an origin) and NodeSelectorSlot's DefaultNode of the event's
// context (context tracking on) of every event, created on first sight; the map slots go to ev_node, and a resource
// with an origin event is walked by k_lwalk_cx in this batch. Runs only for a batch that passed validation (a
// rejected batch creates nothing). The host sized the map for every event's keys at load <= 1/2.
__global__ void __launch_bounds__(256) k_lnode_assign(LArgs a) {
    if (*a.err) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_local_event e = a.ev[i];
        const uint32_t res = e.resource & SG_KEY_INDEX;
        uint2 v = make_uint2(kNoNode, kNoNode);
        if (res < a.K) {
            if (e.origin > 0) {
                v.x = lnode_slot(a, lnode_key(res, 0, (uint32_t)e.origin));
                if (a.dyn[res] != a.epoch) a.dyn[res] = a.epoch;
            }
            if (a.track_ctx) v.y = lnode_slot(a, lnode_key(res, kLNodeCtx, a.ext ? a.ext[i].context : 0u));
        }
        a.ev_node[i] = v;
    }
}

// Every event's map slots → node indices (after k_lnode_assign: the inserting lanes have written them), so the walkers
// read an event's nodes with one load.
__global__ void __launch_bounds__(256) k_lnode_resolve(LArgs a) {
    if (*a.err) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint2 s = a.ev_node[i];
        a.ev_node[i] = make_uint2(s.x != kNoNode ? a.nvals[s.x] : kNoNode, s.y != kNoNode ? a.nvals[s.y] : kNoNode);
    }
}

__global__ void k_lnode_find(const uint64_t* keys, const uint32_t* vals, uint64_t mask, uint64_t key, uint32_t* out) {
    uint64_t s = lnode_hash(key) & mask;
    uint32_t r = kNoNode;
    for (uint64_t probes = 0; probes <= mask; ++probes, s = (s + 1) & mask) {
        if (keys[s] == key) {
            r = vals[s];
            break;
        }
        if (keys[s] == 0) break;
    }
    *out = r;
}

// ----------------------------------------------------------------------------- per-resource state

// The state of one resource during a walk. In the wave walker every field is wave-uniform and every lane
// executes the serial step identically (stores from all lanes carry the same value).
struct LNode {
    const LArgs& a;
    LRule R;
    uint32_t k;
    LBucket* sec;
    LFuture* bor;
    LBucket* mnt;
    Cursor cs, cm;     // second / minute window periods
    int64_t P0s, P0m;
    // open second-window bucket
    int64_t sc[kLEv], s_min, s_ws, s_wo;  // s_wo: Σ PASS of the other valid buckets
    int sI;
    // open minute-window bucket
    int64_t mc[kLEv], m_min, m_ws;
    int mI;
    int64_t threads;
    int64_t created;   // LHead.created (set by the walkers for a resource with events: ClusterBuilderSlot)
    LBreaker cb[2];

    // a node the event does not touch (no origin / context node): nothing loaded, never opened or finished
    struct None {};
    __device__ LNode(const LArgs& a_, None) : a(a_), k(0) {
        R = LRule{};
        sec = nullptr;
        bor = nullptr;
        mnt = nullptr;
        cs = cm = Cursor{nullptr, 0, 0xFFFFFFFFu, 0};
        P0s = P0m = 0;
        sI = mI = -1;
        s_ws = m_ws = s_wo = 0;
        s_min = m_min = kStatMaxRt;
        for (int e = 0; e < kLEv; ++e) sc[e] = mc[e] = 0;
        threads = created = 0;
        cb[0] = cb[1] = LBreaker{};
    }

    // a pool node (origin / context) of the same batch as `like`: its window cursors and period bases are like's
    // (the batch's), only its head is read
    __device__ LNode(const LArgs& a_, const LNode& like, uint32_t k_) : a(a_), k(k_) {
        R = LRule{};
        R.flow_grade = -1;
        R.b[0].stat_ms = R.b[1].stat_ms = 1;
        sec = a.sec + (size_t)k * a.S;
        bor = a.bor + (size_t)k * a.S;
        mnt = a.minute + (size_t)k * kMinuteS;
        cs = Cursor{like.cs.bnd, like.cs.np, 0xFFFFFFFFu, 0};
        cm = Cursor{like.cm.bnd, like.cm.np, 0xFFFFFFFFu, 0};
        P0s = like.P0s;
        P0m = like.P0m;
        sI = mI = -1;
        s_ws = m_ws = 0;
        s_wo = 0;
        s_min = m_min = kStatMaxRt;
        for (int e = 0; e < kLEv; ++e) sc[e] = mc[e] = 0;
        const LHead h = a.head[k];
        threads = h.threads;
        created = h.created;
        cb[0] = h.cb[0];
        cb[1] = h.cb[1];
    }

    __device__ LNode(const LArgs& a_, const uint32_t* const* bndp, uint32_t k_) : a(a_), k(k_) {
        if (k_ < a.K) {
            R = a.rules[k_];
        } else {  // a pool node (origin / context): no rules, no breakers
            R = LRule{};
            R.flow_grade = -1;
            R.b[0].stat_ms = R.b[1].stat_ms = 1;
        }
        sec = a.sec + (size_t)k * a.S;
        bor = a.bor + (size_t)k * a.S;
        mnt = a.minute + (size_t)k * kMinuteS;
        cs = Cursor{bndp[a.wsec], a.np[a.wsec], 0xFFFFFFFFu, 0};
        cm = Cursor{bndp[a.wmin], a.np[a.wmin], 0xFFFFFFFFu, 0};
        P0s = a.p0[a.wsec];
        P0m = a.p0[a.wmin];
        sI = mI = -1;
        s_ws = m_ws = 0;
        s_wo = 0;
        s_min = m_min = kStatMaxRt;
        for (int e = 0; e < kLEv; ++e) sc[e] = mc[e] = 0;
        const LHead h = a.head[k];
        threads = h.threads;
        created = h.created;
        cb[0] = h.cb[0];
        cb[1] = h.cb[1];
    }

    // -------- second window (OccupiableBucketLeapArray) --------
    __device__ void sec_close() {
        if (sI < 0) return;
        LBucket b;
        b.start = s_ws;
        for (int e = 0; e < kLEv; ++e) b.c[e] = sc[e];
        b.min_rt = s_min;
        sec[sI] = b;
    }

    // currentWindow(t) for the period q (LeapArray.java:116-202; newEmptyBucket / resetWindowTo of
    // OccupiableBucketLeapArray.java:40-63 read the borrow bucket of the same window), then the PASS sum
    // of the other valid buckets (values(t): valid iff start >= windowStart - (S-1)*windowLength).
    __device__ void sec_open(uint32_t q) {
        sec_close();
        cs.seek(q);
        const int S = a.S;
        const int64_t P = P0s + (int64_t)q;
        const int I = (int)(P % S);
        const int64_t ws = P * a.wl2;
        const LBucket old = sec[I];
        const LFuture fb = bor[I];
        const bool borrow = fb.start == ws;  // borrowArray.getWindowValue(t): same window
        if (old.start == ws) {
            for (int e = 0; e < kLEv; ++e) sc[e] = old.c[e];
            s_min = old.min_rt;
        } else {
            for (int e = 0; e < kLEv; ++e) sc[e] = 0;
            s_min = kStatMaxRt;
            if (borrow) {
                if (old.start == INT64_MIN) sc[kLPass] = fb.pass;  // new bucket: reset(borrowBucket) copies it
                else sc[kLPass] += (int64_t)(int32_t)fb.pass;      // reset: addPass((int) borrowBucket.pass())
            }
        }
        sI = I;
        s_ws = ws;
        const int64_t lo = ws - (int64_t)(S - 1) * a.wl2;
        int64_t wo = 0;
        for (int j = 0; j < S; ++j) {
            if (j == I) continue;
            const int64_t st = sec[j].start;
            if (st != INT64_MIN && st >= lo) wo += sec[j].c[kLPass];
        }
        s_wo = wo;
    }

    // -------- minute window (BucketLeapArray, 60 x 1000 ms) --------
    __device__ void min_close() {
        if (mI < 0) return;
        LBucket b;
        b.start = m_ws;
        for (int e = 0; e < kLEv; ++e) b.c[e] = mc[e];
        b.min_rt = m_min;
        mnt[mI] = b;
    }

    __device__ void min_open(uint32_t q) {
        min_close();
        cm.seek(q);
        const int64_t P = P0m + (int64_t)q;
        const int I = (int)(P % kMinuteS);
        const int64_t ws = P * kMinuteWl;
        const LBucket old = mnt[I];
        if (old.start == ws) {
            for (int e = 0; e < kLEv; ++e) mc[e] = old.c[e];
            m_min = old.min_rt;
        } else {
            for (int e = 0; e < kLEv; ++e) mc[e] = 0;
            m_min = kStatMaxRt;
        }
        mI = I;
        m_ws = ws;
    }

    __device__ __forceinline__ void at(uint32_t qs, uint32_t qm) {
        if (qs != cs.q) sec_open(qs);
        if (qm != cm.q) min_open(qm);
    }
    // one window only: each read or add of the reference calls currentWindow on the window it touches, and a node
    // the event leaves alone keeps its stale buckets (the full-chain walker opens exactly what the reference touches)
    __device__ __forceinline__ void at_s(uint32_t qs) {
        if (qs != cs.q) sec_open(qs);
    }
    __device__ __forceinline__ void at_m(uint32_t qm) {
        if (qm != cm.q) min_open(qm);
    }

    __device__ __forceinline__ double pass_qps() const { return qps_of(s_wo + sc[kLPass], a.isec); }

    // -------- borrow array (FutureBucketLeapArray; memory only, prioritized path) --------
    __device__ int bor_window(int64_t t) {  // currentWindow(t): slot, or -2 for a detached bucket
        const int S = a.S;
        const int idx = (int)((t / a.wl2) % S);
        const int64_t ws = t - t % a.wl2;
        const int64_t st = bor[idx].start;
        if (st == INT64_MIN || ws > st) {
            LFuture f;
            f.start = ws;
            f.pass = 0;
            bor[idx] = f;
            return idx;
        }
        return ws == st ? idx : -2;
    }
    // OccupiableBucketLeapArray.currentWaiting (:66-75): future buckets only (deprecated iff t >= start)
    __device__ int64_t waiting(int64_t t) {
        bor_window(t);
        int64_t w = 0;
        for (int j = 0; j < a.S; ++j) {
            const LFuture f = bor[j];
            if (f.start != INT64_MIN && t < f.start) w += f.pass;
        }
        return w;
    }
    // ArrayMetric.getWindowPass(t) = data.getWindowValue(t).pass(): the second-window bucket holding t
    __device__ int64_t window_pass(int64_t t) {
        if (t < 0) return 0;
        const int idx = (int)((t / a.wl2) % a.S);
        if (idx == sI) return (s_ws <= t && t < s_ws + a.wl2) ? sc[kLPass] : 0;  // the open bucket
        const LBucket b = sec[idx];
        if (b.start == INT64_MIN || !(b.start <= t && t < b.start + a.wl2)) return 0;
        return b.c[kLPass];
    }
    // StatisticNode.tryOccupyNext, StatisticNode.java:288-320
    __device__ int64_t try_occupy_next(int64_t now, int32_t acquire, double threshold) {
        const double max_count = threshold * a.interval / 1000;
        const int64_t borrow = waiting(now);
        if ((double)borrow >= max_count) return a.occupy_timeout;
        const int32_t wlen = a.interval / a.S;
        int64_t earliest = now - now % wlen + wlen - a.interval;
        int32_t idx = 0;
        int64_t current_pass = s_wo + sc[kLPass];  // pass(): the open period's window sum
        while (earliest < now) {
            const int64_t wait = (int64_t)(int32_t)((uint32_t)idx * (uint32_t)wlen) + wlen - now % wlen;
            if (wait >= a.occupy_timeout) break;
            const int64_t wp = window_pass(earliest);
            if ((double)(current_pass + borrow + (int64_t)acquire - wp) <= max_count) return wait;
            earliest += wlen;
            current_pass -= wp;
            ++idx;
        }
        return a.occupy_timeout;
    }

    // -------- circuit breakers --------
    __device__ __forceinline__ void cb_to_open(int j, int64_t t) {
        cb[j].state = kCbOpen;
        cb[j].next_retry = t + (int64_t)R.b[j].recovery_ms;
    }
    __device__ __forceinline__ void cb_stat_window(int j, int64_t t) {  // LeapArray(1, statIntervalMs).currentWindow
        // events are time-ordered: t >= the bucket's start, so the bucket is current iff t < start + length
        if (cb[j].stat_start != INT64_MIN && t - cb[j].stat_start < R.b[j].stat_ms) return;
        cb[j].stat_start = t - t % R.b[j].stat_ms;
        cb[j].bad = cb[j].total = 0;
    }
    __device__ __forceinline__ bool cb_bad(int j, int64_t rt, bool error) const {
        return R.b[j].grade == SG_DEGRADE_RT ? rt > R.b[j].max_rt : error;
    }
    // CLOSED: would the counts (bad, total) open the breaker? (ResponseTimeCircuitBreaker.java:101-118,
    // ExceptionCircuitBreaker.java:88-108)
    __device__ __forceinline__ bool cb_trips(int j, int64_t bad, int64_t total) const {
        if (total < R.b[j].min_request) return false;
        if (R.b[j].grade == SG_DEGRADE_RT) {
            const double ratio = bad * 1.0 / total;
            return ratio > R.b[j].slow_ratio || (ratio == R.b[j].slow_ratio && R.b[j].slow_ratio == 1.0);
        }
        const double cur = R.b[j].grade == SG_DEGRADE_EXCEPTION_RATIO ? bad * 1.0 / total : (double)bad;
        return cur > R.b[j].count;
    }
    // onRequestComplete at exit time t
    __device__ __forceinline__ void cb_complete(int j, int64_t t, int64_t rt, bool error) {
        cb_stat_window(j, t);
        const bool bad = cb_bad(j, rt, error);
        cb[j].bad += bad ? 1 : 0;
        cb[j].total += 1;
        if (cb[j].state == kCbOpen) return;
        if (cb[j].state == kCbHalfOpen) {
            if (bad) {
                cb_to_open(j, t);
            } else {  // fromHalfOpenToClose → resetStat(): currentWindow().value().reset()
                cb[j].state = kCbClosed;
                cb[j].bad = cb[j].total = 0;
            }
            return;
        }
        if (cb_trips(j, cb[j].bad, cb[j].total)) cb_to_open(j, t);
    }

    // DegradeSlot.performChecking: AbstractCircuitBreaker.tryPass (:73-84) in rule order; the loops are fully
    // unrolled so the breaker state stays in registers. ts() yields the entry's time (read only when needed).
    template <class TS>
    __device__ __forceinline__ bool degrade_blocks(TS&& ts) {
        bool blocked = false, half0 = false, half1 = false;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j >= R.nb || blocked) continue;
            if (cb[j].state == kCbClosed) continue;
            if (cb[j].state == kCbOpen && ts() >= cb[j].next_retry) {
                cb[j].state = kCbHalfOpen;
                if (j == 0) half0 = true;
                else half1 = true;
            } else {
                blocked = true;
            }
        }
        if (blocked) {  // DegradeException; whenTerminate of a blocked probe: back to OPEN
            if (half0 && cb[0].state == kCbHalfOpen) cb[0].state = kCbOpen;
            if (half1 && cb[1].state == kCbHalfOpen) cb[1].state = kCbOpen;
        }
        return blocked;
    }

    // StatisticNode.previousPassQps at t: the minute window's previous bucket (ArrayMetric.previousWindowPass,
    // LeapArray.getPreviousWindow :210-227; t < 1000 reads as null, see the oracle)
    __device__ int64_t prev_pass(int64_t t) const {
        if (t < kMinuteWl) return 0;
        const int idx = (int)(((t - kMinuteWl) / kMinuteWl) % kMinuteS);
        int64_t st, pass;
        if (idx == mI) {
            st = m_ws;
            pass = mc[kLPass];
        } else {
            st = mnt[idx].start;
            pass = mnt[idx].c[kLPass];
        }
        if (st == INT64_MIN || t - st > (int64_t)kMinuteS * kMinuteWl) return 0;
        if (st + kMinuteWl < t - kMinuteWl) return 0;
        return pass;
    }

    // -------- one event, sequentially (the oracle's or_local_decide step) --------
    // Entry: FlowSlot (DefaultController.canPass) → DegradeSlot.performChecking → StatisticSlot.
    // t: the entry's timestamp, or INT64_MIN when not loaded yet (read only on the paths that need it:
    // the prioritized occupy and an OPEN breaker's retry check)
    __device__ void entry(const LEvent& e, int64_t t) {
        auto ts = [&]() {
            if (t == INT64_MIN) t = a.ev[e.idx].ts_ms;
            return t;
        };
        int32_t status = SG_LOCAL_PASS;
        int64_t wait = 0;
        if (R.flow_grade >= 0) {
            const int32_t cur = R.flow_grade == 0 ? (int32_t)threads : java_d2i(pass_qps());
            const int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)e.count);  // int + int wraps
            if ((double)sum > R.flow_count) {
                status = SG_LOCAL_BLOCK_FLOW;
                if (e.prio && R.flow_grade == 1) {
                    wait = try_occupy_next(ts(), e.count, R.flow_count);
                    if (wait < a.occupy_timeout) {
                        const int s = bor_window(t + wait);  // addWaitingRequest
                        if (s >= 0) bor[s].pass += e.count;
                        mc[kLOccPass] += e.count;  // addOccupiedPass: minute window (StatisticNode.java:333-336)
                        mc[kLPass] += e.count;
                        status = SG_LOCAL_PASS_WAIT;
                    }
                }
            }
        }
        if (status == SG_LOCAL_PASS && degrade_blocks(ts)) status = SG_LOCAL_BLOCK_DEGRADE;
        if (status == SG_LOCAL_PASS) {
            threads += 1;
            sc[kLPass] += e.count;
            mc[kLPass] += e.count;
        } else if (status == SG_LOCAL_PASS_WAIT) {
            threads += 1;
        } else {
            sc[kLBlock] += e.count;
            mc[kLBlock] += e.count;
        }
        if (status != SG_LOCAL_BLOCK_FLOW) lstore(a, e.idx, status, status == SG_LOCAL_PASS_WAIT ? (int32_t)wait : 0);
    }

    // Exit: StatisticSlot.exit (addRtAndSuccess, decreaseThreadNum, increaseExceptionQps) → DegradeSlot.exit.
    __device__ void exit(const LEvent& e, int64_t t, int64_t create) {
        const int64_t rt = t - create;
        const bool error = e.kind == SG_LOCAL_EXIT_ERROR;
        sc[kLSucc] += e.count;
        sc[kLRt] += rt;
        if (rt < s_min) s_min = rt;
        mc[kLSucc] += e.count;
        mc[kLRt] += rt;
        if (rt < m_min) m_min = rt;
        threads -= 1;
        if (error) {
            sc[kLExc] += e.count;
            mc[kLExc] += e.count;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (j < R.nb) cb_complete(j, t, rt, error);
    }

    __device__ void step(const LEvent& e, int64_t t, int64_t create) {
        at(cs.of(e.idx), cm.of(e.idx));
        if (e.kind == SG_LOCAL_ENTRY) entry(e, t);
        else exit(e, t, create);
    }

    __device__ void finish() {
        sec_close();
        min_close();
        LHead h;
        h.threads = threads;
        h.created = created;
        h.cb[0] = cb[0];
        h.cb[1] = cb[1];
        h.pad2[0] = h.pad2[1] = 0;
        a.head[k] = h;
    }
};

// ------------------------------------------------------------------------------ short walker

__device__ __forceinline__ void stage_lperiods(const LArgs& a, uint32_t* sbnd, const uint32_t** bndp) {
    uint32_t tot = 0;
    for (int w = 0; w < a.n_wl; ++w) tot += a.np[w];
    const bool lds = tot <= (uint32_t)kLdsBnd;
    uint32_t off = 0;
    for (int w = 0; w < a.n_wl; ++w) {
        const uint32_t npw = a.np[w];
        const uint32_t* g = a.bnd + (size_t)w * kMaxPeriods;
        if (lds) {
            for (uint32_t i = threadIdx.x; i < npw; i += blockDim.x) sbnd[off + i] = g[i];
            if (threadIdx.x == 0) bndp[w] = sbnd + off;
        } else if (threadIdx.x == 0) {
            bndp[w] = g;
        }
        off += npw;
    }
    __syncthreads();
}

// One lane per resource segment: the serial step for every event.
#ifndef SG_LWALK_BLOCKS
#define SG_LWALK_BLOCKS 1
#endif
__global__ void __launch_bounds__(256, SG_LWALK_BLOCKS) k_lwalk_short(LArgs a, BatchArgs sg) {
    __shared__ uint32_t sbnd[kLdsBnd];
    __shared__ const uint32_t* bndp[kMaxWl];
    if (*a.err) return;
    stage_lperiods(a, sbnd, bndp);
    const int lane = lane_id();
    uint32_t cnt[kClasses], grp_end[kClasses];
    uint32_t total = 0;
    for (int c = kClasses - 1; c >= 0; --c) {
        cnt[c] = sg.short_count[c];
        total += (cnt[c] + 63) / 64;
        grp_end[c] = total;
    }
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t g = wave; g < total; g += nwaves) {
        int c = kClasses - 1;
        uint32_t g0 = 0;
        while (g >= grp_end[c]) {
            g0 = grp_end[c];
            --c;
        }
        const uint32_t i = (g - g0) * 64 + (uint32_t)lane;
        if (i >= cnt[c]) continue;
        const uint64_t j = sg.short_list[sg.class_off[c] + i];
        const uint32_t k = (uint32_t)(a.rec_sorted[j] >> a.kshift);
        if (a.rules[k].cx || (a.dyn && a.dyn[k] == a.epoch)) continue;  // k_lwalk_cx
        LNode nd(a, bndp, k);
        nd.created = 1;  // the resource has events, so an entry reached ClusterBuilderSlot
        // software pipeline: records kRecAhead ahead, exit timestamps kEvAhead ahead (a lane walks up to
        // short_max contiguous records; one load in flight per record would leave it latency-bound)
        constexpr int kRecAhead = 8, kEvAhead = 4;
        uint64_t r[kRecAhead];
        int64_t ets[kEvAhead], ecr[kEvAhead];
        uint64_t nextp = j;
#pragma unroll
        for (int u = 0; u < kRecAhead; ++u, ++nextp) r[u] = nextp < a.n ? a.rec_sorted[nextp] : ~0ull;
        auto ev_load = [&](uint64_t rec, int64_t& ts, int64_t& cr) {
            ts = cr = 0;
            if ((uint32_t)(rec >> a.kshift) == k && ((rec & a.amask) >> 1 & 3ull) != 0) {
                const sg_local_event* p = a.ev + ((rec >> a.abits) & a.imask);
                ts = p->ts_ms;
                cr = p->create_ts;
            }
        };
#pragma unroll
        for (int u = 0; u < kEvAhead; ++u) ev_load(r[u], ets[u], ecr[u]);
        for (;;) {
            const uint64_t cur = r[0];
            if ((uint32_t)(cur >> a.kshift) != k) break;
            const int64_t t = ets[0], cr = ecr[0];
#pragma unroll
            for (int u = 0; u < kRecAhead - 1; ++u) r[u] = r[u + 1];
            r[kRecAhead - 1] = nextp < a.n ? a.rec_sorted[nextp] : ~0ull;
            ++nextp;
#pragma unroll
            for (int u = 0; u < kEvAhead - 1; ++u) {
                ets[u] = ets[u + 1];
                ecr[u] = ecr[u + 1];
            }
            ev_load(r[kEvAhead - 1], ets[kEvAhead - 1], ecr[kEvAhead - 1]);
            const LEvent e = ldecode(a, cur);
            nd.at(nd.cs.of(e.idx), nd.cm.of(e.idx));
            if (e.kind == SG_LOCAL_ENTRY) nd.entry(e, INT64_MIN);
            else nd.exit(e, t, cr);
        }
        nd.finish();
    }
}

// First position p in [lo, hi) with pred(p) (monotone), hi if none: 64-way wave search.
template <class Pred>
__device__ __forceinline__ uint64_t lwave_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
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

// ------------------------------------------------------------------------------- wave walker

// One wave per hot resource. Events come 64 at a time (lane = event); a chunk is cut into runs of equal
// second/minute window periods and breaker statistic windows, and each run into epochs that end at the
// next event needing the serial step:
//   - an entry whose flow check fails and that is prioritized (occupy path), or any entry of a
//     thread-grade rule;
//   - an entry that passes the flow check while a breaker is OPEN with its retry time reached (→ HALF_OPEN);
//   - an exit that would open a CLOSED breaker, or the first exit while a breaker is HALF_OPEN.
// Inside an epoch the breakers are fixed, so entries are decided by the flow rule alone (greedy admit by a
// wave prefix scan, then "fits on its own" for the rest, exactly like ClusterFlowChecker's walker) or are
// all blocked (a breaker rejects whatever passes the flow check), and exits only accumulate.
__device__ void lwalk_wave(const LArgs& a, const uint32_t* const* bndp, uint32_t k, uint64_t s, uint64_t e_end) {
    const int lane = lane_id();
    LNode nd(a, bndp, k);
    nd.created = 1;
    const int nb = nd.R.nb;
    const bool thread_grade = nd.R.flow_grade == 0;
    // a saturated second window (not even acquireCount 1 fits) FLOW-blocks every entry until the period
    // ends, whatever the breakers are, unless an entry may occupy (prioritized) or has a count <= 0
    const bool may_skip = nd.R.flow_grade == 1 && !(*a.flags & (kLFlagPrio | kLFlagNonPos));
    uint64_t skip_retry = 0;  // after a failed attempt: retry once the walk is past the obstacle
    // the resource's exits in the sorted exit list, consumed in order; the end of the current pair of
    // window periods, found once per pair
    const uint32_t ne = a.exit_cnt[0];
    uint64_t xi = may_skip ? lwave_search(0, ne, [&](uint64_t i) { return (uint64_t)a.exit_pos[i] >= s; }, lane) : ne;
    uint32_t pe_qs = 0xFFFFFFFFu, pe_qm = 0xFFFFFFFFu;
    uint64_t pe = 0;
    // the next chunk's records and event timestamps are loaded while this chunk is decided (records at the chunk's
    // start, events once its records have arrived): two dependent loads per chunk off the critical path. Loads are
    // unconditional with clamped indices; lanes past the segment ignore what they read.
    const uint64_t n1 = a.n - 1;
    // an entry's time matters only while a breaker is not CLOSED (the retry check) and in the serial step (which
    // reads it itself when not loaded): entries' times are prefetched only while some breaker is open or half-open,
    // and loaded on demand when one opens inside a chunk (a random 32-B event read per entry otherwise)
    auto breakers_closed = [&]() {
        bool c = true;
#pragma unroll
        for (int x = 0; x < 2; ++x) c = c && (x >= nb || nd.cb[x].state == kCbClosed);
        return c;
    };
    auto ev_ts = [&](uint64_t rec, int64_t& tt, int64_t& cc, bool ents) {  // exits always (rt, statistic window)
        const LEvent x = ldecode(a, rec);
        const sg_local_event* le = a.ev + min((uint64_t)x.idx, n1);
        const bool need = x.kind != SG_LOCAL_ENTRY || ents;
        tt = need ? le->ts_ms : INT64_MIN;
        cc = need ? le->create_ts : 0;
    };
    uint64_t pf = s;  // position of the prefetched chunk
    uint64_t rec_n = a.rec_sorted[min(s + lane, n1)];
    int64_t t_n, c_n;
    bool ents_n = nb > 0 && !breakers_closed();  // the prefetched chunk's entries carry their times
    ev_ts(rec_n, t_n, c_n, ents_n);
    for (uint64_t base = s; base < e_end;) {
        const uint64_t j = base + lane;
        const bool act = j < e_end;
        if (pf != base) {  // wave-uniform: a skip moved past the prefetched chunk
            rec_n = a.rec_sorted[min(j, n1)];
            ents_n = nb > 0 && !breakers_closed();
            ev_ts(rec_n, t_n, c_n, ents_n);
        }
        const uint64_t rec_c = rec_n;
        const int64_t t_c = t_n, c_c = c_n;
        bool t_ok = ents_n || nb == 0;  // wave-uniform: the chunk's entries have their times
        pf = base + 64;
        rec_n = a.rec_sorted[min(pf + lane, n1)];
        LEvent ev;
        ev.idx = 0;
        ev.count = 0;
        ev.kind = -1;
        ev.prio = false;
        int64_t t = 0, create = 0;
        uint32_t qs = 0xFFFFFFFFu, qm = 0xFFFFFFFFu;
        int64_t sw0 = 0, sw1 = 0;  // breaker statistic windows of this event (exits)
        if (act) {
            ev = ldecode(a, rec_c);
            qs = nd.cs.of(ev.idx);
            qm = nd.cm.of(ev.idx);
            t = t_c;
            create = c_c;
            if (ev.kind != SG_LOCAL_ENTRY) {
                if (nb > 0) sw0 = t - t % nd.R.b[0].stat_ms;
                if (nb > 1) sw1 = t - t % nd.R.b[1].stat_ms;
            }
        }
        base += 64;
        const int nact = (int)__popcll(__ballot(act));
        const bool is_entry = act && ev.kind == SG_LOCAL_ENTRY;
        const bool is_exit = act && ev.kind != SG_LOCAL_ENTRY;
        const int64_t rt = t - create;
        int pos = 0;
        while (pos < nact) {
            // run: lanes [pos, rend) with the same windows as lane pos
            const uint32_t qs0 = (uint32_t)bcast32((int)qs, pos), qm0 = (uint32_t)bcast32((int)qm, pos);
            const uint64_t exr = __ballot(is_exit) & ~below(pos);
            const int fx = exr ? __builtin_ctzll(exr) : pos;  // the run's first exit fixes its statistic windows
            const int64_t a0 = bcast64(sw0, fx), a1 = bcast64(sw1, fx);
            const uint64_t diff = __ballot(act && lane > pos &&
                                           (qs != qs0 || qm != qm0 || (is_exit && (sw0 != a0 || sw1 != a1))));
            const int rend = diff ? __builtin_ctzll(diff) : nact;
            nd.at(qs0, qm0);
            int p = pos;
            while (p < rend) {
                const bool in = lane >= p && lane < rend;
                // ---- the breakers' fixed verdict for entries passing the flow check in this epoch
                // the first breaker (in order) that is not CLOSED decides: HALF_OPEN rejects, OPEN rejects
                // before its retry time and lets a probe through after it
                bool all_closed = true;
                int64_t retry = INT64_MAX;
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    if (x >= nb || !all_closed || nd.cb[x].state == kCbClosed) continue;
                    all_closed = false;
                    if (nd.cb[x].state == kCbOpen) retry = nd.cb[x].next_retry;
                }
                // ---- first lane needing the serial step (epoch end), from everything that does not
                // depend on this epoch's entry decisions
                uint64_t special = 0;
                if (thread_grade) special |= __ballot(in && is_entry);
                // exits: would a CLOSED breaker open here? first exit while HALF_OPEN.
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    if (x >= nb || nd.cb[x].state == kCbOpen) continue;
                    const bool ex = in && is_exit;
                    if (nd.cb[x].state == kCbHalfOpen) {
                        special |= __ballot(ex);
                        continue;
                    }
                    const int64_t swx = x == 0 ? a0 : a1;  // the run's statistic window for breaker x
                    const bool fresh = nd.cb[x].stat_start == INT64_MIN || swx > nd.cb[x].stat_start;
                    const int64_t b0 = fresh ? 0 : nd.cb[x].bad, t0 = fresh ? 0 : nd.cb[x].total;
                    const bool bad = ex && nd.cb_bad(x, rt, ev.kind == SG_LOCAL_EXIT_ERROR);
                    const int64_t pb = wave_incl_scan(bad ? 1 : 0, lane), pt = wave_incl_scan(ex ? 1 : 0, lane);
                    special |= __ballot(ex && nd.cb_trips(x, b0 + pb, t0 + pt));
                }
                // entries: flow decisions. The window sum moves only through passes of this epoch.
                const double thr = nd.R.flow_count;
                const bool flow_rule = nd.R.flow_grade == 1;
                uint64_t pass_m = 0, blk_flow = 0, blk_deg = 0;
                const uint64_t entries = __ballot(in && is_entry);
                uint64_t todo = entries & ~below(p);
                int E = special ? __builtin_ctzll(special) : rend;
                todo &= below(E);
                if (!all_closed) {
                    if (!t_ok) {  // a breaker opened inside this chunk: the entries' times, on demand
                        if (act && ev.kind == SG_LOCAL_ENTRY) t = a.ev[ev.idx].ts_ms;
                        t_ok = true;
                    }
                    // fixed window: an entry passes the flow check iff it fits on its own
                    const int32_t cur = java_d2i(nd.pass_qps());
                    const bool fits = !flow_rule || !((double)(int32_t)((uint32_t)cur + (uint32_t)ev.count) > thr);
                    const uint64_t fm = __ballot(fits) & todo;
                    // a flow-passing entry at or after the retry time is a probe (serial); a prioritized
                    // flow failure may occupy (serial)
                    const uint64_t sp = (__ballot(fits && t >= retry) | (__ballot(!fits && ev.prio && flow_rule))) & todo;
                    if (sp) {
                        E = __builtin_ctzll(sp);
                        todo &= below(E);
                    }
                    blk_deg = fm & todo;
                    blk_flow = todo & ~fm;
                } else if (!flow_rule) {
                    pass_m = todo;  // no flow rule (or none that counts QPS): every entry passes
                } else {
                    // greedy admit (DefaultController.canPass with a window that grows by the passes)
                    uint64_t pending = todo;
                    int64_t W = nd.s_wo + nd.sc[kLPass];
                    int guard = 0;
                    while (pending) {
                        if (++guard > 130) {
                            atomicOr(a.err, kErrInternal);
                            break;
                        }
                        const bool pl = (pending >> lane) & 1ull;
                        const int64_t av = pl ? (int64_t)ev.count : 0;
                        const int64_t ex = wave_incl_scan(av, lane) - av;
                        const int32_t cur = java_d2i(qps_of(W + ex, a.isec));
                        const bool ok = !((double)(int32_t)((uint32_t)cur + (uint32_t)ev.count) > thr);
                        const uint64_t fails = __ballot(pl && !ok);
                        const uint64_t adm = fails ? (pending & below(__builtin_ctzll(fails))) : pending;
                        pass_m |= adm;
                        W += wave_sum(((adm >> lane) & 1ull) ? (int64_t)ev.count : 0);
                        if (!fails) break;
                        const int f = __builtin_ctzll(fails);
                        const bool fprio = bcast32((int)ev.prio, f) != 0;
                        if (fprio) {  // a prioritized failure may occupy: serial step
                            E = f;
                            break;
                        }
                        blk_flow |= 1ull << f;
                        pending &= ~below(f + 1);
                        // skip mode: the window is fixed until the next entry that fits on its own
                        const int32_t curw = java_d2i(qps_of(W, a.isec));
                        const bool fit = pl && !((double)(int32_t)((uint32_t)curw + (uint32_t)ev.count) > thr);
                        const uint64_t stop = (__ballot(fit) | __ballot(pl && ev.prio)) & pending;
                        const uint64_t blk = stop ? (pending & below(__builtin_ctzll(stop))) : pending;
                        blk_flow |= blk;
                        pending &= ~blk;
                    }
                    todo &= below(E);
                    pass_m &= todo;
                    blk_flow &= todo;
                }
                // ---- apply lanes [p, E): entries by their verdict, exits accumulate
                const uint64_t ex_m = __ballot(in && is_exit) & below(E) & ~below(p);
                const bool mp = (pass_m >> lane) & 1ull, mf = (blk_flow >> lane) & 1ull, md = (blk_deg >> lane) & 1ull;
                const bool mx = (ex_m >> lane) & 1ull;
                if (mp) lstore(a, ev.idx, SG_LOCAL_PASS, 0);
                if (md) lstore(a, ev.idx, SG_LOCAL_BLOCK_DEGRADE, 0);
                const int64_t c = ev.count;
                const int64_t passed = wave_sum(mp ? c : 0), blocked = wave_sum((mf || md) ? c : 0);
                const int64_t succ = wave_sum(mx ? c : 0), rts = wave_sum(mx ? rt : 0);
                const int64_t excs = wave_sum((mx && ev.kind == SG_LOCAL_EXIT_ERROR) ? c : 0);
                const int64_t rmin = wave_min(mx ? rt : INT64_MAX);
                nd.sc[kLPass] += passed;
                nd.mc[kLPass] += passed;
                nd.sc[kLBlock] += blocked;
                nd.mc[kLBlock] += blocked;
                nd.sc[kLSucc] += succ;
                nd.mc[kLSucc] += succ;
                nd.sc[kLRt] += rts;
                nd.mc[kLRt] += rts;
                nd.sc[kLExc] += excs;
                nd.mc[kLExc] += excs;
                if (rmin < nd.s_min) nd.s_min = rmin;
                if (rmin < nd.m_min) nd.m_min = rmin;
                nd.threads += (int64_t)__popcll(pass_m) - (int64_t)__popcll(ex_m);
#pragma unroll
                for (int x = 0; x < 2; ++x) {  // breaker statistics of the exits (no state change by construction)
                    if (x >= nb || !ex_m) continue;
                    const int64_t swx = x == 0 ? a0 : a1;
                    nd.cb_stat_window(x, swx);
                    nd.cb[x].bad += wave_sum((mx && nd.cb_bad(x, rt, ev.kind == SG_LOCAL_EXIT_ERROR)) ? 1 : 0);
                    nd.cb[x].total += (int64_t)__popcll(ex_m);
                }
                if (E >= rend) break;
                // ---- lane E: the serial step
                {
                    LEvent es;
                    es.idx = (uint32_t)bcast32((int)ev.idx, E);
                    es.count = bcast32(ev.count, E);
                    es.kind = bcast32(ev.kind, E);
                    es.prio = bcast32((int)ev.prio, E) != 0;
                    const int64_t te = bcast64(t, E), ce = bcast64(create, E);
                    if (es.kind == SG_LOCAL_ENTRY) nd.entry(es, nb > 0 ? te : INT64_MIN);
                    else nd.exit(es, te, ce);
                }
                p = E + 1;
            }
            pos = rend;
        }
        ents_n = nb > 0 && !breakers_closed();
        ev_ts(rec_n, t_n, c_n, ents_n);  // the next chunk's events (its records have arrived meanwhile)
        // dead-period skip: the open second window admits nothing any more → jump to the first of (end of
        // this second-window period, end of this minute period, next exit of the resource); k_lskip_apply
        // adds the skipped entries' BLOCK counts to both windows
        if (may_skip && base < e_end && base >= skip_retry &&
            (double)(int32_t)((uint32_t)java_d2i(nd.pass_qps()) + 1u) > nd.R.flow_count) {
            if (nd.cs.q != pe_qs || nd.cm.q != pe_qm) {
                pe_qs = nd.cs.q;
                pe_qm = nd.cm.q;
                const uint32_t nbs = nd.cs.next_b, nbm = nd.cm.next_b;
                pe = gallop_search(base, e_end, [&](uint64_t p) {
                    const uint32_t idx = (uint32_t)((a.rec_sorted[p] >> a.abits) & a.imask);
                    return idx >= nbs || idx >= nbm;
                }, lane);
            }
            for (;;) {  // advance to the first exit at or after base, 64 entries per step
                const uint64_t i = xi + (uint64_t)lane;
                const uint64_t m = __ballot(i >= ne || (uint64_t)a.exit_pos[i] >= base);
                if (m) {
                    xi += (uint64_t)__builtin_ctzll(m);
                    break;
                }
                xi += 64;
            }
            const uint64_t nx = xi < ne ? min((uint64_t)a.exit_pos[xi], e_end) : e_end;
            const uint64_t end = min(pe, nx);
            skip_retry = end + 1;
            if (end > base && end - base >= kSkipMin) {
                const uint32_t np = (uint32_t)((end - base + kSkipPiece - 1) / kSkipPiece);
                uint32_t slot = 0;
                if (lane == 0) slot = atomicAdd(a.skip_count, np);
                slot = (uint32_t)bcast32((int)slot, 0);
                if (slot + np <= a.skip_cap) {
                    for (uint32_t pi = lane; pi < np; pi += 64) {
                        LSkip sk;
                        sk.k = k;
                        sk.qs = nd.cs.q;
                        sk.qm = nd.cm.q;
                        sk.b0 = (uint32_t)(base + (uint64_t)pi * kSkipPiece);
                        sk.b1 = (uint32_t)min(end, base + (uint64_t)(pi + 1) * kSkipPiece);
                        sk.pad[0] = sk.pad[1] = sk.pad[2] = 0;
                        a.skips[slot + pi] = sk;
                    }
                    base = end;
                }
            }
        }
    }
    nd.finish();
}

__global__ void __launch_bounds__(256, SG_LWALK_BLOCKS) k_lwalk_long(LArgs a, BatchArgs sg) {
    __shared__ uint32_t sbnd[kLdsBnd];
    __shared__ const uint32_t* bndp[kMaxWl];
    if (*a.err) return;
    stage_lperiods(a, sbnd, bndp);
    const int lane = lane_id();
    const uint32_t n_long = *sg.long_count;
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t item = wave; item < n_long; item += nwaves) {
        const uint64_t s = sg.long_list[item];
        const uint32_t k = (uint32_t)(a.rec_sorted[s] >> a.kshift);
        if (a.rules[k].cx || (a.dyn && a.dyn[k] == a.epoch)) continue;  // k_lwalk_cx
        const uint64_t e = gallop_search(s + (sg.short_max ? sg.short_max : 1), a.n, [&](uint64_t p) {
            return (uint32_t)(a.rec_sorted[p] >> a.kshift) != k;
        }, lane);
        lwalk_wave(a, bndp, k, s, e);
    }
}

// ------------------------------------------------------------------------ the flow-rule layer (cx)
//
// Resources whose flow rules are more than the fast walkers' one DefaultController rule with limitApp
// "default" — several rules (FlowRuleChecker.checkFlow, FlowRuleChecker.java:44-57: in FlowRuleComparator
// order, the first failing rule throws), limitApp origin / "other" rules reading the origin's StatisticNode
// (selectNodeByRequesterAndStrategy :115-145), WarmUp / RateLimiter / WarmUpRateLimiter controllers — are
// walked one event at a time, one lane per resource segment, by k_lwalk_cx. The resource's ClusterNode stays
// in registers (LNode); an origin node is opened from memory for the event that needs it.

namespace {

__device__ __forceinline__ int64_t java_d2l(double x) {  // JLS §5.1.3
    if (x != x) return 0;
    if (x >= 9223372036854775807.0) return INT64_MAX;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t java_round(double a) {  // Math.round(double), floor(a + 1/2) on the bits
    const int64_t bits = __double_as_longlong(a);
    const int64_t shift = (52 - 1 + 1023) - ((bits & 0x7FF0000000000000LL) >> 52);
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000FFFFFFFFFFFFFLL) | 0x0010000000000000LL;
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return java_d2l(a);
}

// WarmUpController.coolDownTokens (WarmUpController.java:161-175)
__device__ int64_t warm_cool_down(const LFlowRule& r, const LCtl& c, int64_t ct, int64_t pass_qps) {
    const int64_t old = c.stored;
    int64_t nv = old;
    if (old < r.warning_token || (old > r.warning_token && pass_qps < java_d2i(r.count) / r.cold))
        nv = java_d2l((double)old + (double)(ct - c.last_filled) * r.count / 1000);
    return nv < r.max_token ? nv : (int64_t)r.max_token;
}

// WarmUpController.syncToken (:140-159)
__device__ void warm_sync(const LFlowRule& r, LCtl& c, int64_t now, int64_t pass_qps) {
    const int64_t ct = now - now % 1000;
    if (ct <= c.last_filled) return;
    const int64_t cur = (int64_t)((uint64_t)warm_cool_down(r, c, ct, pass_qps) - (uint64_t)pass_qps);
    c.stored = cur < 0 ? 0 : cur;
    c.last_filled = ct;
}

__device__ __forceinline__ double warm_qps(const LFlowRule& r, int64_t above) {  // Math.nextUp(1 / (…))
    return nextafter(1.0 / ((double)above * r.slope + 1.0 / r.count), (double)INFINITY);
}

// RateLimiterController.canPass (:46-91) / the tail of WarmUpRateLimiterController.canPass (:61-86) with the
// cost already known; *wait = the sleep. The acquire/count checks only exist in RateLimiterController.
__device__ bool pace_step(const LFlowRule& r, LCtl& c, int64_t now, int64_t cost, int64_t* wait) {
    *wait = 0;
    if (cost + c.latest <= now) {
        c.latest = now;
        return true;
    }
    if (cost + c.latest - now > r.max_queue_ms) return false;
    c.latest += cost;
    const int64_t w = c.latest - now;
    if (w > r.max_queue_ms) {  // unreachable without concurrent callers
        c.latest -= cost;
        return false;
    }
    *wait = w > 0 ? w : 0;
    return true;
}

// ---- the embedded token server (ClusterStateManager SERVER) ----

__device__ __forceinline__ double c3_qps(int64_t sum, double isec) { return avg_div((double)sum, isec); }

// DefaultTokenService.requestToken (DefaultTokenService.java:39-50) → ClusterFlowChecker.acquireClusterToken
// (ClusterFlowChecker.java:55-112) for one request at time t, on the flowId's ClusterMetric ring in HBM
// (ClusterMetric / ClusterMetricLeapArray: currentWindow with the occupy transfer on reset, :49-71; tryOccupyNext,
// ClusterMetric.java:79-98). The same arithmetic as the cluster walkers (engine.hip), one request at a time.
__device__ int32_t embedded_token(const LArgs& a, uint32_t key, int64_t t, int32_t acq, bool prio, int32_t* wait) {
    *wait = 0;
    key &= SG_KEY_INDEX;
    if (key == SG_KEY_BAD || acq <= 0) return SG_STATUS_BAD_REQUEST;
    if (key >= a.c3_K) return SG_STATUS_NO_RULE_EXISTS;
    const uint8_t ls = a.c3_rule_lim ? a.c3_rule_lim[key] : (uint8_t)0xFF;
    if (ls != 0xFF && !emb_lim_try_pass(a.lim_ring + ls, t, a.lim_qps[ls])) return SG_STATUS_TOO_MANY_REQUEST;
    const Rule R = a.c3_rules[key];
    Bucket* ring = a.c3_ring + (size_t)key * a.c3_stride;
    const Occ o = a.c3_occ[key];
    int64_t occ_pass = o.pass, occ_req = o.pass_req;
    // currentWindow(t) on slot I, then values(t) of the other slots
    const int64_t P = t / R.wl;
    const int S = R.S;
    const int I = (int)(P % S);
    const int64_t ws = P * R.wl;
    const int64_t lo = ws - (int64_t)(S - 1) * R.wl;
    const int h = (int)((P + 1) % S);
    int64_t wo_pass = 0, wo_wait = 0, head_other = 0;
    for (int q = 0; q < S; ++q) {
        const int64_t st = ring[q].start;
        const bool v = q != I && st != INT64_MIN && st >= lo;
        wo_pass += v ? ring[q].c[SG_EV_PASS] : 0;
        wo_wait += v ? ring[q].c[SG_EV_WAITING] : 0;
        if (q == h && v) head_other = ring[q].c[SG_EV_PASS];
    }
    int64_t cur[SG_NUM_EVENTS];
    const int64_t stI = ring[I].start;
    if (stI == ws) {
        for (int e = 0; e < SG_NUM_EVENTS; ++e) cur[e] = ring[I].c[e];
    } else {
        for (int e = 0; e < SG_NUM_EVENTS; ++e) cur[e] = 0;
        if (stI != INT64_MIN && occ_req > 0) {  // resetWindowTo transfers the occupied quota (not a creation)
            cur[SG_EV_OCCUPIED_PASS] += occ_pass;
            cur[SG_EV_PASS] += occ_pass;
            cur[SG_EV_PASS_REQUEST] += occ_req;
            occ_pass = occ_req = 0;
        }
    }
    int32_t st = SG_STATUS_BLOCKED;
    const double latest = c3_qps(wo_pass + cur[SG_EV_PASS], R.isec);
    const double next_remaining = R.thr - latest - (double)acq;
    if (next_remaining >= 0) {
        cur[SG_EV_PASS] += acq;
        cur[SG_EV_PASS_REQUEST] += 1;
        if (prio) cur[SG_EV_OCCUPIED_PASS] += acq;
        st = SG_STATUS_OK;
    } else {
        bool waited = false;
        if (prio) {
            const double occupy_avg = c3_qps(wo_wait + cur[SG_EV_WAITING], R.isec);
            if (occupy_avg <= a.max_occ_ratio * R.thr) {
                const int64_t head = (S == 1) ? cur[SG_EV_PASS] : head_other;
                if (latest + (double)(acq + occ_pass) - (double)head <= R.thr) {
                    occ_pass += acq;  // addOccupyPass
                    occ_req += 1;
                    cur[SG_EV_WAITING] += acq;
                    if (R.wait_ms > 0) {
                        *wait = R.wait_ms;
                        st = SG_STATUS_SHOULD_WAIT;
                        waited = true;
                    }
                }
            }
        }
        if (!waited) {
            cur[SG_EV_BLOCK] += acq;
            cur[SG_EV_BLOCK_REQUEST] += 1;
            if (prio) cur[SG_EV_OCCUPIED_BLOCK] += acq;
        }
    }
    ring[I].start = ws;
    for (int e = 0; e < SG_NUM_EVENTS; ++e) ring[I].c[e] = cur[e];
    store_hot(a.c3_hot + (size_t)key * a.c3_stride + I, ws, cur[SG_EV_PASS], cur[SG_EV_WAITING]);
    if (occ_pass != o.pass || occ_req != o.pass_req) {
        Occ no;
        no.pass = occ_pass;
        no.pass_req = occ_req;
        a.c3_occ[key] = no;
    }
    return st;
}

// FlowRuleChecker.selectNodeByRequesterAndStrategy (:115-145) with selectReferenceNode (:96-112): 0 the ClusterNode,
// 1 the origin node, 2 the resource's DefaultNode of the current context (CHAIN), 3 the ClusterNode of r.ref
// (RELATE; ref_exists() says whether ClusterBuilderSlot created it), -1 none (the rule passes)
template <class RefExists>
__device__ int cx_select(const LArgs& a, const LRule& R, const LFlowRule& r, int origin, int ctx, RefExists&& ref_exists) {
    int matched;
    if (origin > 0 && r.limit_app == origin) {
        matched = 1;
    } else if (r.limit_app == SG_LIMIT_APP_DEFAULT) {
        matched = 0;
    } else if (r.limit_app == SG_LIMIT_APP_OTHER && origin > 0) {  // FlowRuleManager.isOtherOrigin (:132-148)
        for (uint32_t i = 0; i < R.fr_n; ++i)
            if (a.frules[R.fr_begin + i].limit_app == origin) return -1;
        matched = 1;
    } else {
        return -1;
    }
    if (r.strategy == SG_STRATEGY_DIRECT) return matched;
    if (r.ref < 0) return -1;  // StringUtil.isEmpty(refResource)
    if (r.strategy == SG_STRATEGY_RELATE) return ref_exists() ? 3 : -1;
    if (r.strategy == SG_STRATEGY_CHAIN) return r.ref == ctx ? 2 : -1;
    return -1;
}

// One rule's canPass on the selected node: 0 block, 1 pass (*wait: the controller's sleep), 2 PriorityWaitException.
// The node's windows are opened as the controller reads them: passQps the second window, previousPassQps the minute
// window, the occupy path both (tryOccupyNext, addWaitingRequest, addOccupiedPass); a THREAD rule reads neither.
__device__ int cx_rule(const LArgs& a, LNode& n, const LFlowRule& r, LCtl& c, const LEvent& e, int64_t t,
                       uint32_t qs, uint32_t qm, int64_t* wait) {
    *wait = 0;
    switch (r.behavior) {
    case SG_CONTROL_WARM_UP: {  // WarmUpController.canPass (:113-138)
        n.at_s(qs);
        n.at_m(qm);
        const int64_t pass_qps = java_d2l(n.pass_qps());
        warm_sync(r, c, t, java_d2l((double)n.prev_pass(t)));
        const int64_t sum = (int64_t)((uint64_t)pass_qps + (uint64_t)(int64_t)e.count);
        const double lim = c.stored >= r.warning_token ? warm_qps(r, c.stored - r.warning_token) : r.count;
        return (double)sum <= lim ? 1 : 0;
    }
    case SG_CONTROL_RATE_LIMITER:
        if (e.count <= 0) return 1;
        if (r.count <= 0) return 0;
        return pace_step(r, c, t, java_round(1.0 * (double)e.count / r.count * 1000), wait) ? 1 : 0;
    case SG_CONTROL_WARM_UP_RATE_LIMITER: {  // WarmUpRateLimiterController.canPass (:43-87)
        n.at_m(qm);
        warm_sync(r, c, t, java_d2l((double)n.prev_pass(t)));
        const double q = c.stored >= r.warning_token ? warm_qps(r, c.stored - r.warning_token) : r.count;
        return pace_step(r, c, t, java_round(1.0 * (double)e.count / q * 1000), wait) ? 1 : 0;
    }
    default: {  // DefaultController.canPass (:49-76)
        if (r.grade != 0) n.at_s(qs);
        const int32_t cur = r.grade == 0 ? (int32_t)n.threads : java_d2i(n.pass_qps());
        if (!((double)(int32_t)((uint32_t)cur + (uint32_t)e.count) > r.count)) return 1;
        if (e.prio && r.grade == 1) {
            n.at_m(qm);
            const int64_t w = n.try_occupy_next(t, e.count, r.count);
            if (w < a.occupy_timeout) {
                const int s = n.bor_window(t + w);  // addWaitingRequest
                if (s >= 0) n.bor[s].pass += e.count;
                n.mc[kLOccPass] += e.count;         // addOccupiedPass: the minute window
                n.mc[kLPass] += e.count;
                *wait = w;
                return 2;
            }
        }
        return 0;
    }
    }
}

// The nodes StatisticSlot updates for one event besides the ClusterNode: the origin node (ClusterBuilderSlot, origin
// o of the event) and the DefaultNode of the event's context (NodeSelectorSlot, context tracking on), from the pool.
__device__ __forceinline__ uint2 event_nodes(const LArgs& a, uint32_t idx) {
    if (!a.nkeys) return make_uint2(kNoNode, kNoNode);
    return a.ev_node[idx];  // node indices (k_lnode_resolve)
}

// One entry of a cx resource, the slot chain in SPI order inside StatisticSlot.entry (StatisticSlot.java:55-122):
// ParamFlowSlot.checkFlow (ParamFlowSlot.java:66-93, the event's arguments) → FlowSlot (every rule,
// FlowRuleChecker.checkFlow :44-57; cluster-mode rules as on a node that is neither token client nor server,
// passClusterCheck → fallbackToLocalOrPass :147-175) → DegradeSlot, then the StatisticSlot updates of the
// ClusterNode, the origin node and the context's DefaultNode, and ParamFlowStatisticEntryCallback.onPass.
// The lane cx walker's per-lane resource node lives in dynamic LDS (kCxNdBytes per lane): the out-of-line serial
// step takes it by reference, which kept it in scratch.
constexpr uint32_t kCxNdBytes = (uint32_t)((sizeof(LNode) + 15) / 16 * 16);
constexpr uint32_t kCxLdsBytes = 256 * kCxNdBytes;

// The origin / context / RELATE nodes of one event: on the stack (the lane walker: one per lane), or — W, the wave
// walker, whose serial step every lane runs on wave-uniform values — in the wave's three LDS slots `slots`
// (kCxNdBytes each), one copy instead of 64 private ones in scratch.
template <bool W>
struct CxNodes;
template <>
struct CxNodes<false> {
    LNode on, cn;
    __device__ CxNodes(const LArgs& a, const LNode& nd, uint32_t on_idx, uint32_t cn_idx, unsigned char*)
        : on(on_idx != kNoNode ? LNode(a, nd, on_idx) : LNode(a, LNode::None{})),
          cn(cn_idx != kNoNode ? LNode(a, nd, cn_idx) : LNode(a, LNode::None{})) {}
};
template <>
struct CxNodes<true> {
    LNode& on;
    LNode& cn;
    __device__ CxNodes(const LArgs& a, const LNode& nd, uint32_t on_idx, uint32_t cn_idx, unsigned char* slots)
        : on(on_idx != kNoNode ? *::new (slots) LNode(a, nd, on_idx) : *::new (slots) LNode(a, LNode::None{})),
          cn(cn_idx != kNoNode ? *::new (slots + kCxNdBytes) LNode(a, nd, cn_idx)
                               : *::new (slots + kCxNdBytes) LNode(a, LNode::None{})) {}
};

template <bool W>
__device__ void cx_entry(const LArgs& a, const uint32_t* const* bndp, LNode& nd, const LEvent& e, int64_t t, int origin,
                         int ctx, const sg_slot_ext* x, uint32_t qs, uint32_t qm, uint2 nodes, unsigned char* slots) {
    const LRule& R = nd.R;
    const uint32_t on_idx = nodes.x, cn_idx = nodes.y;
    const bool have_on = on_idx != kNoNode, have_cn = cn_idx != kNoNode;
    // windows opened as touched (cx_rule, the StatisticSlot adds); an absent node loads nothing
    CxNodes<W> nn(a, nd, on_idx, cn_idx, slots);
    LNode& on = nn.on;
    LNode& cn = nn.cn;
    const bool params = R.ps && a.has_ps && x && !x->args_null;
    int32_t status = SG_LOCAL_PASS;
    int64_t wait = 0;
    if (params) {  // ParamFlowSlot (@Spi order -3000): before FlowSlot
        // the resource's one QPS rule, its (rule, value) slot looked up by k_local_prep (LArgs::pslot), else every rule
        const uint64_t psl = a.pslot ? a.pslot[e.idx] : kPsUnknown;
        int32_t pr = -1;
        if (psl != kPsUnknown) {
            const uint32_t ri = a.ps.res_rules[a.ps.res_begin[nd.k]];
            a.ps.inited[ri] = 1;  // initParamMetricsFor (the arguments are not null here)
            bool ok = psl != kPsEarlyFail;
            if (ok && psl != kPsNoCheckInit && psl != kPsNoCheck) {
                const PRule r = a.ps.p.rules[ri];
                PSlot& sl = a.ps.p.table[psl];
                const int64_t tc = r.hot_count ? param_token_count(a.ps.p, r, sl.value) : r.token_count;
                PState st{sl.time, sl.tokens, sl.flags};
                ok = r.behavior == 2 ? param_throttle_step(st, throttle_cost(r, tc, e.count), r.max_queueing_ms, t)
                                     : param_default_step(st, tc, tc + r.burst, r.duration_sec * 1000, t, e.count);
                sl.time = st.time;
                sl.tokens = st.tokens;
                sl.flags = st.flags;
            }
            if (!ok) pr = (int32_t)ri;
        } else {
            pr = ps_check_entry(a.ps, nd.k, t, e.count, x->arg_begin, x->arg_count);
        }
        if (pr >= 0) {
            status = SG_LOCAL_BLOCK_PARAM;
            wait = pr;  // reported in wait_ms: the rule that threw ParamFlowException
        }
    }
    // the rules in check order; a resource whose one DefaultController rule the fast walkers read from R (it is
    // walked here because of its param rules) gets that rule back as a plain DIRECT / "default" rule
    const uint32_t n_rules = R.fr_n ? R.fr_n : (R.flow_grade >= 0 ? 1u : 0u);
    LCtl stateless{0, 0, -1, 0};
    for (uint32_t i = 0; status == SG_LOCAL_PASS && i < n_rules; ++i) {
        LFlowRule r;
        if (R.fr_n) {
            r = a.frules[R.fr_begin + i];
        } else {
            r = LFlowRule{};
            r.count = R.flow_count;
            r.grade = R.flow_grade;
            r.behavior = SG_CONTROL_DEFAULT;
            r.limit_app = SG_LIMIT_APP_DEFAULT;
            r.strategy = SG_STRATEGY_DIRECT;
            r.ref = -1;
            r.cluster_mode = SG_CLUSTER_MODE_OFF;
        }
        if (r.cluster_mode != SG_CLUSTER_MODE_OFF && a.emb) {
            // passClusterCheck on the embedded server (FlowRuleChecker.java:147-164), applyTokenResult (:186-209)
            int32_t tw = 0;
            const int32_t ts = embedded_token(a, r.cluster_key, t, e.count, e.prio, &tw);
            if (ts == SG_STATUS_OK) continue;
            if (ts == SG_STATUS_SHOULD_WAIT) {  // Thread.sleep(waitInMs), then the rule passes
                wait += tw;
                continue;
            }
            if (ts == SG_STATUS_BLOCKED) {
                status = SG_LOCAL_BLOCK_FLOW;
                break;
            }
            // NO_RULE_EXISTS / BAD_REQUEST / FAIL / TOO_MANY_REQUEST: fallbackToLocalOrPass
        }
        if (r.cluster_mode == SG_CLUSTER_MODE_NO_FALLBACK) continue;  // cluster rule not activated: passes
        const int sel = cx_select(a, R, r, origin, ctx, [&]() {
            if (r.ref == (int32_t)nd.k) return true;  // this entry reached ClusterBuilderSlot
            return (uint32_t)r.ref < a.K && a.head[r.ref].created != 0;
        });
        if (sel < 0 || (sel == 1 && !have_on) || (sel == 2 && !have_cn)) continue;
        LCtl& c = R.fr_n ? a.ctl[R.fr_begin + i] : stateless;
        int64_t w = 0;
        int v;
        if (sel == 0 || (sel == 3 && r.ref == (int32_t)nd.k)) {
            v = cx_rule(a, nd, r, c, e, t, qs, qm, &w);
        } else if (sel == 1) {
            v = cx_rule(a, on, r, c, e, t, qs, qm, &w);
        } else if (sel == 2) {
            v = cx_rule(a, cn, r, c, e, t, qs, qm, &w);
        } else if constexpr (W) {  // (a RELATE group is walked by the lane walker; kept for completeness)
            LNode& rn = *::new (slots + 2 * kCxNdBytes) LNode(a, bndp, (uint32_t)r.ref);
            v = cx_rule(a, rn, r, c, e, t, qs, qm, &w);
            rn.finish();
        } else {  // RELATE: another resource of this key group, kept in memory between its events
            LNode rn(a, bndp, (uint32_t)r.ref);
            v = cx_rule(a, rn, r, c, e, t, qs, qm, &w);
            rn.finish();
        }
        if (v == 0) {
            status = SG_LOCAL_BLOCK_FLOW;
            break;
        }
        if (v == 2) {
            status = SG_LOCAL_PASS_WAIT;
            wait = w;
            break;
        }
        wait += w;  // each rate limiter sleeps in turn
    }
    if (status == SG_LOCAL_PASS && nd.degrade_blocks([&]() { return t; })) status = SG_LOCAL_BLOCK_DEGRADE;
    if (status == SG_LOCAL_PASS) {  // addPassRequest: both windows of each node
        nd.at(qs, qm);
        nd.threads += 1;
        nd.sc[kLPass] += e.count;
        nd.mc[kLPass] += e.count;
        if (have_on) {
            on.at(qs, qm);
            on.threads += 1;
            on.sc[kLPass] += e.count;
            on.mc[kLPass] += e.count;
        }
        if (have_cn) {
            cn.at(qs, qm);
            cn.threads += 1;
            cn.sc[kLPass] += e.count;
            cn.mc[kLPass] += e.count;
        }
    } else if (status == SG_LOCAL_PASS_WAIT) {  // PriorityWaitException: thread counts only
        nd.threads += 1;
        if (have_on) on.threads += 1;
        if (have_cn) cn.threads += 1;
    } else {  // increaseBlockQps: both windows
        nd.at(qs, qm);
        nd.sc[kLBlock] += e.count;
        nd.mc[kLBlock] += e.count;
        if (have_on) {
            on.at(qs, qm);
            on.sc[kLBlock] += e.count;
            on.mc[kLBlock] += e.count;
        }
        if (have_cn) {
            cn.at(qs, qm);
            cn.sc[kLBlock] += e.count;
            cn.mc[kLBlock] += e.count;
        }
        if (status != SG_LOCAL_BLOCK_PARAM) wait = 0;
    }
    if (params && (status == SG_LOCAL_PASS || status == SG_LOCAL_PASS_WAIT))
        ps_threads(a.ps, nd.k, x->arg_begin, x->arg_count, +1);  // ParamFlowStatisticEntryCallback.onPass
    lstore(a, e.idx, status, wait > INT32_MAX ? INT32_MAX : (int32_t)wait);
    if (have_on) on.finish();
    if (have_cn) cn.finish();
}

// One exit of a cx resource: StatisticSlot.exit (:124-165) on the ClusterNode (+ DegradeSlot.exit), the origin node
// and the context's DefaultNode; ParamFlowStatisticExitCallback.onExit (decreaseThreadCount of the exit's args).
template <bool W>
__device__ void cx_exit(const LArgs& a, const uint32_t* const* bndp, LNode& nd, const LEvent& e, int64_t t,
                        int64_t create, int origin, int ctx, const sg_slot_ext* x, uint32_t qs, uint32_t qm, uint2 nodes,
                        unsigned char* slots) {
    nd.exit(e, t, create);
    const uint32_t on_idx = nodes.x, cn_idx = nodes.y;
    auto node_exit = [&](uint32_t idx, unsigned char* slot) {
        if constexpr (W) {
            LNode& m = *::new (slot) LNode(a, nd, idx);
            m.at(qs, qm);
            m.exit(e, t, create);
            m.finish();
        } else {
            LNode m(a, nd, idx);
            m.at(qs, qm);
            m.exit(e, t, create);
            m.finish();
        }
    };
    if (on_idx != kNoNode) node_exit(on_idx, slots);  // recordCompleteFor(originNode)
    if (cn_idx != kNoNode) node_exit(cn_idx, slots ? slots + kCxNdBytes : nullptr);
    if (nd.R.ps && a.has_ps && x && !x->args_null) ps_threads(a.ps, nd.k, x->arg_begin, x->arg_count, -1);
}

}  // namespace

// One lane per segment of a cx resource (or a RELATE key group), from every length class of k_seg's lists. A lone
// resource keeps its ClusterNode in registers for the whole segment; a group's events belong to several resources
// (one reads another's ClusterNode), so each event opens its resource's node from memory and writes it back.
__device__ bool cxw_dead_able(const LArgs& a, const LRule& R, uint32_t k, int32_t* prule);
__device__ bool cxw_saturated(const LArgs& a, const LNode& nd);

// Work items of the lane cx walker: k_seg's long list, then its length classes longest first (the lanes with the
// longest chains start first).
__device__ __forceinline__ uint32_t cx_items(const BatchArgs& sg) {
    uint32_t total = *sg.long_count;
    for (int c = 0; c < kClasses; ++c) total += sg.short_count[c];
    return total;
}

// Item i: the head of a segment the lane cx walker takes (a cx or origin-event resource the wave walker leaves; a
// RELATE group), else ~0. (Returned, not written through an out-parameter: that form, inlined into k_lcx_list under
// -O3, stored 0 for the origin-event segments — test_local_rules_gpu.py::test_mixed_rule_sets with one lane per
// segment caught it.)
__device__ __forceinline__ uint64_t cx_item(const LArgs& a, const BatchArgs& sg, uint32_t i) {
    uint32_t r = i;
    uint64_t j;
    bool wave = false;  // the wave walker's (k_lwalk_cxw), unless a RELATE group
    if (r < *sg.long_count) {
        j = sg.long_list[r];
        wave = a.cxw != 0;
    } else {
        r -= *sg.long_count;
        int c = kClasses - 1;
        while (r >= sg.short_count[c]) r -= sg.short_count[c--];
        j = sg.short_list[sg.class_off[c] + r];
        wave = a.cxw != 0 && c >= a.cxw_cls;
    }
    const uint32_t k = (uint32_t)(a.rec_sorted[j] >> a.kshift);
    const LRule& R = a.rules[k];
    const bool dyn = a.dyn && a.dyn[k] == a.epoch;
    const bool take = (R.cx || dyn) && !(wave && !R.grp);
    return take ? j : ~0ull;
}

// The lane cx walker's segments, compacted in item order (wave-aggregated appends): a cx resource is ~10 % of the
// batch's segments, so walking k_seg's lists directly left ~9 of every 10 lanes of its waves idle.
__global__ void __launch_bounds__(256) k_lcx_list(LArgs a, BatchArgs sg) {
    if (*a.err) return;
    const uint32_t total = cx_items(sg);
    const int lane = lane_id();
    for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < total; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + (uint32_t)lane;
        const uint64_t j = i < total ? cx_item(a, sg, i) : ~0ull;
        const bool take = j != ~0ull;
        const uint64_t m = __ballot(take);
        if (!m) continue;
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(a.cx_count, (uint32_t)__popcll(m));
        at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
        if (take) a.cx_list[at + (uint32_t)__popcll(m & below(lane))] = (uint32_t)j;
    }
}

// The cx walkers' serial step (cx_entry / cx_exit / cxw_step, out of line) takes the batch arguments by reference:
// taken from the kernel parameter, that reference made the compiler copy all 1,248 B of LArgs to every lane's
// scratch at kernel entry and read the fields from there. A copy in LDS, staged once per block straight from the
// kernarg segment (LArgs is the first parameter), serves those reads instead.
__device__ __forceinline__ void stage_largs(LArgs* dst) {
    const uint32_t* src = (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (uint32_t i = threadIdx.x; i < (uint32_t)(sizeof(LArgs) / 4); i += blockDim.x) d[i] = src[i];
    __syncthreads();
}
static_assert(sizeof(LArgs) % 4 == 0, "LArgs staged by dwords");


__global__ void __launch_bounds__(256) k_lwalk_cx(LArgs a_arg, BatchArgs sg) {
    __shared__ uint32_t sbnd[kLdsBnd];
    __shared__ const uint32_t* bndp[kMaxWl];
    __shared__ LArgs a_lds;
    extern __shared__ __attribute__((aligned(16))) unsigned char cx_nd_lds[];
    void* const nd_mem = cx_nd_lds + (size_t)threadIdx.x * kCxNdBytes;
    (void)a_arg;
    stage_largs(&a_lds);
    const LArgs& a = a_lds;
    if (*a.err) return;
    stage_lperiods(a, sbnd, bndp);
    // the segments k_lcx_list compacted (64 of them per wave), else every segment of k_seg's lists
    const bool listed = a.cx_list != nullptr;
    const uint32_t total = listed ? *a.cx_count : cx_items(sg);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const uint64_t j = listed ? (uint64_t)a.cx_list[i] : cx_item(a, sg, i);
        if (j == ~0ull) continue;
        const uint32_t k = (uint32_t)(a.rec_sorted[j] >> a.kshift);
        if (a.rules[k].grp) {
            for (uint64_t p = j; p < a.n; ++p) {
                const uint64_t rec = a.rec_sorted[p];
                if ((uint32_t)(rec >> a.kshift) != k) break;
                const LEvent e = ldecode(a, rec);
                const sg_local_event le = a.ev[e.idx];
                const sg_slot_ext* x = a.ext ? a.ext + e.idx : nullptr;
                const int ctx = x ? (int)x->context : 0;
                LNode& nd = *::new (nd_mem) LNode(a, bndp, le.resource & SG_KEY_INDEX);
                nd.created = 1;
                const uint32_t qs = nd.cs.of(e.idx), qm = nd.cm.of(e.idx);
                if (e.kind != SG_LOCAL_ENTRY) nd.at(qs, qm);  // an entry opens what it touches (cx_entry)
                const uint2 nodes = event_nodes(a, e.idx);
                if (e.kind == SG_LOCAL_ENTRY) cx_entry<false>(a, bndp, nd, e, le.ts_ms, le.origin, ctx, x, qs, qm, nodes, nullptr);
                else cx_exit<false>(a, bndp, nd, e, le.ts_ms, le.create_ts, le.origin, ctx, x, qs, qm, nodes, nullptr);
                nd.finish();
            }
            continue;
        }
        LNode& nd = *::new (nd_mem) LNode(a, bndp, k);
        nd.created = 1;
        // Dead periods as in the wave walker (cx_wave), one lane at a time: once a QPS rule every entry reaches is
        // saturated, the period's further entries need only their ParamFlowSlot check and BLOCK counts (ClusterNode
        // and origin node, added when the period ends), not the whole chain.
        int32_t prule = -1;
        const bool dead_ok =
            a.cxw && !(*a.flags & (kLFlagPrio | kLFlagNonPos)) && cxw_dead_able(a, nd.R, k, &prule);
        PRule pr{};
        if (prule >= 0) pr = a.ps.p.rules[prule];
        bool dead = false, inited = false;
        uint32_t dqs = 0, dqm = 0, dend = 0;
        int64_t dblk = 0;
        uint32_t onode[2] = {kNoNode, kNoNode};
        int64_t osum[2] = {0, 0};
        auto flush_origins = [&]() {
            for (int q = 0; q < 2; ++q) {
                if (onode[q] == kNoNode) continue;
                LNode on(a, nd, onode[q]);
                on.at(dqs, dqm);
                on.sc[kLBlock] += osum[q];
                on.mc[kLBlock] += osum[q];
                on.finish();
                onode[q] = kNoNode;
                osum[q] = 0;
            }
        };
        for (uint64_t p = j; p < a.n; ++p) {
            const uint64_t rec = a.rec_sorted[p];
            if ((uint32_t)(rec >> a.kshift) != k) break;
            const LEvent e = ldecode(a, rec);
            if (dead && e.idx >= dend) {  // the dead period ended
                nd.at(dqs, dqm);
                nd.sc[kLBlock] += dblk;
                nd.mc[kLBlock] += dblk;
                dblk = 0;
                flush_origins();
                dead = false;
            }
            if (dead && e.kind == SG_LOCAL_ENTRY) {
                uint64_t psl = kPsNoCheck;
                int64_t t = 0;
                uint32_t node;
                if (a.cxside) {
                    const CxSide z = a.cxside[p];
                    node = z.node;
                    if (prule >= 0) {
                        t = z.t;
                        psl = z.psl >= 0xFFFFFFFCu ? ~0ull - (uint64_t)(0xFFFFFFFFu - z.psl) : (uint64_t)z.psl;
                    }
                } else {
                    node = event_nodes(a, e.idx).x;
                    if (prule >= 0) {
                        psl = a.pslot ? a.pslot[e.idx] : kPsUnknown;
                        t = a.ev[e.idx].ts_ms;
                    }
                }
                if (psl != kPsUnknown) {
                    bool pfail = false;
                    if (prule >= 0 && psl != kPsNoCheck) {
                        if (!inited) {  // initParamMetricsFor
                            a.ps.inited[prule] = 1;
                            inited = true;
                        }
                        if (psl == kPsEarlyFail) {
                            pfail = true;
                        } else if (psl != kPsNoCheckInit) {
                            PSlot& sl = a.ps.p.table[psl];
                            const int64_t tc = pr.hot_count ? param_token_count(a.ps.p, pr, sl.value) : pr.token_count;
                            PState st{sl.time, sl.tokens, sl.flags};
                            const bool ok =
                                pr.behavior == 2
                                    ? param_throttle_step(st, throttle_cost(pr, tc, e.count), pr.max_queueing_ms, t)
                                    : param_default_step(st, tc, tc + pr.burst, pr.duration_sec * 1000, t, e.count);
                            sl.time = st.time;
                            sl.tokens = st.tokens;
                            sl.flags = st.flags;
                            pfail = !ok;
                        }
                    }
                    if (pfail) lstore(a, e.idx, SG_LOCAL_BLOCK_PARAM, prule);  // (FLOW: the default result)
                    dblk += e.count;
                    if (node != kNoNode) {
                        int q = onode[0] == node ? 0 : onode[1] == node ? 1 : onode[0] == kNoNode ? 0 : onode[1] == kNoNode ? 1 : -1;
                        if (q < 0) {
                            flush_origins();
                            q = 0;
                        }
                        onode[q] = node;
                        osum[q] += e.count;
                    }
                    continue;
                }
            }
            const sg_local_event le = a.ev[e.idx];
            const sg_slot_ext* x = a.ext ? a.ext + e.idx : nullptr;
            const int ctx = x ? (int)x->context : 0;
            const uint32_t qs = nd.cs.of(e.idx), qm = nd.cm.of(e.idx);
            if (e.kind != SG_LOCAL_ENTRY) nd.at(qs, qm);
            const uint2 nodes = event_nodes(a, e.idx);
            if (e.kind == SG_LOCAL_ENTRY) {
                cx_entry<false>(a, bndp, nd, e, le.ts_ms, le.origin, ctx, x, qs, qm, nodes, nullptr);
                if (dead_ok && !dead && nd.cs.q == qs && nd.cm.q == qm && cxw_saturated(a, nd)) {
                    dead = true;
                    dqs = qs;
                    dqm = qm;
                    dend = min(nd.cs.next_b, nd.cm.next_b);
                }
            } else {
                cx_exit<false>(a, bndp, nd, e, le.ts_ms, le.create_ts, le.origin, ctx, x, qs, qm, nodes, nullptr);
            }
        }
        if (dead) {
            nd.at(dqs, dqm);
            nd.sc[kLBlock] += dblk;
            nd.mc[kLBlock] += dblk;
            flush_origins();
        }
        nd.finish();
    }
}

// ------------------------------------------------------------------------------ the cx wave walker
//
// One wave per long segment of a cx resource (not a RELATE group): the lanes load 64 events at a time (record,
// event, arguments, origin / context nodes) and every lane runs the same serial step for each event in turn
// (cx_entry / cx_exit with the values broadcast from that event's lane), so the resource's ClusterNode stays in
// registers and an event costs no dependent loads of its own. Once a window period goes "dead" — a QPS rule that
// every entry reaches is saturated (DefaultController: (int)(passQps + 1) > count; a lone WarmUp rule: passQps + 1 >
// its synced warning-zone QPS), and every rule before it is side-effect free — every further entry of the period is
// FLOW-blocked: its only effects are BLOCK counts (ClusterNode, origin node) and its ParamFlowSlot check, which the
// wave decides 64 entries at a time (the rule's token chains of equal values in lane order, ParamFlowChecker
// .passDefaultLocalCheck / passThrottleLocalCheck :127-254); exits stay serial. Prioritized entries, entries with
// acquireCount <= 0, context tracking, shaping controllers other than a lone WarmUp, several ParamFlowRules or
// collection arguments keep the serial step.

// The wave walker's serial step as a called function: its registers (the entry's origin / context nodes, the
// controllers) stay out of the walker's loop, whose dead-period chunks then run without spilling.
__device__ __noinline__ bool cxw_step(const LArgs& a, const uint32_t* const* bndp, LNode& nd, const LEvent& es,
                                      int64_t te, int64_t ce, int og, const sg_slot_ext* xp, uint32_t qs0, uint32_t qm0,
                                      uint2 nn, unsigned char* slots) {
    const int ctx = xp ? (int)xp->context : 0;
    if (es.kind == SG_LOCAL_ENTRY) {
        cx_entry<true>(a, bndp, nd, es, te, og, ctx, xp, qs0, qm0, nn, slots);
        return true;
    }
    nd.at(qs0, qm0);
    cx_exit<true>(a, bndp, nd, es, te, ce, og, ctx, xp, qs0, qm0, nn, slots);
    return false;
}

// Whether resource k's periods can go dead; *prule = its one QPS ParamFlowRule (-1: none).
__device__ bool cxw_dead_able(const LArgs& a, const LRule& R, uint32_t k, int32_t* prule) {
    *prule = -1;
    if (a.track_ctx) return false;
    if (R.fr_n == 0) {
        if (R.flow_grade != 1) return false;
    } else {
        bool any = false;
        for (uint32_t i = 0; i < R.fr_n; ++i) {
            const LFlowRule r = a.frules[R.fr_begin + i];
            if (r.strategy != SG_STRATEGY_DIRECT || r.cluster_mode != SG_CLUSTER_MODE_OFF) return false;
            if (r.behavior == SG_CONTROL_WARM_UP) {
                if (R.fr_n != 1 || r.limit_app != SG_LIMIT_APP_DEFAULT) return false;
            } else if (r.behavior != SG_CONTROL_DEFAULT) {
                return false;
            }
            any = any || (r.grade == 1 && r.limit_app == SG_LIMIT_APP_DEFAULT);
        }
        if (!any) return false;
    }
    if (R.ps && a.has_ps) {
        const uint32_t rb = a.ps.res_begin[k], re = a.ps.res_begin[k + 1];
        if (re - rb > 1) return false;
        if (re == rb + 1) {
            const uint32_t ri = a.ps.res_rules[rb];
            const int32_t cm = a.ps.cmode ? a.ps.cmode[ri] : SG_CLUSTER_MODE_OFF;
            if (a.ps.grade[ri] != 1 || cm != SG_CLUSTER_MODE_OFF || a.ps.cur_idx[ri] < 0) return false;
            *prule = (int32_t)ri;
        }
    }
    return true;
}

// Is the open second-window period saturated for a rule every entry reaches? (nd's windows are at the period.)
__device__ bool cxw_saturated(const LArgs& a, const LNode& nd) {
    const LRule& R = nd.R;
    const double qps = nd.pass_qps();
    if (R.fr_n == 0) return (double)(int32_t)((uint32_t)java_d2i(qps) + 1u) > R.flow_count;
    for (uint32_t i = 0; i < R.fr_n; ++i) {
        const LFlowRule r = a.frules[R.fr_begin + i];
        if (r.grade != 1 || r.limit_app != SG_LIMIT_APP_DEFAULT) continue;
        if (r.behavior == SG_CONTROL_WARM_UP) {
            const LCtl c = a.ctl[R.fr_begin + i];
            if (c.last_filled < nd.m_ws) return false;  // no entry reached it in this second yet: syncToken pending
            const double lim = c.stored >= r.warning_token ? warm_qps(r, c.stored - r.warning_token) : r.count;
            if ((double)(int64_t)((uint64_t)java_d2l(qps) + 1ull) > lim) return true;
        } else if ((double)(int32_t)((uint32_t)java_d2i(qps) + 1u) > r.count) {
            return true;
        }
    }
    return false;
}

__device__ void cx_wave(const LArgs& a, const BatchArgs& sg, const uint32_t* const* bndp, uint32_t k, uint64_t s,
                        uint64_t e_end, void* nd_mem, unsigned char* slots) {
    const int lane = lane_id();
    // SG_DEBUG & 64: counters into sg.dbg_ctr[20..]: segments, wave ticks (sum, max), dead / general chunks, serial
    // entry / exit steps, ticks in dead chunks, in serial steps (s_memrealtime, 100 MHz); [12..14] the param dead
    // loop's phases (decode + prefetch + fix-up, token chains, stores); [17] dead-chunk heads; [18..19], [29..] and
    // [32..127] the segments over 5 ms
    const bool dg = (sg.dbg & 64) && sg.dbg_ctr;
    const uint64_t tw0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t c_dead = 0, c_gen = 0, c_sent = 0, c_sexit = 0, t_dead = 0, t_ser = 0;
    uint64_t ph[3] = {0, 0, 0};
    // the resource's node in the wave's LDS slot: its fields are wave-uniform, and the out-of-line serial step takes it
    // by reference — on the stack every lane kept its own copy in scratch, 64 private copies of one value
    LNode& nd = *::new (nd_mem) LNode(a, bndp, k);
    nd.created = 1;
    int32_t prule = -1;
    const bool dead_ok = !(*a.flags & (kLFlagPrio | kLFlagNonPos)) && cxw_dead_able(a, nd.R, k, &prule);
    prule = __builtin_amdgcn_readfirstlane(prule);
    PRule pr{};  // the ParamFlowRule the dead periods check
    if (prule >= 0) pr = a.ps.p.rules[prule];
    bool inited = false;  // this walker set the rule's initParamMetricsFor flag
    bool dead = false;
    uint32_t dead_qs = 0xFFFFFFFFu, dead_qm = 0xFFFFFFFFu;
    uint32_t dead_end = 0;  // first event index past the dead period (its records are sorted by index)
    int64_t dblk = 0;       // this lane's BLOCK counts of the dead period's entries (the ClusterNode's, at its end)
    // ... per origin node: this lane's {node, sum} of its own entries (4 slots, no cross-lane work per chunk), merged
    // into the wave's table — one slot per lane {node, sum} — when a lane runs out of slots or the period ends; the
    // nodes get the sums when the period ends (before any later period can reuse their bucket slots)
    uint32_t ln[4] = {kNoNode, kNoNode, kNoNode, kNoNode};
    int64_t ls[4] = {0, 0, 0, 0};
    uint32_t ob_node = kNoNode;
    int64_t ob_sum = 0;
    auto table_add = [&](uint32_t node0, int64_t sum) {  // wave-uniform
        const uint64_t hit = __ballot(ob_node == node0);
        if (hit) {
            if (lane == __builtin_ctzll(hit)) ob_sum += sum;
            return false;
        }
        const uint64_t fr = __ballot(ob_node == kNoNode);
        if (!fr) return true;  // full: the caller flushes and retries
        if (lane == __builtin_ctzll(fr)) {
            ob_node = node0;
            ob_sum = sum;
        }
        return false;
    };
    auto lane_add = [&](uint32_t node, int64_t c) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (ln[q] == node) {
                ls[q] += c;
                return true;
            }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (ln[q] == kNoNode) {
                ln[q] = node;
                ls[q] = c;
                return true;
            }
        return false;
    };
    auto flush_origins = [&]() {
        uint64_t used = __ballot(ob_node != kNoNode);
        while (used) {
            const int j = __builtin_ctzll(used);
            used &= used - 1;
            LNode& on = *::new (slots) LNode(a, nd, (uint32_t)bcast32((int)ob_node, j));  // the wave's LDS slot
            on.at(dead_qs, dead_qm);
            const int64_t sum = bcast64(ob_sum, j);
            on.sc[kLBlock] += sum;
            on.mc[kLBlock] += sum;
            on.finish();
        }
        ob_node = kNoNode;
        ob_sum = 0;
    };
    auto merge_lanes = [&]() {  // wave-uniform: every lane's {node, sum} slots into the wave's table
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint64_t todo = __ballot(ln[q] != kNoNode);
            while (todo) {
                const uint32_t node0 = (uint32_t)bcast32((int)ln[q], __builtin_ctzll(todo));
                const bool mine = ln[q] == node0;
                todo &= ~__ballot(mine);
                const int64_t sum = wave_sum(mine ? ls[q] : 0);
                if (table_add(node0, sum)) {
                    flush_origins();
                    table_add(node0, sum);
                }
            }
            ln[q] = kNoNode;
            ls[q] = 0;
        }
    };
    auto end_dead = [&]() {
        nd.at(dead_qs, dead_qm);
        const int64_t b = wave_sum(dblk);
        nd.sc[kLBlock] += b;
        nd.mc[kLBlock] += b;
        dblk = 0;
        merge_lanes();
        flush_origins();
        dead = false;
    };
    // Records are read two chunks ahead and the next chunk's per-event words (time and ParamFlowSlot lookup of an
    // entry, origin / context nodes) one chunk ahead, so a dead chunk waits on one load latency (its slot states).
    // The chunk step runs twice per loop turn with the two register sets swapped: the prefetched values then need
    // no copy at the turn's end (a copy would wait for their loads).
    struct Pf {
        int64_t t;
        uint64_t psl;
        uint2 nodes;
    };
    auto gather = [&](uint64_t j, uint64_t rec) {
        Pf f;
        f.t = 0;
        f.psl = kPsUnknown;
        f.nodes = make_uint2(kNoNode, kNoNode);
        if (j < e_end) {
            const LEvent e = ldecode(a, rec);
            f.nodes = event_nodes(a, e.idx);
            if (prule >= 0 && a.pslot && e.kind == SG_LOCAL_ENTRY) {
                f.t = a.ev[e.idx].ts_ms;
                f.psl = a.pslot[e.idx];
            }
        }
        return f;
    };
    // one chunk at base: rec_c its records (then the records two chunks ahead), rec_n the next chunk's, fc its
    // prefetched words, fn the next chunk's (issued here); false: the segment is done
    uint64_t t_head = 0;  // SG_DEBUG & 64: ticks from a dead chunk's start to its dead-period work
    auto chunk = [&](uint64_t& base, uint64_t& rec_c, uint64_t& rec_n, Pf& fc, Pf& fn) -> bool {
        const uint64_t th0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
        // ---- dead period, no ParamFlowSlot rule: four chunks per step while they hold only the period's entries
        // (count and origin node are all an entry needs; every load of the step issued together)
        if (dead && prule < 0) {
            const uint64_t b0 = base;
            for (;;) {
                uint64_t r[4];
                uint32_t sn[4];  // the entries' origin nodes from the side words (read beside the records)
                r[0] = base + (uint64_t)lane < e_end ? a.rec_sorted[base + lane] : 0;
#pragma unroll
                for (int u = 1; u < 4; ++u) {
                    const uint64_t jj = base + (uint64_t)(u * 64 + lane);
                    r[u] = jj < e_end ? a.rec_sorted[jj] : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint64_t jj = base + (uint64_t)(u * 64 + lane);
                    sn[u] = (a.cxside && jj < e_end) ? a.cxside[jj].node : kNoNode;
                }
                bool ok = true;
                LEvent eu[4];
                uint2 nu[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint64_t jj = base + (uint64_t)(u * 64 + lane);
                    eu[u].kind = -1;
                    eu[u].count = 0;
                    eu[u].idx = 0;
                    if (jj < e_end) {
                        eu[u] = ldecode(a, r[u]);
                        ok = ok && eu[u].kind == SG_LOCAL_ENTRY && eu[u].idx < dead_end;
                    }
                }
                if (__ballot(!ok) || base + 256 > e_end) break;
#pragma unroll
                for (int u = 0; u < 4; ++u) nu[u] = a.cxside ? make_uint2(sn[u], kNoNode) : event_nodes(a, eu[u].idx);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    dblk += eu[u].count;
                    const bool on = nu[u].x != kNoNode;
                    const bool ovf = on && !lane_add(nu[u].x, eu[u].count);
                    if (__ballot(ovf)) {
                        merge_lanes();
                        if (ovf) lane_add(nu[u].x, eu[u].count);
                    }
                }
                base += 256;
                if (dg) c_dead += 4;
            }
            if (base != b0) {
                if (base >= e_end) return false;
                rec_c = a.rec_sorted[min(base + (uint64_t)lane, a.n - 1)];
                rec_n = base + 64 + (uint64_t)lane < e_end ? a.rec_sorted[base + 64 + lane] : 0;
                fc = gather(base + (uint64_t)lane, rec_c);
            }
        }
        // ---- dead period, one QPS ParamFlowRule: chunks of entries decided from their side words (k_lcx_side), the
        // next chunk's slot states read while this one is decided — a slot this chunk writes is then taken from its
        // writer lane — until a chunk holds an exit, an entry past the period or one the lookup left to the serial step
        if (dead && prule >= 0 && a.cxside) {
            const uint64_t b0 = base;
            const uint64_t td0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
            const uint32_t ri = (uint32_t)prule;
            const int64_t dur = pr.duration_sec * 1000;
            const uint64_t* const recs = a.rec_sorted;
            const CxSide* const side = a.cxside;
            PSlot* const tab = a.ps.p.table;
            auto ld_rec = [&](uint64_t c) {
                const uint64_t jj = c + (uint64_t)lane;
                return jj < e_end ? gload(recs + jj) : 0ull;
            };
            auto ld_side = [&](uint64_t c) {
                const uint64_t jj = c + (uint64_t)lane;
                CxSide z;
                z.t = 0;
                z.psl = 0xFFFFFFFCu;  // no check
                z.node = kNoNode;
                if (jj < e_end) z = gload(side + jj);
                return z;
            };
            struct Sv {  // a slot's value and state
                uint64_t value;
                PState st;
            };
            auto ld_state = [&](const CxSide& z) {
                Sv v{0ull, {0, 0, 0u}};
                if (z.psl < 0xFFFFFFFCu) {
                    const PSlot sl = gload(tab + z.psl);
                    v.value = sl.value;
                    v.st.time = sl.time;
                    v.st.tokens = sl.tokens;
                    v.st.flags = sl.flags;
                }
                return v;
            };
            uint64_t r_c = ld_rec(base), r_n = ld_rec(base + 64);
            CxSide s_c = ld_side(base), s_n = ld_side(base + 64);
            Sv v_c = ld_state(s_c);
            uint32_t w_g = 0xFFFFFFFFu;  // the slot this lane (its last request) wrote in the previous chunk
            PState w_st{0, 0, 0u};
            for (;;) {
                const bool act = base + (uint64_t)lane < e_end;
                LEvent e;
                e.kind = SG_LOCAL_ENTRY;
                e.count = 0;
                e.idx = 0;
                if (act) e = ldecode(a, r_c);
                const uint64_t tp0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;  // SG_DEBUG & 64: phase ticks
                const bool okl = !act || (e.kind == SG_LOCAL_ENTRY && e.idx < dead_end && s_c.psl != 0xFFFFFFFFu);
                if (__ballot(!okl)) break;
                // two chunks ahead: records and side words; the next chunk: its slot states
                const uint64_t r_n2 = ld_rec(base + 128);
                const CxSide s_n2 = ld_side(base + 128);
                const Sv v_n = ld_state(s_n);
                // this chunk's states were read before the previous chunk's writes landed
                uint64_t wm = __ballot(w_g != 0xFFFFFFFFu);
                while (wm) {
                    const int q = __builtin_ctzll(wm);
                    wm &= wm - 1;
                    const uint32_t g0 = (uint32_t)bcast32((int)w_g, q);
                    const int64_t tm = bcast64(w_st.time, q), tk = bcast64(w_st.tokens, q);
                    const uint32_t fl = (uint32_t)bcast32((int)w_st.flags, q);
                    if (s_c.psl == g0) {
                        v_c.st.time = tm;
                        v_c.st.tokens = tk;
                        v_c.st.flags = fl;
                    }
                }
                const uint64_t tp1 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
                const uint32_t psl = s_c.psl;
                if (!inited && __ballot(act && psl != 0xFFFFFFFEu)) {  // initParamMetricsFor
                    a.ps.inited[ri] = 1;
                    inited = true;
                }
                const bool has = act && psl != 0xFFFFFFFEu && psl != 0xFFFFFFFCu;
                const bool early = has && psl == 0xFFFFFFFDu;
                const bool chain0 = has && !early;
                const int64_t tc = !chain0 ? 0 : pr.hot_count ? param_token_count(a.ps.p, pr, v_c.value) : pr.token_count;
                PState st = v_c.st;
                const bool stuck = chain0 && pr.behavior != 2 && (st.flags & 3u) == 3u && s_c.t - st.time <= dur &&
                                   st.tokens <= 0;
                const bool chain = chain0 && !stuck;
                int rank = 0, prev = lane;
                uint64_t gm = 0;
                uint64_t todo = __ballot(chain);
                int maxrank = 0;  // the longest chain's last rank
                while (todo) {
                    const int l0 = __builtin_ctzll(todo);
                    const uint32_t g0 = (uint32_t)bcast32((int)psl, l0);
                    const uint64_t m = __ballot(chain && psl == g0);
                    todo &= ~m;
                    maxrank = max(maxrank, (int)__popcll(m) - 1);
                    if (chain && psl == g0) {
                        gm = m;
                        const uint64_t lo = m & below(lane);
                        rank = (int)__popcll(lo);
                        prev = lo ? 63 - __builtin_clzll(lo) : lane;
                    }
                }
                bool ok = !stuck;
                for (int r = 0; r <= maxrank; ++r) {
                    const int64_t ptm = __shfl((long long)st.time, prev, 64);
                    const int64_t ptk = __shfl((long long)st.tokens, prev, 64);
                    const uint32_t pfl = (uint32_t)__shfl((int)st.flags, prev, 64);
                    if (chain && rank == r) {
                        if (r > 0) {
                            st.time = ptm;
                            st.tokens = ptk;
                            st.flags = pfl;
                        }
                        ok = pr.behavior == 2
                                 ? param_throttle_step(st, throttle_cost(pr, tc, e.count), pr.max_queueing_ms, s_c.t)
                                 : param_default_step(st, tc, tc + pr.burst, dur, s_c.t, e.count);
                    }
                }
                const uint64_t tp2 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
                w_g = 0xFFFFFFFFu;
                if (chain && (gm & ~below(lane + 1)) == 0) {  // the slot's last request writes it back
                    PSlot* const sl = tab + psl;
                    gstore(&sl->time, st.time);
                    gstore(&sl->tokens, st.tokens);
                    gstore(&sl->flags, st.flags);
                    w_g = psl;
                    w_st = st;
                }
                if (has && (early || !ok)) lstore(a, e.idx, SG_LOCAL_BLOCK_PARAM, prule);
                // BLOCK counts of the ClusterNode and the origin nodes (added when the period ends)
                if (act) dblk += e.count;
                const bool on = act && s_c.node != kNoNode;
                const bool ovf = on && !lane_add(s_c.node, e.count);
                if (__ballot(ovf)) {
                    merge_lanes();
                    if (ovf) lane_add(s_c.node, e.count);
                }
                if (dg) {
                    ++c_dead;
                    const uint64_t tp3 = __builtin_amdgcn_s_memrealtime();
                    ph[0] += tp1 - tp0;
                    ph[1] += tp2 - tp1;
                    ph[2] += tp3 - tp2;
                }
                base += 64;
                if (base >= e_end) break;
                r_c = r_n;
                r_n = r_n2;
                s_c = s_n;
                s_n = s_n2;
                v_c = v_n;
            }
            if (dg) t_dead += __builtin_amdgcn_s_memrealtime() - td0;
            if (base != b0) {
                if (base >= e_end) return false;
                rec_c = a.rec_sorted[base + (uint64_t)lane < e_end ? base + lane : base];
                rec_n = base + 64 + (uint64_t)lane < e_end ? a.rec_sorted[base + 64 + lane] : 0;
                fc = gather(base + (uint64_t)lane, rec_c);
            }
        }
        const uint64_t j = base + (uint64_t)lane;
        const bool act = j < e_end;
        fn = gather(j + 64, rec_n);
        LEvent ev;
        ev.idx = 0;
        ev.count = 0;
        ev.kind = -1;
        ev.prio = false;
        int64_t t = 0, cr = 0;
        int32_t org = 0;
        sg_slot_ext xx;
        xx.context = 0;
        xx.arg_begin = xx.arg_count = 0;
        xx.args_null = 1;
        uint2 nodes = make_uint2(kNoNode, kNoNode);
        uint32_t qs = 0xFFFFFFFFu, qm = 0xFFFFFFFFu;
        uint64_t psl = kPsUnknown;
        if (act) ev = ldecode(a, rec_c);
        rec_c = j + 128 < e_end ? a.rec_sorted[j + 128] : 0;  // in flight meanwhile
        auto load_full = [&]() {  // the event record, its arguments and (param rule) lookup
            const sg_local_event le = a.ev[ev.idx];
            t = le.ts_ms;
            cr = le.create_ts;
            org = le.origin;
            if (a.ext) xx = a.ext[ev.idx];
            if (a.pslot && prule >= 0 && ev.kind == SG_LOCAL_ENTRY) psl = a.pslot[ev.idx];
        };
        // the serial step of lane q, every lane with lane q's values
        auto step = [&](int q, uint32_t qs0, uint32_t qm0) {
            const uint64_t ts0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
            LEvent es;
            es.idx = (uint32_t)bcast32((int)ev.idx, q);
            es.count = bcast32(ev.count, q);
            es.kind = bcast32(ev.kind, q);
            es.prio = bcast32((int)ev.prio, q) != 0;
            const int64_t te = bcast64(t, q), ce = bcast64(cr, q);
            const int og = bcast32(org, q);
            sg_slot_ext xe;
            xe.context = (uint32_t)bcast32((int)xx.context, q);
            xe.arg_begin = (uint32_t)bcast32((int)xx.arg_begin, q);
            xe.arg_count = (uint32_t)bcast32((int)xx.arg_count, q);
            xe.args_null = bcast32(xx.args_null, q);
            const uint2 nn = make_uint2((uint32_t)bcast32((int)nodes.x, q), (uint32_t)bcast32((int)nodes.y, q));
            const sg_slot_ext* xp = a.ext ? &xe : nullptr;
            const bool entry = cxw_step(a, bndp, nd, es, te, ce, og, xp, qs0, qm0, nn, slots);
            if (dg) {
                if (entry) ++c_sent;
                else ++c_sexit;
                t_ser += __builtin_amdgcn_s_memrealtime() - ts0;
            }
            return entry;
        };
        // Lanes `in` of the dead period: entries FLOW-blocked unless their ParamFlowSlot check fails, exits serial.
        // Returns false (nothing done) when an entry needs the serial step (a collection argument).
        auto dead_lanes = [&](bool in) {
            const bool ent = in && ev.kind == SG_LOCAL_ENTRY;
            bool pfail = false;
            if (prule >= 0) {
                const uint32_t ri = (uint32_t)prule;
                int64_t tc = 0;
                uint64_t g = ~0ull;
                bool has = false, early = false;
                if (a.pslot) {  // k_local_prep looked the entries up
                    if (__ballot(ent && psl == kPsUnknown)) return false;
                    if (!inited && __ballot(ent && psl != kPsNoCheck)) {  // initParamMetricsFor
                        a.ps.inited[ri] = 1;
                        inited = true;
                    }
                    has = ent && psl != kPsNoCheck && psl != kPsNoCheckInit;
                    early = has && psl == kPsEarlyFail;
                    if (has && !early) {
                        g = psl;
                        tc = pr.hot_count ? param_token_count(a.ps.p, pr, a.ps.p.table[g].value) : pr.token_count;
                    }
                } else {
                    const int32_t pidx = a.ps.cur_idx[ri];
                    const bool args = ent && a.ext && !xx.args_null;
                    has = args && (int32_t)xx.arg_count > pidx;
                    sg_pslot_arg ag;
                    ag.kind = SG_ARG_NULL;
                    ag.value_begin = ag.value_count = 0;
                    if (has) {
                        ag = a.ps.args[xx.arg_begin + (uint32_t)pidx];
                        has = ag.kind != SG_ARG_NULL;
                    }
                    if (__ballot(has && ag.kind == SG_ARG_COLLECTION)) return false;
                    if (__ballot(args)) a.ps.inited[ri] = 1;  // initParamMetricsFor (ParamFlowSlot.checkFlow :84)
                    if (has) {
                        const uint64_t v = a.ps.values[ag.value_begin];
                        tc = param_token_count(a.ps.p, pr, v);
                        if (tc == 0 || (pr.behavior != 2 && (int64_t)ev.count > tc + pr.burst)) {
                            early = true;
                        } else {
                            g = param_slot(a.ps.p, pr, v);
                            if (g == ~0ull) {
                                atomicOr(a.ps.err, kErrTableFull);
                                early = true;
                            }
                        }
                    }
                }
                // every request reads its slot; one the state already refuses — a token bucket within its
                // duration with no token left — leaves the slot as it is, and so does every earlier request of the
                // slot in the chunk (times non-decreasing, acquireCount >= 1): only the requests after them chain
                const bool chain0 = has && !early;
                PState st{0, 0, 0u};
                if (chain0) {
                    const PSlot& sl = a.ps.p.table[g];
                    st.time = sl.time;
                    st.tokens = sl.tokens;
                    st.flags = sl.flags;
                }
                const bool stuck = chain0 && pr.behavior != 2 && (st.flags & 3u) == 3u &&
                                   t - st.time <= pr.duration_sec * 1000 && st.tokens <= 0;
                // token chains: the lanes of one (rule, value) slot in lane (event) order
                const bool chain = chain0 && !stuck;
                int rank = 0, prev = lane;
                uint64_t gm = 0;
                uint64_t todo = __ballot(chain);
                int maxrank = 0;  // the longest chain's last rank
                while (todo) {
                    const int l0 = __builtin_ctzll(todo);
                    const uint64_t g0 = (uint64_t)bcast64((int64_t)g, l0);
                    const uint64_t m = __ballot(chain && g == g0);
                    todo &= ~m;
                    maxrank = max(maxrank, (int)__popcll(m) - 1);
                    if (chain && g == g0) {
                        gm = m;
                        const uint64_t lo = m & below(lane);
                        rank = (int)__popcll(lo);
                        prev = lo ? 63 - __builtin_clzll(lo) : lane;
                    }
                }
                bool ok = !stuck;
                for (int r = 0; r <= maxrank; ++r) {
                    const int64_t ptm = __shfl((long long)st.time, prev, 64);
                    const int64_t ptk = __shfl((long long)st.tokens, prev, 64);
                    const uint32_t pfl = (uint32_t)__shfl((int)st.flags, prev, 64);
                    if (chain && rank == r) {
                        if (r > 0) {
                            st.time = ptm;
                            st.tokens = ptk;
                            st.flags = pfl;
                        }
                        ok = pr.behavior == 2
                                 ? param_throttle_step(st, throttle_cost(pr, tc, ev.count), pr.max_queueing_ms, t)
                                 : param_default_step(st, tc, tc + pr.burst, pr.duration_sec * 1000, t, ev.count);
                    }
                }
                if (chain && (gm & ~below(lane + 1)) == 0) {  // the slot's last request writes it back
                    PSlot& sl = a.ps.p.table[g];
                    sl.time = st.time;
                    sl.tokens = st.tokens;
                    sl.flags = st.flags;
                }
                pfail = has && (early || !ok);
            }
            if (pfail) lstore(a, ev.idx, SG_LOCAL_BLOCK_PARAM, prule);  // ParamFlowException (FLOW: the default)
            // increaseBlockQps of the ClusterNode and the origin nodes, both windows (added when the period ends)
            if (ent) dblk += ev.count;
            const bool on = ent && nodes.x != kNoNode;
            const bool ovf = on && !lane_add(nodes.x, ev.count);
            if (__ballot(ovf)) {
                merge_lanes();
                if (ovf) lane_add(nodes.x, ev.count);
            }
            // exits, in order (they change no pass count: the period stays dead)
            uint64_t ex = __ballot(in && ev.kind != SG_LOCAL_ENTRY);
            while (ex) {
                const int q = __builtin_ctzll(ex);
                ex &= ex - 1;
                step(q, dead_qs, dead_qm);
            }
            return true;
        };
        // ---- a chunk wholly inside the dead period: its entries need only count, node, time and param lookup
        if (dead && (prule < 0 || a.pslot != nullptr)) {
            const bool in = act && ev.idx < dead_end;
            if (__ballot(act && !in) == 0) {
                const uint64_t td0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
                if (dg) t_head += td0 - th0;
                if (act) {
                    if (ev.kind != SG_LOCAL_ENTRY) {
                        load_full();
                    } else {
                        t = fc.t;
                        psl = fc.psl;
                    }
                    nodes = fc.nodes;
                }
                if (dead_lanes(in)) {
                    if (dg) {
                        ++c_dead;
                        t_dead += __builtin_amdgcn_s_memrealtime() - td0;
                    }
                    base += 64;
                    return base < e_end;
                }
                // a collection argument: the general path below (its serial steps)
                if (act && ev.kind == SG_LOCAL_ENTRY) load_full();
            }
        }
        // ---- the general path: runs of equal window periods, serial until dead
        if (dg) ++c_gen;
        if (act) {
            if (ev.kind != SG_LOCAL_ENTRY || !(dead && ev.idx < dead_end) || psl == kPsUnknown) load_full();
            nodes = fc.nodes;
            qs = nd.cs.of(ev.idx);
            qm = nd.cm.of(ev.idx);
        }
        const int nact = (int)__popcll(__ballot(act));
        int p = 0;
        while (p < nact) {
            // run: lanes [p, rend) in the window periods of lane p
            const uint32_t qs0 = (uint32_t)bcast32((int)qs, p), qm0 = (uint32_t)bcast32((int)qm, p);
            const uint64_t diff = __ballot(act && lane > p && (qs != qs0 || qm != qm0));
            const int rend = diff ? __builtin_ctzll(diff) : nact;
            if (dead && (qs0 != dead_qs || qm0 != dead_qm)) end_dead();  // the dead period ended
            while (p < rend && !dead) {
                const bool entry = step(p, qs0, qm0);
                ++p;
                if (entry && dead_ok && nd.cs.q == qs0 && nd.cm.q == qm0 && cxw_saturated(a, nd)) {
                    dead = true;
                    dead_qs = qs0;
                    dead_qm = qm0;
                    dead_end = min(nd.cs.next_b, nd.cm.next_b);
                }
            }
            if (p >= rend) continue;
            const bool in = act && lane >= p && lane < rend;
            if (!dead_lanes(in)) {
                while (p < rend) step(p++, qs0, qm0);
                continue;
            }
            p = rend;
        }
        base += 64;
        return base < e_end;
    };
    uint64_t ra = s + (uint64_t)lane < e_end ? a.rec_sorted[s + lane] : 0;
    uint64_t rb = s + 64 + (uint64_t)lane < e_end ? a.rec_sorted[s + 64 + lane] : 0;
    Pf fa = gather(s + (uint64_t)lane, ra), fb;
    for (uint64_t base = s; chunk(base, ra, rb, fa, fb) && chunk(base, rb, ra, fb, fa);) {
    }
    if (dead) end_dead();
    nd.finish();
    if (dg && lane == 0) {
        const uint64_t tw = __builtin_amdgcn_s_memrealtime() - tw0;
        atomicAdd(&sg.dbg_ctr[20], 1ull);
        atomicAdd(&sg.dbg_ctr[21], (unsigned long long)tw);
        atomicMax(&sg.dbg_ctr[22], (unsigned long long)tw);
        atomicAdd(&sg.dbg_ctr[23], (unsigned long long)c_dead);
        atomicAdd(&sg.dbg_ctr[24], (unsigned long long)c_gen);
        atomicAdd(&sg.dbg_ctr[25], (unsigned long long)c_sent);
        atomicAdd(&sg.dbg_ctr[26], (unsigned long long)c_sexit);
        atomicAdd(&sg.dbg_ctr[27], (unsigned long long)t_dead);
        atomicAdd(&sg.dbg_ctr[28], (unsigned long long)t_ser);
        atomicAdd(&sg.dbg_ctr[17], (unsigned long long)t_head);
        atomicAdd(&sg.dbg_ctr[12], (unsigned long long)ph[0]);
        atomicAdd(&sg.dbg_ctr[13], (unsigned long long)ph[1]);
        atomicAdd(&sg.dbg_ctr[14], (unsigned long long)ph[2]);
        if (tw > 500000ull) {  // segments over 5 ms: their serial steps, serial ticks, dead chunks
            atomicAdd(&sg.dbg_ctr[29], (unsigned long long)(c_sent + c_sexit));
            atomicAdd(&sg.dbg_ctr[30], (unsigned long long)t_ser);
            atomicAdd(&sg.dbg_ctr[31], (unsigned long long)c_dead);
            atomicAdd(&sg.dbg_ctr[19], 1ull);
            const unsigned long long sl = atomicAdd(&sg.dbg_ctr[18], 1ull);
            if (sl < 12) {  // [32 + 8 * sl]: resource, records, wave ticks, dead ticks, dead chunks, serial steps /
                            // ticks, param rule
                unsigned long long* o = sg.dbg_ctr + 32 + 8 * sl;
                o[0] = k;
                o[1] = e_end - s;
                o[2] = tw;
                o[3] = t_dead;
                o[4] = c_dead;
                o[5] = c_sent + c_sexit;
                o[6] = t_ser;
                o[7] = (unsigned long long)(int64_t)prule;
            }
        }
    }
}

// The cx walkers' dead-period words of every sorted record of a cx resource (CxSide), so that a dead chunk reads them
// contiguously rather than through a gather per word and entry.
__global__ void __launch_bounds__(256) k_lcx_side(LArgs a) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.n; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = a.rec_sorted[p];
        const uint32_t k = (uint32_t)(r >> a.kshift);
        if (k >= a.K || !(a.rules[k].cx || (a.dyn && a.dyn[k] == a.epoch))) continue;
        const LEvent e = ldecode(a, r);
        CxSide z;
        z.t = a.ev[e.idx].ts_ms;
        const uint64_t ps = (a.pslot && e.kind == SG_LOCAL_ENTRY) ? a.pslot[e.idx] : kPsUnknown;
        z.psl = (ps >= kPsNoCheckInit || ps < 0xFFFFFFFCull) ? (uint32_t)ps : 0xFFFFFFFFu;  // a slot that looks like a code
        z.node = event_nodes(a, e.idx).x;
        a.cxside[p] = z;
    }
}

__global__ void __launch_bounds__(256, SG_LWALK_BLOCKS) k_lwalk_cxw(LArgs a_arg, BatchArgs sg) {
    __shared__ uint32_t sbnd[kLdsBnd];
    __shared__ const uint32_t* bndp[kMaxWl];
    __shared__ LArgs a_lds;  // as k_lwalk_cx
    __shared__ alignas(16) unsigned char cxw_nd[4][kCxNdBytes];         // each wave's resource node (cx_wave)
    __shared__ alignas(16) unsigned char cxw_slots[4][3 * kCxNdBytes];  // and its event's origin / context nodes
    (void)a_arg;
    stage_largs(&a_lds);
    const LArgs& a = a_lds;
    if (*a.err) return;
    stage_lperiods(a, sbnd, bndp);
    const int lane = lane_id();
    const uint32_t n_long = *sg.long_count;
    uint32_t total = n_long;  // the long list, then the short classes >= cxw_cls (longest first)
    for (int c = a.cxw_cls; c < kClasses; ++c) total += sg.short_count[c];
    // a wave takes the next item when it is free: the waves that start on the longest segments take no more
    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(a.cxw_next, 1u);
        item = (uint32_t)__builtin_amdgcn_readfirstlane((int)item);
        if (item >= total) break;
        uint64_t s, lo;
        if (item < n_long) {
            s = sg.long_list[item];
            lo = sg.short_max ? sg.short_max : 1;
        } else {
            uint32_t r = item - n_long;
            int c = kClasses - 1;
            while (r >= sg.short_count[c]) r -= sg.short_count[c--];
            s = sg.short_list[sg.class_off[c] + r];
            lo = c == 0 ? 1 : kClassMax[c - 1];
        }
        const uint32_t k = (uint32_t)(a.rec_sorted[s] >> a.kshift);
        const LRule& R = a.rules[k];
        if (!(R.cx || (a.dyn && a.dyn[k] == a.epoch)) || R.grp) continue;  // k_lwalk_long / k_lwalk_short / k_lwalk_cx
        const uint64_t e = gallop_search(s + lo, a.n, [&](uint64_t p) {
            return (uint32_t)(a.rec_sorted[p] >> a.kshift) != k;
        }, lane);
        cx_wave(a, sg, bndp, k, s, e, cxw_nd[threadIdx.x >> 6], cxw_slots[threadIdx.x >> 6]);
    }
}

// Sorted positions of the exit records, in ascending order: per-tile counts, a one-block exclusive scan,
// then each tile writes its positions in order (the dead-period skip stops at the next exit).
__global__ void __launch_bounds__(256) k_lexit_count(LArgs a) {
    __shared__ uint32_t wc[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kLTile;
    uint32_t c = 0;
    for (uint64_t j = t0 + threadIdx.x; j < min(a.n, t0 + kLTile); j += blockDim.x) {
        const uint64_t r = a.rec_sorted[j];
        c += ((uint32_t)(r >> a.kshift) < a.K && ((r & a.amask) >> 1 & 3ull) != 0) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
    if (lane_id() == 0) wc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) a.exit_cnt[1 + blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ void __launch_bounds__(1024) k_lexit_scan(LArgs a, uint32_t tiles) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < tiles; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < tiles ? a.exit_cnt[1 + i] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint32_t x = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += x;
            __syncthreads();
        }
        const uint32_t c = carry;
        if (i < tiles) a.exit_cnt[1 + i] = c + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = c + part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.exit_cnt[0] = carry;
}

__global__ void __launch_bounds__(256) k_lexit_write(LArgs a) {
    __shared__ uint32_t wc[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kLTile;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    uint32_t off = a.exit_cnt[1 + blockIdx.x];
    for (uint64_t r0 = t0; r0 < min(a.n, t0 + kLTile); r0 += blockDim.x) {
        const uint64_t j = r0 + threadIdx.x;
        bool x = false;
        if (j < a.n) {
            const uint64_t r = a.rec_sorted[j];
            x = (uint32_t)(r >> a.kshift) < a.K && ((r & a.amask) >> 1 & 3ull) != 0;
        }
        const uint64_t m = __ballot(x);
        if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t pre = off;
        for (int w = 0; w < wave; ++w) pre += wc[w];
        if (x) a.exit_pos[pre + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)j;
        off += wc[0] + wc[1] + wc[2] + wc[3];
        __syncthreads();
    }
}

// BLOCK counts of the skipped entries (one wave per piece; their FlowException results are k_local_prep's
// default), added to the second- and minute-window buckets of their periods unless a later period of the
// batch reset that slot.
constexpr int kLSkipU = 8;
__global__ void __launch_bounds__(256) k_lskip_apply(LArgs a) {
    if (*a.err) return;
    const uint32_t cnt = min(*a.skip_count, a.skip_cap);
    const int lane = lane_id();
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    for (uint32_t i = wave; i < cnt; i += nwaves) {
        const LSkip sk = a.skips[i];
        int64_t sum = 0;
        // kLSkipU rows of 64 records loaded together (one row per round trip left the wave latency-bound)
        for (uint64_t j0 = (uint64_t)sk.b0; j0 < sk.b1; j0 += 64ull * kLSkipU) {
            uint64_t r[kLSkipU];
#pragma unroll
            for (int u = 0; u < kLSkipU; ++u) {
                const uint64_t j = j0 + (uint64_t)u * 64 + lane;
                r[u] = j < sk.b1 ? a.rec_sorted[j] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < kLSkipU; ++u)
                if (j0 + (uint64_t)u * 64 + lane < sk.b1) sum += ldecode(a, r[u]).count;
        }
        sum = wave_sum(sum);
        if (lane == 0) {
            const int64_t Ps = a.p0[a.wsec] + (int64_t)sk.qs, Pm = a.p0[a.wmin] + (int64_t)sk.qm;
            LBucket& bs = a.sec[(size_t)sk.k * a.S + (int)(Ps % a.S)];
            if (bs.start == Ps * a.wl2) atomicAdd((unsigned long long*)&bs.c[kLBlock], (unsigned long long)sum);
            LBucket& bm = a.minute[(size_t)sk.k * kMinuteS + (int)(Pm % kMinuteS)];
            if (bm.start == Pm * kMinuteWl) atomicAdd((unsigned long long*)&bm.c[kLBlock], (unsigned long long)sum);
        }
    }
}

// The pipelined batch's first timestamp against the previous batch's last (k_local_prep ran before that batch ended).
__global__ void k_local_check_last(LArgs a) {
    if (a.n > 0 && a.ev[0].ts_ms < *a.last_ts) atomicOr(a.err, kErrTime);
}

__global__ void k_local_finish(LArgs a) {
    if (*a.err == 0 && a.n > 0) {
        *a.last_ts = a.ev[a.n - 1].ts_ms;
        if (a.c3_last_ts) *a.c3_last_ts = a.ev[a.n - 1].ts_ms;  // the embedded server's token requests came up to here
        if (a.has_ps && a.ps.emb) *a.ps.cp_last_ts = a.ev[a.n - 1].ts_ms;
    }
}

// ------------------------------------------------------------------------------- metric rows

// StatisticNode.metrics() at now (StatisticNode.java:116-147, ArrayMetric.details / fromBucket :156-204), one
// thread per resource over its 60 minute buckets. An inbound resource's buckets newer than the ENTRY_NODE's
// lastFetchTime are also summed into a.entry_acc: StatisticSlot adds every EntryType.IN entry and exit to
// Constants.ENTRY_NODE as to the resource (StatisticSlot.java:71-75, :139-141), so the ENTRY_NODE's bucket of a
// second is the sum of the inbound resources' buckets of that second (k_local_entry_rows emits its rows).
__device__ __forceinline__ bool metric_row_valid(const LBucket& b) {  // MetricNode validity (isValidMetricNode)
    const int64_t succ = b.c[kLSucc];
    const int64_t rt = succ != 0 ? b.c[kLRt] / succ : b.c[kLRt];
    return b.c[kLPass] > 0 || b.c[kLBlock] > 0 || succ > 0 || b.c[kLExc] > 0 || rt > 0 || b.c[kLOccPass] > 0;
}

__global__ void __launch_bounds__(256) k_local_metrics(LArgs a, int64_t now, sg_metric_node* out,
                                                       unsigned long long* count, int emit, int raw, const int* gate) {
    if (gate && !*gate) return;  // sg_local_metrics_raw_enqueue: more rows than the caller's capacity, no side effect
    // the ENTRY_NODE sums of this block's inbound resources, per minute slot, in LDS (one global atomic per slot and
    // event per block instead of one per resource); rows placed with one counter atomic per wave
    __shared__ unsigned long long eacc[kMinuteS][kLEv];
    __shared__ int64_t estart[kMinuteS];
    for (int i = threadIdx.x; i < kMinuteS * kLEv; i += blockDim.x) (&eacc[0][0])[i] = 0ull;
    for (int i = threadIdx.x; i < kMinuteS; i += blockDim.x) estart[i] = INT64_MIN;
    __syncthreads();
    const int64_t cur = now - now % 1000;
    const int I = (int)((now / kMinuteWl) % kMinuteS);
    const int64_t efetch = a.entry_fetch ? *a.entry_fetch : INT64_MAX;
    const int lane = threadIdx.x & 63;
    for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < a.K; k0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = k0 + threadIdx.x;
        const bool act = k < a.K;
        LBucket* m = a.minute + (act ? k : 0) * kMinuteS;
        bool reset_I = false;
        int64_t last = 0, s_lo = 0, newest = 0;
        uint32_t rows = 0;
        if (act) {
            // data.currentWindow(now): an absent or stale bucket in now's slot becomes an empty one (emit: for real;
            // counting: as if, so that both passes list the same buckets)
            reset_I = m[I].start == INT64_MIN || m[I].start < cur;
            if (emit && reset_I) {
                LBucket b;
                b.start = cur;
                for (int e = 0; e < kLEv; ++e) b.c[e] = 0;
                b.min_rt = kStatMaxRt;
                m[I] = b;
            }
            const bool inb = a.inbound && a.inbound[k];
            last = a.last_fetch[k];
            newest = last;
            // Only buckets that start after the earlier of the two fetch times (the resource's, and the ENTRY_NODE's
            // for an inbound resource), before cur and inside the minute can yield a row or an ENTRY_NODE sum: their
            // seconds s in [cur - 59 s, cur) past that fetch time, slot (s / 1000) mod 60 — one bucket per resource
            // when the listener fetches every second, instead of all 60 (a bucket whose start is some other second
            // fails the checks below, as in the full scan).
            const int64_t lo_f = (inb && efetch < last) ? efetch : last;
            s_lo = cur - (int64_t)(kMinuteS - 1) * kMinuteWl;
            if (lo_f >= s_lo) s_lo = (lo_f >= 0 ? lo_f / kMinuteWl : -((-lo_f + kMinuteWl - 1) / kMinuteWl)) * kMinuteWl + kMinuteWl;
            if (s_lo < 0) s_lo = 0;
            for (int64_t s = s_lo; s < cur; s += kMinuteWl) {  // data.list(now): present and not deprecated
                const int j = (int)((s / kMinuteWl) % kMinuteS);
                if (j == I && reset_I) continue;  // the fresh bucket at cur is never in time
                const LBucket b = m[j];
                if (b.start == INT64_MIN || now - b.start > (int64_t)kMinuteS * kMinuteWl) continue;
                if (inb && b.start > efetch && b.start < cur) {  // the ENTRY_NODE's bucket of that second
                    estart[j] = b.start;  // every inbound bucket of slot j in the window has this start
                    for (int e = 0; e < kLEv; ++e)
                        if (b.c[e]) atomicAdd(&eacc[j][e], (unsigned long long)b.c[e]);
                }
                if (!(b.start > last && b.start < cur)) continue;  // isNodeInTime
                if (!metric_row_valid(b)) continue;
                newest = b.start > newest ? b.start : newest;
                ++rows;
            }
        }
        // the wave's rows: one counter atomic, each lane's rows after its lower lanes'
        uint32_t incl = rows;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, (unsigned)o, 64);
            if (lane >= o) incl += y;
        }
        const uint32_t wtot = (uint32_t)__shfl((int)incl, 63, 64);
        unsigned long long base = 0;
        if (lane == 0 && wtot) base = atomicAdd(count, (unsigned long long)wtot);
        base = (unsigned long long)__shfl((long long)base, 0, 64);
        if (!emit || !act) continue;
        unsigned long long pos = base + incl - rows;
        for (int64_t s = s_lo; rows && s < cur; s += kMinuteWl) {  // the same buckets again, now written out
            const int j = (int)((s / kMinuteWl) % kMinuteS);
            if (j == I && reset_I) continue;
            const LBucket b = m[j];
            if (b.start == INT64_MIN || now - b.start > (int64_t)kMinuteS * kMinuteWl) continue;
            if (!(b.start > last && b.start < cur) || !metric_row_valid(b)) continue;
            const int64_t pass = b.c[kLPass], block = b.c[kLBlock], succ = b.c[kLSucc], exc = b.c[kLExc];
            sg_metric_node r;
            r.timestamp = b.start;
            r.pass_qps = pass;
            r.block_qps = block;
            r.success_qps = succ;
            r.exception_qps = exc;
            r.rt = (succ != 0 && !raw) ? b.c[kLRt] / succ : b.c[kLRt];
            r.occupied_pass_qps = b.c[kLOccPass];
            r.resource = (uint32_t)k;
            r.concurrency = 0;
            out[pos++] = r;
        }
        a.last_fetch[k] = newest;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kMinuteS * kLEv; i += blockDim.x) {
        const unsigned long long v = (&eacc[0][0])[i];
        if (v) atomicAdd((unsigned long long*)&a.entry_acc[i / kLEv].c[i % kLEv], v);
    }
    for (int i = threadIdx.x; i < kMinuteS; i += blockDim.x)
        if (estart[i] != INT64_MIN) a.entry_acc[i].start = estart[i];
}

// Constants.ENTRY_NODE.metrics() rows from the summed buckets (one thread per minute slot; resource id
// SG_ENTRY_NODE_RESOURCE); emit advances the ENTRY_NODE's lastFetchTime.
__global__ void __launch_bounds__(64) k_local_entry_rows(LArgs a, int64_t now, sg_metric_node* out,
                                                         unsigned long long* count, int emit, int raw, const int* gate) {
    if (gate && !*gate) return;
    const int j = threadIdx.x;
    const int64_t cur = now - now % 1000;
    bool row = false;
    LBucket b;
    if (j < kMinuteS) {
        b = a.entry_acc[j];
        // StatisticNode.addOccupiedPass raises the minute PASS and OCCUPIED_PASS of the selected node only: the
        // ENTRY_NODE sees StatisticSlot's addPassRequest of real passes, never a prioritized wait's occupied pass
        b.c[kLPass] -= b.c[kLOccPass];
        b.c[kLOccPass] = 0;
        row = b.start != INT64_MIN && b.start > *a.entry_fetch && b.start < cur && metric_row_valid(b);
    }
    if (row) {
        if (emit) {
            const int64_t succ = b.c[kLSucc];
            sg_metric_node r;
            r.timestamp = b.start;
            r.pass_qps = b.c[kLPass];
            r.block_qps = b.c[kLBlock];
            r.success_qps = succ;
            r.exception_qps = b.c[kLExc];
            r.rt = (succ != 0 && !raw) ? b.c[kLRt] / succ : b.c[kLRt];
            r.occupied_pass_qps = 0;
            r.resource = SG_ENTRY_NODE_RESOURCE;
            r.concurrency = 0;
            out[atomicAdd(count, 1ull)] = r;
        } else {
            atomicAdd(count, 1ull);
        }
    }
    // newest row start → lastFetchTime (wave max; one wave)
    int64_t nb = row ? b.start : INT64_MIN;
    for (int o = 32; o > 0; o >>= 1) nb = max(nb, (int64_t)__shfl_xor((long long)nb, o, 64));
    if (emit && j == 0 && nb != INT64_MIN && nb > *a.entry_fetch) *a.entry_fetch = nb;
}

// ---------------------------------------------------------------------------------- launchers

static unsigned lgrid(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

static unsigned lresident(const void* kernel) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0);
    return (unsigned)((cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1));
}

hipError_t launch_local_prep(const LArgs& a, hipStream_t stream) {
    lds_poison(stream);
    hipLaunchKernelGGL(k_local_prep, dim3((unsigned)((a.n + 256 * kLPrepItems - 1) / (256 * kLPrepItems))), dim3(256), 0,
                       stream, a);
    return hipGetLastError();
}

hipError_t launch_local_metrics(const LArgs& a, int64_t now, sg_metric_node* out, unsigned long long* count, int emit,
                                int raw, hipStream_t stream, const int* gate) {
    if (a.K == 0) return hipSuccess;
    lds_poison(stream);
    hipLaunchKernelGGL(k_local_metrics, dim3(lgrid(a.K, 256, 4096)), dim3(256), 0, stream, a, now, out, count, emit, raw,
                       gate);
    return hipGetLastError();
}

// The count pass's rows against the caller's capacity: the count for the caller, and whether the emit pass runs.
__global__ void k_metrics_gate(const unsigned long long* cnt, uint64_t cap, unsigned long long* count_out, int* gate) {
    const unsigned long long c = *cnt;
    *count_out = c;
    *gate = c <= cap ? 1 : 0;
}

hipError_t launch_metrics_gate(const unsigned long long* cnt, uint64_t cap, unsigned long long* count_out, int* gate,
                               hipStream_t stream) {
    hipLaunchKernelGGL(k_metrics_gate, dim3(1), dim3(1), 0, stream, cnt, cap, count_out, gate);
    return hipGetLastError();
}

__global__ void k_entry_acc_reset(LBucket* acc) {  // the ENTRY_NODE's summed buckets, empty before a metric pass
    const int j = threadIdx.x;
    if (j >= kMinuteS) return;
    LBucket b;
    b.start = INT64_MIN;
    for (int e = 0; e < kLEv; ++e) b.c[e] = 0;
    b.min_rt = kStatMaxRt;
    acc[j] = b;
}

hipError_t launch_entry_acc_reset(LBucket* acc, hipStream_t stream) {
    hipLaunchKernelGGL(k_entry_acc_reset, dim3(1), dim3(64), 0, stream, acc);
    return hipGetLastError();
}

hipError_t launch_local_entry_rows(const LArgs& a, int64_t now, sg_metric_node* out, unsigned long long* count, int emit,
                                   int raw, hipStream_t stream, const int* gate) {
    hipLaunchKernelGGL(k_local_entry_rows, dim3(1), dim3(64), 0, stream, a, now, out, count, emit, raw, gate);
    return hipGetLastError();
}

hipError_t launch_local_init(const LArgs& a, hipStream_t stream) { return launch_local_init_range(a, 0, a.K, stream); }

hipError_t launch_local_init_range(const LArgs& a, uint64_t lo, uint64_t hi, hipStream_t stream) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_local_init, dim3(lgrid((hi - lo) * kMinuteS, 256, 8192)), dim3(256), 0, stream, a, lo, hi);
    return hipGetLastError();
}

hipError_t launch_lnode_assign(const LArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_lnode_assign, dim3(lgrid(a.n, 256, 8192)), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(k_lnode_resolve, dim3(lgrid(a.n, 256, 8192)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_lnode_find(const uint64_t* keys, const uint32_t* vals, uint64_t mask, uint64_t key, uint32_t* out,
                             hipStream_t stream) {
    hipLaunchKernelGGL(k_lnode_find, dim3(1), dim3(1), 0, stream, keys, vals, mask, key, out);
    return hipGetLastError();
}

hipError_t launch_local_exits(const LArgs& a, hipStream_t stream, bool counted) {
    const uint32_t tiles = (uint32_t)((a.n + kLTile - 1) / kLTile);
    lds_poison(stream);
    if (!counted) hipLaunchKernelGGL(k_lexit_count, dim3(tiles), dim3(256), 0, stream, a);
    lds_poison(stream);
    hipLaunchKernelGGL(k_lexit_scan, dim3(1), dim3(1024), 0, stream, a, tiles);
    lds_poison(stream);
    hipLaunchKernelGGL(k_lexit_write, dim3(tiles), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_local_back(const LArgs& a, const BatchArgs& sg, bool has_cx, hipStream_t aux, hipStream_t stream,
                             hipEvent_t fork, hipEvent_t join) {
    static unsigned bl = 0, bs = 0;
    if (bl == 0) bl = lresident((const void*)k_lwalk_long);
    if (bs == 0) bs = lresident((const void*)k_lwalk_short);
    if (a.defer_last) hipLaunchKernelGGL(k_local_check_last, dim3(1), dim3(1), 0, stream, a);
    // the side words are read by both cx walkers (the lane walker on `aux` in its dead periods): they are
    // written before the fork, so `aux` is ordered after them
    if (has_cx && a.cxw && a.cxside) {
        // test aid (env SG_TEST_CXSIDE_POISON=1): the side words start as garbage, so a walker that read them before
        // k_lcx_side wrote them would fail every time (the lane walker's fork comes after k_lcx_side)
        if (const char* p = std::getenv("SG_TEST_CXSIDE_POISON"))
            if (std::atoi(p)) (void)hipMemsetAsync(a.cxside, 0xFF, sizeof(CxSide) * a.n, stream);
        hipLaunchKernelGGL(k_lcx_side, dim3(lgrid(a.n, 256, 8192)), dim3(256), 0, stream, a);
    }
    hipError_t e = hipEventRecord(fork, stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    if (e != hipSuccess) return e;
    // the hot cx segments' waves first (the batch's longest serial chains), the lane walker of the other cx
    // segments beside them after the plain wave walker
    if (has_cx && a.cxw) {
        static unsigned bw = 0;
        if (bw == 0) bw = lresident((const void*)k_lwalk_cxw);
        e = hipMemsetAsync(a.cxw_next, 0, sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_lwalk_cxw, dim3(bw), dim3(256), 0, stream, a, sg);
    }
    hipLaunchKernelGGL(k_lwalk_long, dim3(bl), dim3(256), 0, aux, a, sg);
    if (has_cx) {
        if (a.cx_list) {
            e = hipMemsetAsync(a.cx_count, 0, sizeof(uint32_t), aux);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k_lcx_list, dim3(lgrid(a.n, 256, 4096)), dim3(256), 0, aux, a, sg);
        }
        static const bool lds_ok = hipFuncSetAttribute((const void*)k_lwalk_cx, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)kCxLdsBytes) == hipSuccess;
        if (!lds_ok) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_lwalk_cx, dim3(bs), dim3(256), kCxLdsBytes, aux, a, sg);
    }
    hipLaunchKernelGGL(k_lwalk_short, dim3(bs), dim3(256), 0, stream, a, sg);
    e = hipEventRecord(join, aux);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, join, 0);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lskip_apply, dim3(1024), dim3(256), 0, stream, a);
    hipLaunchKernelGGL(k_local_finish, dim3(1), dim3(1), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_local_walk(const LArgs& a, const BatchArgs& sg, bool has_cx, hipStream_t aux, hipStream_t stream,
                             hipEvent_t fork, hipEvent_t join) {
    const hipError_t e = launch_local_exits(a, stream, false);
    if (e != hipSuccess) return e;
    return launch_local_back(a, sg, has_cx, aux, stream, fork, join);
}

}  // namespace sg
