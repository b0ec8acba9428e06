// limiter.hip — the namespace QPS limiter pre-pass (GlobalRequestLimiter / RequestLimiter).
//
// ClusterFlowChecker.acquireClusterToken first calls allowProceed → GlobalRequestLimiter.tryPass(ns)
// (srv/flow/ClusterFlowChecker.java:50-53, srv/flow/statistic/limit/GlobalRequestLimiter.java:46-55):
// RequestLimiter.tryPass (srv/flow/statistic/limit/RequestLimiter.java:72-87) admits a request iff
// Σ UnaryLeapArray(10, 1000) + 1 <= qpsAllowed and then adds 1. The check depends on nothing but the
// namespace's arrival sequence, so it runs before the per-flowId partition:
//   within one 100 ms limiter period q the window is base_q + (passes so far in q), hence the passes of
//   period q are exactly the first pass_q arrivals, pass_q = min(arrivals_q, cap(base_q)), and base_q
//   only depends on earlier periods' passes. A request of namespace slot l in period q is admitted iff
//   its rank among l's arrivals in q is < pass_q; rank = C_l(i) − Σ_{p<q} arrivals[l][p] where C_l(i)
//   counts l's requests before index i.
//   k_lim_count  per tile: each valid request's limiter slot, per-slot tile totals, per-(slot, period)
//                arrivals (LDS-aggregated over the few periods a tile spans, then global atomics)
//   k_lim_plan   one block: exclusive scan of the tile totals per slot; per slot, the sequential walk over
//                the batch's limiter periods with the 10-bucket ring (quota, period prefix, ring update)
//   k_lim_apply  per tile: C_l(i) by an in-tile ranked count; over-quota requests → TOO_MANY_REQUEST and
//                their record becomes the sentinel so the flow walkers never see them.
//
// Sharded: each GPU holds a share of the flowIds, but one namespace window for the node. The node's
// arrival order is (ts, shard rank, position in the shard's batch); every shard counts its arrivals per
// (slot, millisecond) (k_limx_arrivals), the node all-gathers those counts, and every shard walks the same global
// per-period arrivals (so its replica of the window stays equal to the others') and gives its request i of
// millisecond m the global rank  Σ_{m' < m in i's period} all + Σ_{r < rank} arrivals_r(m) + (C_l(i) − C_l(m)).
#include "engine.h"

namespace sg {

constexpr int kLimThreads = 256;
constexpr int kLimTile = 4096;
constexpr int kLimRounds = kLimTile / kLimThreads;
constexpr int kLimLocalPeriods = 8;  // periods a tile aggregates in LDS before falling back to atomics

__device__ __forceinline__ uint32_t lim_period_of(const uint32_t* bnd, uint32_t np, uint32_t idx) {
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bnd[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kLimThreads) k_lim_count(BatchArgs a, LimArgs L) {
    __shared__ uint32_t tot[kMaxLim];
    __shared__ uint32_t arr[kMaxLim][kLimLocalPeriods];
    __shared__ uint32_t q_first;
    const int tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kLimTile;
    const uint32_t* bnd = a.bnd + (size_t)L.wl_idx * kMaxPeriods;
    const uint32_t np = a.np[L.wl_idx];
    if (tid < kMaxLim) tot[tid] = 0;
    if (tid < kMaxLim * kLimLocalPeriods) arr[tid / kLimLocalPeriods][tid % kLimLocalPeriods] = 0;
    if (tid == 0) q_first = lim_period_of(bnd, np, (uint32_t)base);
    __syncthreads();
    const uint32_t q0 = q_first;
    for (int r = 0; r < kLimRounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kLimThreads + tid;
        uint8_t slot = 0xFF;
        if (i < a.n) {
            const uint64_t rec = a.rec[i];
            const uint32_t k = (uint32_t)(rec >> a.kshift);
            if (k < a.K) slot = (uint8_t)L.rule_lim[k];
            L.slot[i] = slot;
        }
        if (slot != 0xFF && L.xg) {
            atomicAdd(&tot[slot], 1u);
            const int64_t m = L.ts[i * L.ts_stride] - L.t_base;
            if (m < 0 || m >= (int64_t)L.n_ms) atomicOr(a.err, kErrExchange);
        } else if (slot != 0xFF) {
            atomicAdd(&tot[slot], 1u);
            const uint32_t q = lim_period_of(bnd, np, (uint32_t)i);
            if (q - q0 < (uint32_t)kLimLocalPeriods) atomicAdd(&arr[slot][q - q0], 1u);
            else atomicAdd(&L.arrivals[(size_t)slot * kMaxPeriods + q], 1u);
        }
    }
    __syncthreads();
    if (tid < kMaxLim) L.tile_tot[(size_t)blockIdx.x * kMaxLim + tid] = tot[tid];
    if (tid < kMaxLim * kLimLocalPeriods && !L.xg) {
        const int l = tid / kLimLocalPeriods, dq = tid % kLimLocalPeriods;
        const uint32_t v = arr[l][dq];
        if (v && q0 + dq < np) atomicAdd(&L.arrivals[(size_t)l * kMaxPeriods + q0 + dq], v);
    }
}

// Largest integer x with (double)x + 1.0 <= qps (RequestLimiter.canPass), or INT64_MAX if unbounded.
__device__ int64_t lim_xmax(double qps) {
    if (!(qps >= 1.0)) return -1;
    if (qps >= 9.0e18) return INT64_MAX;
    int64_t x = (int64_t)floor(qps - 1.0);
    while ((double)(x + 1) + 1.0 <= qps) ++x;
    while (x >= 0 && !((double)x + 1.0 <= qps)) --x;
    return x;
}

// tryPass of `arr` arrivals in limiter period P (absolute): currentWindow create/reset, then the first
// cap(base) of them pass (RequestLimiter.java:72-87 over UnaryLeapArray(10, 1000)). Returns the passes.
__device__ uint32_t lim_ring_step(LimRing* ring, int64_t P, uint32_t arr, int64_t xmax) {
    const int I = (int)(P % kLimSamples);
    const int64_t ws = P * kLimWindowMs;
    if (ring->start[I] != ws) {  // currentWindow: create or reset (UnaryLeapArray.resetWindowTo)
        ring->start[I] = ws;
        ring->count[I] = 0;
    }
    const int64_t lo = ws - (int64_t)(kLimSamples - 1) * kLimWindowMs;
    int64_t base = 0;
    for (int j = 0; j < kLimSamples; ++j)
        if (j != I && ring->start[j] != INT64_MIN && ring->start[j] >= lo) base += ring->count[j];
    base += ring->count[I];
    const int64_t cap = xmax == INT64_MAX ? INT64_MAX : (xmax >= base ? xmax - base + 1 : 0);
    const uint32_t pass = cap >= (int64_t)arr ? arr : (uint32_t)cap;
    ring->count[I] += pass;
    return pass;
}

// Sharded plan, one block: per slot, exclusive prefixes over the exchange's milliseconds of the node's arrivals
// (PT, into L.prefix) and of this shard's (PL); per-period quotas by the ring walk over the node's arrivals; then
// xoff[m] = PT[m] − PT[first ms of m's period] + Σ_{r < rank} arrivals_r(m) − PL[m] (xoff reuses L.arrivals).
__device__ void limx_plan(const LimArgs& L) {
    __shared__ uint32_t pt[kLimThreads], pl[kLimThreads];
    const int tid = threadIdx.x;
    const uint32_t nm = L.n_ms;
    const int64_t P0 = L.t_base / kLimWindowMs;
    const uint32_t r0 = (uint32_t)(L.t_base % kLimWindowMs);
    for (int l = 0; l < L.n_lim; ++l) {
        uint32_t* PT = L.prefix + (size_t)l * kMaxPeriods;
        int32_t* xoff = (int32_t*)L.arrivals + (size_t)l * kMaxPeriods;
        uint32_t ct = 0, cl = 0;
        for (uint32_t m0 = 0; m0 < nm; m0 += kLimThreads) {
            const uint32_t m = m0 + (uint32_t)tid;
            uint32_t tot = 0, bef = 0, loc = 0;
            if (m < nm) {
                for (int r = 0; r < L.world; ++r) {
                    const uint32_t v = L.xg[((size_t)r * L.n_lim + l) * nm + m];
                    tot += v;
                    if (r < L.rank) bef += v;
                    if (r == L.rank) loc = v;
                }
            }
            pt[tid] = tot;
            pl[tid] = loc;
            __syncthreads();
            for (int o = 1; o < kLimThreads; o <<= 1) {
                const uint32_t xt = tid >= o ? pt[tid - o] : 0u, xl = tid >= o ? pl[tid - o] : 0u;
                __syncthreads();
                pt[tid] += xt;
                pl[tid] += xl;
                __syncthreads();
            }
            if (m < nm) {
                PT[m] = ct + pt[tid] - tot;
                xoff[m] = (int32_t)((int64_t)bef - (int64_t)(cl + pl[tid] - loc));
            }
            ct += pt[kLimThreads - 1];
            cl += pl[kLimThreads - 1];
            __syncthreads();
        }
        if (tid == 0) {
            const int64_t xmax = lim_xmax(L.qps[l]);
            const uint32_t nq = (r0 + nm - 1) / kLimWindowMs + 1;
            for (uint32_t q = 0; q < nq; ++q) {
                const uint32_t lo = q == 0 ? 0u : q * kLimWindowMs - r0;
                const uint32_t hi = min(nm, (q + 1) * kLimWindowMs - r0);
                const uint32_t arr = (hi < nm ? PT[hi] : ct) - PT[lo];
                L.quota[(size_t)l * kMaxPeriods + q] = arr ? lim_ring_step(L.ring + l, P0 + (int64_t)q, arr, xmax) : 0u;
            }
        }
        __syncthreads();
        for (uint32_t m = (uint32_t)tid; m < nm; m += kLimThreads) {
            const uint32_t q = (m + r0) / kLimWindowMs;
            const uint32_t lo = q == 0 ? 0u : q * kLimWindowMs - r0;
            xoff[m] += (int32_t)(PT[m] - PT[lo]);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kLimThreads) k_lim_plan(BatchArgs a, LimArgs L, uint32_t ntiles) {
    if (*a.err) {
        // a rejected batch leaves the limiter untouched — except a shard's replica of the node-wide windows,
        // which walks the gathered node arrivals whatever this shard's batch was (every shard charges them)
        if (L.xg) limx_plan(L);
        return;
    }
    const int tid = threadIdx.x;
    // (1) exclusive scan of per-tile totals, slot by slot (thread-strided partial sums + carry)
    __shared__ uint32_t part[kLimThreads];
    for (int l = 0; l < L.n_lim; ++l) {
        uint32_t carry = 0;
        for (uint32_t t0 = 0; t0 < ntiles; t0 += kLimThreads) {
            const uint32_t t = t0 + tid;
            const uint32_t v = t < ntiles ? L.tile_tot[(size_t)t * kMaxLim + l] : 0u;
            part[tid] = v;
            __syncthreads();
            for (int o = 1; o < kLimThreads; o <<= 1) {
                const uint32_t x = tid >= o ? part[tid - o] : 0u;
                __syncthreads();
                part[tid] += x;
                __syncthreads();
            }
            if (t < ntiles) L.tile_off[(size_t)t * kMaxLim + l] = carry + part[tid] - v;
            const uint32_t tot = part[kLimThreads - 1];
            __syncthreads();
            carry += tot;
        }
    }
    if (L.xg) {
        limx_plan(L);
        return;
    }
    // (2) per slot: sequential walk over the limiter periods with the UnaryLeapArray(10, 1000) ring
    if (tid < L.n_lim) {
        const int l = tid;
        const int64_t xmax = lim_xmax(L.qps[l]);
        const uint32_t np = a.np[L.wl_idx];
        const int64_t P0 = a.p0[L.wl_idx];
        uint32_t prefix = 0;
        for (uint32_t q = 0; q < np; ++q) {
            const uint32_t arr = L.arrivals[(size_t)l * kMaxPeriods + q];
            L.prefix[(size_t)l * kMaxPeriods + q] = prefix;
            prefix += arr;
            // no tryPass in a period without arrivals: the ring is not touched
            L.quota[(size_t)l * kMaxPeriods + q] = arr ? lim_ring_step(L.ring + l, P0 + (int64_t)q, arr, xmax) : 0u;
        }
    }
}

__global__ void __launch_bounds__(kLimThreads) k_lim_apply(BatchArgs a, LimArgs L) {
    __shared__ uint32_t run[kMaxLim];
    __shared__ uint32_t wcnt[kLimThreads / 64][kMaxLim];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kLimTile;
    const uint32_t* bnd = a.bnd + (size_t)L.wl_idx * kMaxPeriods;
    const uint32_t np = a.np[L.wl_idx];
    const uint64_t sentinel = (uint64_t)a.K << a.kshift;
    if (*a.err) return;
    if (tid < kMaxLim) run[tid] = L.tile_off[(size_t)blockIdx.x * kMaxLim + tid];
    // every (wave, slot) count starts at 0: a round sets only the slots present in a wave, and the first round would
    // otherwise read what an earlier kernel left in this CU's LDS for the others
    if (tid < (kLimThreads / 64) * kMaxLim) wcnt[tid / kMaxLim][tid % kMaxLim] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int r = 0; r < kLimRounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kLimThreads + tid;
        const uint8_t slot = i < a.n ? L.slot[i] : (uint8_t)0xFF;
        // rank among this wave's lanes of the same slot, then across waves of this round
        uint64_t peers = ~0ull;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((slot >> b) & 1u);
            peers &= ((slot >> b) & 1u) ? m : ~m;
        }
        const uint32_t rank_w = (uint32_t)__popcll(peers & lt);
        if (slot != 0xFF && lane == __builtin_ctzll(peers)) wcnt[wave][slot] = (uint32_t)__popcll(peers);
        if (slot == 0xFF && lane == 0) {}
        __syncthreads();
        uint32_t before = 0;
        if (slot != 0xFF) {
            before = run[slot];
            for (int w = 0; w < wave; ++w) before += wcnt[w][slot];
        }
        __syncthreads();
        if (tid < kMaxLim) {
            uint32_t add = 0;
            for (int w = 0; w < kLimThreads / 64; ++w) {
                add += wcnt[w][tid];
                wcnt[w][tid] = 0;
            }
            run[tid] += add;
        }
        if (slot != 0xFF) {
            const uint32_t C = before + rank_w;  // slot-l requests before index i in the whole batch
            uint32_t q;
            int64_t rank;
            if (L.xg) {  // the node-wide rank within the period (k_lim_plan's xoff)
                const uint32_t m = (uint32_t)(L.ts[i * L.ts_stride] - L.t_base);
                q = (m + (uint32_t)(L.t_base % kLimWindowMs)) / kLimWindowMs;
                rank = (int64_t)C + (int64_t)((const int32_t*)L.arrivals)[(size_t)slot * kMaxPeriods + m];
            } else {
                q = lim_period_of(bnd, np, (uint32_t)i);
                rank = (int64_t)C - (int64_t)L.prefix[(size_t)slot * kMaxPeriods + q];
            }
            if (rank >= (int64_t)L.quota[(size_t)slot * kMaxPeriods + q]) {
                sg_result res;
                res.status = SG_STATUS_TOO_MANY_REQUEST;
                res.remaining = 0;
                res.wait_ms = 0;
                a.out[i] = res;
                a.rec[i] = sentinel;
            }
        }
        __syncthreads();
    }
}

hipError_t launch_limiter(const BatchArgs& a, const LimArgs& L, hipStream_t stream) {
    const uint32_t ntiles = (uint32_t)((a.n + kLimTile - 1) / kLimTile);
    hipError_t e = hipMemsetAsync(L.arrivals, 0, sizeof(uint32_t) * kMaxLim * kMaxPeriods, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lim_count, dim3(ntiles), dim3(kLimThreads), 0, stream, a, L);
    hipLaunchKernelGGL(k_lim_plan, dim3(1), dim3(kLimThreads), 0, stream, a, L, ntiles);
    lds_poison(stream);
    hipLaunchKernelGGL(k_lim_apply, dim3(ntiles), dim3(kLimThreads), 0, stream, a, L);
    return hipGetLastError();
}

hipError_t launch_limiter_plan_only(const BatchArgs& a, const LimArgs& L, hipStream_t stream) {
    hipLaunchKernelGGL(k_lim_plan, dim3(1), dim3(kLimThreads), 0, stream, a, L, 0u);
    return hipGetLastError();
}

constexpr uint32_t kLimxWin = 256;  // milliseconds a tile aggregates in LDS (a time-ordered tile spans few)

// The limiter's tryPass candidates of a flow batch (DefaultTokenService.requestToken validation, as k_prep) and of a
// cluster param batch (requestParamToken validation, as k_cp_prep2): key = rule index, or none.
struct LimxFlowReq {
    __device__ static uint32_t key(const sg_req& q, uint32_t K) {
        const uint32_t k = q.key & SG_KEY_INDEX;
        return (k == SG_KEY_BAD || q.acquire <= 0 || k >= K) ? 0xFFFFFFFFu : k;
    }
};
struct LimxParamReq {
    __device__ static uint32_t key(const sg_cparam_req& q, uint32_t K) {
        const uint32_t k = q.key & SG_KEY_INDEX;
        return (k == SG_KEY_BAD || q.acquire <= 0 || q.value_count == 0 || k >= K) ? 0xFFFFFFFFu : k;
    }
};

template <class Req, class V>
__global__ void __launch_bounds__(kLimThreads) k_limx_arrivals(const Req* req, uint64_t n, uint32_t K,
                                                              const uint8_t* rule_lim, int64_t t_base, uint32_t n_ms,
                                                              uint32_t* counts, int* err) {
    __shared__ uint32_t hist[kMaxLim][kLimxWin];
    __shared__ int64_t m_first;
    const int tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kLimTile;
    for (uint32_t x = (uint32_t)tid; x < kMaxLim * kLimxWin; x += kLimThreads) hist[x / kLimxWin][x % kLimxWin] = 0;
    if (tid == 0) m_first = req[base].ts_ms - t_base;
    __syncthreads();
    const int64_t m0 = m_first;
    for (int r = 0; r < kLimRounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kLimThreads + tid;
        if (i >= n) break;
        const Req q = req[i];
        const uint32_t key = V::key(q, K);
        if (key == 0xFFFFFFFFu) continue;
        const uint8_t slot = rule_lim[key];
        if (slot == 0xFF) continue;
        const int64_t m = q.ts_ms - t_base;
        if (m < 0 || m >= (int64_t)n_ms) {
            atomicOr(err, kErrExchange);
        } else if (m >= m0 && m - m0 < (int64_t)kLimxWin) {
            atomicAdd(&hist[slot][m - m0], 1u);
        } else {
            atomicAdd(&counts[(size_t)slot * n_ms + (uint64_t)m], 1u);
        }
    }
    __syncthreads();
    for (uint32_t x = (uint32_t)tid; x < kMaxLim * kLimxWin; x += kLimThreads) {
        const uint32_t v = hist[x / kLimxWin][x % kLimxWin];
        const int64_t m = m0 + (int64_t)(x % kLimxWin);
        if (v) atomicAdd(&counts[(size_t)(x / kLimxWin) * n_ms + (uint64_t)m], v);
    }
}

hipError_t launch_lim_arrivals(const sg_req* req, uint64_t n, uint32_t K, const uint8_t* rule_lim, int64_t t_base,
                               uint32_t n_ms, uint32_t* counts, int* err, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t ntiles = (uint32_t)((n + kLimTile - 1) / kLimTile);
    lds_poison(stream);
    hipLaunchKernelGGL((k_limx_arrivals<sg_req, LimxFlowReq>), dim3(ntiles), dim3(kLimThreads), 0, stream, req, n, K,
                       rule_lim, t_base, n_ms, counts, err);
    return hipGetLastError();
}

hipError_t launch_lim_arrivals_param(const sg_cparam_req* req, uint64_t n, uint32_t K, const uint8_t* rule_lim,
                                     int64_t t_base, uint32_t n_ms, uint32_t* counts, int* err, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t ntiles = (uint32_t)((n + kLimTile - 1) / kLimTile);
    lds_poison(stream);
    hipLaunchKernelGGL((k_limx_arrivals<sg_cparam_req, LimxParamReq>), dim3(ntiles), dim3(kLimThreads), 0, stream, req,
                       n, K, rule_lim, t_base, n_ms, counts, err);
    return hipGetLastError();
}

}  // namespace sg
