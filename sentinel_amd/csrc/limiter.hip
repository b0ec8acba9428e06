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
        if (slot != 0xFF) {
            atomicAdd(&tot[slot], 1u);
            const uint32_t q = lim_period_of(bnd, np, (uint32_t)i);
            if (q - q0 < (uint32_t)kLimLocalPeriods) atomicAdd(&arr[slot][q - q0], 1u);
            else atomicAdd(&L.arrivals[(size_t)slot * kMaxPeriods + q], 1u);
        }
    }
    __syncthreads();
    if (tid < kMaxLim) L.tile_tot[(size_t)blockIdx.x * kMaxLim + tid] = tot[tid];
    if (tid < kMaxLim * kLimLocalPeriods) {
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

__global__ void __launch_bounds__(kLimThreads) k_lim_plan(BatchArgs a, LimArgs L, uint32_t ntiles) {
    if (*a.err) return;  // a rejected batch leaves the limiter untouched
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
    // (2) per slot: sequential walk over the limiter periods with the UnaryLeapArray(10, 1000) ring
    if (tid < L.n_lim) {
        const int l = tid;
        const int64_t xmax = lim_xmax(L.qps[l]);
        const uint32_t np = a.np[L.wl_idx];
        const int64_t P0 = a.p0[L.wl_idx];
        LimRing* ring = L.ring + l;
        uint32_t prefix = 0;
        for (uint32_t q = 0; q < np; ++q) {
            const uint32_t arr = L.arrivals[(size_t)l * kMaxPeriods + q];
            L.prefix[(size_t)l * kMaxPeriods + q] = prefix;
            prefix += arr;
            if (arr == 0) {
                L.quota[(size_t)l * kMaxPeriods + q] = 0;
                continue;  // no tryPass in this period: the ring is not touched
            }
            const int64_t P = P0 + (int64_t)q;
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
            int64_t cap = xmax == INT64_MAX ? INT64_MAX : (xmax >= base ? xmax - base + 1 : 0);
            const uint32_t pass = cap >= (int64_t)arr ? arr : (uint32_t)cap;
            L.quota[(size_t)l * kMaxPeriods + q] = pass;
            ring->count[I] += pass;
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
            const uint32_t q = lim_period_of(bnd, np, (uint32_t)i);
            const uint32_t rank = C - L.prefix[(size_t)slot * kMaxPeriods + q];
            if (rank >= L.quota[(size_t)slot * kMaxPeriods + q]) {
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
    hipLaunchKernelGGL(k_lim_apply, dim3(ntiles), dim3(kLimThreads), 0, stream, a, L);
    return hipGetLastError();
}

}  // namespace sg
