// node.hip — the node handle's request routing (include/sentinel_gpu.h, sg_node_*): one token server's batch split
// over G shard handles by flowId owner, and the shards' results put back in the caller's order.
//
// The reference serves every flowId from one TokenService (DefaultTokenService.requestToken, DefaultTokenService.java
// :39-50, called by all Netty workers, NettyTransportServer.java:53-54). Here the flowIds are hashed over G shards
// (splitmix64(flowId) mod G); the node's front handle has already validated the batch and run the
// namespace limiter over it in caller order (k_prep + the limiter pre-pass), so each request of its packed records
// that survived carries its node rule index. Routing is a stable multisplit of those records by shard:
//   k_route_count    per 4096-record tile: requests per shard (LDS counters)
//   k_route_scan     one block per shard: the exclusive scan of its tile counts, its total; k_route_bases lays the
//                    shard slices out one after the other (shard g at base[g]) in one sub-batch buffer
//   k_route_scatter  per tile: each wave ranks its 64-record rounds by shard (match ballots, as the radix scatter)
//                    and writes the sub-request {ts, local rule index | prio, acquire} and the node position of
//                    every routed request — time order within a shard is kept (stable), so each slice is a valid
//                    batch for its shard
//   k_route_gather   out[pos[j]] = sub_out[j]: the shards' results in caller order
// Shards on the front's device take packed records instead (RouteArgs::sub_rec): 8 B read and 8 B written per routed
// request, and the shards write the caller's results in place (no gather).
// HBM-bound byte work: 16 B read + 16 B + 4 B written per request (scatter), 12 B + 4 B read and 12 B written
// (gather); no MFMA.
#include "engine.h"

namespace sg {

namespace {

constexpr int kRouteThreads = 256;
constexpr int kRouteRounds = 16;
constexpr uint32_t kRouteTile = kRouteThreads * kRouteRounds;
constexpr int kRouteWaveRecs = kRouteTile / (kRouteThreads / 64);

__device__ __forceinline__ int route_lane() { return (int)__lane_id(); }

// Lanes of the wave whose 6-bit shard equals this lane's (shard 64: not routed).
__device__ __forceinline__ uint64_t match_shard(uint32_t s) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint64_t m = __ballot((s >> b) & 1u);
        peers &= ((s >> b) & 1u) ? m : ~m;
    }
    return peers;
}

__device__ __forceinline__ uint32_t shard_of_rec(const RouteArgs& r, uint64_t rec) {
    const uint32_t k = (uint32_t)(rec >> r.kshift);
    return k < r.K ? (uint32_t)r.shard_of[k] : (uint32_t)kRouteNone;
}

}  // namespace

__global__ void __launch_bounds__(kRouteThreads) k_route_count(RouteArgs r) {
    __shared__ uint32_t cnt[kMaxShards];
    const int tid = threadIdx.x;
    if (tid < kMaxShards) cnt[tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
    // every record's load, then every owner lookup, issued before any is used (two round trips per thread)
    uint64_t rec[kRouteRounds];
    uint32_t sh[kRouteRounds];
#pragma unroll
    for (int it = 0; it < kRouteRounds; ++it) {
        const uint64_t i = base + (uint64_t)it * kRouteThreads + tid;
        rec[it] = i < r.n ? r.rec[i] : ~0ull;
    }
#pragma unroll
    for (int it = 0; it < kRouteRounds; ++it) sh[it] = shard_of_rec(r, rec[it]);
#pragma unroll
    for (int it = 0; it < kRouteRounds; ++it)
        if (sh[it] < (uint32_t)r.G) atomicAdd(&cnt[sh[it]], 1u);
    __syncthreads();
    if (tid < r.G) r.tile_cnt[(size_t)blockIdx.x * kMaxShards + tid] = cnt[tid];
}

// One block per shard: the exclusive scan of the shard's column of tile counts (1024 threads, a few tiles each,
// then a block scan), the shard's total for the host. (A serial column walk was one dependent load per tile:
// 1.4 ms for a 16M-request batch.)
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) k_route_scan(RouteArgs r, uint32_t ntiles) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const int g = blockIdx.x, tid = threadIdx.x, lane = route_lane(), wave = tid >> 6;
    const uint32_t per = (ntiles + kScanThreads - 1) / kScanThreads;
    const uint32_t t0 = (uint32_t)tid * per, t1 = min(t0 + per, ntiles);
    uint32_t mine = 0;
    for (uint32_t t = t0; t < t1; ++t) mine += r.tile_cnt[(size_t)t * kMaxShards + g];
    uint32_t x = mine;  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t run = x - mine, total = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) {
        if (w < wave) run += wsum[w];
        total += wsum[w];
    }
    for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t c = r.tile_cnt[(size_t)t * kMaxShards + g];
        r.tile_cnt[(size_t)t * kMaxShards + g] = run;
        run += c;
    }
    if (tid == 0) r.shard_tot[g] = total;
}

// The shard slices one after the other: base[g] = Σ totals before g (G <= 64: one wave).
__global__ void __launch_bounds__(64) k_route_bases(RouteArgs r) {
    const int lane = route_lane();
    const uint32_t v = lane < r.G ? r.shard_tot[lane] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
        if (lane >= o) x += y;
    }
    if (lane < r.G) r.shard_base[lane] = x - v;
    if (lane == 63) r.shard_base[r.G] = x;
}

__global__ void __launch_bounds__(kRouteThreads) k_route_scatter(RouteArgs r) {
    __shared__ uint32_t wrun[kRouteThreads / 64][kMaxShards];  // each wave's running count per shard in its range
    __shared__ uint32_t wtot[kRouteThreads / 64][kMaxShards];  // each wave's total per shard (its range's prefix)
    const int tid = threadIdx.x, lane = route_lane(), wave = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kRouteTile;
    const uint64_t w0 = base + (uint64_t)wave * kRouteWaveRecs;  // the wave's contiguous records
    for (int x = lane; x < kMaxShards; x += 64) {
        wrun[wave][x] = 0;
        wtot[wave][x] = 0;
    }
    // every record, then every owner and local index, loaded before any is used (kept for both passes: a dependent
    // load chain per round was the kernel's time beside the walkers)
    constexpr int kR = kRouteWaveRecs / 64;
    uint64_t recs[kR];
    uint32_t sh[kR], loc[kR];
#pragma unroll
    for (int it = 0; it < kR; ++it) {
        const uint64_t i = w0 + (uint64_t)it * 64 + lane;
        recs[it] = i < r.n ? r.rec[i] : ~0ull;
    }
#pragma unroll
    for (int it = 0; it < kR; ++it) {
        sh[it] = shard_of_rec(r, recs[it]);
        const uint32_t k = (uint32_t)(recs[it] >> r.kshift);
        loc[it] = sh[it] < (uint32_t)r.G ? r.local_of[k] : 0u;
    }
    // 1. per wave: records per shard over its range (the tile's stable order is wave 0's records, then wave 1's …)
#pragma unroll
    for (int it = 0; it < kR; ++it) {
        const uint32_t s = sh[it];
        const uint64_t peers = match_shard(s);
        if (s < (uint32_t)r.G && (peers & ((1ull << lane) - 1ull)) == 0) wtot[wave][s] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_sched_barrier(0);  // round by round (hoisted ballots spilled)
    }
    __syncthreads();
    // 2. place: position = shard base + the tile's offset + earlier waves of the tile + earlier rounds + rank in round
#pragma unroll
    for (int it = 0; it < kR; ++it) {
        const uint64_t rec = recs[it];
        const uint32_t s = sh[it];
        const uint64_t peers = match_shard(s);
        const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (s < (uint32_t)r.G) {
            uint32_t before = 0;
            for (int w = 0; w < wave; ++w) before += wtot[w][s];
            const uint32_t pos = r.shard_base[s] + r.tile_cnt[(size_t)blockIdx.x * kMaxShards + s] + before +
                                 wrun[wave][s] + rank;
            if (r.sub_rec) {
                r.sub_rec[pos] = ((uint64_t)loc[it] << r.skshift[s]) | (rec & r.low_mask);
            } else {
                const uint32_t idx = (uint32_t)((rec >> r.abits) & r.imask);
                const sg_req q = r.req[idx];
                sg_req o;
                o.ts_ms = q.ts_ms;
                o.key = loc[it] | (q.key & SG_KEY_PRIO);
                o.acquire = q.acquire;
                r.sub_req[pos] = o;
                r.sub_pos[pos] = idx;
            }
        }
        if (s < (uint32_t)r.G && rank == 0) wrun[wave][s] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_sched_barrier(0);
    }
}

__global__ void __launch_bounds__(256) k_route_gather(const sg_result* sub_out, const uint32_t* sub_pos, uint64_t total,
                                                      sg_result* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (uint64_t)gridDim.x * blockDim.x)
        out[sub_pos[j]] = sub_out[j];
}

hipError_t launch_route(const RouteArgs& r, hipStream_t stream) {
    const uint32_t tiles = (uint32_t)((r.n + kRouteTile - 1) / kRouteTile);
    if (tiles == 0) return hipSuccess;
    lds_poison(stream);
    hipLaunchKernelGGL(k_route_count, dim3(tiles), dim3(kRouteThreads), 0, stream, r);
    hipLaunchKernelGGL(k_route_scan, dim3((unsigned)r.G), dim3(kScanThreads), 0, stream, r, tiles);
    hipLaunchKernelGGL(k_route_bases, dim3(1), dim3(64), 0, stream, r);
    lds_poison(stream);
    hipLaunchKernelGGL(k_route_scatter, dim3(tiles), dim3(kRouteThreads), 0, stream, r);
    return hipGetLastError();
}

hipError_t launch_route_gather(const sg_result* sub_out, const uint32_t* sub_pos, uint64_t total, sg_result* out,
                               hipStream_t stream) {
    if (total == 0) return hipSuccess;
    uint64_t g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_route_gather, dim3((unsigned)g), dim3(256), 0, stream, sub_out, sub_pos, total, out);
    return hipGetLastError();
}

uint64_t route_tiles(uint64_t n) { return (n + kRouteTile - 1) / kRouteTile; }

}  // namespace sg
