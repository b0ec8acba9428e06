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

// ---- cluster param and concurrent token batches over the node (sg_node_cparam_*, sg_node_conc_*) ----
//
// DefaultTokenService.requestParamToken / requestConcurrentToken / releaseConcurrentToken (DefaultTokenService.java
// :53-85) for the whole node: a request goes to the shard that owns its flowId (a param rule's flowId; a flow rule's
// for concurrent tokens; a release to the shard whose token it names: node token id = (shard token id - 1) * G +
// shard + 1), and every shard decides its slice in the node's order. Requests nothing owns (invalid keys, null
// tokens) go to shard 0, whose validation answers them. Routing is a stable partition by owner: a record {owner : 8 |
// request index} per request, one 8-bit radix pass, then the slices gathered (keys and token ids made shard-local;
// a param request's values copied after the slice's earlier ones, its value_begin rebased).

__global__ void __launch_bounds__(256) k_nreq_keys(NodeReqArgs q) {
    __shared__ uint32_t cnt[kMaxShards], vcnt[kMaxShards];
    const int tid = threadIdx.x;
    if (tid < kMaxShards) cnt[tid] = vcnt[tid] = 0;
    __syncthreads();
    // the loop runs block-uniformly (the shard counts below are wave-wide)
    for (uint64_t b0 = (uint64_t)blockIdx.x * 256; b0 < q.n; b0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = b0 + tid;
        const bool act = i < q.n;
        uint32_t g = 0, nv = 0;
        if (act) {
            {  // the node's time order (a batch older than the node's previous one, or unsorted, is refused whole)
                const int64_t t = q.cp ? q.cp[i].ts_ms : q.cc[i].ts_ms;
                const int64_t tp = i == 0 ? q.last_ts : (q.cp ? q.cp[i - 1].ts_ms : q.cc[i - 1].ts_ms);
                if (t < 0 || t < tp) atomicOr(q.err, kErrTime);
            }
            if (q.cp) {
                const sg_cparam_req r = q.cp[i];
                const uint32_t key = r.key & SG_KEY_INDEX;
                if (key < q.K) g = q.shard_of[key];
                // only a valid request's values are read (DefaultTokenService answers the others without them); an
                // invalid one reaches its shard with no values, and the shard answers it as one handle would
                const bool valid = key < q.K && r.acquire > 0 && r.value_count > 0;
                nv = valid ? r.value_count : 0u;
                if (nv && ((uint64_t)r.value_begin + nv > q.n_values)) {  // the whole batch is refused (SG_E_INVAL)
                    atomicOr(q.err, kErrBounds);
                    nv = 0;
                }
            } else {
                const sg_conc_req r = q.cc[i];
                if (r.kind == SG_CONC_RELEASE) g = r.token_id ? (uint32_t)((r.token_id - 1) % (uint64_t)q.G) : 0u;
                else if ((r.key & SG_KEY_INDEX) < q.K) g = q.shard_of[r.key & SG_KEY_INDEX];
            }
            q.rec[i] = ((uint64_t)g << 56) | i;
            q.nvals[i] = nv;
        }
        // per shard present in the wave: one LDS add of its request count and value count (the lanes of a wave hit
        // G addresses at most; per-lane atomics serialised on them and held back the next request's loads)
        bool todo = act;
        while (__ballot(todo)) {
            const uint32_t g0 = (uint32_t)__shfl((int)g, __builtin_ctzll(__ballot(todo)), 64);
            const bool mine = todo && g == g0;
            const uint64_t m = __ballot(mine);
            uint32_t v = mine ? nv : 0u;
            for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
            if (__lane_id() == (uint32_t)__builtin_ctzll(m)) {
                atomicAdd(&cnt[g0], (uint32_t)__popcll(m));
                if (v) atomicAdd(&vcnt[g0], v);
            }
            todo = todo && !mine;
        }
    }
    __syncthreads();
    if (tid < q.G) {
        if (cnt[tid]) atomicAdd(&q.cnt[tid], cnt[tid]);
        if (vcnt[tid]) atomicAdd(&q.vcnt[tid], vcnt[tid]);
    }
}

// Exclusive scan of the sorted requests' value counts (param batches): per 4096-request tile sums, one block over the
// tile sums, then each tile's requests (nvals in node order, read through the sorted records).
constexpr uint32_t kNvTile = 4096;
__global__ void __launch_bounds__(256) k_nreq_vsum(NodeReqArgs q, const uint64_t* sorted) {
    __shared__ uint32_t ws[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kNvTile;
    uint32_t s = 0;
    for (uint64_t j = t0 + threadIdx.x; j < min(q.n, t0 + kNvTile); j += 256)
        s += q.nvals[sorted[j] & 0xFFFFFFFFFFFFFFull];
    for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) q.tsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void __launch_bounds__(1024) k_nreq_vscan(NodeReqArgs q, uint32_t tiles) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < tiles; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < tiles ? q.tsum[i] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint32_t x = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += x;
            __syncthreads();
        }
        const uint32_t c = carry;
        if (i < tiles) q.tsum[i] = c + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = c + part[1023];
        __syncthreads();
    }
}

// The slices: sub_req[j] = the request of sorted record j with its key (and token id) made shard-local, its value
// range copied and rebased (param), sub_pos[j] its node position. One block per 4096 sorted records; the value
// offsets inside the tile by a block scan.
__global__ void __launch_bounds__(256) k_nreq_gather(NodeReqArgs q, const uint64_t* sorted) {
    __shared__ uint32_t ws[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kNvTile;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t run = q.cp ? q.tsum[blockIdx.x] : 0u;
    for (uint64_t b0 = t0; b0 < min(q.n, t0 + kNvTile); b0 += 256) {
        const uint64_t j = b0 + threadIdx.x;
        const bool act = j < q.n;
        const uint64_t rec = act ? sorted[j] : 0ull;
        const uint32_t g = (uint32_t)(rec >> 56);
        const uint64_t i = rec & 0xFFFFFFFFFFFFFFull;
        uint32_t nv = (act && q.cp) ? q.nvals[i] : 0u;
        // block-exclusive scan of nv
        uint32_t x = nv;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        uint32_t off = run + x - nv;
        uint32_t tot = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wave) off += ws[w];
            tot += ws[w];
        }
        __syncthreads();
        run += tot;
        if (!act) continue;
        q.sub_pos[j] = (uint32_t)i;
        if (q.cp) {
            sg_cparam_req r = q.cp[i];
            if ((r.key & SG_KEY_INDEX) < q.K) r.key = q.local_of[r.key & SG_KEY_INDEX] | (r.key & ~SG_KEY_INDEX);
            for (uint32_t v = 0; v < nv; ++v) q.sub_vals[off + v] = q.values[r.value_begin + v];
            r.value_begin = nv ? off - q.vbase[g] : 0u;
            q.sub_cp[j] = r;
        } else {
            sg_conc_req r = q.cc[i];
            if (r.kind == SG_CONC_RELEASE) {
                if (r.token_id) r.token_id = (r.token_id - 1) / (uint64_t)q.G + 1;
            } else if ((r.key & SG_KEY_INDEX) < q.K) {
                r.key = q.local_of[r.key & SG_KEY_INDEX] | (r.key & ~SG_KEY_INDEX);
            }
            q.sub_cc[j] = r;
        }
    }
}

// Concurrent results back in node order, shard g's slice [base, base + cnt): an acquire's token id in node terms.
__global__ void __launch_bounds__(256) k_nconc_scatter(const sg_conc_result* sub_out, const uint32_t* sub_pos,
                                                       const sg_conc_req* sub_req, uint64_t base, uint64_t cnt,
                                                       uint32_t g, uint32_t G, sg_conc_result* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < cnt; j += (uint64_t)gridDim.x * 256) {
        sg_conc_result r = sub_out[base + j];
        if (sub_req[base + j].kind != SG_CONC_RELEASE && r.token_id) r.token_id = (r.token_id - 1) * G + g + 1;
        out[sub_pos[base + j]] = r;
    }
}

// The node snapshot from shard g's part (its local rule order): out[2 node_key[j] + c] = part[2 j + c].
__global__ void __launch_bounds__(256) k_nsnap_scatter(const double* part, const uint32_t* node_key, uint64_t cnt,
                                                       double* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < cnt; j += (uint64_t)gridDim.x * 256) {
        const uint32_t k = node_key[j];
        out[2 * (uint64_t)k] = part[2 * j];
        out[2 * (uint64_t)k + 1] = part[2 * j + 1];
    }
}

hipError_t launch_nsnap_scatter(const double* part, const uint32_t* node_key, uint64_t cnt, double* out,
                                hipStream_t stream) {
    if (cnt == 0) return hipSuccess;
    uint64_t b = (cnt + 255) / 256;
    if (b > 8192) b = 8192;
    hipLaunchKernelGGL(k_nsnap_scatter, dim3((unsigned)b), dim3(256), 0, stream, part, node_key, cnt, out);
    return hipGetLastError();
}

// The contract on a param batch's value ranges (sg_cparam_decide_batch): the valid requests' ranges follow request
// order and do not overlap — each begins at or after the largest end of the earlier valid requests. One handle
// checks it slot by slot on its sorted records (k_cp_order); the node copies each request's values into its slice,
// so it checks the node batch as a whole: per 4096-request tile the largest end, one block's exclusive prefix max
// over the tiles, then each tile against that carry (16 consecutive requests per thread, a block-wide prefix max).
__device__ __forceinline__ bool nreq_valid(const NodeReqArgs& q, const sg_cparam_req& r) {
    return (r.key & SG_KEY_INDEX) < q.K && r.acquire > 0 && r.value_count > 0;
}

__global__ void __launch_bounds__(256) k_nreq_vmax(NodeReqArgs q) {
    __shared__ uint32_t wm[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kNvTile;
    uint32_t m = 0;
    for (uint64_t i = t0 + threadIdx.x; i < min(q.n, t0 + kNvTile); i += 256) {
        const sg_cparam_req r = q.cp[i];
        if (nreq_valid(q, r)) m = max(m, r.value_begin + r.value_count);
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) q.tsum[blockIdx.x] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
}

__global__ void __launch_bounds__(1024) k_nreq_vmax_scan(NodeReqArgs q, uint32_t tiles) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < tiles; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < tiles ? q.tsum[i] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint32_t x = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] = max(part[threadIdx.x], x);
            __syncthreads();
        }
        const uint32_t c = carry;
        const uint32_t excl = threadIdx.x ? part[threadIdx.x - 1] : 0u;
        if (i < tiles) q.tsum[i] = max(c, excl);
        __syncthreads();
        if (threadIdx.x == 1023) carry = max(c, part[1023]);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_nreq_vorder(NodeReqArgs q) {
    __shared__ uint32_t tm[256];
    constexpr int kPer = (int)(kNvTile / 256);
    const uint64_t i0 = (uint64_t)blockIdx.x * kNvTile + (uint64_t)threadIdx.x * kPer;
    uint32_t m = 0;
    for (int u = 0; u < kPer && i0 + u < q.n; ++u) {
        const sg_cparam_req r = q.cp[i0 + u];
        if (nreq_valid(q, r)) m = max(m, r.value_begin + r.value_count);
    }
    tm[threadIdx.x] = m;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive prefix max of the threads' maxima
        const uint32_t x = threadIdx.x >= (unsigned)o ? tm[threadIdx.x - o] : 0u;
        __syncthreads();
        tm[threadIdx.x] = max(tm[threadIdx.x], x);
        __syncthreads();
    }
    uint32_t carry = max(q.tsum[blockIdx.x], threadIdx.x ? tm[threadIdx.x - 1] : 0u);
    bool bad = false;
    for (int u = 0; u < kPer && i0 + u < q.n; ++u) {
        const sg_cparam_req r = q.cp[i0 + u];
        if (!nreq_valid(q, r)) continue;
        bad |= r.value_begin < carry;
        carry = max(carry, r.value_begin + r.value_count);
    }
    if (bad) atomicOr(q.err, kErrBounds);
}

hipError_t launch_nreq_keys(const NodeReqArgs& q, hipStream_t stream) {
    if (q.n == 0) return hipSuccess;
    uint64_t g = (q.n + 255) / 256;
    if (g > 4096) g = 4096;
    lds_poison(stream);
    hipLaunchKernelGGL(k_nreq_keys, dim3((unsigned)g), dim3(256), 0, stream, q);
    if (q.cp) {  // the value ranges' order (the tile maxima use tsum before the gather's value scan does)
        const uint32_t tiles = (uint32_t)((q.n + kNvTile - 1) / kNvTile);
        hipLaunchKernelGGL(k_nreq_vmax, dim3(tiles), dim3(256), 0, stream, q);
        hipLaunchKernelGGL(k_nreq_vmax_scan, dim3(1), dim3(1024), 0, stream, q, tiles);
        hipLaunchKernelGGL(k_nreq_vorder, dim3(tiles), dim3(256), 0, stream, q);
    }
    return hipGetLastError();
}

hipError_t launch_nreq_gather(const NodeReqArgs& q, const uint64_t* sorted, hipStream_t stream) {
    if (q.n == 0) return hipSuccess;
    const uint32_t tiles = (uint32_t)((q.n + kNvTile - 1) / kNvTile);
    if (q.cp) {
        hipLaunchKernelGGL(k_nreq_vsum, dim3(tiles), dim3(256), 0, stream, q, sorted);
        hipLaunchKernelGGL(k_nreq_vscan, dim3(1), dim3(1024), 0, stream, q, tiles);
    }
    hipLaunchKernelGGL(k_nreq_gather, dim3(tiles), dim3(256), 0, stream, q, sorted);
    return hipGetLastError();
}

uint64_t nreq_tiles(uint64_t n) { return (n + kNvTile - 1) / kNvTile; }

hipError_t launch_nconc_scatter(const sg_conc_result* sub_out, const uint32_t* sub_pos, const sg_conc_req* sub_req,
                                uint64_t base, uint64_t cnt, uint32_t g, uint32_t G, sg_conc_result* out,
                                hipStream_t stream) {
    if (cnt == 0) return hipSuccess;
    uint64_t b = (cnt + 255) / 256;
    if (b > 8192) b = 8192;
    hipLaunchKernelGGL(k_nconc_scatter, dim3((unsigned)b), dim3(256), 0, stream, sub_out, sub_pos, sub_req, base, cnt, g,
                       G, out);
    return hipGetLastError();
}

}  // namespace sg
