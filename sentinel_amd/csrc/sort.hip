// sort.hip — stable LSD radix sort of the 64-bit request records by their flowId field.
//
// The walkers need each flowId's requests contiguous and still in (timestamp, arrival) order, i.e. a
// stable partition by flowId. Records are sorted on bits [lo_bit, 64) only, 8 bits per pass:
//   k_radix_hist     per 4096-record tile: digit histogram (wave match-any aggregation, then LDS)
//   k_scan_*         exclusive scan of the digit-major histogram [256][tiles]
//   k_radix_scatter  per tile, 16 rounds of 256 records in index order: wave match-any gives each
//                    record its rank among equal digits in its wave, an LDS prefix over the 4 waves and
//                    the running per-digit count give its rank in the tile; record → global offset.
// Stability follows from ranking strictly in index order (rounds, then waves, then lanes).
#include "engine.h"

namespace sg {

constexpr int kRadixBits = 8;
constexpr int kBins = 1 << kRadixBits;
constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRounds = 16;
constexpr int kTile = kSortThreads * kRounds;  // 4096 records per tile
constexpr int kScanItems = 8;
constexpr int kScanChunk = kSortThreads * kScanItems;  // 2048 counters per scan block

// Lanes of this wave whose `digit` equals this lane's (8 ballots).
__device__ __forceinline__ uint64_t match_digit(uint32_t digit) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < kRadixBits; ++b) {
        const uint64_t m = __ballot((digit >> b) & 1u);
        peers &= ((digit >> b) & 1u) ? m : ~m;
    }
    return peers;
}

__global__ void __launch_bounds__(kSortThreads) k_radix_hist(const uint64_t* in, uint64_t n, int shift, uint32_t* hist,
                                                             uint32_t ntiles) {
    __shared__ uint32_t cnt[kBins];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    cnt[tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = base + (uint64_t)r * kSortThreads + tid;
        const bool valid = idx < n;
        const uint32_t d = valid ? (uint32_t)(in[idx] >> shift) & (kBins - 1) : 0u;
        const uint64_t peers = match_digit(d) & __ballot(valid);
        if (valid && lane == __builtin_ctzll(peers)) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    hist[(size_t)tid * ntiles + blockIdx.x] = cnt[tid];
}

// Block-local exclusive scan of kScanChunk counters; writes the chunk total to sums[blockIdx.x].
__global__ void __launch_bounds__(kSortThreads) k_scan_local(uint32_t* data, uint64_t n, uint32_t* sums) {
    __shared__ uint32_t part[kSortThreads];
    const int tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)tid * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        v[i] = (base + i < n) ? data[base + i] : 0u;
        s += v[i];
    }
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < kSortThreads; o <<= 1) {  // Hillis-Steele inclusive scan of per-thread sums
        uint32_t x = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    uint32_t run = part[tid] - s;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        if (base + i < n) data[base + i] = run;
        run += v[i];
    }
    if (tid == kSortThreads - 1) sums[blockIdx.x] = part[tid];
}

// Single-block exclusive scan of the chunk totals (any count, carried across 256-wide steps).
__global__ void __launch_bounds__(kSortThreads) k_scan_top(uint32_t* sums, uint32_t nb) {
    __shared__ uint32_t part[kSortThreads];
    __shared__ uint32_t carry;
    const int tid = threadIdx.x;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += kSortThreads) {
        const uint32_t i = b0 + tid;
        const uint32_t v = i < nb ? sums[i] : 0u;
        part[tid] = v;
        __syncthreads();
        for (int o = 1; o < kSortThreads; o <<= 1) {
            uint32_t x = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += x;
            __syncthreads();
        }
        const uint32_t c = carry;
        if (i < nb) sums[i] = c + part[tid] - v;
        __syncthreads();
        if (tid == kSortThreads - 1) carry = c + part[tid];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(kSortThreads) k_radix_scatter(const uint64_t* in, uint64_t* out, uint64_t n, int shift,
                                                                const uint32_t* hist, const uint32_t* sums,
                                                                uint32_t ntiles) {
    __shared__ uint32_t gbase[kBins];
    __shared__ uint32_t run[kBins];
    __shared__ uint32_t wcnt[kSortWaves][kBins];
    __shared__ uint32_t wbase[kSortWaves][kBins];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    {
        const uint64_t hi = (uint64_t)tid * ntiles + blockIdx.x;
        gbase[tid] = hist[hi] + sums[hi / kScanChunk];
        run[tid] = 0;
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) wcnt[w][tid] = 0;
    }
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = base + (uint64_t)r * kSortThreads + tid;
        const bool valid = idx < n;
        const uint64_t rec = valid ? in[idx] : 0ull;
        const uint32_t d = (uint32_t)(rec >> shift) & (kBins - 1);
        const uint64_t peers = match_digit(d) & __ballot(valid);
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && lane == __builtin_ctzll(peers)) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {  // digit owner: offsets of each wave's group in this round, then advance the digit's count
            uint32_t x = run[tid];
#pragma unroll
            for (int w = 0; w < kSortWaves; ++w) {
                wbase[w][tid] = x;
                x += wcnt[w][tid];
                wcnt[w][tid] = 0;
            }
            run[tid] = x;
        }
        __syncthreads();
        if (valid) out[(uint64_t)gbase[d] + wbase[wave][d] + rank] = rec;
    }
}

size_t radix_hist_words(uint64_t n) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const uint64_t words = ntiles * kBins;
    const uint64_t nb = (words + kScanChunk - 1) / kScanChunk;
    return (size_t)(words + nb + 64);
}

// Sorts n records on bits [lo_bit, hi_bit) in passes of 8 bits (bits above hi_bit must be zero or
// already grouped), ping-ponging between a and b.
// Returns the buffer that holds the result through *result.
hipError_t radix_sort_records(uint64_t* a, uint64_t* b, uint64_t n, int lo_bit, uint32_t* hist_ws,
                              uint64_t** result, hipStream_t stream, int hi_bit) {
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    const uint64_t words = (uint64_t)ntiles * kBins;
    const uint32_t nb = (uint32_t)((words + kScanChunk - 1) / kScanChunk);
    uint32_t* hist = hist_ws;
    uint32_t* sums = hist_ws + words;
    uint64_t* src = a;
    uint64_t* dst = b;
    for (int shift = lo_bit; shift < hi_bit; shift += kRadixBits) {
        hipLaunchKernelGGL(k_radix_hist, dim3(ntiles), dim3(kSortThreads), 0, stream, src, n, shift, hist, ntiles);
        hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(kSortThreads), 0, stream, hist, words, sums);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kSortThreads), 0, stream, sums, nb);
        hipLaunchKernelGGL(k_radix_scatter, dim3(ntiles), dim3(kSortThreads), 0, stream, src, dst, n, shift, hist,
                           sums, ntiles);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *result = src;
    return hipGetLastError();
}

}  // namespace sg
