// sort.hip — stable LSD radix sort of the 64-bit request records by their key field.
//
// The walkers need each key's requests contiguous and still in (timestamp, arrival) order, i.e. a stable
// partition by key. Records are sorted on bits [lo_bit, hi_bit) in 8-bit digits, reduce-then-scan per
// pass (no inter-block look-back: the 8 XCDs' L2s are not coherent, so a chained scan pays an uncached
// round trip per link — measured 149 µs per pass against 77 µs for this scheme):
//   k_radix_hist     per 4096-record tile: digit histogram (LDS atomics), stored digit-major [bins][tiles]
//   k_scan_*         exclusive scan of that histogram (the global position of each tile's digit run)
//   k_radix_scatter  per tile: each wave ranks its contiguous 1024 records, 64 at a time, against a
//                    wave-private running count per digit (match-any ballots give the rank among equal
//                    digits of a round; no block barrier inside the loop), then the records are placed
//                    digit-sorted in LDS and written in that order (consecutive lanes → consecutive addresses
//                    of one digit's run: coalesced stores, no partial-line write amplification).
// Stability: waves in index order within a tile, rounds then lanes within a wave.
#include "engine.h"

namespace sg {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRounds = 16;
constexpr int kTile = kSortThreads * kRounds;  // 4096 records per tile
constexpr int kWaveRecs = kTile / kSortWaves;  // 1024 contiguous records per wave
constexpr int kBins = 256;                     // 8-bit digits; one digit per thread
constexpr int kScanItems = 8;
constexpr int kScanChunk = kSortThreads * kScanItems;  // 2048 counters per scan block
static_assert(kBins == kSortThreads, "one digit per thread");

// Lanes of this wave whose `digit` equals this lane's (8 ballots).
__device__ __forceinline__ uint64_t match_digit(uint32_t digit) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint64_t m = __ballot((digit >> b) & 1u);
        peers &= ((digit >> b) & 1u) ? m : ~m;
    }
    return peers;
}

__global__ void __launch_bounds__(kSortThreads) k_radix_hist(const uint64_t* in, uint64_t n, int shift, uint32_t* hist,
                                                             uint32_t ntiles) {
    __shared__ uint32_t cnt[kBins];
    const int tid = threadIdx.x;
    cnt[tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    uint64_t rec[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = base + (uint64_t)r * kSortThreads + tid;
        rec[r] = idx < n ? in[idx] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r)
        if (base + (uint64_t)r * kSortThreads + tid < n) atomicAdd(&cnt[(uint32_t)(rec[r] >> shift) & (kBins - 1)], 1u);
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
    __shared__ uint64_t stage[kTile];
    __shared__ uint32_t wcnt[kSortWaves][kBins];  // per-wave running digit count, then per-wave base
    __shared__ uint32_t dstart[kBins];            // tile-local start of each digit's run
    __shared__ uint32_t gbase[kBins];             // global start of each digit's run of this tile
    __shared__ uint32_t wtot[kSortWaves];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    {
        const uint64_t hi = (uint64_t)tid * ntiles + blockIdx.x;
        gbase[tid] = hist[hi] + sums[hi / kScanChunk];
    }
#pragma unroll
    for (int w = 0; w < kSortWaves; ++w) wcnt[w][tid] = 0;
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    const uint64_t wbase = base + (uint64_t)wave * kWaveRecs;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t rec[kRounds];
    uint32_t rank[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = wbase + (uint64_t)r * 64 + lane;
        rec[r] = idx < n ? in[idx] : 0ull;
    }
    __syncthreads();
    // 1. rank within the wave (wave-private counters: LDS ops of one wave execute in order)
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const bool valid = wbase + (uint64_t)r * 64 + lane < n;
        const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
        const uint64_t peers = match_digit(d) & __ballot(valid);
        const uint32_t c = wcnt[wave][d];
        rank[r] = c + (uint32_t)__popcll(peers & lt);
        if (valid && lane == __builtin_ctzll(peers)) wcnt[wave][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // 2. digit `tid`: per-wave bases, tile total, tile-local digit start (block scan over the digits)
    {
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) {
            const uint32_t c = wcnt[w][tid];
            wcnt[w][tid] = tot;
            tot += c;
        }
        uint32_t x = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[wave] = x;
        __syncthreads();
        uint32_t off = x - tot;
        for (int w = 0; w < wave; ++w) off += wtot[w];
        dstart[tid] = off;
    }
    __syncthreads();
    // 3. place the records digit-sorted in LDS
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if (wbase + (uint64_t)r * 64 + lane < n) {
            const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
            stage[dstart[d] + wcnt[wave][d] + rank[r]] = rec[r];
        }
    }
    __syncthreads();
    // 4. write out in digit order
    const uint32_t cnt = (uint32_t)min((uint64_t)kTile, n - base);
    for (uint32_t p = tid; p < cnt; p += kSortThreads) {
        const uint64_t v = stage[p];
        const uint32_t d = (uint32_t)(v >> shift) & (kBins - 1);
        out[(uint64_t)gbase[d] + (p - dstart[d])] = v;
    }
}

size_t radix_hist_words(uint64_t n) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const uint64_t words = ntiles * kBins;
    const uint64_t nb = (words + kScanChunk - 1) / kScanChunk;
    return (size_t)(words + nb + 64);
}

static void radix_pass(uint64_t* src, uint64_t* dst, uint64_t n, int shift, uint32_t* hist_ws, hipStream_t stream,
                       bool hist_ready) {
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    const uint64_t words = (uint64_t)ntiles * kBins;
    const uint32_t nb = (uint32_t)((words + kScanChunk - 1) / kScanChunk);
    uint32_t* hist = hist_ws;
    uint32_t* sums = hist_ws + words;
    if (!hist_ready)
        hipLaunchKernelGGL(k_radix_hist, dim3(ntiles), dim3(kSortThreads), 0, stream, src, n, shift, hist, ntiles);
    hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(kSortThreads), 0, stream, hist, words, sums);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kSortThreads), 0, stream, sums, nb);
    hipLaunchKernelGGL(k_radix_scatter, dim3(ntiles), dim3(kSortThreads), 0, stream, src, dst, n, shift, hist, sums,
                       ntiles);
}

// Sorts n records on bits [lo_bit, hi_bit) (bits above hi_bit must be zero or already grouped),
// ping-ponging between a and b. Returns the buffer that holds the result through *result.
// first_hist_ready: the first pass's per-tile histogram is already in hist_ws (k_prep counted it).
hipError_t radix_sort_records(uint64_t* a, uint64_t* b, uint64_t n, int lo_bit, uint32_t* hist_ws,
                              uint64_t** result, hipStream_t stream, int hi_bit, bool first_hist_ready) {
    uint64_t* src = a;
    uint64_t* dst = b;
    for (int shift = lo_bit; shift < hi_bit && n > 0; shift += 8) {
        radix_pass(src, dst, n, shift, hist_ws, stream, shift == lo_bit && first_hist_ready);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *result = src;
    return hipGetLastError();
}

}  // namespace sg
