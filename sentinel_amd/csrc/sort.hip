// sort.hip — stable LSD radix sort of the 64-bit request records by their key field.
//
// The walkers need each key's requests contiguous and still in (timestamp, arrival) order, i.e. a stable
// partition by key. Records are sorted on bits [lo_bit, hi_bit) only, in as few passes as possible:
// digits of 8 bits, or of 10 bits when that saves a pass (a 20-bit key: 2 passes instead of 3).
//   k_radix_hist     per 4096-record tile: digit histogram (wave match-any aggregation, then LDS)
//   k_scan_*         exclusive scan of the digit-major histogram [bins][tiles]
//   k_radix_scatter  per tile, 16 rounds of 256 records in index order: wave match-any gives each record
//                    its rank among equal digits in its wave, an LDS prefix over the 4 waves and the
//                    running per-digit count give its rank in the tile; records are placed digit-sorted
//                    in LDS and written out in that order (consecutive lanes → consecutive addresses of one
//                    digit's run: coalesced stores, no partial-line write amplification).
// Stability follows from ranking strictly in index order (rounds, then waves, then lanes).
#include "engine.h"

namespace sg {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRounds = 16;
constexpr int kTile = kSortThreads * kRounds;  // 4096 records per tile
constexpr int kScanItems = 8;
constexpr int kScanChunk = kSortThreads * kScanItems;  // 2048 counters per scan block
constexpr int kMaxBins = 1024;
constexpr bool kSortWideDigits = false;

// Lanes of this wave whose `digit` equals this lane's (RB ballots).
template <int RB>
__device__ __forceinline__ uint64_t match_digit(uint32_t digit) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < RB; ++b) {
        const uint64_t m = __ballot((digit >> b) & 1u);
        peers &= ((digit >> b) & 1u) ? m : ~m;
    }
    return peers;
}

template <int RB>
__global__ void __launch_bounds__(kSortThreads) k_radix_hist(const uint64_t* in, uint64_t n, int shift, uint32_t* hist,
                                                             uint32_t ntiles) {
    constexpr int kBins = 1 << RB;
    __shared__ uint32_t cnt[kBins];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    for (int d = tid; d < kBins; d += kSortThreads) cnt[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    uint64_t rec[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = base + (uint64_t)r * kSortThreads + tid;
        rec[r] = idx < n ? in[idx] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const bool valid = base + (uint64_t)r * kSortThreads + tid < n;
        const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
        const uint64_t peers = match_digit<RB>(d) & __ballot(valid);
        if (valid && lane == __builtin_ctzll(peers)) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    for (int d = tid; d < kBins; d += kSortThreads) hist[(size_t)d * ntiles + blockIdx.x] = cnt[d];
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

template <int RB>
__global__ void __launch_bounds__(kSortThreads) k_radix_scatter(const uint64_t* in, uint64_t* out, uint64_t n, int shift,
                                                                const uint32_t* hist, const uint32_t* sums,
                                                                uint32_t ntiles) {
    constexpr int kBins = 1 << RB;
    constexpr int kPer = kBins / kSortThreads;  // digits owned per thread
    __shared__ uint64_t stage[kTile];
    __shared__ uint32_t gbase[kBins];  // global start of each digit's run for this tile
    __shared__ uint32_t run[kBins];    // running count per digit, then the tile-local digit start
    __shared__ uint32_t wcnt[kSortWaves][kBins];
    __shared__ uint32_t wbase[kSortWaves][kBins];
    __shared__ uint32_t wtot[kSortWaves];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int d = tid * kPer + i;
        const uint64_t hi = (uint64_t)d * ntiles + blockIdx.x;
        gbase[d] = hist[hi] + sums[hi / kScanChunk];
        run[d] = 0;
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) wcnt[w][d] = 0;
    }
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t rec[kRounds];
    uint32_t rank[kRounds];  // rank among the tile's records of the same digit (bit 31: invalid)
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint64_t idx = base + (uint64_t)r * kSortThreads + tid;
        rec[r] = idx < n ? in[idx] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const bool valid = base + (uint64_t)r * kSortThreads + tid < n;
        const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
        const uint64_t peers = match_digit<RB>(d) & __ballot(valid);
        const uint32_t wr = (uint32_t)__popcll(peers & lt);
        if (valid && lane == __builtin_ctzll(peers)) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kPer; ++i) {  // digit owner: offsets of each wave's group in this round
            const int dd = tid * kPer + i;
            uint32_t x = run[dd];
#pragma unroll
            for (int w = 0; w < kSortWaves; ++w) {
                wbase[w][dd] = x;
                x += wcnt[w][dd];
                wcnt[w][dd] = 0;
            }
            run[dd] = x;
        }
        __syncthreads();
        rank[r] = valid ? wbase[wave][d] + wr : 0x80000000u;
    }
    // tile-local digit starts: exclusive scan of the per-digit totals over the digits (kPer per thread)
    {
        uint32_t v[kPer], t = 0;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            v[i] = run[tid * kPer + i];
            t += v[i];
        }
        uint32_t x = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[wave] = x;
        __syncthreads();
        uint32_t off = x - t;
        for (int w = 0; w < wave; ++w) off += wtot[w];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            run[tid * kPer + i] = off;
            off += v[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r)
        if (!(rank[r] & 0x80000000u)) stage[run[(uint32_t)(rec[r] >> shift) & (kBins - 1)] + rank[r]] = rec[r];
    __syncthreads();
    const uint32_t cnt = (uint32_t)min((uint64_t)kTile, n - base);
    for (uint32_t p = tid; p < cnt; p += kSortThreads) {
        const uint64_t v = stage[p];
        const uint32_t d = (uint32_t)(v >> shift) & (kBins - 1);
        out[(uint64_t)gbase[d] + (p - run[d])] = v;
    }
}

size_t radix_hist_words(uint64_t n) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const uint64_t words = ntiles * kMaxBins;
    const uint64_t nb = (words + kScanChunk - 1) / kScanChunk;
    return (size_t)(words + nb + 64);
}

template <int RB>
static void radix_pass(uint64_t* src, uint64_t* dst, uint64_t n, int shift, uint32_t* hist_ws, hipStream_t stream) {
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    const uint64_t words = (uint64_t)ntiles << RB;
    const uint32_t nb = (uint32_t)((words + kScanChunk - 1) / kScanChunk);
    uint32_t* hist = hist_ws;
    uint32_t* sums = hist_ws + words;
    hipLaunchKernelGGL(k_radix_hist<RB>, dim3(ntiles), dim3(kSortThreads), 0, stream, src, n, shift, hist, ntiles);
    hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(kSortThreads), 0, stream, hist, words, sums);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kSortThreads), 0, stream, sums, nb);
    hipLaunchKernelGGL(k_radix_scatter<RB>, dim3(ntiles), dim3(kSortThreads), 0, stream, src, dst, n, shift, hist, sums,
                       ntiles);
}

// Sorts n records on bits [lo_bit, hi_bit) (bits above hi_bit must be zero or already grouped),
// ping-ponging between a and b. Returns the buffer that holds the result through *result.
hipError_t radix_sort_records(uint64_t* a, uint64_t* b, uint64_t n, int lo_bit, uint32_t* hist_ws,
                              uint64_t** result, hipStream_t stream, int hi_bit) {
    uint64_t* src = a;
    uint64_t* dst = b;
    const int bits = hi_bit - lo_bit;
    // 10-bit digits only when they take fewer passes than 8-bit ones AND the caller asks: on MI355X the
    // 1024-bin scatter (72 KB LDS, 2 blocks/CU) costs more per pass than it saves in passes at 16M records
    // (C3: 2 x 10-bit 0.55 ms vs 3 x 8-bit 0.40 ms)
    const bool wide = kSortWideDigits && bits > 0 && (bits + 9) / 10 < (bits + 7) / 8;
    const int step = wide ? 10 : 8;
    for (int shift = lo_bit; shift < hi_bit; shift += step) {
        if (wide) radix_pass<10>(src, dst, n, shift, hist_ws, stream);
        else radix_pass<8>(src, dst, n, shift, hist_ws, stream);
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *result = src;
    return hipGetLastError();
}

}  // namespace sg
