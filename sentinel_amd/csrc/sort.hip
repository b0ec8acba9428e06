// sort.hip — stable LSD radix sort of the 64-bit request records by their key field.
//
// The walkers need each key's requests contiguous and still in (timestamp, arrival) order, i.e. a stable
// partition by key. Records are sorted on bits [lo_bit, hi_bit) in 8-bit digits, or two 10-bit digits for
// 17..20-bit keys (the C3 flowIds: one pass of traffic fewer than three 8-bit passes), reduce-then-scan per
// pass (no inter-block look-back: the 8 XCDs' L2s are not coherent, so a chained scan pays an uncached
// round trip per link — measured 149 µs per pass against 77 µs for this scheme):
//   k_radix_hist     per 4096-record tile: digit histogram (LDS atomics), one contiguous row per tile [tiles][bins]
//                    (k_prep counts the first pass's row itself)
//   k_colsum, k_chunkscan, k_rescan   exclusive scan of those rows in (digit, tile) order: the global start of
//                    every tile's run of every digit, written over the rows in place
//   k_radix_scatter  per tile: each wave ranks its contiguous 1024 records, 64 at a time, against a
//                    wave-private running count per digit (match-any ballots give the rank among equal
//                    digits of a round; no block barrier inside the loop), then the records are placed
//                    digit-sorted in LDS and written in that order (consecutive lanes → consecutive addresses
//                    of one digit's run); tiles are dealt to XCDs in contiguous ranges, so the partial lines
//                    two adjacent tiles share in a digit's run are completed in one L2.
// Stability: waves in index order within a tile, rounds then lanes within a wave.
#include "engine.h"

#include <cstdlib>
#include <type_traits>

namespace sg {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kRounds = 16;
constexpr int kTile = kSortThreads * kRounds;  // 4096 records per tile
constexpr int kWaveRecs = kTile / kSortWaves;  // 1024 contiguous records per wave
constexpr int kMaxDigit = 10;                  // widest digit (1024 bins)

// Lanes of this wave whose D-bit `digit` equals this lane's (D ballots).
template <int D>
__device__ __forceinline__ uint64_t match_digit(uint32_t digit) {
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < D; ++b) {
        const uint64_t m = __ballot((digit >> b) & 1u);
        peers &= ((digit >> b) & 1u) ? m : ~m;
    }
    return peers;
}

// XCD-aware tile order for the scatter: blocks are dealt round-robin over the 8 XCDs (observed dispatch, a speed
// matter only), so block b takes tile (b % 8) * per + b / 8 and every XCD scatters a contiguous range of tiles.
// Adjacent tiles' runs of one digit are adjacent in the output: their shared partial lines meet in one L2.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles) {
    const uint32_t per = (ntiles + 7) / 8;
    return (b % 8) * per + b / 8;
}

template <int D>
__global__ void __launch_bounds__(kSortThreads) k_radix_hist(const uint64_t* in, uint64_t n, int shift, uint32_t* hist,
                                                             uint32_t ntiles, uint32_t* csum) {
    constexpr int kBins = 1 << D;
    constexpr int kPer = kBins / kSortThreads;
    __shared__ uint32_t cnt[kBins];
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < kPer; ++i) cnt[tid + i * kSortThreads] = 0;
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
#pragma unroll
    for (int i = 0; i < kPer; ++i) hist[(size_t)blockIdx.x * kBins + tid + i * kSortThreads] = cnt[tid + i * kSortThreads];
    if (csum) {  // the chunk's column sums (zeroed before the launch)
        uint32_t* cs = csum + (size_t)(blockIdx.x / kChunkTiles) * kBins;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint32_t v = cnt[tid + i * kSortThreads];
            if (v) atomicAdd(cs + tid + i * kSortThreads, v);
        }
    }
}

// The per-tile histograms are stored tile-major (hist[t][d]: each tile writes and reads one contiguous row); the
// scatter needs each (tile, digit) run's global start, the exclusive scan in (digit, tile) order. In the pipelined
// flow path these kernels run beside the previous batch's walkers, whose random traffic stretches every dependent
// memory round trip to ~20-30 µs (measured: a 4-way longer chunk-scan chain took 4x as long there), so each kernel
// issues all of a thread's loads at once and costs one load round trip:
//   k_colsum    one thread per (chunk of kChunkTiles tiles, digit): the chunk's column sums;
//   k_chunkscan 64 digits x 16 chunk groups per block: column-relative exclusive scan of the chunk sums in place,
//               and each digit's total (tot[d]);
//   k_rescan    one thread per (chunk, digit): each tile's run start (column-relative) written over its row;
//   k_radix_scatter adds each digit's base, an exclusive scan of the totals it does in LDS.
constexpr int kScanGroups = 16;  // chunk groups per digit in k_chunkscan
constexpr int kScanLoads = 8;    // chunk sums per thread loaded at once (nchunks <= 128: 16M-record batches)

template <int D>
__global__ void __launch_bounds__(1 << D) k_colsum(const uint32_t* hist, uint32_t ntiles, uint32_t* csum) {
    constexpr int kBins = 1 << D;
    const uint32_t t0 = blockIdx.x * kChunkTiles, nt = min(kChunkTiles, ntiles - t0);
    const int d = threadIdx.x;
    uint32_t v[kChunkTiles];
#pragma unroll
    for (uint32_t u = 0; u < kChunkTiles; ++u) v[u] = hist[(size_t)(t0 + min(u, nt - 1)) * kBins + d];
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t u = 0; u < kChunkTiles; ++u) acc += u < nt ? v[u] : 0u;
    csum[(size_t)blockIdx.x * kBins + d] = acc;
}

template <int D>
__global__ void __launch_bounds__(1024) k_chunkscan(uint32_t* csum, uint32_t nchunks, uint32_t* tot) {
    constexpr int kBins = 1 << D;
    __shared__ uint32_t gs[kScanGroups][64];
    const int dl = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int d = blockIdx.x * 64 + dl;
    const uint32_t G = (nchunks + kScanGroups - 1) / kScanGroups;  // chunks per group
    const uint32_t c0 = grp * G, c1 = min(c0 + G, nchunks);
    const uint32_t last = nchunks - 1;
    uint32_t v[kScanLoads];
    uint32_t sum = 0;
    for (uint32_t b0 = c0; b0 < c1; b0 += kScanLoads) {
#pragma unroll
        for (int u = 0; u < kScanLoads; ++u) v[u] = csum[(size_t)min(b0 + u, last) * kBins + d];
#pragma unroll
        for (int u = 0; u < kScanLoads; ++u) sum += b0 + u < c1 ? v[u] : 0u;
    }
    gs[grp][dl] = sum;
    __syncthreads();
    if (grp == 0) {  // exclusive scan over the groups of digit d, and its total
        uint32_t run = 0;
#pragma unroll
        for (int g = 0; g < kScanGroups; ++g) {
            const uint32_t x = gs[g][dl];
            gs[g][dl] = run;
            run += x;
        }
        tot[d] = run;
    }
    __syncthreads();
    uint32_t run = gs[grp][dl];
    for (uint32_t b0 = c0; b0 < c1; b0 += kScanLoads) {
        if (b0 != c0) {  // more than kScanLoads chunks per group (batches > 16M records): reload
#pragma unroll
            for (int u = 0; u < kScanLoads; ++u) v[u] = csum[(size_t)min(b0 + u, last) * kBins + d];
        } else if (G > (uint32_t)kScanLoads) {
#pragma unroll
            for (int u = 0; u < kScanLoads; ++u) v[u] = csum[(size_t)min(b0 + u, last) * kBins + d];
        }
#pragma unroll
        for (int u = 0; u < kScanLoads; ++u) {
            if (b0 + u < c1) {
                csum[(size_t)(b0 + u) * kBins + d] = run;
                run += v[u];
            }
        }
    }
}

template <int D>
__global__ void __launch_bounds__(1 << D) k_rescan(uint32_t* hist, const uint32_t* csum, uint32_t ntiles) {
    constexpr int kBins = 1 << D;
    const uint32_t t0 = blockIdx.x * kChunkTiles, nt = min(kChunkTiles, ntiles - t0);
    const int d = threadIdx.x;
    uint32_t run = csum[(size_t)blockIdx.x * kBins + d];
    uint32_t v[kChunkTiles];
#pragma unroll
    for (uint32_t u = 0; u < kChunkTiles; ++u) v[u] = hist[(size_t)(t0 + min(u, nt - 1)) * kBins + d];
#pragma unroll
    for (uint32_t u = 0; u < kChunkTiles; ++u) {
        if (u < nt) hist[(size_t)(t0 + u) * kBins + d] = run;
        run += v[u];  // (past nt: unused)
    }
}

// MARK (the last pass of a sort whose key is a flowId index, SegMark): besides the records, each key's segment in
// the sorted output — within a digit's run of the tile the records are sorted by the whole key, so the first and
// last record of every key in the run are found by comparing LDS neighbours; the segment's start is the smallest of
// its runs' firsts (atomicMin on seg_start, 0xFFFFFFFF between batches) and its end the largest of their lasts + 1
// (atomicMax on seg_end, 0 between batches; k_seg_classify consumes and clears both). This replaces a separate pass
// over the sorted records (k_seg_mark).
// BIN (the binned front half's one pass, engine.h kBinDigit): the digit is the bin digit k_prep wrote into the
// record's middle bits; it is cleared on the way out, and the records of regular bins (digit < R) go to `reg` (k_bin_sort
// sorts them from there into `out`), the hot bins' and rejected requests' records to `out`, at the same positions.
struct BinSplit {
    uint64_t* reg;
    uint32_t R;
};

template <int D, bool MARK>
__global__ void __launch_bounds__(kSortThreads) k_radix_scatter(const uint64_t* in, uint64_t* out, uint64_t n, int shift,
                                                                const uint32_t* hist, uint32_t ntiles,
                                                                const uint32_t* tot, SegMark mk, BinSplit bs) {
    constexpr int kBins = 1 << D;
    constexpr int kPer = kBins / kSortThreads;  // digits per thread
    using Cnt = typename std::conditional<(D > 8), uint16_t, uint32_t>::type;  // wave counts <= 1024
    __shared__ uint64_t stage[kTile];
    __shared__ Cnt wcnt[kSortWaves][kBins];  // per-wave running digit count, then per-wave base
    __shared__ uint32_t dstart[kBins];       // tile-local start of each digit's run
    __shared__ uint32_t gbase[kBins];        // global start of each digit's run of this tile
    __shared__ uint32_t wtot[kSortWaves];
    __shared__ uint32_t btot[kSortWaves];
    const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
    if (tile >= ntiles) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t tv[kPer];  // totals of digits tid*kPer .. (k_chunkscan)
#pragma unroll
    for (int i = 0; i < kPer; ++i) tv[i] = tot[tid * kPer + i];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int d = tid + i * kSortThreads;
        gbase[d] = hist[(size_t)tile * kBins + d];  // the tile's row of column-relative run offsets (k_rescan)
#pragma unroll
        for (int w = 0; w < kSortWaves; ++w) wcnt[w][d] = 0;
    }
    // digit bases: exclusive scan of the totals (digits tid*kPer .. contiguous per thread), added after the barrier
    uint32_t bsum = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) bsum += tv[i];
    uint32_t bx = bsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)bx, (unsigned)o, 64);
        if (lane >= o) bx += y;
    }
    if (lane == 63) btot[wave] = bx;
    const uint64_t base = (uint64_t)tile * kTile;
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
    {
        uint32_t b = bx - bsum;
        for (int w = 0; w < wave; ++w) b += btot[w];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            gbase[tid * kPer + i] += b;
            b += tv[i];
        }
    }
    // 1. rank within the wave (wave-private counters: LDS ops of one wave execute in order)
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const bool valid = wbase + (uint64_t)r * 64 + lane < n;
        const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
        const uint64_t peers = match_digit<D>(d) & __ballot(valid);
        const uint32_t c = wcnt[wave][d];
        rank[r] = c + (uint32_t)__popcll(peers & lt);
        if (valid && lane == __builtin_ctzll(peers)) wcnt[wave][d] = (Cnt)(c + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    // 2. digits tid*kPer .. +kPer-1: per-wave bases, tile totals, tile-local digit starts (block scan)
    {
        uint32_t tot[kPer], sum = 0;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int d = tid * kPer + i;
            uint32_t t = 0;
#pragma unroll
            for (int w = 0; w < kSortWaves; ++w) {
                const uint32_t c = wcnt[w][d];
                wcnt[w][d] = (Cnt)t;
                t += c;
            }
            tot[i] = t;
            sum += t;
        }
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[wave] = x;
        __syncthreads();
        uint32_t off = x - sum;
        for (int w = 0; w < wave; ++w) off += wtot[w];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            dstart[tid * kPer + i] = off;
            off += tot[i];
        }
    }
    __syncthreads();
    // 3. place the records digit-sorted in LDS
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if (wbase + (uint64_t)r * 64 + lane < n) {
            const uint32_t d = (uint32_t)(rec[r] >> shift) & (kBins - 1);
            stage[dstart[d] + (uint32_t)wcnt[wave][d] + rank[r]] = rec[r];
        }
    }
    __syncthreads();
    // 4. write out in digit order
    const uint32_t cnt = (uint32_t)min((uint64_t)kTile, n - base);
    const uint64_t keep = bs.reg ? ~((uint64_t)(kBins - 1) << shift) : ~0ull;
    for (uint32_t p = tid; p < cnt; p += kSortThreads) {
        const uint64_t v = stage[p];
        const uint32_t d = (uint32_t)(v >> shift) & (kBins - 1);
        const uint32_t gp = gbase[d] + (p - dstart[d]);
        (bs.reg && d < bs.R ? bs.reg : out)[gp] = v & keep;
        if constexpr (MARK) {
            const uint32_t k = (uint32_t)(v >> mk.kshift);
            if (k < mk.K) {
                const uint32_t r0 = dstart[d];
                const uint32_t r1 = d + 1 < (uint32_t)kBins ? dstart[d + 1] : cnt;  // the digit's run in the tile
                if (p == r0 || (uint32_t)(stage[p - 1] >> mk.kshift) != k) atomicMin(mk.seg_start + k, gp);
                if (p + 1 == r1 || (uint32_t)(stage[p + 1] >> mk.kshift) != k) atomicMax(mk.seg_end + k, gp + 1);
            }
        }
    }
}

bool radix_csum_atomic() {  // read per sort (a getenv per batch): tests switch it per engine
    const char* e = std::getenv("SG_CSUM_ATOMIC");
    return e ? std::atoi(e) != 0 : true;
}

uint32_t* radix_csum(uint32_t* hist_ws, uint64_t n, int D) {
    return hist_ws + (size_t)((n + kTile - 1) / kTile) * (1u << D);
}

size_t radix_csum_bytes(uint64_t n, int D) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    return sizeof(uint32_t) * (size_t)((ntiles + kChunkTiles - 1) / kChunkTiles) * (1u << D);
}

size_t radix_hist_words(uint64_t n) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const uint64_t nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    return (size_t)((ntiles + nchunks + 1) * (1ull << kMaxDigit) + 64);  // rows, chunk sums, digit totals
}

// Digit width of a sort over `bits` key bits: 8-bit digits, except 10-bit ones where they save a pass: 2 passes for
// 17..20 bits (the C3 flowIds), 3 for 25..30 (hot-parameter value slots) instead of 3 / 4 8-bit passes.
int radix_digit_bits(int bits) { return ((bits > 16 && bits <= 20) || (bits > 24 && bits <= 30)) ? 10 : 8; }

template <int D>
static hipError_t radix_pass(uint64_t* src, uint64_t* dst, uint64_t n, int shift, uint32_t* hist_ws, hipStream_t stream,
                       bool hist_ready, const SegMark* mark, bool csum_ready, BinSplit bs = BinSplit{}) {
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    const uint32_t nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    uint32_t* hist = hist_ws;                                   // [ntiles][bins], then run offsets in place
    uint32_t* csum = hist_ws + (size_t)ntiles * (1u << D);       // [nchunks][bins]
    uint32_t* tot = csum + (size_t)nchunks * (1u << D);          // [bins]
    if (!hist_ready) {
        const bool atom = radix_csum_atomic();
        if (atom) {
            const hipError_t e = hipMemsetAsync(csum, 0, radix_csum_bytes(n, D), stream);
            if (e != hipSuccess) return e;
        }
        lds_poison(stream);
        hipLaunchKernelGGL(k_radix_hist<D>, dim3(ntiles), dim3(kSortThreads), 0, stream, src, n, shift, hist, ntiles,
                           atom ? csum : nullptr);
        csum_ready = atom;
    }
    if (!csum_ready) hipLaunchKernelGGL(k_colsum<D>, dim3(nchunks), dim3(1u << D), 0, stream, hist, ntiles, csum);
    hipLaunchKernelGGL(k_chunkscan<D>, dim3((1u << D) / 64), dim3(1024), 0, stream, csum, nchunks, tot);
    hipLaunchKernelGGL(k_rescan<D>, dim3(nchunks), dim3(1u << D), 0, stream, hist, csum, ntiles);
    const uint32_t grid = 8 * ((ntiles + 7) / 8);  // xcd_tile: blocks past ntiles return at once
    lds_poison(stream);
    if (mark)
        hipLaunchKernelGGL((k_radix_scatter<D, true>), dim3(grid), dim3(kSortThreads), 0, stream, src, dst, n, shift,
                           hist, ntiles, tot, *mark, BinSplit{});
    else
        hipLaunchKernelGGL((k_radix_scatter<D, false>), dim3(grid), dim3(kSortThreads), 0, stream, src, dst, n, shift,
                           hist, ntiles, tot, SegMark{}, bs);
    return hipGetLastError();
}

// The digit totals radix_pass<D> leaves in hist_ws (k_chunkscan), [1 << D].
const uint32_t* radix_tot(const uint32_t* hist_ws, uint64_t n, int D) {
    const uint64_t ntiles = (n + kTile - 1) / kTile;
    const uint64_t nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    return hist_ws + (size_t)(ntiles + nchunks) * (1ull << D);
}

// The binned front half's scatter pass (engine.h kBinDigit): records by bin digit at bit `shift`, regular bins
// (digit < R) into `reg`, the rest into `out`.
hipError_t radix_bin_pass(uint64_t* src, uint64_t* out, uint64_t* reg, uint32_t R, uint64_t n, int shift,
                          uint32_t* hist_ws, bool hist_ready, bool csum_ready, hipStream_t stream) {
    static_assert(kBinDigit == 10, "radix_pass<10>");
    return radix_pass<10>(src, out, n, shift, hist_ws, stream, hist_ready, nullptr, csum_ready, BinSplit{reg, R});
}

// Sorts n records on bits [lo_bit, hi_bit) (bits above hi_bit must be zero or already grouped),
// ping-ponging between a and b. Returns the buffer that holds the result through *result.
// first_hist_ready: the first pass's per-tile histogram (radix_digit_bits wide) is already in hist_ws (k_prep).
hipError_t radix_sort_records(uint64_t* a, uint64_t* b, uint64_t n, int lo_bit, uint32_t* hist_ws,
                              uint64_t** result, hipStream_t stream, int hi_bit, bool first_hist_ready,
                              const SegMark* mark, bool first_csum_ready) {
    uint64_t* src = a;
    uint64_t* dst = b;
    const int D = radix_digit_bits(hi_bit - lo_bit);
    for (int shift = lo_bit; shift < hi_bit && n > 0; shift += D) {
        const bool ready = shift == lo_bit && first_hist_ready;
        const SegMark* mk = shift + D >= hi_bit ? mark : nullptr;  // the last pass marks the segments
        const bool cready = ready && first_csum_ready;
        const hipError_t e = D == 10 ? radix_pass<10>(src, dst, n, shift, hist_ws, stream, ready, mk, cready)
                                     : radix_pass<8>(src, dst, n, shift, hist_ws, stream, ready, mk, cready);
        if (e != hipSuccess) return e;
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    *result = src;
    return hipGetLastError();
}

}  // namespace sg
