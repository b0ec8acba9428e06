// search_dev.h — device helpers shared by the walkers: wave-wide searches over the sorted records, the window
// average's division.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sg {

// First q in [lo, hi) with pred(q) (pred monotone false → true), hi if none: 64 evenly spaced probes per step.
template <class Pred>
__device__ __forceinline__ uint64_t search64(uint64_t lo, uint64_t hi, Pred pred, int lane) {
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t q = lo + (uint64_t)lane * step;
        const uint64_t m = __ballot(q >= hi || pred(q));
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
    const uint64_t q = lo + (uint64_t)lane;
    const uint64_t m = __ballot(q < hi && pred(q));
    return m ? lo + (uint64_t)__builtin_ctzll(m) : hi;
}

// As search64 for an answer expected near lo (a segment's end seen from inside it, a window period's end): lane l
// probes lo + 2^l - 1, which brackets the answer between two probes (the first few share lo's cache line), then
// search64 inside the bracket. search64 over [lo, hi) alone spreads its first rounds over the whole range — 64 far
// cache lines per round when hi is the end of the batch.
template <class Pred>
__device__ __forceinline__ uint64_t gallop_search(uint64_t lo, uint64_t hi, Pred pred, int lane) {
    if (lo >= hi) return hi;
    const uint64_t span = hi - lo;
    const uint64_t off = lane < 63 ? (1ull << lane) - 1ull : ~0ull;
    const bool in = off < span;
    const uint64_t m = __ballot(!in || pred(lo + off));  // lane 63 is never in: m != 0
    const int f = __builtin_ctzll(m);
    if (f == 0) return lo;
    const uint64_t b0 = lo + (1ull << (f - 1));            // probe f - 1 (at b0 - 1) was false
    const uint64_t b1 = lo + ((1ull << f) - 1ull);          // probe f: true, or past hi
    return search64(b0, b1 < hi ? b1 : hi, pred, lane);
}

// sum / intervalInSecond (LeapArray averages: ClusterMetric.getAvg, StatisticNode.passQps, …) as Java computes it.
// For a power-of-two interval (1 s, 2 s, 0.5 s, …) the quotient is the product with the exact reciprocal, built from
// the exponent bits; the fp64 division sequence (~13 instructions a record on the walkers' hot path) runs only
// for other intervals. (A test for isec == 1.0 alone is folded away by the compiler: x / 1.0 == x.)
__device__ __forceinline__ double avg_div(double x, double isec) {
#ifdef SG_NO_AVGDIV
    return x / isec;
#endif
    const uint64_t b = (uint64_t)__double_as_longlong(isec);
    const uint64_t e = (b >> 52) & 0x7FF;
    if ((b & 0x800FFFFFFFFFFFFFull) == 0 && e - 1 < 0x7FD)
        return x * __longlong_as_double((long long)((0x7FEull - e) << 52));
    return x / isec;
}

// Streaming stores for the prep kernels' outputs (default results, packed records: written once, read by a later
// kernel): non-temporal, so a batch's front half does not fill L2 with lines the walkers beside it would have used.
// SG_NT_PREP=0 builds plain stores.
#ifndef SG_NT_PREP
#define SG_NT_PREP 1
#endif
template <class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
#if SG_NT_PREP
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

}  // namespace sg
