// conc.hip — concurrent (thread-grade) cluster tokens on the device: TokenService.requestConcurrentToken /
// releaseConcurrentToken (srv/flow/DefaultTokenService.java:66-85) → ConcurrentClusterFlowChecker
// (srv/flow/ConcurrentClusterFlowChecker.java:48-101) over CurrentConcurrencyManager's nowCalls per flowId and
// TokenCacheNodeManager's token map, and RegularExpireStrategy.clearToken
// (…/statistic/concurrent/expire/RegularExpireStrategy.java:94-137).
//
// A batch (time-ordered acquires and releases):
//   k_conc_prep    validation (BAD_REQUEST / NO_RULE_EXISTS), and every release resolved to the rule that owns
//                  its token: a token of this batch through the acquire it names (token id = base + index + 1), an
//                  older one through the token table (unknown → ALREADY_RELEASE, rule gone → NO_RULE_EXISTS);
//                  packs {rule | request index}
//   radix sort by rule (sort.hip): each rule's acquires and releases contiguous, in arrival order
//   k_conc_walk    one lane per rule: nowCalls in a register, acquire iff nowCalls + acquireCount <= threshold
//                  (int sum, double compare), releases give the count back (only this lane touches the rule's
//                  tokens, so the table needs no atomics here)
//   k_conc_insert  the batch's tokens still live at its end go into the table (CAS on the id word)
// State lives in HBM between batches: nowCalls[K] and the token table (48 B per token).
#include "engine.h"

namespace sg {

namespace {

__device__ __forceinline__ uint64_t tok_hash(uint64_t id) {  // splitmix64 finaliser
    uint64_t z = id + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t fid_hash2(int64_t fid) {
    return tok_hash((uint64_t)fid);
}

// Slot of a live token, or -1 (TokenCacheNodeManager.getTokenCacheNode)
__device__ int64_t tok_find(const ConcArgs& c, uint64_t id) {
    for (uint64_t h = tok_hash(id) & c.tmask, probes = 0; probes <= c.tmask; h = (h + 1) & c.tmask, ++probes) {
        const uint64_t s = c.tab[h].id;
        if (s == id) return c.tab[h].state == 1 ? (int64_t)h : -1;
        if (s == 0) return -1;
    }
    return -1;
}

// Rule index of a flowId (ClusterFlowRuleManager.getFlowRuleById), or -1
__device__ int64_t rule_of(const ConcArgs& c, int64_t fid) {
    if (!c.fid) return -1;
    for (uint64_t h = fid_hash2(fid) & c.fid_mask;; h = (h + 1) & c.fid_mask) {
        const FidSlot s = c.fid[h];
        if (s.fid == fid) return (int64_t)s.idx;
        if (s.fid == 0) return -1;
    }
}

__device__ __forceinline__ void put(const ConcArgs& c, uint64_t i, int32_t status, uint64_t token) {
    sg_conc_result r;
    r.status = status;
    r.reserved = 0;
    r.token_id = token;
    c.out[i] = r;
}

__device__ __forceinline__ bool acquire_valid(const sg_conc_req& q, uint32_t K) {
    const uint32_t k = q.key & SG_KEY_INDEX;
    return q.kind == SG_CONC_ACQUIRE && q.client != 0 && k != SG_KEY_BAD && q.acquire > 0 && k < K;
}

}  // namespace

__global__ void __launch_bounds__(256) k_conc_prep(ConcArgs c) {
    const uint64_t sentinel = (uint64_t)c.K << c.kshift;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const sg_conc_req q = c.req[i];
        if (q.ts_ms < 0 || (i == 0 ? q.ts_ms < *c.last_ts : q.ts_ms < c.req[i - 1].ts_ms)) atomicOr(c.err, kErrTime);
        c.alive[i] = 0;
        uint64_t rec = sentinel | i;
        if (q.kind == SG_CONC_ACQUIRE) {
            const uint32_t k = q.key & SG_KEY_INDEX;
            if (q.client == 0 || k == SG_KEY_BAD || q.acquire <= 0) put(c, i, SG_STATUS_BAD_REQUEST, 0);
            else if (k >= c.K) put(c, i, SG_STATUS_NO_RULE_EXISTS, 0);
            else rec = ((uint64_t)k << c.kshift) | i;
        } else if (q.kind == SG_CONC_RELEASE) {
            const uint64_t id = q.token_id;
            if (id == 0) {
                put(c, i, SG_STATUS_BAD_REQUEST, 0);
            } else if (id > c.base && id - c.base <= c.n) {  // a token of this batch: the acquire it names
                const uint64_t j = id - c.base - 1;
                const sg_conc_req a = c.req[j];
                if (j < i && acquire_valid(a, c.K)) rec = ((uint64_t)(a.key & SG_KEY_INDEX) << c.kshift) | i;
                else put(c, i, SG_STATUS_ALREADY_RELEASE, 0);
            } else {
                const int64_t s = tok_find(c, id);
                if (s < 0) {
                    put(c, i, SG_STATUS_ALREADY_RELEASE, 0);
                } else {
                    const int64_t r = rule_of(c, c.tab[s].flow_id);
                    if (r < 0) put(c, i, SG_STATUS_NO_RULE_EXISTS, 0);
                    else rec = ((uint64_t)r << c.kshift) | i;
                }
            }
        } else {
            put(c, i, SG_STATUS_BAD_REQUEST, 0);
        }
        c.rec[i] = rec;
    }
}

// One lane per rule segment of the sorted records.
__global__ void __launch_bounds__(256) k_conc_walk(ConcArgs c) {
    if (*c.err) return;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < c.n; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r0 = c.rec_sorted[p];
        const uint32_t k = (uint32_t)(r0 >> c.kshift);
        if (k >= c.K || (p > 0 && (uint32_t)(c.rec_sorted[p - 1] >> c.kshift) == k)) continue;
        int32_t now = c.now[k];
        const double thr = c.thr[k];
        for (uint64_t q = p; q < c.n; ++q) {
            const uint64_t r = c.rec_sorted[q];
            if ((uint32_t)(r >> c.kshift) != k) break;
            const uint64_t i = r & c.imask;
            const sg_conc_req e = c.req[i];
            if (e.kind == SG_CONC_ACQUIRE) {
                const int32_t sum = (int32_t)((uint32_t)now + (uint32_t)e.acquire);
                if ((double)sum > thr) {
                    put(c, i, SG_STATUS_BLOCKED, 0);
                } else {
                    now = sum;
                    c.alive[i] = 1;
                    put(c, i, SG_STATUS_OK, c.base + i + 1);
                }
            } else if (e.token_id > c.base && e.token_id - c.base <= c.n) {
                const uint64_t j = e.token_id - c.base - 1;
                if (c.alive[j]) {
                    c.alive[j] = 0;
                    now = (int32_t)((uint32_t)now - (uint32_t)c.req[j].acquire);
                    put(c, i, SG_STATUS_RELEASE_OK, 0);
                } else {
                    put(c, i, SG_STATUS_ALREADY_RELEASE, 0);
                }
            } else {
                const int64_t s = tok_find(c, e.token_id);
                if (s < 0) {
                    put(c, i, SG_STATUS_ALREADY_RELEASE, 0);
                } else {
                    c.tab[s].state = 2;
                    now = (int32_t)((uint32_t)now - (uint32_t)c.tab[s].acquire);
                    put(c, i, SG_STATUS_RELEASE_OK, 0);
                }
            }
        }
        c.now[k] = now;
    }
}

__device__ void tok_insert(CTok* tab, uint64_t tmask, const CTok& t, int* err) {
    for (uint64_t h = tok_hash(t.id) & tmask, probes = 0;; h = (h + 1) & tmask, ++probes) {
        if (probes > tmask) {
            atomicOr(err, kErrTableFull);
            return;
        }
        if (atomicCAS((unsigned long long*)&tab[h].id, 0ull, (unsigned long long)t.id) == 0ull) {
            tab[h].flow_id = t.flow_id;
            tab[h].client_to = t.client_to;
            tab[h].res_to = t.res_to;
            tab[h].acquire = t.acquire;
            tab[h].client = t.client;
            tab[h].pad = 0;
            tab[h].state = t.state;
            return;
        }
    }
}

// TokenCacheNode.generateTokenCacheNode + putTokenCacheNode for the batch's tokens still live
__global__ void __launch_bounds__(256) k_conc_insert(ConcArgs c) {
    if (*c.err) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!c.alive[i]) continue;
        const sg_conc_req q = c.req[i];
        const uint32_t k = q.key & SG_KEY_INDEX;
        CTok t;
        t.id = c.base + i + 1;
        t.flow_id = c.flow_id[k];
        t.client_to = c.client_off[k] + q.ts_ms;
        t.res_to = c.res_to[k] + q.ts_ms;
        t.acquire = q.acquire;
        t.client = q.client;
        t.state = 1;
        t.pad = 0;
        tok_insert(c.tab, c.tmask, t, c.err);
    }
}

__global__ void __launch_bounds__(256) k_conc_finish(ConcArgs c) {
    if (*c.err == 0 && c.n > 0) *c.last_ts = c.req[c.n - 1].ts_ms;
}

// RegularExpireStrategy.clearToken over every live token (removal order does not change the sums)
__global__ void __launch_bounds__(256) k_conc_expire(ConcArgs c, int64_t now, const uint8_t* online, uint32_t n_clients,
                                                     unsigned long long* removed) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= c.tmask; s += (uint64_t)gridDim.x * blockDim.x) {
        const CTok t = c.tab[s];
        if (t.id == 0 || t.state != 1) continue;
        const bool on = t.client < n_clients && online[t.client] != 0;
        const int64_t r = rule_of(c, t.flow_id);
        bool drop = !on && t.client_to - now < 0;
        if (!drop && r >= 0 && now - t.res_to > c.res_to[r]) drop = true;
        if (!drop) continue;
        c.tab[s].state = 2;
        atomicAdd(removed, 1ull);
        if (r >= 0) atomicSub((unsigned int*)&c.now[r], (unsigned int)t.acquire);
    }
}

__global__ void __launch_bounds__(256) k_conc_count(ConcArgs c, unsigned long long* live) {
    unsigned long long n = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= c.tmask; s += (uint64_t)gridDim.x * blockDim.x)
        n += (c.tab[s].id != 0 && c.tab[s].state == 1) ? 1ull : 0ull;
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if (__lane_id() == 0) atomicAdd(live, n);
}

__global__ void __launch_bounds__(256) k_conc_rehash(const CTok* old_tab, uint64_t old_slots, CTok* tab, uint64_t tmask,
                                                     int* err) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < old_slots; s += (uint64_t)gridDim.x * blockDim.x) {
        const CTok t = old_tab[s];
        if (t.id != 0 && t.state == 1) tok_insert(tab, tmask, t, err);
    }
}

static unsigned cgrid(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

hipError_t launch_conc_batch(ConcArgs& c, uint64_t* b_buf, uint32_t* hist, hipStream_t stream) {
    hipLaunchKernelGGL(k_conc_prep, dim3(cgrid(c.n, 8192)), dim3(256), 0, stream, c);
    uint64_t* sorted = nullptr;
    hipError_t e = radix_sort_records(c.rec, b_buf, c.n, c.kshift, hist, &sorted, stream);
    if (e != hipSuccess) return e;
    c.rec_sorted = sorted;
    hipLaunchKernelGGL(k_conc_walk, dim3(cgrid(c.n, 8192)), dim3(256), 0, stream, c);
    hipLaunchKernelGGL(k_conc_insert, dim3(cgrid(c.n, 8192)), dim3(256), 0, stream, c);
    hipLaunchKernelGGL(k_conc_finish, dim3(1), dim3(1), 0, stream, c);
    return hipGetLastError();
}

hipError_t launch_conc_expire(const ConcArgs& c, int64_t now, const uint8_t* online, uint32_t n_clients,
                              unsigned long long* removed, hipStream_t stream) {
    hipLaunchKernelGGL(k_conc_expire, dim3(cgrid(c.tmask + 1, 8192)), dim3(256), 0, stream, c, now, online, n_clients,
                       removed);
    return hipGetLastError();
}

hipError_t launch_conc_count(const ConcArgs& c, unsigned long long* live, hipStream_t stream) {
    hipLaunchKernelGGL(k_conc_count, dim3(cgrid(c.tmask + 1, 4096)), dim3(256), 0, stream, c, live);
    return hipGetLastError();
}

hipError_t launch_conc_rehash(const CTok* old_tab, uint64_t old_slots, CTok* tab, uint64_t tmask, int* err,
                              hipStream_t stream) {
    hipLaunchKernelGGL(k_conc_rehash, dim3(cgrid(old_slots, 8192)), dim3(256), 0, stream, old_tab, old_slots, tab, tmask,
                       err);
    return hipGetLastError();
}

}  // namespace sg
