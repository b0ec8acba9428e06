// codec.hip — the token server's wire codec on the device.
//
// Frames arrive from the Netty pipeline length-delimited (LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2),
// srv/server/NettyTransportServer.java:89); a batching front-end appends each payload to one buffer and
// records its start. k_codec_decode turns frame i into the engine's request record (one thread per frame,
// big-endian fields read byte-wise: frames are not aligned), resolving flowId → rule index in an exact
// open-addressing table built at rule load (ClusterFlowRuleManager.getFlowRuleById). k_codec_encode writes
// each TokenResult as a fixed 16-byte response frame, one aligned 16-byte store per thread.
#include "engine.h"

namespace sg {

__device__ __forceinline__ uint64_t fid_hash(int64_t fid) {  // splitmix64 finaliser
    uint64_t z = (uint64_t)fid + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t rd_be32(const uint8_t* p) {
    return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}

__device__ __forceinline__ int64_t rd_be64(const uint8_t* p) {
    return (int64_t)(((uint64_t)(uint32_t)rd_be32(p) << 32) | (uint64_t)(uint32_t)rd_be32(p + 4));
}

constexpr int kDecFrames = 256;        // frames per block step (one per thread)
constexpr uint32_t kDecStage = 16384;  // LDS bytes staged per step

// Decode one frame from `p` (LDS or HBM) of `len` bytes.
__device__ __forceinline__ void decode_frame(const CodecArgs& c, uint64_t i, const uint8_t* p, uint32_t len) {
    sg_req r;
    r.ts_ms = c.ts[i];
    r.key = SG_KEY_BAD;
    r.acquire = 0;
    int32_t xid = 0;
    uint8_t kind;
    if (len < 5) {  // DefaultRequestEntityDecoder.decode: readableBytes() >= 5, else null (:37)
        kind = SG_FRAME_SHORT;
    } else {
        xid = rd_be32(p);                        // readInt() (:38)
        const int type = (int)(int8_t)p[4];      // readByte() (:39)
        const uint32_t rem = len - 5;
        if (type != SG_MSG_TYPE_FLOW) {
            kind = SG_FRAME_OTHER;
        } else if (rem < 12) {  // FlowRequestDataDecoder.decode: readableBytes() >= 12, else null (:33)
            kind = SG_FRAME_NO_DATA;
        } else {
            kind = SG_FRAME_FLOW;
            const int64_t fid = rd_be64(p + 5);             // readLong() (:35)
            r.acquire = rd_be32(p + 13);                    // readInt() (:36)
            const bool prio = rem >= 13 && p[17] != 0;      // readBoolean() if a byte is left (:37-39)
            if (fid <= 0) {
                r.key = SG_KEY_BAD;  // DefaultTokenService.notValidRequest → badRequest() (:87-89)
            } else {
                uint32_t key = SG_KEY_NO_RULE;  // rule == null → NO_RULE_EXISTS (:44-47)
                for (uint64_t h = fid_hash(fid) & c.fid_mask;; h = (h + 1) & c.fid_mask) {
                    const FidSlot s = c.fid_tab[h];
                    if (s.fid == fid) {
                        key = s.idx;
                        break;
                    }
                    if (s.fid == 0) break;  // empty slot: not present (the table is never full)
                }
                r.key = key;
            }
            if (prio) r.key |= SG_KEY_PRIO;
        }
    }
    c.req[i] = r;
    c.xid[i] = xid;
    c.kind[i] = kind;
}

// One block step = kDecFrames consecutive frames. Their payload bytes are contiguous, so when they fit the
// block stages them in LDS with coalesced aligned 4-byte loads (the word holding a frame's last byte never
// crosses the allocation's end) and parses from there; larger steps read their bytes from HBM directly.
__global__ void __launch_bounds__(kDecFrames) k_codec_decode(CodecArgs c) {
    __shared__ uint32_t stage[kDecStage / 4];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(stage);
    for (uint64_t i0 = (uint64_t)blockIdx.x * kDecFrames; i0 < c.n; i0 += (uint64_t)gridDim.x * kDecFrames) {
        const uint64_t i1 = min(i0 + (uint64_t)kDecFrames, c.n);
        const uint32_t lo = c.offsets[i0], hi = c.offsets[i1];
        const uint32_t a0 = lo & ~3u;
        const bool staged = hi >= lo && hi - a0 <= kDecStage;  // (offsets running backwards: read in place)
        if (staged && hi > lo) {
            const uint32_t words = (hi - a0 + 3) / 4;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(c.payload) + a0 / 4;
            for (uint32_t w = threadIdx.x; w < words; w += kDecFrames) stage[w] = src[w];
        }
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        if (i < i1) {
            const uint32_t off = c.offsets[i], end = c.offsets[i + 1];
            const uint32_t len = end >= off ? end - off : 0u;  // a backwards frame decodes as SG_FRAME_SHORT
            decode_frame(c, i, staged ? sb + (off - a0) : c.payload + off, len);
        }
        __syncthreads();  // the stage is refilled by the next step
    }
}

__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

__global__ void __launch_bounds__(256) k_codec_encode(CodecArgs c) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (c.kind_in[i] == SG_FRAME_FLOW) {
            const sg_result r = c.res[i];
            const uint32_t x = (uint32_t)c.xid_in[i];
            // bytes: [0, 14] length (LengthFieldPrepender(2)), xid, type, status (DefaultResponseEntityWriter
            // .writeHead), remaining, waitInMs (FlowResponseDataWriter.writeTo); big-endian, little-endian words
            w.x = (14u << 8) | ((x >> 24) << 16) | (((x >> 16) & 0xFFu) << 24);
            w.y = ((x >> 8) & 0xFFu) | ((x & 0xFFu) << 8) | ((uint32_t)SG_MSG_TYPE_FLOW << 16) |
                  (((uint32_t)r.status & 0xFFu) << 24);
            w.z = bswap((uint32_t)r.remaining);
            w.w = bswap((uint32_t)r.wait_ms);
        }
        reinterpret_cast<uint4*>(c.frames)[i] = w;
    }
}

static unsigned codec_grid(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 8192 ? (b ? b : 1) : 8192);
}

hipError_t launch_codec_decode(const CodecArgs& c, hipStream_t stream) {
    if (((uintptr_t)c.payload & 3u) != 0) return hipErrorInvalidValue;  // staged loads are 4-byte words
    lds_poison(stream);
    hipLaunchKernelGGL(k_codec_decode, dim3(codec_grid(c.n)), dim3(kDecFrames), 0, stream, c);
    return hipGetLastError();
}

hipError_t launch_codec_encode(const CodecArgs& c, hipStream_t stream) {
    hipLaunchKernelGGL(k_codec_encode, dim3(codec_grid(c.n)), dim3(256), 0, stream, c);
    return hipGetLastError();
}

}  // namespace sg
