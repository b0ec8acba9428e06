// engine.h — internal device-side types and launch entry points of libsentinel_gpu.so.
// Not part of the public ABI (that is include/sentinel_gpu.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/sentinel_gpu.h"
#include "search_dev.h"

namespace sg {

// Per-flowId rule record, 32 B. thr/isec/S/wl describe the flow's ClusterMetric; the window shape is
// that of the metric created when the flowId first appeared (ClusterFlowRuleManager.java:361 keeps
// an existing metric across rule reloads), the threshold that of the current rule.
struct alignas(16) Rule {
    double thr;       // calcGlobalThreshold(rule) * exceedCount   (ClusterFlowChecker.java:38-48, :68)
    double isec;      // LeapArray.intervalInSecond = intervalInMs / 1000.0 (LeapArray.java:68)
    int32_t S;        // sampleCount
    int32_t wl;       // windowLengthInMs = intervalInMs / sampleCount
    int32_t wl_idx;   // index into the batch's distinct-window-length table
    int32_t wait_ms;  // 1000 / sampleCount (ClusterMetric.java:86)
};
static_assert(sizeof(Rule) == 32, "Rule layout");

// One ClusterMetricBucket + its WindowWrap start, 64 B (one bucket per cache half-line pair).
// start == INT64_MIN encodes a never-created slot (AtomicReferenceArray element == null).
struct alignas(64) Bucket {
    int64_t start;
    int64_t c[SG_NUM_EVENTS];
};
static_assert(sizeof(Bucket) == 64, "Bucket layout");

// The fields of a bucket the window sums read — its start, PASS and WAITING — kept beside the ring, 16 B per bucket
// (PASS / WAITING in int32: read only under BatchArgs::narrow, where every count is proven below 2^30). The short
// walkers gather a flowId's ten buckets from here in 160 contiguous bytes instead of five 128-B lines of the ring;
// every writer of a bucket's start, PASS or WAITING writes both (store_bucket), bulk changes resync it (k_hot_sync).
struct alignas(16) BucketHot {
    int64_t start;
    int32_t pass;
    int32_t wait;
};
static_assert(sizeof(BucketHot) == 16, "BucketHot layout");

__device__ __forceinline__ void store_hot(BucketHot* h, int64_t start, int64_t pass, int64_t wait) {
    BucketHot x;
    x.start = start;
    x.pass = (int32_t)pass;
    x.wait = (int32_t)wait;
    *h = x;
}

// ClusterMetricLeapArray.occupyCounter[PASS], [PASS_REQUEST]; hasOccupied == (pass_req > 0).
struct alignas(16) Occ {
    int64_t pass;
    int64_t pass_req;
};

#ifndef SG_SORT_ROUNDS
#define SG_SORT_ROUNDS 16
#endif
constexpr int kSortRounds = SG_SORT_ROUNDS;  // records per thread of a sort tile (256 threads): 4096-record tiles
constexpr int kMaxWl = 8;                 // distinct window lengths per handle
constexpr uint32_t kMaxPeriods = 1u << 16; // window periods a single batch may span per window length
constexpr int kShortMax = 256;            // default: segments longer than this are walked by a whole wave
constexpr int kLdsBnd = 4096;             // period-table entries the walk kernel stages in LDS
constexpr int kLdsBndFlow = 1024;         // the same for the cluster flow walkers (LDS budget of the short walker)
#ifndef SG_RECW
#define SG_RECW 32
#endif
constexpr int kRecW = SG_RECW;            // records per lane the short walker stages in LDS at a time
// Short segments are grouped by length class (length <= 4, 16, 64, 256, 1024, more) so that the 64 lanes
// of a short-walker wave walk segments of similar length.
constexpr int kClasses = 6;
constexpr uint32_t kClassMax[kClasses - 1] = {4, 16, 64, 256, 1024};

// error bits reported through BatchArgs::err
constexpr int kErrTime = 1;      // negative or decreasing timestamps
constexpr int kErrPeriods = 2;   // batch spans more than kMaxPeriods windows
constexpr int kErrInternal = 16; // a walker loop exceeded its bound (never expected)
constexpr int kErrExchange = 64; // a limited request lies outside the sharded limiter exchange's time range

struct BatchArgs {
    const sg_req* req;
    sg_result* out;
    uint64_t n;
    uint64_t* rec;       // packed records, request order
    uint32_t* hist0;     // k_prep: per-tile histogram of the first sort digit (radix_hist layout), or nullptr
    uint32_t* csum0;     // k_prep also adds each tile's counts to its chunk's column sums (radix_csum), or nullptr
    int hist0_bits;      // width of that digit (radix_digit_bits of the key width)
    uint64_t* rec_sorted;
    // record layout: [key : kbits][0 …][idx : ibits][acode : abits], acode = acquire << 1 | prio, abits <= 8;
    // with abits == 8 and ibits <= 24 the low 32 bits {idx, acode} are the compact record the short walker stages
    // in LDS
    int kshift;          // = 64 - kbits
    int abits;
    uint64_t imask;      // (1 << ibits) - 1
    uint64_t amask;      // (1 << abits) - 1
    uint64_t aesc;       // acquire field value meaning "read req[idx].acquire"
    uint32_t K;          // number of rules
    const Rule* rules;
    Bucket* ring;        // [K][stride]
    BucketHot* hot;      // [K][stride] start / PASS / WAITING of every bucket (the short walkers' gather)
    Occ* occ;            // [K]
    int stride;          // buckets per flowId (max sampleCount)
    double max_occ_ratio;
    int n_wl;
    int32_t wl[kMaxWl];
    uint32_t* bnd;       // [kMaxWl][kMaxPeriods]: first request index of each window period
    int64_t* p0;         // [kMaxWl]: first window period of the batch
    uint32_t* np;        // [kMaxWl]: number of window periods the batch spans
    int* err;
    int64_t* last_ts;    // max timestamp of all earlier batches (-1 before the first)
    int check_last;      // k_prep checks the first timestamp against last_ts (0: k_check_last does, pipelined)
    int64_t* front_ts;   // pipelined batches with namespace limiters: the last timestamp of the latest front half that
                         // passed validation (k_prep also checks against it; k_front_ts advances it); else nullptr
    int walk_cus;        // CUs the walkers' stream may use (CU-masked pipeline streams), 0 = all
    uint32_t* long_list; // segment starts handed to the wave walker
    uint32_t* long_count;
    uint32_t* short_list; // segment starts walked one lane each, per length class (slices, see class_off)
    uint32_t* short_count; // [kClasses] per length class
    uint32_t* short_key;   // flowId of each short_list entry (nullptr: not written)
    uint32_t* long_key;    // flowId of each long_list entry (nullptr: not written)
    uint32_t* seg_end;     // [K] end of each present key's segment in rec_sorted (nullptr: not written)
    uint32_t* seg_start;   // [K] start of each present key's segment (k_seg_mark), 0xFFFFFFFF between batches
    uint32_t* short_end;   // end of each short_list entry's segment (k_seg_classify)
    uint32_t* long_end;    // end of each long_list entry's segment (k_seg_classify; nullptr: seg_end[long_key])
    int seg_marked;        // the sort's last pass marked seg_start / seg_end (launch_seg_flow skips k_seg_mark)
    uint32_t* long_pend;   // [kLongTab][kLongPeriods]: position in rec_sorted where period q + 1 of long segment
                           // i begins (k_long_bounds; nullptr: the wave walker searches for it)
    uint64_t class_off[kClasses]; // first entry of each class slice in short_list
    uint32_t short_max;  // segments longer than this go to the wave walker
    uint32_t* exit_cnt;  // local chain: k_seg also counts the exit records per kLTile-record tile into exit_cnt[1 + t]
    uint64_t exit_amask; // (zeroed before; an exit is a record of a resource whose kind bits (amask >> 1 & 3) are set)
    int dbg;             // debugging switches (env SG_DEBUG): 1 = period table from HBM, 2 = one stream
                         // (serialised walkers, for per-kernel profiles), 64 = short-walker counters into dbg_ctr,
                         // 128 = length class 0 through k_walk_tiny; timing experiments only (wrong results):
                         // 4096 = no k_walk_long, 8192 = no k_walk_short, 16384 = k_prep writes no default results
    int narrow;          // PASS / WAITING of every bucket provably < 2^30 (short walker's 12 B LDS snapshot)
    int generic_walker;  // SG_FLAG_RING_REREAD: short walker re-reads the ring (no register snapshot)
    int tiny;            // 1: length class 0 (<= kClassMax[0] records) is walked by k_walk_tiny, not k_walk_short
    unsigned long long* dbg_ctr;  // [32]
    // ranges of records the wave walker skipped as certainly BLOCKED: {flow key, period q, begin, end}
    uint4* skips;
    uint32_t* skip_count;
    uint32_t skip_cap;
    // Binned front half (bin_on = 1, see k_bin_sort): k_prep writes a 10-bit bin digit into the record's free
    // middle bits [bin_dshift, bin_dshift + 10) — the flowId's hot slot (R + slot) for the hot flowIds of the previous
    // batch, else its key range (key >> bin_bsh), kBinDrop for rejected requests — and counts it for the one global
    // scatter pass; hot bins hold one flowId each, already in order, the regular bins are sorted in LDS by k_bin_sort.
    int hist0_shift;       // k_prep's histogram digit: (rec >> hist0_shift) & mask (kshift, or bin_dshift)
    int bin_on;
    int prep_tiles;        // tiles (of the sort's 4096 records) per k_prep block on the binned path (env SG_PREP_TILES)
    int bin_dshift;
    int bin_bsh;
    uint32_t bin_R;        // regular bins [0, R) (R = ((K - 1) >> bin_bsh) + 1 <= kBinRegular)
    uint2* hot_tab;        // [kHotTab] {flowId, hot slot} open-addressing table (k_prep stages it in LDS)
    uint32_t* hot_key;     // [kBinHot] flowId of each hot slot
    uint64_t* bin_buf;     // the regular bins after the scatter (k_bin_sort's input, rec_sorted's index space)
    const uint32_t* bin_tot;  // [1 << kBinDigit] digit totals (k_chunkscan)
};

constexpr int kBinDigit = 10;                        // bin digit width: one radix_pass<10>
constexpr uint32_t kBinRegular = 512;                // regular bins (key ranges)
constexpr uint32_t kBinHot = (1u << kBinDigit) - kBinRegular - 1;  // hot slots: one flowId each
constexpr uint32_t kBinDrop = (1u << kBinDigit) - 1; // rejected requests
constexpr int kBinMaxBsh = 11;                       // keys per regular bin <= 2048 (k_bin_sort's LDS counters)
// The hot set's table: 512 buckets of 4 {flowId, slot} entries (16 KB), a flowId only in its home bucket (k_hot_update
// leaves a flowId whose bucket is full out of the hot set), so k_prep's lookup is two independent 16-B LDS reads.
constexpr int kHotBucketBits = 9;
constexpr uint32_t kHotWays = 4;
constexpr uint32_t kHotTab = kHotWays << kHotBucketBits;
constexpr uint32_t kHotEmpty = 0xFFFFFFFFu;
__host__ __device__ __forceinline__ uint32_t hot_hash(uint32_t key) {
    return (key * 2654435761u) >> (32 - kHotBucketBits);
}

constexpr int kLongPeriods = 16;       // period-end table of the wave walker: batches of <= 16 window periods
constexpr uint32_t kLongTab = 65536;  // long segments with a table (later ones search)
constexpr uint32_t kSkipMin = 256;    // shortest all-BLOCKED tail worth skipping (records)
constexpr uint32_t kSkipPiece = 4096; // skipped ranges are handed to k_skip_apply in pieces of this size

// ---- namespace QPS limiter (limiter.hip) ----
constexpr int kMaxLim = 8;          // namespaces with a RequestLimiter on the device path
constexpr int kLimSamples = 10;     // RequestLimiter: new UnaryLeapArray(10, 1000) (RequestLimiter.java:35-37)
constexpr int kLimWindowMs = 100;

struct LimRing {                    // one UnaryLeapArray(10, 1000); start INT64_MIN = never created
    int64_t start[kLimSamples];
    int64_t count[kLimSamples];
};

static_assert(sizeof(sg_req) % sizeof(int64_t) == 0 && sizeof(sg_cparam_req) % sizeof(int64_t) == 0 &&
                  offsetof(sg_req, ts_ms) == 0 && offsetof(sg_cparam_req, ts_ms) == 0,
              "LimArgs::ts strides over the request records");
struct LimArgs {
    int n_lim;
    int wl_idx;                     // index of the 100 ms window length in the period table
    double qps[kMaxLim];            // RequestLimiter.qpsAllowed per slot
    const uint8_t* rule_lim;        // [K]: limiter slot of the rule's namespace, 0xFF = none
    uint8_t* slot;                  // [n]: limiter slot per request (0xFF = not subject to a limiter)
    uint32_t* tile_tot;             // [tiles][kMaxLim]
    uint32_t* tile_off;             // [tiles][kMaxLim]
    uint32_t* arrivals;             // [kMaxLim][kMaxPeriods]
    uint32_t* prefix;               // [kMaxLim][kMaxPeriods]
    uint32_t* quota;                // [kMaxLim][kMaxPeriods]
    LimRing* ring;                  // [kMaxLim]
    // sharded limiter: per-millisecond arrivals of every shard, gathered by the node; null = this
    // handle sees the namespace's whole arrival sequence
    const uint32_t* xg;             // [world][n_lim][n_ms]
    const int64_t* ts;              // request i's ts_ms at ts[i * ts_stride] (sg_req: 2 words, sg_cparam_req: 3)
    uint32_t ts_stride;
    int64_t t_base;                 // the exchange's first millisecond (node-wide)
    uint32_t n_ms;                  // milliseconds covered, <= kMaxPeriods
    int world, rank;
};

hipError_t launch_limiter(const BatchArgs& a, const LimArgs& L, hipStream_t stream);
// A shard with no requests in a node batch still advances its replica of the namespace windows.
hipError_t launch_limiter_plan_only(const BatchArgs& a, const LimArgs& L, hipStream_t stream);
// This shard's arrivals per (limiter slot, millisecond) for the exchange: counts[slot * n_ms + (ts - t_base)].
hipError_t launch_lim_arrivals(const sg_req* req, uint64_t n, uint32_t K, const uint8_t* rule_lim, int64_t t_base,
                               uint32_t n_ms, uint32_t* counts, int* err, hipStream_t stream);
hipError_t launch_lim_arrivals_param(const sg_cparam_req* req, uint64_t n, uint32_t K, const uint8_t* rule_lim,
                                     int64_t t_base, uint32_t n_ms, uint32_t* counts, int* err, hipStream_t stream);

// ---- hot-parameter flow control (param.hip) ----
constexpr int kErrNonPositive = 4;  // some acquireCount <= 0 in the batch (disables the skip shortcut)
constexpr int kErrTableFull = 8;    // a rule's value table is full

struct PRule {
    int64_t token_count;    // (long) ParamFlowRule.count
    int64_t duration_sec;
    int32_t burst;
    int32_t behavior;       // 2 = CONTROL_BEHAVIOR_RATE_LIMITER (throttle), else token bucket
    int32_t max_queueing_ms;
    uint32_t hot_begin, hot_count;
    uint32_t pad;
    uint64_t table_base;    // first slot of this rule's sub-table
    uint64_t table_mask;    // 2^capacity_log2 - 1; slot table_base + mask + 1 holds the value ~0
};

// The words a dead period of the cx wave walker reads per entry of a resource with a param rule, in sorted-record order
// (k_lcx_side): the event time, its ParamFlowSlot lookup (LArgs::pslot in 32 bits: 0xFFFFFFFC.. = the kPs* codes,
// else the slot) and its origin node.
struct alignas(16) CxSide {
    int64_t t;
    uint32_t psl;
    uint32_t node;
};

struct alignas(32) PSlot {  // one (rule, value): timeCounters / tokenCounters entries
    uint64_t value;         // ~0 = empty (except in the side slot)
    uint32_t flags;         // bit0 time counter present, bit1 token counter present
    uint32_t pad;
    int64_t time;
    int64_t tokens;
};

constexpr uint32_t kPcBuckets = 2048;  // request buckets of the index → millisecond lookup (pace, hot params)

struct PArgs {
    const sg_param_req* req;
    int32_t* out;
    uint64_t n;
    uint64_t* rec;          // {global slot : high bits | request index : ibits} (ParamFlowSlot chain), or for the
                            // hot-parameter batch {slot : 64 - gshift | acquire code : 8 | request index : ibits}
    uint64_t* rec_sorted;
    int ibits;
    uint64_t imask;
    int gshift;             // the hot-parameter batch's slot shift (ibits + 8); acquire code 255 = read req[i].acquire
    uint32_t* msb;          // [kMaxPeriods] first request index of each millisecond of the batch (entry 0 unused)
    int64_t* mt0;           // the batch's first timestamp
    uint32_t* mnp;          // milliseconds the batch spans (> kMaxPeriods: the walkers read the timestamps)
    uint16_t* mbk;          // [n >> bshift buckets] millisecond (from the first) of request bucket << bshift
    int bshift;
    const PRule* rules;
    uint32_t n_rules;
    const sg_param_hot_item* hot;  // per rule, sorted by value
    PSlot* table;
    uint64_t total_slots;   // all sub-tables; records of requests rejected early carry this as slot
    int* err;
    int64_t* last_ts;
    uint32_t* long_list;
    uint32_t* long_count;
    uint32_t short_max;
};

// ParameterMetric's thread counts of the ParamFlowSlot chain (PSArgs below)
struct alignas(32) PSThread {  // ParameterMetric.threadCountMap entry: (resource, paramIdx) owner word + value
    unsigned long long owner;  // 0 = empty, else (resource + 1) << 32 | (paramIdx + 1)
    uint64_t value;
    int64_t count;
    int64_t pad;
};

hipError_t launch_param_clear(PSlot* table, uint64_t n, hipStream_t stream);
// The long-segment walker runs on `aux` beside the short one (fork / join events).
// sg: the length-class lists (short_list / short_count / class_off) and a zero error word for k_seg.
hipError_t launch_param_batch(const PArgs& p, const BatchArgs& sg, uint64_t* a_buf, uint64_t* b_buf, uint32_t* hist,
                              int lo_bit, int hi_bit, uint64_t** sorted_out, hipStream_t stream, hipStream_t aux,
                              hipEvent_t fork, hipEvent_t join);

// ---- pace controller: RateLimiterController per FlowRule (pace.hip) ----
struct PaceRule {
    double count;           // FlowRule.count
    int32_t max_queueing_ms;
    int32_t pad;
};

struct PaceArgs {
    const sg_pace_req* req;
    int32_t* out;           // wait ms or SG_PACE_BLOCKED
    uint64_t n;
    uint64_t* rec;          // {rule : high bits | request index : ibits}
    uint64_t* rec_sorted;
    int ibits;
    uint64_t imask;
    const PaceRule* rules;
    uint32_t n_rules;       // records of requests decided before the walk carry n_rules as rule
    int64_t* latest;        // [n_rules] latestPassedTime
    int* err;
    int64_t* last_ts;
    uint32_t* long_list;
    uint32_t* long_count;   // [0] long segments, [1 + c] short segments of length class c
    uint32_t* short_list;
    uint32_t short_max;
    int gshift;             // records {rule : high bits | acquire code : 8 | request index : ibits}: rule at gshift
    uint32_t* msb;          // the millisecond table: first request index of every millisecond of the batch
    int64_t* mt0;           // [0] the batch's first timestamp, then {millisecond count, zero word}
    uint32_t* mnp;
    uint16_t* mbk;          // [n >> bshift buckets] millisecond (from the first) of request bucket << bshift
    int bshift;
    uint64_t class_off[kClasses];  // the lane walker's length classes in short_list (counts at long_count[1 + c])
};

// The long-rule walker runs on `aux` beside the short one (fork / join events).
hipError_t launch_pace_batch(const PaceArgs& p, uint64_t* a_buf, uint64_t* b_buf, uint32_t* hist, int lo_bit, int hi_bit,
                             uint64_t** sorted_out, hipStream_t stream, hipStream_t aux, hipEvent_t fork,
                             hipEvent_t join);

// ---- cluster hot-parameter tokens (cparam.hip) ----
constexpr int kErrBounds = 32;      // a request's values lie outside the batch's value array

struct CPRule {
    double count;             // ParamFlowRule.count
    double isec;              // windowIntervalMs / 1000.0
    int32_t S;                // sampleCount of the flowId's metric
    int32_t wl;               // windowIntervalMs / sampleCount
    int32_t global;           // thresholdType == FLOW_THRESHOLD_GLOBAL
    int32_t connected;        // connectedCount of its namespace (AVG_LOCAL)
    uint32_t hot_begin, hot_count;
    uint64_t table_base;      // first slot of this rule's (value → ring) sub-table
    uint64_t table_mask;      // 2^capacity_log2 - 1; slot table_base + mask + 1 holds the value ~0
    int32_t wl_idx;           // index of wl in the handle's distinct window lengths (the batch's period tables)
    int32_t pad;
};

struct CPBucket {             // one bucket of a (flowId, value) ring: window start, the value's count
    int64_t start;            // INT64_MIN: never written
    int64_t count;
};

struct CPArgs {
    const sg_cparam_req* req;
    const uint64_t* values;
    uint64_t n_values;
    sg_result* out;
    uint64_t n;
    uint64_t* rec;            // {slot : high bits | request index - lo : ibits}
    int ibits;
    uint64_t imask;
    const CPRule* rules;
    uint32_t n_rules;
    const sg_param_hot_item* hot;  // per rule, sorted by value
    uint64_t* keys;           // [total_slots] value of each slot (~0 = empty)
    CPBucket* ring;           // [total_slots][stride]
    int stride;
    uint64_t total_slots;
    uint64_t per;             // slots per rule (every sub-table has 2^capacity_log2 + 1): rule of slot g = g / per
    int* err;
    int64_t* last_ts;
};

// One pipeline for single- and multi-value requests (cparam.hip): per-value records sorted by (slot, value
// position), a lane per slot, and a fixed point over the multi-value requests' all-or-nothing outcomes.
struct CPBatch {
    uint32_t* owner;          // [n_values] request that owns value position p (~0 = none)
    uint8_t* chk;             // [n_values] the value's check at its request (multi-value requests)
    uint8_t* assume;          // [n] multi-value request: assumed outcome of this iteration (k_cp_prep2 writes 3 for
                              // a valid multi-value request: bit 1 lists it for k_cp_mlist; k_cp_combine writes 0 / 1)
    // value records, sorted by slot: {slot : 64 - pbits | payload : pbits}, payload = {multi : 1 | acquire code : 7 |
    // id : idbits}; id = the request index of a single-value request, the value position of a multi-value one (its
    // request: owner[id]); acquire code 127 = read req[i].acquire. The walkers read nothing else per single-value record
    // but the period of its request (the batch's period tables: request index -> window period, per window length).
    uint64_t* rec;
    int pbits;
    uint64_t pmask;
    int idbits;
    uint64_t idmask;
    int n_wl;
    int32_t wl[kMaxWl];
    uint32_t* bnd;            // [kMaxWl][kMaxPeriods] first request index of each window period
    int64_t* p0;              // [kMaxWl] first window period of the batch
    uint32_t* np;             // [kMaxWl] window periods the batch spans
    int* changed;             // k_cp_prep2: the batch has multi-value requests; rounds: this round's combine changed an outcome
    const int* changed_prev;  // rounds > 0: the previous round's flag (0: converged, the round's kernels return at once)
    CPBucket* save;           // [touched slots][stride] pre-batch rings of the touched slots (null: no re-walks)
    uint32_t* pslot;          // [n_values] slot of value position p
    uint32_t* dflag;          // [work items] the item is listed for the next re-walk (an assumed outcome changed)
    uint32_t* item_start;     // [work items] segment start of item t (long items first, then short: k_cp_items)
    uint32_t* item_end;       // [work items] its end
    uint32_t* item_slot;      // [work items] its slot
    uint32_t* slot_item;      // [total slots] work item of each slot this batch touches
    uint32_t* din;            // re-walk lists walked this round: [2][dcap] long / short items
    uint32_t* din_count;      // [2]
    uint32_t* dout;           // re-walk lists k_cp_combine fills for the next round
    uint32_t* dout_count;     // [2], zeroed by k_cp_combine before k_cp_relist fills it
    uint32_t dcap;
    uint32_t* mlist;          // valid multi-value requests (k_cp_prep2 appends, any order)
    uint32_t* mcount;
    int round;                // 0: first walk (saves the rings); > 0: re-walk the listed items from the saves
    int lim;                  // the namespace limiter already ran (TOO_MANY_REQUEST results stand)
    uint32_t* dq;             // [work items] earliest window period (batch-relative) a changed outcome touches (~0: none)
    CPBucket* ckpt;           // [long items][ck_np][stride] hot-slot ring at the opening of each window period (null:
                              // re-walks start at the slot's first record)
    uint32_t ck_np;
    uint2* skips;             // saturated ranges [x, y) of sorted records handed to k_cp_skipfill (null: no skipping)
    uint32_t* skip_count;     // zeroed by the host before round 0, by k_cp_relist before the next round
    uint32_t skip_cap;
};
hipError_t launch_cp_prep2(const CPArgs& c, const CPBatch& b, hipStream_t stream);
hipError_t launch_cp_walk2(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, hipStream_t stream, hipStream_t aux,
                           hipEvent_t fork, hipEvent_t join);
hipError_t launch_cp_items(const CPBatch& b, const BatchArgs& sg, uint64_t items, hipStream_t stream);
hipError_t launch_cp_mlist(const CPArgs& c, const CPBatch& b, hipStream_t stream);
hipError_t launch_cp_combine(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, uint64_t items, hipStream_t stream);
hipError_t launch_cp_saverings(const CPArgs& c, const CPBatch& b, const BatchArgs& sg, int restore, hipStream_t stream);
// Fallback when the fixed point's rounds run out: the work items linked by multi-value requests grouped into
// connected components, each group's requests replayed in arrival order on one lane (cparam.hip, k_cpfb_*).
struct CPGroups {
    uint32_t items;        // work items (touched slots)
    uint32_t* label;       // [items] group label (the smallest item of the group once settled)
    uint32_t* flag;        // [items] label l names a group the last round still changed
    int* changed;          // a hooking launch moved a label
    uint64_t* ent;         // [valid requests] {label : 64 - ibits | request index : ibits} of the linked groups
    uint64_t* ent_sorted;  // the entries sorted (radix_sort_records)
    uint32_t* ent_count;
    uint32_t* heads;       // first entry of every group
    uint32_t* head_count;
    int ibits;
    int all;               // no round ran (a zero round budget): every group is replayed, over the untouched rings
};
// step 0: labels; 1: one hook + jump iteration over the m multi-value requests; 2: flags, restore, entries;
// 3: replay of the m sorted entries
hipError_t launch_cpfb(const CPArgs& c, const CPBatch& b, const CPGroups& g, int step, uint32_t m, hipStream_t stream);
hipError_t launch_cp_finish_batch(const CPArgs& c, hipStream_t stream);
hipError_t launch_cp_order(const CPArgs& c, const CPBatch& b, const uint64_t* sorted, uint64_t n, hipStream_t stream);
// The namespace limiter for a cparam batch: 100 ms period table (row 0 of a.bnd) and per-request records with the
// cparam rule index as key; then launch_limiter marks TOO_MANY_REQUEST.
hipError_t launch_cp_limprep(const CPArgs& c, BatchArgs& a, hipStream_t stream);
hipError_t launch_cp_clear(uint64_t* keys, CPBucket* ring, uint64_t slots, int stride, hipStream_t stream);
hipError_t launch_cp_copy(const uint64_t* okeys, const CPBucket* oring, uint64_t obase, int ostride, uint64_t* nkeys,
                          CPBucket* nring, uint64_t nbase, int nstride, uint64_t slots, int S, hipStream_t stream);
hipError_t launch_cp_read(const CPArgs& c, uint32_t rule, uint64_t value, int64_t now, int64_t* out_dev, hipStream_t stream);
struct CPTop {                // a (rule, value) window sum for ClusterParamMetric.getTopValues
    uint64_t value;
    int64_t sum;
    uint32_t rule;
    uint32_t pad;
};
hipError_t launch_cp_top(const CPArgs& c, int64_t now, uint64_t per, CPTop* out, unsigned long long* count,
                         hipStream_t stream);

// ParamFlowSlot chain (param.hip): every param rule of a resource on one lane per resource (or key group)
struct PSArgs {
    PArgs p;                  // rules (token / throttle parameters), hot items, token table
    const sg_pslot_event* ev;
    const sg_pslot_arg* args;
    uint64_t n_args;
    const uint64_t* values;
    uint64_t n_values;
    sg_pslot_result* out;
    uint64_t n;
    uint32_t n_res;
    const uint32_t* res_begin;  // [n_res + 1] the resource's rules: res_rules[res_begin[r] .. res_begin[r + 1])
    const uint32_t* res_rules;  // rule indices in load order
    const int32_t* grade;       // per rule
    int32_t* cur_idx;           // per rule: paramIdx (applyRealParamIdx rewrites a negative one once)
    int32_t* inited;            // per rule: initParamMetricsFor ran (its paramIdx has a thread map)
    PSThread* tc;
    uint64_t tc_mask;
    uint64_t* rec;              // [resource : high bits][event index]
    int kshift;
    uint64_t imask;
    int* err;
    int64_t* last_ts;
    // cluster-mode rules (ParamFlowChecker.passCheck :71-73 → passClusterCheck :278-303)
    const int32_t* cmode;        // per rule: SG_CLUSTER_MODE_* (null: every rule is local)
    const uint32_t* ckey;        // per rule: its flowId's rule index in the embedded server's cluster param state
    int32_t emb;                 // 1: ClusterStateManager SERVER, the cluster rules request param tokens from `cp`
    CPArgs cp;                   // the embedded token server's ClusterParamMetrics (rules, hot items, keys, rings)
    const uint8_t* cp_rule_lim;  // limiter slot of each cluster param rule's namespace (0xFF none), or null
    LimRing* lim_ring;
    double lim_qps[kMaxLim];
    int64_t* cp_last_ts;         // emb: the cluster param batches' last timestamp (time order across both paths)
    const uint32_t* gkey;        // [n_res] record key of each resource (its embedded-server key group), or null
};

hipError_t launch_pslot_batch(PSArgs& s, uint64_t* b_buf, uint32_t* hist, hipStream_t stream);
hipError_t launch_pslot_clear(PSThread* tc, uint64_t n, hipStream_t stream);
hipError_t launch_pslot_thread_read(const PSArgs& s, uint32_t res, int32_t idx, uint64_t value, int64_t* out,
                                    hipStream_t stream);

struct FidSlot {      // flowId → rule index, open addressing with linear probing (fid 0 = empty)
    int64_t fid;
    uint32_t idx;
    uint32_t pad;
};

// ---- concurrent cluster tokens (conc.hip): ConcurrentClusterFlowChecker + TokenCacheNodeManager ----
struct alignas(16) CTok {     // TokenCacheNode in an open-addressing table keyed by token id
    uint64_t id;              // 0 = empty slot
    int64_t flow_id;
    int64_t client_to;        // clientOfflineTime + creation time
    int64_t res_to;           // resourceTimeout + creation time
    int32_t acquire;
    uint32_t client;
    int32_t state;            // 1 live, 2 removed (slots are never reused until the table is rebuilt)
    int32_t pad;
};
static_assert(sizeof(CTok) == 48, "CTok layout");

struct ConcArgs {
    const sg_conc_req* req;
    sg_conc_result* out;
    uint64_t n;
    uint64_t base;            // requests decided before this batch: token id of acquire i = base + i + 1
    uint32_t K;
    const double* thr;        // calcGlobalThreshold per rule
    int32_t* now;             // nowCalls per rule
    const int64_t* client_off;
    const int64_t* res_to;
    const int64_t* flow_id;
    CTok* tab;
    uint64_t tmask;
    const FidSlot* fid;
    uint64_t fid_mask;
    uint64_t* rec;            // [rule : K bits][request index]
    uint64_t* rec_sorted;
    int kshift;
    uint64_t imask;
    uint8_t* alive;           // per request: an acquire of this batch whose token is live
    int* err;
    int64_t* last_ts;
};

hipError_t launch_conc_batch(ConcArgs& c, uint64_t* b_buf, uint32_t* hist, hipStream_t stream);
hipError_t launch_conc_expire(const ConcArgs& c, int64_t now, const uint8_t* online, uint32_t n_clients,
                              unsigned long long* removed, hipStream_t stream);
hipError_t launch_conc_count(const ConcArgs& c, unsigned long long* live, hipStream_t stream);
hipError_t launch_conc_rehash(const CTok* old_tab, uint64_t old_slots, CTok* tab, uint64_t tmask, int* err,
                              hipStream_t stream);

// ---- local slot chain: StatisticSlot → FlowSlot(DefaultController) → DegradeSlot (local.hip) ----
constexpr int kLEv = 6;             // MetricEvent PASS, BLOCK, EXCEPTION, SUCCESS, RT, OCCUPIED_PASS
constexpr int kLPass = 0, kLBlock = 1, kLExc = 2, kLSucc = 3, kLRt = 4, kLOccPass = 5;
constexpr int64_t kStatMaxRt = 5000; // SentinelConfig.statisticMaxRt default (MetricBucket.initMinRt)
constexpr int kMinuteS = 60;         // StatisticNode.rollingCounterInMinute = ArrayMetric(60, 60000, false)
constexpr int kMinuteWl = 1000;
constexpr int kCbClosed = 0, kCbOpen = 1, kCbHalfOpen = 2;

struct alignas(64) LBucket {  // WindowWrap<MetricBucket>: start (INT64_MIN = null slot), 6 counters, minRt
    int64_t start;
    int64_t c[kLEv];
    int64_t min_rt;
};
static_assert(sizeof(LBucket) == 64, "LBucket layout");

struct alignas(16) LFuture {  // borrow ring (FutureBucketLeapArray) slot: only PASS is ever added
    int64_t start;
    int64_t pass;
};

struct LBreaker {             // AbstractCircuitBreaker state + its LeapArray(1, statIntervalMs) bucket
    int64_t next_retry;
    int64_t stat_start;       // INT64_MIN = bucket never created
    int64_t bad;              // slowCount / errorCount
    int64_t total;
    int32_t state;            // kCb*
    int32_t pad;
};

struct alignas(64) LHead {    // per resource: curThreadNum + up to two breakers (128 B)
    int64_t threads;
    int64_t created;          // 1: the resource's ClusterNode exists (ClusterBuilderSlot ran for an entry)
    LBreaker cb[2];
    int64_t pad2[2];
};
static_assert(sizeof(LHead) == 128, "LHead layout");

struct LBreakerRule {
    double count;             // RT: maxAllowedRt source; ratio / count threshold
    double slow_ratio;        // maxSlowRequestRatio (RT)
    int64_t max_rt;           // Math.round(count) (ResponseTimeCircuitBreaker.java:52)
    int32_t grade;            // SG_DEGRADE_*
    int32_t min_request;
    int32_t recovery_ms;      // timeWindow * 1000, int (AbstractCircuitBreaker.java:54)
    int32_t stat_ms;          // statIntervalMs
};

struct alignas(16) LRule {
    double flow_count;
    int32_t flow_grade;       // 0 thread, 1 QPS, -1 no flow rule (the fast walkers' one DefaultController rule)
    int32_t nb;               // breakers 0..2
    LBreakerRule b[2];
    uint32_t fr_begin, fr_n;  // cx: the resource's flow rules frules[fr_begin .. + fr_n) in check order
    int32_t cx;               // 1: walked by k_lwalk_cx (several rules, limitApps, shaping controllers, param rules,
                              // context DefaultNodes, RELATE groups); a batch's events from an origin make their
                              // resource cx for that batch (LArgs::dyn)
    int32_t ps;               // 1: the resource has ParamFlowSlot rules (sg_pslot_load_rules)
    int32_t grp;              // 1: in a RELATE key group (walked event by event from memory, k_lwalk_cx)
    int32_t pad_;
};
constexpr uint32_t kNoNode = 0xFFFFFFFFu;

// The node pool of the local chain: nodes besides the resources' ClusterNodes — ClusterNode.getOrCreateOriginNode
// (ClusterBuilderSlot.java:99-102: every entry with an origin) and NodeSelectorSlot's DefaultNode per context
// (NodeSelectorSlot.java:156-170: every entry in a context) — created at the first event that needs them, as the
// reference does, and kept for the life of the resources (they outlive flow-rule reloads). An open-addressing map
// {(resource, kind, id) → node index} in HBM; pool nodes follow the K resources in the node arrays.
constexpr uint64_t kLNodeCtx = 1ull << 31;  // key bit: a context DefaultNode (else an origin node)
__host__ __device__ __forceinline__ uint64_t lnode_key(uint32_t res, uint64_t kind, uint32_t id) {
    return ((uint64_t)(res + 1u) << 32) | kind | (uint64_t)id;  // never 0 (the empty slot)
}
__host__ __device__ __forceinline__ uint64_t lnode_hash(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// A flow rule of the local chain with its controller's constants (FlowRuleUtil.generateRater, WarmUpController
// .construct :83-106).
struct alignas(16) LFlowRule {
    double count;
    double slope;
    int32_t grade;            // 0 thread, 1 QPS
    int32_t behavior;         // SG_CONTROL_* actually used (THREAD rules: DEFAULT)
    int32_t limit_app;        // SG_LIMIT_APP_DEFAULT / _OTHER / origin id
    int32_t max_queue_ms;
    int32_t warning_token, max_token, cold;
    int32_t strategy;         // SG_STRATEGY_*
    int32_t ref;              // RELATE: resource index; CHAIN: context id; < 0: refResource blank
    int32_t cluster_mode;     // SG_CLUSTER_MODE_* (cluster-mode rules are checked last)
    uint32_t cluster_key;     // embedded token server: the flowId's rule index in the cluster flow state
    int32_t pad_[3];
};

struct alignas(32) LCtl {     // the controller's state: storedTokens, lastFilledTime, latestPassedTime
    int64_t stored, last_filled, latest, pad;
};

struct LArgs {
    const sg_local_event* ev;
    sg_local_result* out;
    uint64_t n;
    uint64_t* rec;            // [res : kbits][idx : ibits][count << 3 | kind << 1 | prio : abits]
    uint64_t* rec_sorted;
    uint32_t* hist0;          // k_local_prep: per-tile histogram of the first sort digit (radix_hist layout), or null
    uint32_t* csum0;          // and its chunk column sums (radix_csum), or null
    int hist0_bits;
    int kshift, abits;
    uint64_t imask, amask, aesc;
    uint32_t K;               // resources (record keys)
    uint32_t N;               // nodes: the K resources, then the pool (origin / context nodes)
    const LRule* rules;       // [K]
    const LFlowRule* frules;  // flow rules of the cx resources
    LCtl* ctl;                // [frules] controller state
    int32_t n_origins;
    LHead* head;              // [K]
    LBucket* sec;             // [K][S]   second window (OccupiableBucketLeapArray)
    LFuture* bor;             // [K][S]   its borrow array
    LBucket* minute;          // [K][60]  minute window (BucketLeapArray)
    int S;                    // SampleCountProperty.SAMPLE_COUNT
    int32_t wl2;              // INTERVAL / SAMPLE_COUNT
    int32_t interval;         // IntervalProperty.INTERVAL
    double isec;              // INTERVAL / 1000.0
    int32_t occupy_timeout;   // OccupyTimeoutProperty
    int wsec, wmin;           // period-table indices of the second / minute window lengths
    int n_wl;
    int32_t wl[kMaxWl];
    uint32_t* bnd;
    int64_t* p0;
    uint32_t* np;
    int* err;
    int64_t* last_ts;
    int32_t defer_last;       // 1 (pipelined batches): k_local_check_last, in the back half, compares the first
                              // timestamp with last_ts once the previous batch has advanced it; 0: k_local_prep does
    const sg_slot_ext* ext;   // per event: context and arguments (nullable: context 0, null args)
    int32_t n_contexts;       // context ids 0 .. n_contexts - 1
    const uint32_t* gkey;     // [K] record key of each resource (its RELATE group's first resource), or null
    PSArgs ps;                // ParamFlowSlot rules, value tables and thread counts; ps.args / ps.values: the batch's
    int32_t has_ps;           // 1: ps is loaded (resources with LRule.ps run ParamFlowSlot)
    int* flags;               // kLFlag*: batch properties that rule out the dead-period skip
    uint32_t* exit_pos;       // sorted positions of exit records (ascending), exit_cnt[0] of them
    uint32_t* exit_cnt;       // [0] total, then per-tile counts / offsets
    struct LSkip* skips;      // dead-period ranges handed to k_lskip_apply
    uint32_t* skip_count;
    uint32_t skip_cap;
    // node pool (null nkeys: no origins / contexts tracked)
    uint64_t* nkeys;          // [nmask + 1] lnode_key, 0 = empty
    uint32_t* nvals;          // node index of each key
    uint64_t nmask;
    uint32_t node_base;       // index of the batch's first new pool node (K + pool nodes before the batch)
    uint32_t* node_new;       // pool nodes the batch created (k_lnode_assign)
    uint2* ev_node;           // [n] map slots of each event's {origin node, context DefaultNode}, kNoNode = none
    uint32_t* dyn;            // [K] epoch of the last batch with an origin event of the resource (walked as cx)
    uint32_t epoch;
    int32_t track_ctx;        // 1: every event updates its context's DefaultNode (n_contexts >= 1)
    int32_t cxw;              // 1: long cx segments (not RELATE groups) go to the wave walker k_lwalk_cxw
    int32_t cxw_cls;          // ... and so do those of the short length classes >= cxw_cls (kClasses: none)
    uint32_t* cxw_next;       // the wave walker's next work item (zeroed before it starts; waves take items in turn)
    uint32_t* cx_list;        // [n] or null: the lane cx walker's segment heads (k_lcx_list), cx_count of them
    uint32_t* cx_count;
    uint64_t* pslot;          // [n] or null: k_local_prep's ParamFlowSlot lookup of each entry of a resource with one
                              // QPS param rule (kPsNoCheck / kPsEarlyFail / kPsUnknown, else the (rule, value) slot)
    CxSide* cxside;           // [n] or null: k_lcx_side's words of the sorted records of the cx resources
    // the embedded token server (ClusterStateManager SERVER, emb = 1): the handle's cluster flow state
    int32_t emb;
    const Rule* c3_rules;
    Bucket* c3_ring;
    BucketHot* c3_hot;
    Occ* c3_occ;
    int c3_stride;
    uint32_t c3_K;
    double max_occ_ratio;
    const uint8_t* c3_rule_lim;   // limiter slot of each cluster rule's namespace (0xFF none)
    LimRing* lim_ring;
    double lim_qps[kMaxLim];
    int64_t* c3_last_ts;          // the cluster flow batches' last timestamp (time order across both paths)
    int64_t* last_fetch;      // [K] StatisticNode.lastFetchTime (metric rows already reported)
    const uint8_t* inbound;   // [K] 1: the resource's entries are EntryType.IN (Constants.ENTRY_NODE), or null
    LBucket* entry_acc;       // [60] the ENTRY_NODE's minute buckets summed from the inbound resources' (metric rows)
    int64_t* entry_fetch;     // the ENTRY_NODE's lastFetchTime
};

constexpr uint64_t kPsUnknown = ~0ull;     // LArgs::pslot codes: not looked up (the walker's own step decides)
constexpr uint64_t kPsNoCheck = ~0ull - 1;  // args null: ParamFlowSlot passes without a look
constexpr uint64_t kPsEarlyFail = ~0ull - 2;  // blocked before the maps (tokenCount 0, acquire > tokens + burst)
constexpr uint64_t kPsNoCheckInit = ~0ull - 3;  // arguments, but none at paramIdx (too short or null): no check
constexpr int kLFlagPrio = 1;    // some entry is prioritized (may occupy in a saturated window)
constexpr int kLFlagNonPos = 2;  // some entry has acquireCount <= 0 (may fit in a saturated window)
constexpr uint32_t kLTile = 4096;  // records per tile of the exit-position compaction

struct LSkip {                   // entries [b0, b1) of resource k, all FLOW-blocked in periods (qs, qm)
    uint32_t k, qs, qm, b0, b1, pad[3];
};

hipError_t launch_local_prep(const LArgs& L, hipStream_t stream);
hipError_t launch_local_walk(const LArgs& L, const BatchArgs& seg, bool has_cx, hipStream_t aux, hipStream_t stream,
                             hipEvent_t fork, hipEvent_t join);
// launch_local_walk in two halves for the pipelined local path: the exit-position list (reads only the batch's
// sorted records: front half), then the cross-batch time check when deferred, the walkers, the skipped BLOCK counts
// and last_ts (back half, in batch order).
hipError_t launch_local_exits(const LArgs& L, hipStream_t stream, bool counted);  // counted: by k_seg
hipError_t launch_local_back(const LArgs& L, const BatchArgs& seg, bool has_cx, hipStream_t aux, hipStream_t stream,
                             hipEvent_t fork, hipEvent_t join);
hipError_t launch_local_init(const LArgs& L, hipStream_t stream);
// Empty nodes [lo, hi) of the node arrays L.head / sec / bor / minute.
hipError_t launch_local_init_range(const LArgs& L, uint64_t lo, uint64_t hi, hipStream_t stream);
// Node pool: every event's origin node / context DefaultNode found or created in the map (after k_local_prep,
// nothing when the batch failed validation); node index of a key (kNoNode if absent) into *out (device).
hipError_t launch_lnode_assign(const LArgs& L, hipStream_t stream);
hipError_t launch_lnode_find(const uint64_t* keys, const uint32_t* vals, uint64_t mask, uint64_t key, uint32_t* out,
                             hipStream_t stream);
// StatisticNode.metrics() of every resource at now: emit == 0 counts the rows (no side effect), emit == 1 writes
// them (any order) and applies currentWindow / lastFetchTime.
// Constants.ENTRY_NODE's metric rows from the summed buckets (k_local_metrics accumulated them into a.entry_acc).
// raw: rt is the bucket's raw sum in every row (sg_local_metrics_raw, for a node rollup) instead of rt / success.
hipError_t launch_entry_acc_reset(LBucket* acc, hipStream_t stream);
hipError_t launch_metrics_gate(const unsigned long long* cnt, uint64_t cap, unsigned long long* count_out, int* gate,
                               hipStream_t stream);
hipError_t launch_local_entry_rows(const LArgs& L, int64_t now, sg_metric_node* out, unsigned long long* count, int emit,
                                   int raw, hipStream_t stream, const int* gate = nullptr);
hipError_t launch_local_metrics(const LArgs& L, int64_t now, sg_metric_node* out, unsigned long long* count, int emit,
                                int raw, hipStream_t stream, const int* gate = nullptr);

// Test aid (env SG_LDS_POISON=1): before every kernel that keeps counters or tables in LDS, a kernel fills the LDS of
// every CU with 0xA5 bytes on the same stream, so a counter a kernel forgets to initialise reads garbage at once.
void lds_poison(hipStream_t stream);

// Launchers (engine.hip). All are asynchronous on `stream`.
hipError_t launch_prep(const BatchArgs& a, hipStream_t stream);

// ---- node handle routing (node.hip) ----
constexpr int kMaxShards = 64;
constexpr uint32_t kRouteNone = 127;  // shard id of a request that is not routed (answered by the front)
struct RouteArgs {
    const sg_req* req;         // the node batch (caller order)
    const uint64_t* rec;       // the front's packed records (request order; rejected ones carry the sentinel key)
    uint64_t n;
    int kshift, abits;
    uint64_t imask;
    uint32_t K;                // node rules
    const uint8_t* shard_of;   // [K] owner shard of each node rule
    const uint32_t* local_of;  // [K] its rule index on that shard
    int G;
    uint32_t* tile_cnt;        // [tiles][kMaxShards]
    uint32_t* shard_base;      // [G + 1] first sub-batch position of each shard
    uint32_t* shard_tot;       // [G] requests routed to each shard
    sg_req* sub_req;           // [n] the shard slices, one after the other
    uint32_t* sub_pos;         // [n] node position of each sub-request
    // shards on the front's device (sub_rec != null): the slices are the shards' packed records instead — the
    // front's record with its key field replaced by the shard-local rule index (shifted by the shard's kshift); the
    // request index stays the node's, so the shards' walkers read the node batch's period tables and write the
    // caller's results in place (no sub_req / sub_pos, no gather)
    uint64_t* sub_rec;
    uint64_t low_mask;         // the record bits below the front's key field (request index, acquire code)
    int skshift[kMaxShards];   // each shard's key shift
};
hipError_t launch_route(const RouteArgs& r, hipStream_t stream);
hipError_t launch_route_gather(const sg_result* sub_out, const uint32_t* sub_pos, uint64_t total, sg_result* out,
                               hipStream_t stream);
uint64_t route_tiles(uint64_t n);
// Node routing of cluster param / concurrent token batches (node.hip k_nreq_*): owner records, the slices.
struct NodeReqArgs {
    uint64_t n;
    const sg_cparam_req* cp;   // a param batch (node order), or null
    const sg_conc_req* cc;     // a concurrent-token batch, or null
    const uint64_t* values;    // param: the batch's values
    uint64_t n_values;
    uint32_t K;                // node rules of the kind (param rules / flow rules)
    const uint8_t* shard_of;   // [K] owner shard
    const uint32_t* local_of;  // [K] the rule's index on its owner
    int G;
    uint64_t* rec;             // [n] {owner : 8 | request index : 56}
    uint32_t* nvals;           // [n] value count per request (param; 0 out of bounds)
    uint32_t* cnt;             // [kMaxShards] requests per shard (zeroed before)
    uint32_t* vcnt;            // [kMaxShards] values per shard (zeroed before)
    uint32_t* tsum;            // [tiles] value-count tile sums, then their exclusive scan
    const uint32_t* vbase;     // [kMaxShards] first value of each shard's slice (node value array)
    sg_cparam_req* sub_cp;     // [n] param slices, one after the other
    sg_conc_req* sub_cc;       // [n] concurrent slices
    uint64_t* sub_vals;        // [n_values] the slices' values
    uint32_t* sub_pos;         // [n] node position of each slice entry
    int* err;
    int64_t last_ts;           // the node's previous batch of this kind: its last timestamp (-1: none)
};
hipError_t launch_nreq_keys(const NodeReqArgs& q, hipStream_t stream);
hipError_t launch_nreq_gather(const NodeReqArgs& q, const uint64_t* sorted, hipStream_t stream);
uint64_t nreq_tiles(uint64_t n);
hipError_t launch_nsnap_scatter(const double* part, const uint32_t* node_key, uint64_t cnt, double* out,
                                hipStream_t stream);
hipError_t launch_nconc_scatter(const sg_conc_result* sub_out, const uint32_t* sub_pos, const sg_conc_req* sub_req,
                                uint64_t base, uint64_t cnt, uint32_t g, uint32_t G, sg_conc_result* out,
                                hipStream_t stream);
// sort.hip: stable LSD radix sort of records on bits [lo_bit, hi_bit); result buffer is a or b.
size_t radix_hist_words(uint64_t n);
int radix_digit_bits(int bits);  // digit width radix_sort_records uses for `bits` key bits (8 or 10)
#ifndef SG_CHUNK_TILES
#define SG_CHUNK_TILES 32
#endif
constexpr uint32_t kChunkTiles = SG_CHUNK_TILES;  // sort tiles per column-sum chunk (sort.hip)
// Column sums by atomics in the histogram kernels (k_prep, k_radix_hist) instead of a k_colsum pass over the rows:
// one dependent launch fewer per sort pass (env SG_CSUM_ATOMIC=0: the k_colsum pass).
bool radix_csum_atomic();
uint32_t* radix_csum(uint32_t* hist_ws, uint64_t n, int D);   // the chunk column sums' place in hist_ws
size_t radix_csum_bytes(uint64_t n, int D);
// Segment marks of a flowId-keyed sort's last pass (seg_start atomicMin / seg_end atomicMax per key, see sort.hip)
struct SegMark {
    uint32_t* seg_start;
    uint32_t* seg_end;
    uint32_t K;
    int kshift;
};
hipError_t radix_sort_records(uint64_t* a, uint64_t* b, uint64_t n, int lo_bit, uint32_t* hist_ws,
                              uint64_t** result, hipStream_t stream, int hi_bit = 64, bool first_hist_ready = false,
                              const SegMark* mark = nullptr, bool first_csum_ready = false);
const uint32_t* radix_tot(const uint32_t* hist_ws, uint64_t n, int D);
hipError_t radix_bin_pass(uint64_t* src, uint64_t* out, uint64_t* reg, uint32_t R, uint64_t n, int shift,
                          uint32_t* hist_ws, bool hist_ready, bool csum_ready, hipStream_t stream);
hipError_t launch_seg(const BatchArgs& a, hipStream_t stream);
hipError_t launch_seg_flow(const BatchArgs& a, hipStream_t stream);  // k_seg_mark + k_seg_classify
// Binned front half after k_prep: the scatter by bin digit (regular bins to a.bin_buf, hot bins and rejected requests
// to a.rec_sorted), k_bin_sort (regular bins sorted in LDS into a.rec_sorted, every segment listed), k_hot_update (the
// next batch's hot flowIds: this batch's longest segments).
hipError_t launch_bin_front(const BatchArgs& a, uint32_t* hist_ws, bool hist_ready, bool csum_ready, hipStream_t stream);
hipError_t launch_hot_reset(uint2* hot_tab, hipStream_t stream);
hipError_t launch_walk_long(const BatchArgs& a, hipStream_t stream);   // on an aux stream, concurrent with
bool tiny_walker_enabled(const BatchArgs& a);
hipError_t launch_walk_tiny(const BatchArgs& a, hipStream_t stream);
hipError_t launch_walk_short(const BatchArgs& a, hipStream_t stream);  // the short walker
hipError_t launch_check_last(const BatchArgs& a, hipStream_t stream);
hipError_t launch_finish(const BatchArgs& a, hipStream_t stream);
hipError_t launch_front_ts(const BatchArgs& a, hipStream_t stream);
// bytes (a multiple of 4) from device memory to a device-accessible host buffer by the shader
hipError_t launch_copy_out(const void* src, void* dst_dev, uint64_t bytes, int blocks, hipStream_t stream);
hipError_t launch_skip_apply(const BatchArgs& a, hipStream_t stream);
hipError_t launch_hot_sync(const Bucket* ring, BucketHot* hot, uint64_t buckets, hipStream_t stream);
hipError_t launch_init_state(Bucket* ring, Occ* occ, uint32_t K, int stride, const int32_t* src_map,
                             const Bucket* old_ring, const Occ* old_occ, int old_stride, hipStream_t stream);
hipError_t launch_snapshot(const Rule* rules, const Bucket* ring, const Occ* occ, uint32_t K, int stride,
                           int64_t now, double* out, hipStream_t stream);

// ---- token-server wire codec (codec.hip) ----

struct CodecArgs {
    uint64_t n;
    // decode
    const uint8_t* payload;
    const uint32_t* offsets;  // [n + 1]
    const int64_t* ts;
    sg_req* req;
    int32_t* xid;
    uint8_t* kind;
    const FidSlot* fid_tab;
    uint64_t fid_mask;
    // encode
    const int32_t* xid_in;
    const uint8_t* kind_in;
    const sg_result* res;
    uint8_t* frames;
};

hipError_t launch_codec_decode(const CodecArgs& c, hipStream_t stream);
hipError_t launch_codec_encode(const CodecArgs& c, hipStream_t stream);

}  // namespace sg
