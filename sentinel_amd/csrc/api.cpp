// api.cpp — the C ABI of libsentinel_gpu.so (include/sentinel_gpu.h): handle, rule tables, batch
// driver. Device work is in engine.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "engine.h"

using namespace sg;

constexpr int kAsyncSlots = 3;  // batches of one handle in flight on the host pipeline
constexpr int kDevSlots = 4;    // device-buffer batches of one handle in flight (sg_flow_enqueue)

struct sg_handle {
    int device = 0;
    sg_config cfg{};
    std::string err;

    std::vector<sg_namespace> ns;
    std::vector<sg_flow_rule> rules;  // as loaded (current rule per key)
    std::vector<Rule> rule_tab;       // device image
    uint32_t K = 0;
    int stride = 0;                   // buckets per flowId
    int n_wl = 0;
    int32_t wl[kMaxWl]{};

    Rule* d_rules = nullptr;
    Bucket* d_ring = nullptr;
    BucketHot* d_hot = nullptr;       // start / PASS / WAITING of every bucket (the short walkers' gather)
    Occ* d_occ = nullptr;
    uint32_t* d_seg_end = nullptr;   // [2K] end, then start (k_seg_mark) of each flowId's segment in the sorted records
    // binned front half (engine.hip k_bin_sort): the hot flowIds of the previous batch and workspace 0's bin buffer
    uint32_t* d_hot_key = nullptr;    // [kBinHot] flowId per hot slot, then the table [kHotTab] {flowId, slot}
    uint64_t hot_gen = ~0ull;         // rules_gen the hot set was reset for
    uint64_t rules_gen = 0;           // flow rule loads so far (a reload renumbers flowIds: the hot set restarts)
    uint64_t* d_bin_buf = nullptr;
    int bin_mode = 1;                 // env SG_BIN: 0 off, 1 on for >= 2^14 flowIds, 2 on whenever the records allow
    int prep_tiles = 4;               // env SG_PREP_TILES: sort tiles per k_prep block on the binned path

    // batch workspace (sized for cfg.max_batch)
    uint64_t* d_rec = nullptr;
    uint64_t* d_rec_sorted = nullptr;
    uint64_t* last_sorted = nullptr;  // whichever of d_rec / d_rec_sorted holds the last sort result
    uint32_t* d_hist = nullptr;       // radix sort histogram workspace
    uint32_t* d_bnd = nullptr;
    int64_t* d_p0 = nullptr;
    uint32_t* d_np = nullptr;
    int* d_err = nullptr;
    int64_t* d_last_ts = nullptr;
    int64_t* d_front_ts = nullptr;    // pipelined limiter batches: last timestamp of the latest accepted front half
    uint32_t* d_long_list = nullptr;
    uint32_t* d_long_count = nullptr;  // [4]: long count, short count, work cursors (long, short)
    uint32_t* d_short_list = nullptr;
    uint32_t* d_short_key = nullptr;  // flowId of each d_short_list entry (cluster flow path)
    uint32_t* d_short_end = nullptr;  // segment end of each d_short_list entry (cluster flow path)
    uint32_t* d_long_key = nullptr;   // flowId of each d_long_list entry (cluster flow path)
    uint32_t* d_long_end = nullptr;   // segment end of each d_long_list entry (cluster flow path)
    uint32_t* d_long_pend = nullptr;
    FidSlot* d_fid = nullptr;         // flowId → rule index (wire codec), 2^k slots
    uint64_t fid_mask = 0;  // [kLongTab][kLongPeriods] period ends of the long segments
    uint64_t class_off[kClasses]{};
    unsigned long long* d_dbg = nullptr;   // [128] debug counters (SG_DEBUG & 64)
    uint4* d_skips = nullptr;
    uint32_t* d_skip_count = nullptr;
    int* h_err = nullptr;       // pinned
    uint32_t* h_long = nullptr; // pinned: long segment count, skipped range count

    // host-buffer convenience path
    sg_req* d_req_h = nullptr;
    sg_result* d_out_h = nullptr;

    // namespace QPS limiters (GlobalRequestLimiter): slot per namespace, device rings and scratch
    std::vector<int> ns_slot;
    int n_lim = 0;
    double lim_qps[kMaxLim]{};
    int lim_wl_idx = -1;
    LimRing* d_lim_ring = nullptr;
    uint8_t* d_rule_lim = nullptr;
    uint8_t* d_lim_slot = nullptr;
    uint32_t* d_lim_tile = nullptr;   // tile totals then tile offsets
    uint32_t* d_lim_period = nullptr; // arrivals, prefix, quota

    // hot-parameter flow control
    std::vector<sg_param_rule> prules;
    std::vector<PRule> ptab;
    PRule* d_prules = nullptr;
    sg_param_hot_item* d_phot = nullptr;
    PSlot* d_ptable = nullptr;
    uint64_t ptotal = 0;             // slots over all rule sub-tables
    int64_t* d_plast_ts = nullptr;
    sg_param_req* d_preq_h = nullptr;
    int32_t* d_pout_h = nullptr;

    // pace controller (RateLimiterController per FlowRule)
    std::vector<PaceRule> pace_tab;
    PaceRule* d_pace_rules = nullptr;
    int64_t* d_pace_latest = nullptr;
    int64_t* d_pace_last_ts = nullptr;
    sg_pace_req* d_pace_req_h = nullptr;
    int32_t* d_pace_out_h = nullptr;

    // cluster hot-parameter tokens
    std::vector<sg_cparam_rule> cprules;
    std::vector<CPRule> cptab;
    CPRule* d_cprules = nullptr;
    sg_param_hot_item* d_cphot = nullptr;
    uint64_t* d_cpkeys = nullptr;
    CPBucket* d_cpring = nullptr;
    uint64_t cptotal = 0;
    int cpstride = 1;
    int64_t* d_cplast_ts = nullptr;
    // one-pipeline batch scratch (value-position records, fixed point over multi-value requests)
    uint32_t* d_cp_owner = nullptr;
    uint32_t* d_cp_pslot = nullptr;
    uint32_t* d_cp_long = nullptr;    // segment lists over the value records (capacity cp_val_cap)
    uint32_t* d_cp_short = nullptr;
    uint64_t cp_class_off[kClasses]{};
    uint32_t* d_p_msb = nullptr;      // hot-parameter batch: first request index of each millisecond
    int64_t* d_p_mt = nullptr;        // its first timestamp, then the millisecond count (uint32)
    uint16_t* d_p_mbk = nullptr;      // pace: the millisecond of every kPcBuckets-th request
    std::vector<int32_t> cp_wls;      // distinct window lengths of the cluster param rules (CPRule::wl_idx)
    uint32_t* d_cp_bnd = nullptr;     // [kMaxWl][kMaxPeriods] the batch's period tables (request index -> period)
    int64_t* d_cp_p0 = nullptr;
    uint32_t* d_cp_np = nullptr;
    uint32_t* d_cp_slot_item = nullptr;  // [cptotal] work item of each touched slot (k_cp_items)
    uint64_t cp_slot_item_cap = 0;
    uint32_t* d_cp_items = nullptr;   // [4 * cp_val_cap] per work item: re-walk flag, segment start; re-walk lists x2
    uint32_t* d_cp_counts = nullptr;  // [6]: re-walk list counts (2 buffers x {long, short}), multi-value count
    uint32_t* d_cp_mlist = nullptr;   // [max_batch] multi-value requests
    uint8_t* d_cp_chk = nullptr;
    uint8_t* d_cp_assume = nullptr;
    uint64_t* d_cp_rec = nullptr;
    uint64_t* d_cp_rec2 = nullptr;
    uint32_t* d_cp_hist = nullptr;
    uint64_t cp_val_cap = 0;
    CPBucket* d_cp_save = nullptr;
    CPBucket* d_cp_ckpt = nullptr;    // hot-slot ring checkpoints, one per window period of the batch
    uint64_t cp_ckpt_cap = 0;
    uint2* d_cp_skips = nullptr;      // saturated ranges of the hot-slot walker (k_cp_skipfill), [cp_skip_cap]
    uint32_t* d_cp_skip_count = nullptr;
    uint64_t cp_skip_cap = 0;
    uint64_t cp_save_cap = 0;
    int* d_cp_changed = nullptr;
    uint8_t* d_cp_rule_lim = nullptr; // [cparam rules] limiter slot of the rule's namespace (0xFF none)
    std::vector<uint8_t> cp_rule_lim_host;
    bool cp_any_lim = false;          // some cluster param rule's namespace has a limiter
    uint32_t cp_rounds = 0;           // fixed-point rounds of the last batch (stats / tests)
    uint32_t cp_max_rounds = 64;      // env SG_CP_MAX_ROUNDS overrides (tests force the serial fallback)
    sg_cparam_req* d_cpreq_h = nullptr;
    uint64_t* d_cpval_h = nullptr;
    uint64_t cpval_cap = 0;
    sg_result* d_cpout_h = nullptr;

    // local slot chain
    sg_local_config lcfg{2, 1000, 500, 0};
    std::vector<LRule> ltab;          // [K] the resources (sg_local_load_rules), origin nodes not included
    uint32_t l_nodes = 0;             // node arrays: the resources, then the pool (l_pool_cap nodes)
    int32_t l_n_origins = 0;
    bool l_has_cx = false;
    std::vector<int64_t> l_rule_slot; // loaded flow rule i → its LCtl index, -2 stateless fast-path rule, -1 ignored
    LFlowRule* d_lfrules = nullptr;
    LCtl* d_lctl = nullptr;
    int64_t* d_llast_fetch = nullptr; // [K] StatisticNode.lastFetchTime
    LRule* d_lrules = nullptr;
    LHead* d_lhead = nullptr;
    LBucket* d_lsec = nullptr;
    LFuture* d_lbor = nullptr;
    LBucket* d_lmin = nullptr;
    int64_t* d_llast_ts = nullptr;
    int l_n_wl = 0, l_wsec = 0, l_wmin = 0;
    int32_t l_wl[kMaxWl]{};
    sg_local_event* d_lev_h = nullptr;
    struct LocalWs {                  // the local path's own batch buffers of a pipeline workspace (0: every local
        int* flags = nullptr;         // batch; 1: every other sg_local_enqueue batch), sized for max_batch
        uint32_t* exit_pos = nullptr;
        uint32_t* exit_cnt = nullptr;
        LSkip* skips = nullptr;
        uint32_t* skip_count = nullptr;
        uint64_t* pslot = nullptr;    // [max_batch] LArgs::pslot (param rules loaded and the cx wave walker on)
        CxSide* cxside = nullptr;     // [max_batch] LArgs::cxside (with pslot)
        uint32_t* cxw_next = nullptr; // LArgs::cxw_next
        uint32_t* cx_list = nullptr;  // [max_batch + 1] LArgs::cx_list, then cx_count (cx resources loaded)
    };
    LocalWs lws[2];
    uint32_t lskip_cap = 0;
    sg_local_result* d_lout_h = nullptr;
    // node pool (origin nodes, context DefaultNodes; created by the batches, kept across flow-rule reloads)
    uint32_t l_pool_cap = 0, l_pool_used = 0;
    uint64_t* d_lnkeys = nullptr;     // map (resource, kind, id) → node, l_nmap_cap slots
    uint32_t* d_lnvals = nullptr;
    uint64_t l_nmap_cap = 0;
    uint32_t* d_lnode_new = nullptr;  // pool nodes a batch created
    uint32_t* h_lnode_new = nullptr;  // pinned
    uint2* d_lev_node = nullptr;      // [max_batch] map slots of each event's nodes
    uint32_t* d_ldyn = nullptr;       // [K] batch epoch of each resource's last origin event
    uint32_t l_epoch = 0;
    uint64_t l_batches = 0;           // local batches decided since sg_local_load_rules
    int32_t l_n_contexts = 0;
    int32_t l_cluster_state = SG_CLUSTER_NOT_STARTED;
    bool l_cluster_rules = false;     // some loaded flow rule is in cluster mode
    std::vector<uint8_t> l_base_cx;   // per resource: walked by the cx walker whatever the key groups
    std::vector<std::pair<uint32_t, uint32_t>> l_relate;        // RELATE (resource, referenced resource)
    std::vector<std::pair<uint32_t, uint32_t>> l_cluster_refs;  // cluster-mode rules: (resource, cluster_key)
    bool l_groups_stale = false;      // cluster rules / namespaces / cluster state changed: regroup before a batch
    uint32_t* d_lgkey = nullptr;      // [K] RELATE key groups (record key of each resource), null without groups
    uint64_t l_ps_applied = 0;        // ps_gen whose param flags d_lrules carries (0: none)
    bool l_has_cx_ps = false;         // some resource is cx because of param rules
    sg_slot_ext* d_lext_h = nullptr;  // host-path buffers of sg_slot_decide_batch_host
    uint8_t* d_linbound = nullptr;    // [K] EntryType.IN resources (sg_local_set_entry_types), null = none
    LBucket* d_lentry_acc = nullptr;  // [60] the ENTRY_NODE's buckets, summed per metric call
    unsigned long long* d_lm_cnt = nullptr;  // the metric passes' row counter
    int64_t* d_lentry_fetch = nullptr;// the ENTRY_NODE's lastFetchTime

    int kbits = 0, ibits = 0, abits = 0;
    int32_t shard_rank = 0, shard_world = 1;  // sg_set_shard: this handle's share of a node's flowIds
    // sg_lim_exchange: the node's gathered per-millisecond limiter arrivals for the next flow batch of a shard
    uint32_t* d_xg_ws[2]{};           // the gathered arrivals a pipelined batch of workspace x reads (copied at enqueue)
    uint64_t xg_ws_cap = 0;           // words per buffer
    int* d_limx_err = nullptr;        // sg_lim_arrivals' own error word (the pipelined batches keep theirs)
    int* h_limx_err = nullptr;        // pinned
    const uint32_t* lim_xg = nullptr;
    int64_t lim_xt = 0;
    uint32_t lim_xn = 0;
    bool lim_x_armed = false;
    // ParamFlowSlot chain (sg_pslot_*)
    uint32_t ps_nres = 0;
    bool ps_loaded = false;
    uint32_t* d_ps_begin = nullptr;
    uint32_t* d_ps_rules = nullptr;
    int32_t* d_ps_grade = nullptr;
    int32_t* d_ps_idx = nullptr;
    int32_t* d_ps_init = nullptr;
    PSThread* d_ps_tc = nullptr;
    uint64_t ps_tc_slots = 0;
    int64_t* d_ps_last_ts = nullptr;
    std::vector<uint32_t> ps_res_rules;  // param rules per resource
    uint64_t ps_gen = 0;              // sg_pslot_load_rules calls so far
    int32_t* d_ps_cmode = nullptr;    // per rule: SG_CLUSTER_MODE_*
    uint32_t* d_ps_ckey = nullptr;    // per rule: its flowId's cluster param rule index (embedded server)
    bool ps_cluster = false;          // some loaded param rule is a cluster-mode QPS rule
    std::vector<std::pair<uint32_t, uint32_t>> ps_cluster_refs;  // (resource, cluster_key) of those rules
    uint32_t* d_ps_gkey = nullptr;    // [n_res] key groups of sg_pslot_decide_batch on an embedded server, or null
    bool ps_groups_stale = true;      // param rules / cluster param rules / namespaces / state changed
    // concurrent cluster tokens (sg_conc_*)
    int32_t* d_cnow = nullptr;        // nowCalls per rule
    double* d_cthr = nullptr;
    int64_t* d_coff = nullptr;
    int64_t* d_cres = nullptr;
    int64_t* d_cfid = nullptr;
    CTok* d_ctok = nullptr;
    uint64_t ctok_slots = 0, ctok_used = 0;  // table size; slots taken since the last rehash (upper bound)
    uint8_t* d_calive = nullptr;
    int64_t* d_clast_ts = nullptr;
    sg_conc_req* d_creq_h = nullptr;
    sg_conc_result* d_cout_h = nullptr;
    uint64_t conc_seq = 0;            // requests decided so far (token ids)
    bool conc_dirty = true;           // rules / namespaces / timeouts changed since the last upload
    bool cnow_pending = false;        // cnow_host holds the remapped counters of a rule reload
    std::vector<int32_t> cnow_host;
    std::vector<int64_t> c_off, c_res;
    // asynchronous host pipeline (sg_flow_submit): H2D / compute / D2H streams, kAsyncSlots batches in flight
    struct Slot {
        uint64_t ticket = 0;            // 0 = free
        sg_req* d_req = nullptr;
        sg_result* d_out = nullptr;
        int* h_err = nullptr;           // pinned: the batch's error flags
        hipEvent_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    };
    Slot slots[kAsyncSlots];
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    uint64_t next_ticket = 1;
    std::unordered_map<uint64_t, int> finished;  // tickets completed while making room, not yet collected
    bool stats_on = false;
    uint32_t short_max = kShortMax;   // default walker split (env SG_SHORT_MAX overrides, for tuning)
    bool short_max_env = false;
    int dbg = 0;                      // env SG_DEBUG: see BatchArgs::dbg
    int l_cxw = 1;                    // env SG_CXW=0: long cx segments on the lane walker too (LArgs::cxw)
    uint32_t l_cxw_min = 0xFFFFFFFFu;          // env SG_CXW_MIN: shortest cx segment class the wave walker takes (LArgs::cxw_cls)
    bool wide_seen = false;           // some loaded rule allowed bucket counts >= 2^30 (sticky: the ring keeps them)
    hipEvent_t ev[5]{};
    sg_batch_stats stats{};
    hipStream_t aux = nullptr;        // second stream: the long-segment walker runs beside the short one
    hipEvent_t fork = nullptr, join = nullptr;
    // Pipelined flow batches (sg_flow_enqueue, sg_flow_submit): the front half of a batch (validation, sort,
    // segments) runs on s_front while the previous batch's walkers run on s_back. Two workspaces alternate:
    // workspace 0 is the handle's own batch buffers above, workspace 1 (pws) is allocated on first use.
    struct FlowWs {
        uint64_t* rec = nullptr;
        uint64_t* rec_sorted = nullptr;
        uint32_t* hist = nullptr;
        uint32_t* bnd = nullptr;
        int64_t* p0 = nullptr;
        uint32_t* np = nullptr;
        int* err = nullptr;
        uint32_t* long_list = nullptr;
        uint32_t* long_key = nullptr;
        uint32_t* long_end = nullptr;
        uint32_t* long_pend = nullptr;
        uint32_t* short_list = nullptr;
        uint32_t* short_key = nullptr;
        uint32_t* counts = nullptr;   // [1 + kClasses]: long count, short counts per class
        uint4* skips = nullptr;
        uint32_t* skip_count = nullptr;
        uint32_t* seg_end = nullptr;  // [K]
        uint32_t* seg_start = nullptr;  // [K], all 0xFFFFFFFF between batches
        uint32_t* short_end = nullptr;
        uint64_t* bin_buf = nullptr;    // binned front half: the regular bins after the scatter (max_batch records)
    };
    FlowWs pws{};
    uint32_t pws_segcap = 0;
    hipStream_t s_front = nullptr, s_back = nullptr, s_aux2 = nullptr;
    hipStream_t s_aux3 = nullptr;     // the length-class-0 walker beside the other two (SG_DEBUG & 128, tuning)
    hipEvent_t tjoin = nullptr;
    hipStream_t s_xcopy = nullptr;    // the sharded limiter exchange's copy into a pipeline workspace
    hipEvent_t xcopy_done = nullptr;
    hipEvent_t front_done[2]{}, back_done[2]{}, pfork = nullptr, pjoin = nullptr;
    hipEvent_t lm_in = nullptr, lm_done = nullptr;  // sg_local_metrics_raw_enqueue: the caller's stream <-> s_back
    int* d_lm_gate = nullptr;                        // its capacity gate (count <= cap)
    uint64_t pipe_seq = 0;            // batches put on the pipeline so far (workspace = seq % 2)
    bool d2h_kernel = false;          // sg_flow_submit: results to pinned host buffers by k_copy_out (env SG_D2H=1; the
                                      // copy engine measured faster: 2.64 vs 2.45 G decisions/s end to end)
    int d2h_blocks = 64;              // its workgroups (env SG_D2H_BLOCKS)
    int front_eighths = 4;            // CU partition of the pipeline streams (pipe_setup; round 6: the binned front half
                                      // (k_bin_sort) takes 4/8, -2.5 % against 3/8; the two-pass sort measures the same at 3 or 4)
    int walk_cus = 0;                 // CUs of the walkers' streams when partitioned (0 = all)
    struct DevTicket {                // sg_flow_enqueue batches in flight
        uint64_t ticket = 0;
        int* h_err = nullptr;         // pinned
        hipEvent_t done = nullptr;
        bool local = false;           // an sg_local_enqueue batch (its error flags map through local_status)
    };
    DevTicket dev[kDevSlots];
    bool front_only = false;          // a node handle's front (validation + namespace limiter): no flow state
    // k_seg_mark over the sorted records (default), or the marks fused into the last scatter pass (env SG_SEG_MARK=0:
    // its ~20M atomicMin/Max per 16M-record batch cost more than the separate read — 0.97 vs 0.91 ms/step, same box)
    bool seg_mark_pass = true;
    bool lim_pipe = true;             // limiter batches: the front half does not wait for the previous back half
                                      // (env SG_LIM_PIPE=0: it waits); read once in sg_create
};

namespace {
PSArgs pslot_args(sg_handle* h);          // below: the ParamFlowSlot state's device arguments
int pslot_embed(sg_handle* h, PSArgs& s, hipStream_t stream);  // below: its embedded token server (SERVER)
int ensure_layout(sg_handle* h);          // below: record layout of the loaded rules
int flow_status(sg_handle* h, int err);   // below: batch error flags -> SG_E_*
int drain_async(sg_handle* h);  // below: completes the handle's in-flight host-pipeline batches
int local_apply_groups(sg_handle* h);  // below: key groups of the local chain
}

extern "C" {
static int upload_fid_table(sg_handle* h);  // flowId → rule index for the wire codec (defined below)
}

namespace {

int fail(sg_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

#define HIP_TRY(h, expr)                                                                        \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return fail((h), SG_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e));     \
    } while (0)

int bits_for(uint64_t v) {  // bits needed to represent v (v >= 1)
    int b = 0;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

// calcGlobalThreshold(rule) * exceedCount (ClusterFlowChecker.java:38-48, :68)
double global_threshold(const sg_handle* h, const sg_flow_rule& r) {
    double base;
    if (r.threshold_type == SG_THRESHOLD_GLOBAL) {
        base = r.count;
    } else {
        int connected = 0;
        if (r.namespace_id >= 0 && (size_t)r.namespace_id < h->ns.size()) connected = h->ns[r.namespace_id].connected_count;
        base = r.count * connected;
    }
    return base * h->cfg.exceed_count;
}

// java.lang.Math.round(double) (JDK 7u+): floor(x + 1/2) computed exactly on the bits; saturating.
int64_t java_math_round(double a) {
    int64_t bits;
    std::memcpy(&bits, &a, 8);
    const int64_t biased_exp = (bits & 0x7FF0000000000000LL) >> 52;
    const int64_t shift = (52 - 1 + 1023) - biased_exp;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000FFFFFFFFFFFFFLL) | 0x0010000000000000LL;
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    if (a != a) return 0;
    if (a >= 9223372036854775807.0) return INT64_MAX;
    if (a <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)a;
}


int layout_records(sg_handle* h) {
    h->kbits = bits_for((uint64_t)h->K);  // must hold K itself (sentinel key of rejected requests)
    if (h->kbits < 1) h->kbits = 1;
    h->ibits = bits_for(h->cfg.max_batch > 1 ? h->cfg.max_batch - 1 : 1);
    // acquire field: 7 bits + prio (larger acquireCounts escape to the request), so that {idx, acode} fit the
    // low 32 bits whenever ibits <= 24 (the short walker's compact LDS records)
    h->abits = std::min(8, 64 - h->kbits - h->ibits);
    if (h->abits < 3) return fail(h, SG_E_UNSUPPORTED, "rule count x max_batch too large for 64-bit records");
    return SG_OK;
}

// Distinct window lengths of the loaded flows (+ the limiter's 100 ms when a limiter is on).
int rebuild_wl_table(sg_handle* h) {
    int n_wl = 0;
    int32_t wl[kMaxWl]{};
    auto index_of = [&](int32_t v) -> int {
        for (int w = 0; w < n_wl; ++w)
            if (wl[w] == v) return w;
        if (n_wl == kMaxWl) return -1;
        wl[n_wl] = v;
        return n_wl++;
    };
    for (uint32_t k = 0; k < h->K; ++k) {
        const int w = index_of(h->rule_tab[k].wl);
        if (w < 0) return fail(h, SG_E_UNSUPPORTED, "more than 8 distinct window lengths");
        h->rule_tab[k].wl_idx = w;
    }
    h->lim_wl_idx = -1;
    if (h->n_lim > 0) {
        h->lim_wl_idx = index_of(kLimWindowMs);
        if (h->lim_wl_idx < 0) return fail(h, SG_E_UNSUPPORTED, "more than 8 distinct window lengths");
    }
    h->n_wl = n_wl;
    std::memcpy(h->wl, wl, sizeof(wl));
    return SG_OK;
}

int upload_rule_table(sg_handle* h) {
    h->l_groups_stale = true;  // an embedded token server's key groups follow the cluster rules / namespaces
    h->ps_groups_stale = true;
    int rc = rebuild_wl_table(h);
    if (rc) return rc;
    // Bucket counts stay below thr * (2 + isec) * (2 + maxOccupyRatio): a pass needs PASS sum <= thr * isec,
    // an occupy acquire + occupied <= thr + head and WAITING sum <= ratio * thr * isec before it adds acquire.
    // Below 2^30 the short walker may hold PASS / WAITING in int32 (BatchArgs::narrow).
    const double ratio = h->cfg.max_occupy_ratio > 0 ? h->cfg.max_occupy_ratio : 0.0;
    for (uint32_t k = 0; k < h->K; ++k) {
        Rule& R = h->rule_tab[k];
        R.thr = global_threshold(h, h->rules[k]);
        const double bound = (R.thr > 0 ? R.thr : 0.0) * (2.0 + R.isec) * (2.0 + ratio);
        if (!(bound < 1073741824.0)) h->wide_seen = true;
    }
    if (h->K) HIP_TRY(h, hipMemcpy(h->d_rules, h->rule_tab.data(), sizeof(Rule) * h->K, hipMemcpyHostToDevice));
    // limiter slot of each rule's namespace
    dfree(h->d_rule_lim);
    if (h->K) {
        std::vector<uint8_t> rl(h->K, 0xFF);
        for (uint32_t k = 0; k < h->K; ++k) {
            const int ns = h->rules[k].namespace_id;
            if (ns >= 0 && (size_t)ns < h->ns_slot.size() && h->ns_slot[ns] >= 0) rl[k] = (uint8_t)h->ns_slot[ns];
        }
        if (hipMalloc(&h->d_rule_lim, h->K) != hipSuccess) return fail(h, SG_E_NOMEM, "rule limiter table");
        HIP_TRY(h, hipMemcpy(h->d_rule_lim, rl.data(), h->K, hipMemcpyHostToDevice));
    }
    return SG_OK;
}

}  // namespace

extern "C" {

const char* sg_build_info(void) {
    return "sentinel_gpu: cluster flow-decision engine, HIP for gfx950 (MI355X)";
}

int sg_create(const sg_config* cfg, sg_handle** out) {
    if (!cfg || !out) return SG_E_INVAL;
    *out = nullptr;
    if (cfg->max_batch == 0 || cfg->max_batch > (1ull << 32)) return SG_E_INVAL;
    if (!(cfg->exceed_count >= 0) || !(cfg->max_occupy_ratio >= 0)) return SG_E_INVAL;
    sg_handle* h = new sg_handle();
    h->cfg = *cfg;
    h->device = cfg->device;
    auto bail = [&](int rc) {
        sg_destroy(h);
        return rc;
    };
    if (hipSetDevice(h->device) != hipSuccess) return bail(SG_E_DEVICE);
    const uint64_t n = cfg->max_batch;
    // + kRecW records of slack: the short walker stages record windows past a segment's end unclamped
    if (hipMalloc(&h->d_rec, (n + kRecW) * 8) != hipSuccess || hipMalloc(&h->d_rec_sorted, (n + kRecW) * 8) != hipSuccess)
        return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_bnd, sizeof(uint32_t) * kMaxWl * kMaxPeriods) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_hist, sizeof(uint32_t) * radix_hist_words(n)) != hipSuccess) return bail(SG_E_NOMEM);
    {
        const uint64_t tiles = n / 4096 + 1;
        if (hipMalloc(&h->d_lim_ring, sizeof(LimRing) * kMaxLim) != hipSuccess ||
            hipMalloc(&h->d_lim_slot, n) != hipSuccess ||
            hipMalloc(&h->d_lim_tile, sizeof(uint32_t) * tiles * kMaxLim * 2) != hipSuccess ||
            hipMalloc(&h->d_lim_period, sizeof(uint32_t) * kMaxLim * kMaxPeriods * 3) != hipSuccess)
            return bail(SG_E_NOMEM);
    }
    if (hipMalloc(&h->d_p0, sizeof(int64_t) * kMaxWl) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_np, sizeof(uint32_t) * kMaxWl) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_err, sizeof(int)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_last_ts, 2 * sizeof(int64_t)) != hipSuccess) return bail(SG_E_NOMEM);  // + front_ts
    if (hipMalloc(&h->d_long_list, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&h->d_long_key, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&h->d_long_end, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
        hipMalloc(&h->d_long_pend, sizeof(uint32_t) * (size_t)kLongTab * kLongPeriods) != hipSuccess)
        return bail(SG_E_NOMEM);
    {  // short-segment class slices: class c holds segments longer than kClassMax[c-1], so at most n/(that+1)
        uint64_t off = 0;
        for (int c = 0; c < kClasses; ++c) {
            h->class_off[c] = off;
            off += (c == 0 ? n : n / (kClassMax[c - 1] + 1)) + 1;
        }
        if (hipMalloc(&h->d_short_list, sizeof(uint32_t) * off) != hipSuccess ||
            hipMalloc(&h->d_short_key, sizeof(uint32_t) * off) != hipSuccess ||
            hipMalloc(&h->d_short_end, sizeof(uint32_t) * off) != hipSuccess)
            return bail(SG_E_NOMEM);
    }
    if (hipMalloc(&h->d_dbg, 128 * 8) != hipSuccess || hipMemset(h->d_dbg, 0, 128 * 8) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_long_count, (1 + kClasses) * sizeof(uint32_t)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_skips, sizeof(uint4) * (2 * n / kSkipMin + 1)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMalloc(&h->d_skip_count, sizeof(uint32_t)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipHostMalloc(&h->h_err, sizeof(int)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipHostMalloc(&h->h_long, 2 * sizeof(uint32_t)) != hipSuccess) return bail(SG_E_NOMEM);
    int64_t neg = -1;
    if (hipMemcpy(h->d_last_ts, &neg, sizeof(neg), hipMemcpyHostToDevice) != hipSuccess) return bail(SG_E_DEVICE);
    h->d_front_ts = h->d_last_ts + 1;
    if (hipMemcpy(h->d_front_ts, &neg, sizeof(neg), hipMemcpyHostToDevice) != hipSuccess) return bail(SG_E_DEVICE);
    if (hipMalloc(&h->d_plast_ts, sizeof(int64_t)) != hipSuccess) return bail(SG_E_NOMEM);
    if (hipMemcpy(h->d_plast_ts, &neg, sizeof(neg), hipMemcpyHostToDevice) != hipSuccess) return bail(SG_E_DEVICE);
    for (auto& e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) return bail(SG_E_DEVICE);
    // the auxiliary stream carries the wave walkers beside the lane walkers (pace, hot params, cluster params);
    // env SG_AUX_PRIO=1 (tuning) creates it at the highest stream priority
    int aux_prio = 0;
    if (const char* e = std::getenv("SG_AUX_PRIO"); e && std::atoi(e) == 1) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess) aux_prio = greatest;
    }
    if (hipStreamCreateWithPriority(&h->aux, hipStreamNonBlocking, aux_prio) != hipSuccess ||
        hipEventCreateWithFlags(&h->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->join, hipEventDisableTiming) != hipSuccess)
        return bail(SG_E_DEVICE);
    if (const char* d = std::getenv("SG_DEBUG")) h->dbg = std::atoi(d);
    if (const char* d = std::getenv("SG_CXW")) h->l_cxw = std::atoi(d) != 0 ? 1 : 0;
    if (const char* d = std::getenv("SG_CXW_MIN")) h->l_cxw_min = (uint32_t)std::strtoul(d, nullptr, 10);
    if (const char* d = std::getenv("SG_D2H")) h->d2h_kernel = std::atoi(d) != 0;
    if (const char* d = std::getenv("SG_SEG_MARK")) h->seg_mark_pass = std::atoi(d) != 0;
    if (const char* d = std::getenv("SG_LIM_PIPE")) h->lim_pipe = std::atoi(d) != 0;
    if (const char* d = std::getenv("SG_BIN")) h->bin_mode = std::atoi(d);
    if (const char* d = std::getenv("SG_PREP_TILES")) h->prep_tiles = std::max(1, std::min(64, std::atoi(d)));
    if (const char* d = std::getenv("SG_D2H_BLOCKS")) h->d2h_blocks = std::max(1, std::atoi(d));
    if (const char* sm = std::getenv("SG_SHORT_MAX")) {
        h->short_max = (uint32_t)std::strtoul(sm, nullptr, 10);
        h->short_max_env = true;
    }
    if (const char* mr = std::getenv("SG_CP_MAX_ROUNDS")) h->cp_max_rounds = (uint32_t)std::strtoul(mr, nullptr, 10);
    // default namespace 0, no limiter, 1 connection
    sg_namespace d0{0, 1, 30000.0};
    h->ns.push_back(d0);
    *out = h;
    return SG_OK;
}

void sg_destroy(sg_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    {
        auto& w = h->pws;
        if (h->s_back) (void)hipStreamSynchronize(h->s_back);
        dfree(w.rec);
        dfree(w.rec_sorted);
        dfree(w.hist);
        dfree(w.bnd);
        dfree(w.p0);
        dfree(w.np);
        dfree(w.err);
        dfree(w.long_list);
        dfree(w.long_key);
        dfree(w.long_end);
        dfree(w.long_pend);
        dfree(w.short_list);
        dfree(w.short_key);
        dfree(w.short_end);
        dfree(w.counts);
        dfree(w.skips);
        dfree(w.skip_count);
        dfree(w.seg_end);
        dfree(w.bin_buf);
        for (auto* st : {&h->s_front, &h->s_back, &h->s_aux2, &h->s_aux3, &h->s_xcopy})
            if (*st) (void)hipStreamDestroy(*st);
        if (h->xcopy_done) (void)hipEventDestroy(h->xcopy_done);
        for (int x = 0; x < 2; ++x) {
            if (h->front_done[x]) (void)hipEventDestroy(h->front_done[x]);
            if (h->back_done[x]) (void)hipEventDestroy(h->back_done[x]);
        }
        if (h->tjoin) (void)hipEventDestroy(h->tjoin);
        if (h->lm_in) (void)hipEventDestroy(h->lm_in);
        if (h->lm_done) (void)hipEventDestroy(h->lm_done);
        if (h->pfork) (void)hipEventDestroy(h->pfork);
        if (h->pjoin) (void)hipEventDestroy(h->pjoin);
        for (auto& d : h->dev) {
            if (d.done) (void)hipEventDestroy(d.done);
            if (d.h_err) (void)hipHostFree(d.h_err);
        }
    }
    dfree(h->d_rules);
    dfree(h->d_ring);
    dfree(h->d_hot);
    dfree(h->d_occ);
    dfree(h->d_seg_end);
    dfree(h->d_hot_key);
    dfree(h->d_bin_buf);
    dfree(h->d_rec);
    dfree(h->d_rec_sorted);
    dfree(h->d_hist);
    dfree(h->d_lim_ring);
    dfree(h->d_rule_lim);
    dfree(h->d_lim_slot);
    dfree(h->d_lim_tile);
    dfree(h->d_xg_ws[0]);
    dfree(h->d_xg_ws[1]);
    dfree(h->d_limx_err);
    if (h->h_limx_err) (void)hipHostFree(h->h_limx_err);
    dfree(h->d_lnkeys);
    dfree(h->d_lnvals);
    dfree(h->d_lnode_new);
    dfree(h->d_lev_node);
    dfree(h->d_ldyn);
    if (h->h_lnode_new) (void)hipHostFree(h->h_lnode_new);
    dfree(h->d_lim_period);
    dfree(h->d_bnd);
    dfree(h->d_p0);
    dfree(h->d_np);
    dfree(h->d_err);
    dfree(h->d_last_ts);
    dfree(h->d_long_list);
    dfree(h->d_long_count);
    dfree(h->d_short_list);
    dfree(h->d_short_key);
    dfree(h->d_short_end);
    dfree(h->d_long_key);
    dfree(h->d_long_end);
    dfree(h->d_long_pend);
    dfree(h->d_fid);
    dfree(h->d_dbg);
    dfree(h->d_skips);
    dfree(h->d_prules);
    dfree(h->d_phot);
    dfree(h->d_ptable);
    dfree(h->d_plast_ts);
    dfree(h->d_preq_h);
    dfree(h->d_pout_h);
    dfree(h->d_pace_rules);
    dfree(h->d_pace_latest);
    dfree(h->d_pace_last_ts);
    dfree(h->d_pace_req_h);
    dfree(h->d_pace_out_h);
    dfree(h->d_skip_count);
    dfree(h->d_cprules);
    dfree(h->d_cphot);
    dfree(h->d_cpkeys);
    dfree(h->d_cpring);
    dfree(h->d_cplast_ts);
    dfree(h->d_cpreq_h);
    dfree(h->d_cpval_h);
    dfree(h->d_cpout_h);
    dfree(h->d_lrules);
    dfree(h->d_lfrules);
    dfree(h->d_lctl);
    dfree(h->d_llast_fetch);
    dfree(h->d_ps_begin);
    dfree(h->d_ps_rules);
    dfree(h->d_ps_grade);
    dfree(h->d_ps_idx);
    dfree(h->d_ps_init);
    dfree(h->d_ps_tc);
    dfree(h->d_ps_last_ts);
    dfree(h->d_ps_cmode);
    dfree(h->d_ps_ckey);
    dfree(h->d_ps_gkey);
    dfree(h->d_cp_owner);
    dfree(h->d_cp_pslot);
    dfree(h->d_cp_long);
    dfree(h->d_cp_short);
    dfree(h->d_cp_slot_item);
    dfree(h->d_p_msb);
    dfree(h->d_p_mt);
    dfree(h->d_p_mbk);
    dfree(h->d_cp_bnd);
    dfree(h->d_cp_p0);
    dfree(h->d_cp_np);
    dfree(h->d_cp_items);
    dfree(h->d_cp_counts);
    dfree(h->d_cp_mlist);
    dfree(h->d_cp_chk);
    dfree(h->d_cp_assume);
    dfree(h->d_cp_rec);
    dfree(h->d_cp_rec2);
    dfree(h->d_cp_hist);
    dfree(h->d_cp_save);
    dfree(h->d_cp_ckpt);
    dfree(h->d_cp_skips);
    dfree(h->d_cp_skip_count);
    dfree(h->d_cp_changed);
    dfree(h->d_cp_rule_lim);
    dfree(h->d_cnow);
    dfree(h->d_cthr);
    dfree(h->d_coff);
    dfree(h->d_cres);
    dfree(h->d_cfid);
    dfree(h->d_ctok);
    dfree(h->d_calive);
    dfree(h->d_clast_ts);
    dfree(h->d_creq_h);
    dfree(h->d_cout_h);
    dfree(h->d_lhead);
    dfree(h->d_lsec);
    dfree(h->d_lbor);
    dfree(h->d_lmin);
    dfree(h->d_llast_ts);
    dfree(h->d_lev_h);
    for (auto& w : h->lws) {
        dfree(w.pslot);
        dfree(w.cxside);
        dfree(w.flags);
        dfree(w.cxw_next);
        dfree(w.cx_list);
        dfree(w.exit_pos);
        dfree(w.exit_cnt);
        dfree(w.skips);
        dfree(w.skip_count);
    }
    dfree(h->d_lout_h);
    dfree(h->d_lext_h);
    dfree(h->d_lgkey);
    dfree(h->d_linbound);
    dfree(h->d_lentry_acc);
    dfree(h->d_lm_cnt);
    dfree(h->d_lm_gate);
    dfree(h->d_lentry_fetch);
    dfree(h->d_req_h);
    dfree(h->d_out_h);
    drain_async(h);
    for (auto& sl : h->slots) {
        dfree(sl.d_req);
        dfree(sl.d_out);
        if (sl.h_err) (void)hipHostFree(sl.h_err);
        for (hipEvent_t e : {sl.h2d, sl.comp, sl.d2h})
            if (e) (void)hipEventDestroy(e);
    }
    for (hipStream_t st : {h->s_in, h->s_comp, h->s_out})
        if (st) (void)hipStreamDestroy(st);
    if (h->h_err) (void)hipHostFree(h->h_err);
    if (h->h_long) (void)hipHostFree(h->h_long);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->fork) (void)hipEventDestroy(h->fork);
    if (h->join) (void)hipEventDestroy(h->join);
    if (h->aux) (void)hipStreamDestroy(h->aux);
    delete h;
}

const char* sg_last_error(const sg_handle* h) { return h ? h->err.c_str() : "null handle"; }

int sg_set_shard(sg_handle* h, int32_t rank, int32_t world) {
    if (h) drain_async(h);
    if (!h || world < 1 || rank < 0 || rank >= world) return SG_E_INVAL;
    h->shard_rank = rank;
    h->shard_world = world;
    return SG_OK;
}

int sg_lim_slots(const sg_handle* h, uint32_t* n_lim) {
    if (!h || !n_lim) return SG_E_INVAL;
    *n_lim = (uint32_t)h->n_lim;
    return SG_OK;
}

int sg_lim_arrivals(sg_handle* h, const sg_req* req, uint64_t n, int64_t t_base, uint32_t n_ms, uint32_t* counts_out,
                    uint64_t counts_words, void* stream_) {
    if (!h || (!req && n) || !counts_out) return SG_E_INVAL;
    if (t_base < 0 || n_ms == 0 || n_ms > kMaxPeriods) return fail(h, SG_E_INVAL, "exchange range: t_base >= 0, 1 <= n_ms <= 65536");
    if (counts_words != (uint64_t)h->n_lim * n_ms)
        return fail(h, SG_E_INVAL, "counts buffer must hold n_lim * n_ms words (sg_lim_slots)");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(h, hipSetDevice(h->device));
    // reads only the request batch and the rule → limiter table: batches in flight on the pipeline go on
    int rc = ensure_layout(h);
    if (rc) return rc;
    if (!h->d_limx_err && (hipMalloc(&h->d_limx_err, sizeof(int)) != hipSuccess ||
                           hipHostMalloc(&h->h_limx_err, sizeof(int)) != hipSuccess))
        return fail(h, SG_E_NOMEM, "exchange error word");
    HIP_TRY(h, hipMemsetAsync(counts_out, 0, sizeof(uint32_t) * (size_t)h->n_lim * n_ms, stream));
    HIP_TRY(h, hipMemsetAsync(h->d_limx_err, 0, sizeof(int), stream));
    if (h->n_lim > 0)
        HIP_TRY(h, launch_lim_arrivals(req, n, h->K, h->d_rule_lim, t_base, n_ms, counts_out, h->d_limx_err, stream));
    HIP_TRY(h, hipMemcpyAsync(h->h_limx_err, h->d_limx_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    return flow_status(h, *h->h_limx_err);
}

namespace {
int cp_rule_limiters(sg_handle* h, hipStream_t stream);
}

int sg_lim_arrivals_param(sg_handle* h, const sg_cparam_req* req, uint64_t n, int64_t t_base, uint32_t n_ms,
                          uint32_t* counts_out, uint64_t counts_words, void* stream_) {
    if (!h || (!req && n) || !counts_out) return SG_E_INVAL;
    if (t_base < 0 || n_ms == 0 || n_ms > kMaxPeriods) return fail(h, SG_E_INVAL, "exchange range: t_base >= 0, 1 <= n_ms <= 65536");
    if (counts_words != (uint64_t)h->n_lim * n_ms)
        return fail(h, SG_E_INVAL, "counts buffer must hold n_lim * n_ms words (sg_lim_slots)");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(h, hipSetDevice(h->device));
    int rc = cp_rule_limiters(h, stream);
    if (rc) return rc;
    if (!h->d_limx_err && (hipMalloc(&h->d_limx_err, sizeof(int)) != hipSuccess ||
                           hipHostMalloc(&h->h_limx_err, sizeof(int)) != hipSuccess))
        return fail(h, SG_E_NOMEM, "exchange error word");
    HIP_TRY(h, hipMemsetAsync(counts_out, 0, sizeof(uint32_t) * (size_t)h->n_lim * n_ms, stream));
    HIP_TRY(h, hipMemsetAsync(h->d_limx_err, 0, sizeof(int), stream));
    if (h->n_lim > 0 && h->d_cp_rule_lim)
        HIP_TRY(h, launch_lim_arrivals_param(req, n, (uint32_t)h->cprules.size(), h->d_cp_rule_lim, t_base, n_ms,
                                             counts_out, h->d_limx_err, stream));
    HIP_TRY(h, hipMemcpyAsync(h->h_limx_err, h->d_limx_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    return flow_status(h, *h->h_limx_err);
}

int sg_lim_exchange(sg_handle* h, const uint32_t* gathered, uint64_t gathered_words, int64_t t_base, uint32_t n_ms) {
    if (!h || !gathered) return SG_E_INVAL;
    if (t_base < 0 || n_ms == 0 || n_ms > kMaxPeriods) return fail(h, SG_E_INVAL, "exchange range: t_base >= 0, 1 <= n_ms <= 65536");
    if (gathered_words != (uint64_t)h->shard_world * (uint64_t)h->n_lim * n_ms)
        return fail(h, SG_E_INVAL, "gathered buffer must hold world * n_lim * n_ms words (sg_lim_slots)");
    h->lim_xg = gathered;
    h->lim_xt = t_base;
    h->lim_xn = n_ms;
    h->lim_x_armed = true;
    return SG_OK;
}

int sg_set_namespaces(sg_handle* h, const sg_namespace* ns, uint32_t n) {
    if (!h || (!ns && n)) return SG_E_INVAL;
    int want = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (ns[i].limiter_enabled) {
            if (!(ns[i].max_allowed_qps >= 0)) return fail(h, SG_E_INVAL, "max allowed QPS should >= 0");
            ++want;
        }
    }
    if (want > kMaxLim) return fail(h, SG_E_UNSUPPORTED, "more than 8 namespaces with a QPS limiter");
    h->conc_dirty = true;  // AVG_LOCAL concurrency thresholds read connectedCount
    for (const auto& r : h->rules)
        if (r.namespace_id < 0 || (uint32_t)r.namespace_id >= n)
            return fail(h, SG_E_INVAL, "a loaded rule refers to a namespace that would disappear");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    // A namespace that keeps its limiter keeps its window (GlobalRequestLimiter.initIfAbsent :32-37,
    // applyMaxQpsChange :73-80); a newly enabled one starts empty.
    LimRing old[kMaxLim], nw[kMaxLim];
    if (h->n_lim) HIP_TRY(h, hipMemcpy(old, h->d_lim_ring, sizeof(LimRing) * kMaxLim, hipMemcpyDeviceToHost));
    std::vector<int> slot(n, -1);
    int n_lim = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!ns[i].limiter_enabled) continue;
        const int s_new = n_lim++;
        slot[i] = s_new;
        h->lim_qps[s_new] = ns[i].max_allowed_qps;
        const int s_old = (i < h->ns_slot.size()) ? h->ns_slot[i] : -1;
        if (s_old >= 0) {
            nw[s_new] = old[s_old];
        } else {
            for (int j = 0; j < kLimSamples; ++j) {
                nw[s_new].start[j] = INT64_MIN;
                nw[s_new].count[j] = 0;
            }
        }
    }
    if (n_lim) HIP_TRY(h, hipMemcpy(h->d_lim_ring, nw, sizeof(LimRing) * n_lim, hipMemcpyHostToDevice));
    h->ns.assign(ns, ns + n);
    h->ns_slot = slot;
    h->n_lim = n_lim;
    if (!h->cptab.empty()) {  // AVG_LOCAL param thresholds follow the connected counts
        for (size_t i = 0; i < h->cptab.size(); ++i) {
            const int nsi = h->cprules[i].namespace_id;
            h->cptab[i].connected = (nsi >= 0 && (uint32_t)nsi < n) ? ns[nsi].connected_count : 0;
        }
        HIP_TRY(h, hipMemcpy(h->d_cprules, h->cptab.data(), sizeof(CPRule) * h->cptab.size(), hipMemcpyHostToDevice));
    }
    return upload_rule_table(h);
}

namespace {

// Every check sg_load_flow_rules makes before it changes anything (FlowRuleUtil.isValidRule / checkClusterField,
// FlowRuleUtil.java:167-229, and the device path's limits: sampleCount <= 64 for a surviving metric's window shape
// too, <= 8 distinct window lengths with the limiter's 100 ms): after SG_OK only allocation or device errors remain.
int flow_rules_validate(sg_handle* h, const sg_flow_rule* rules, uint32_t n) {
    if (n >= SG_KEY_BAD) return fail(h, SG_E_INVAL, "too many rules");
    std::unordered_map<int64_t, uint32_t> seen, old_index;
    for (uint32_t k = 0; k < h->K; ++k) old_index.emplace(h->rules[k].flow_id, k);
    std::vector<int32_t> wls;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_flow_rule& r = rules[i];
        if (r.flow_id <= 0) return fail(h, SG_E_INVAL, "flowId must be > 0");
        if (!(r.count >= 0)) return fail(h, SG_E_INVAL, "count must be >= 0");
        if (r.sample_count <= 0 || r.window_interval_ms <= 0 || r.window_interval_ms % r.sample_count != 0)
            return fail(h, SG_E_INVAL, "invalid window config");
        if (r.namespace_id < 0 || (size_t)r.namespace_id >= h->ns.size())
            return fail(h, SG_E_INVAL, "unknown namespace");
        if (!seen.emplace(r.flow_id, i).second) return fail(h, SG_E_INVAL, "duplicate flowId");
        int S = r.sample_count, wl = r.window_interval_ms / r.sample_count;
        auto it = old_index.find(r.flow_id);
        if (it != old_index.end()) {
            S = h->rule_tab[it->second].S;
            wl = h->rule_tab[it->second].wl;
        }
        if (S > SG_MAX_SAMPLE_COUNT) return fail(h, SG_E_UNSUPPORTED, "sampleCount > 64 is not supported by the device path");
        if (std::find(wls.begin(), wls.end(), wl) == wls.end()) wls.push_back(wl);
    }
    if (h->n_lim > 0 && std::find(wls.begin(), wls.end(), (int32_t)kLimWindowMs) == wls.end()) wls.push_back(kLimWindowMs);
    if (wls.size() > (size_t)kMaxWl) return fail(h, SG_E_UNSUPPORTED, "more than 8 distinct window lengths");
    return SG_OK;
}

}  // namespace

namespace {

// The new rule set's device state, built beside the live one (which it only reads: surviving flowIds' rings and
// occupy counters are copied over), so that a failure leaves the handle as it was; flow_rules_commit swaps it in,
// flow_rules_abort frees it. The node handle prepares every shard before it commits any.
struct FlowLoad {
    std::vector<Rule> tab;
    std::vector<int32_t> src;
    int stride = 1;
    int n_wl = 0;
    int32_t wl[kMaxWl]{};
    Rule* d_rules = nullptr;
    Bucket* d_ring = nullptr;
    BucketHot* d_hot = nullptr;
    Occ* d_occ = nullptr;
    uint32_t* d_seg_end = nullptr;
};

void flow_rules_abort(FlowLoad& L) {
    dfree(L.d_rules);
    dfree(L.d_ring);
    dfree(L.d_hot);
    dfree(L.d_occ);
    dfree(L.d_seg_end);
}

int flow_rules_prepare_impl(sg_handle* h, const sg_flow_rule* rules, uint32_t n, FlowLoad& L) {
    // old flowId → old index, to keep the metric of surviving flows (ClusterFlowRuleManager.java:361)
    std::unordered_map<int64_t, uint32_t> old_index;
    for (uint32_t k = 0; k < h->K; ++k) old_index.emplace(h->rules[k].flow_id, k);

    L.tab.assign(n, Rule{});
    L.src.assign(n, -1);
    std::vector<Rule>& tab = L.tab;
    std::vector<int32_t>& src = L.src;
    int& stride = L.stride;
    int& n_wl = L.n_wl;
    int32_t* wl = L.wl;
    for (uint32_t i = 0; i < n; ++i) {
        int S = rules[i].sample_count, interval = rules[i].window_interval_ms;
        auto it = old_index.find(rules[i].flow_id);
        if (it != old_index.end()) {  // the existing ClusterMetric keeps its window shape
            src[i] = (int32_t)it->second;
            S = h->rule_tab[it->second].S;
            interval = h->rule_tab[it->second].S * h->rule_tab[it->second].wl;
        }
        if (S > SG_MAX_SAMPLE_COUNT)
            return fail(h, SG_E_UNSUPPORTED, "sampleCount > 64 is not supported by the device path");
        Rule R{};
        R.S = S;
        R.wl = interval / S;
        R.isec = interval / 1000.0;
        R.wait_ms = 1000 / S;
        int w = 0;
        while (w < n_wl && wl[w] != R.wl) ++w;
        if (w == n_wl) {
            if (n_wl == kMaxWl) return fail(h, SG_E_UNSUPPORTED, "more than 8 distinct window lengths");
            wl[n_wl++] = R.wl;
        }
        R.wl_idx = w;  // final indices come from rebuild_wl_table (adds the limiter's 100 ms)
        stride = std::max(stride, S);
        tab[i] = R;
    }

    Rule*& d_rules = L.d_rules;
    Bucket*& d_ring = L.d_ring;
    BucketHot*& d_hot = L.d_hot;
    Occ*& d_occ = L.d_occ;
    uint32_t*& d_seg_end = L.d_seg_end;
    int32_t* d_src = nullptr;
    if (n && h->front_only) {  // a node's front: rule thresholds and limiter slots only
        if (hipMalloc(&d_rules, sizeof(Rule) * n) != hipSuccess) return fail(h, SG_E_NOMEM, "rule table");
    } else if (n) {
        if (hipMalloc(&d_rules, sizeof(Rule) * n) != hipSuccess || hipMalloc(&d_seg_end, sizeof(uint32_t) * 2 * n) != hipSuccess ||
            hipMalloc(&d_ring, sizeof(Bucket) * (size_t)n * stride) != hipSuccess ||
            hipMalloc(&d_hot, sizeof(BucketHot) * (size_t)n * stride) != hipSuccess ||
            hipMalloc(&d_occ, sizeof(Occ) * n) != hipSuccess || hipMalloc(&d_src, sizeof(int32_t) * n) != hipSuccess) {
            dfree(d_src);
            return fail(h, SG_E_NOMEM, "rule state allocation failed");
        }
        HIP_TRY(h, hipMemset(d_seg_end, 0, sizeof(uint32_t) * n));           // no segment ends marked
        HIP_TRY(h, hipMemset(d_seg_end + n, 0xFF, sizeof(uint32_t) * n));  // no segment starts marked
        HIP_TRY(h, hipMemcpy(d_src, src.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, launch_init_state(d_ring, d_occ, n, stride, d_src, h->d_ring, h->d_occ, h->stride, 0));
        HIP_TRY(h, launch_hot_sync(d_ring, d_hot, (uint64_t)n * stride, 0));
        HIP_TRY(h, hipDeviceSynchronize());
        dfree(d_src);
    }
    return SG_OK;
}

int flow_rules_prepare(sg_handle* h, const sg_flow_rule* rules, uint32_t n, FlowLoad& L) {
    const int rc = flow_rules_prepare_impl(h, rules, n, L);
    if (rc) flow_rules_abort(L);
    return rc;
}

int flow_rules_commit(sg_handle* h, const sg_flow_rule* rules, uint32_t n, FlowLoad& L) {
    std::vector<int32_t>& src = L.src;
    if (h->d_cnow) {  // CurrentConcurrencyManager: surviving flowIds keep nowCalls, new ones start at 0
        // the counters in the current rule order: a reload not yet uploaded (cnow_pending) already holds them
        // remapped to h->K / h->rules; d_cnow is still in the order of the rules before that reload
        std::vector<int32_t> old(h->K, 0);
        if (h->cnow_pending) {
            for (uint32_t k = 0; k < h->K && k < h->cnow_host.size(); ++k) old[k] = h->cnow_host[k];
        } else if (h->K) {
            HIP_TRY(h, hipMemcpy(old.data(), h->d_cnow, sizeof(int32_t) * h->K, hipMemcpyDeviceToHost));
        }
        h->cnow_host.assign(n, 0);
        for (uint32_t i = 0; i < n; ++i)
            if (src[i] >= 0) h->cnow_host[i] = old[src[i]];
        h->cnow_pending = true;
    }
    h->c_off.assign(n, 2000);  // ClusterFlowConfig.clientOfflineTime / resourceTimeout defaults
    h->c_res.assign(n, 2000);
    h->conc_dirty = true;
    dfree(h->d_rules);
    dfree(h->d_ring);
    dfree(h->d_hot);
    dfree(h->d_occ);
    dfree(h->d_seg_end);
    h->d_rules = L.d_rules;
    h->d_ring = L.d_ring;
    h->d_hot = L.d_hot;
    h->d_occ = L.d_occ;
    h->d_seg_end = L.d_seg_end;
    L.d_rules = nullptr;
    L.d_ring = nullptr;
    L.d_hot = nullptr;
    L.d_occ = nullptr;
    L.d_seg_end = nullptr;
    h->rules.assign(rules, rules + n);
    h->rule_tab = L.tab;
    h->K = n;
    ++h->rules_gen;
    h->stride = L.stride;
    h->n_wl = L.n_wl;
    std::memcpy(h->wl, L.wl, sizeof(L.wl));
    int rc = layout_records(h);
    if (rc) return rc;
    rc = upload_fid_table(h);
    if (rc) return rc;
    return upload_rule_table(h);
}

}  // namespace

int sg_load_flow_rules(sg_handle* h, const sg_flow_rule* rules, uint32_t n) {
    if (h) drain_async(h);
    if (!h || (!rules && n)) return SG_E_INVAL;
    (void)hipSetDevice(h->device);
    const int vrc = flow_rules_validate(h, rules, n);
    if (vrc) return vrc;
    FlowLoad L;
    const int rc = flow_rules_prepare(h, rules, n, L);
    if (rc) return rc;
    return flow_rules_commit(h, rules, n, L);
}

// flowId → rule index for the wire codec: open addressing, linear probing, load factor <= 1/2 (the same
// splitmix64 finaliser as codec.hip's fid_hash). flowIds are > 0 and unique (validated above).
static uint64_t host_fid_hash(int64_t fid) {
    uint64_t z = (uint64_t)fid + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int upload_fid_table(sg_handle* h) {
    uint64_t cap = 2;
    while (cap < 2ull * h->K) cap <<= 1;
    std::vector<FidSlot> tab(cap, FidSlot{0, 0, 0});
    for (uint32_t k = 0; k < h->K; ++k) {
        const int64_t fid = h->rules[k].flow_id;
        uint64_t p = host_fid_hash(fid) & (cap - 1);
        while (tab[p].fid != 0) p = (p + 1) & (cap - 1);
        tab[p] = FidSlot{fid, k, 0};
    }
    FidSlot* d = nullptr;
    if (hipMalloc(&d, sizeof(FidSlot) * cap) != hipSuccess) return fail(h, SG_E_NOMEM, "flowId table");
    if (hipMemcpy(d, tab.data(), sizeof(FidSlot) * cap, hipMemcpyHostToDevice) != hipSuccess) {
        dfree(d);
        return fail(h, SG_E_DEVICE, "flowId table upload");
    }
    dfree(h->d_fid);
    h->d_fid = d;
    h->fid_mask = cap - 1;
    return SG_OK;
}

int sg_codec_decode_flow(sg_handle* h, const uint8_t* payload, const uint32_t* offsets, const int64_t* ts_ms,
                         uint64_t n, sg_req* req_out, int32_t* xid_out, uint8_t* kind_out, void* stream) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!payload || !offsets || !ts_ms || !req_out || !xid_out || !kind_out) return fail(h, SG_E_INVAL, "null buffer");
    if (((uintptr_t)payload & 3u) != 0) return fail(h, SG_E_INVAL, "payload must be 4-byte aligned");
    if (!h->d_fid) {
        int rc = upload_fid_table(h);  // no rules loaded yet: every flowId is unknown
        if (rc) return rc;
    }
    HIP_TRY(h, hipSetDevice(h->device));
    CodecArgs c{};
    c.n = n;
    c.payload = payload;
    c.offsets = offsets;
    c.ts = ts_ms;
    c.req = req_out;
    c.xid = xid_out;
    c.kind = kind_out;
    c.fid_tab = h->d_fid;
    c.fid_mask = h->fid_mask;
    HIP_TRY(h, launch_codec_decode(c, (hipStream_t)stream));
    return SG_OK;
}

int sg_codec_encode_flow(sg_handle* h, const int32_t* xid, const uint8_t* kind, const sg_result* res, uint64_t n,
                         uint8_t* frames_out, void* stream) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!xid || !kind || !res || !frames_out) return fail(h, SG_E_INVAL, "null buffer");
    if (((uintptr_t)frames_out & 15u) != 0) return fail(h, SG_E_INVAL, "frames_out must be 16-byte aligned");
    HIP_TRY(h, hipSetDevice(h->device));
    CodecArgs c{};
    c.n = n;
    c.xid_in = xid;
    c.kind_in = kind;
    c.res = res;
    c.frames = frames_out;
    HIP_TRY(h, launch_codec_encode(c, (hipStream_t)stream));
    return SG_OK;
}

int sg_enable_stats(sg_handle* h, int on) {
    if (!h) return SG_E_INVAL;
    h->stats_on = on != 0;
    return SG_OK;
}

int sg_get_stats(const sg_handle* h, sg_batch_stats* out) {
    if (!h || !out) return SG_E_INVAL;
    *out = h->stats;
    return SG_OK;
}

namespace {

// The batch's error flags → return code (the batch is rejected as a whole; no state changed).
int flow_status(sg_handle* h, int err) {
    if (err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (err & kErrPeriods) return fail(h, SG_E_UNSUPPORTED, "batch spans more than 65536 window periods");
    if (err & kErrInternal) return fail(h, SG_E_DEVICE, "internal walker error");
    if (err & kErrExchange)
        return fail(h, SG_E_INVAL, "a request of a limited namespace lies outside the limiter exchange's time range");
    return SG_OK;
}

// A local batch's error flags → return code (rejected as a whole; no state changed).
int local_status(sg_handle* h, int err) {
    if (err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (err & kErrPeriods) return fail(h, SG_E_UNSUPPORTED, "batch spans more than 65536 window periods");
    if (err & kErrBounds)
        return fail(h, SG_E_INVAL, "an event's origin id (0..n_origins), context id (0..n_contexts-1) or arguments "
                                   "(the arg / value arrays) are out of range");
    if (err & kErrTableFull) return fail(h, SG_E_CAPACITY, "a param value or thread-count table is full");
    if (err & kErrInternal) return fail(h, SG_E_DEVICE, "internal walker error");
    return SG_OK;
}

int ticket_status(sg_handle* h, const sg_handle::DevTicket& d) {
    if (!d.local) return flow_status(h, *d.h_err);
    const int rc = local_status(h, *d.h_err);
    // a refused pipelined batch (e.g. its first timestamp behind the previous batch's, found by the back half)
    // decided nothing: it does not count as a batch seen (enqueue_local_pipelined counted it)
    if (rc != SG_OK && h->l_batches > 0) --h->l_batches;
    return rc;
}

// Workspace 0: the handle's own batch buffers.
void main_ws(sg_handle* h, sg_handle::FlowWs& w) {
    w.rec = h->d_rec;
    w.rec_sorted = h->d_rec_sorted;
    w.hist = h->d_hist;
    w.bnd = h->d_bnd;
    w.p0 = h->d_p0;
    w.np = h->d_np;
    w.err = h->d_err;
    w.long_list = h->d_long_list;
    w.long_key = h->d_long_key;
    w.long_end = h->d_long_end;
    w.long_pend = h->d_long_pend;
    w.short_list = h->d_short_list;
    w.short_key = h->d_short_key;
    w.counts = h->d_long_count;
    w.skips = h->d_skips;
    w.skip_count = h->d_skip_count;
    w.seg_end = h->d_seg_end;
    w.seg_start = h->d_seg_end ? h->d_seg_end + h->K : nullptr;
    w.short_end = h->d_short_end;
    w.bin_buf = h->d_bin_buf;
}

// Workspace 1 and the pipeline's streams / events, allocated on first pipelined batch (seg_end grows with K).
int pipe_setup(sg_handle* h) {
    auto& w = h->pws;
    const uint64_t n = h->cfg.max_batch;
    if (!w.rec) {
        uint64_t short_words = 0;
        for (int c = 0; c < kClasses; ++c) short_words += (c == 0 ? n : n / (kClassMax[c - 1] + 1)) + 1;
        if (hipMalloc(&w.rec, (n + kRecW) * 8) != hipSuccess || hipMalloc(&w.rec_sorted, (n + kRecW) * 8) != hipSuccess ||
            hipMalloc(&w.hist, sizeof(uint32_t) * radix_hist_words(n)) != hipSuccess ||
            hipMalloc(&w.bnd, sizeof(uint32_t) * kMaxWl * kMaxPeriods) != hipSuccess ||
            hipMalloc(&w.p0, sizeof(int64_t) * kMaxWl) != hipSuccess ||
            hipMalloc(&w.np, sizeof(uint32_t) * kMaxWl) != hipSuccess || hipMalloc(&w.err, sizeof(int)) != hipSuccess ||
            hipMalloc(&w.long_list, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
            hipMalloc(&w.long_key, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
            hipMalloc(&w.long_end, sizeof(uint32_t) * (n + 1)) != hipSuccess ||
            hipMalloc(&w.long_pend, sizeof(uint32_t) * (size_t)kLongTab * kLongPeriods) != hipSuccess ||
            hipMalloc(&w.short_list, sizeof(uint32_t) * short_words) != hipSuccess ||
            hipMalloc(&w.short_key, sizeof(uint32_t) * short_words) != hipSuccess ||
            hipMalloc(&w.short_end, sizeof(uint32_t) * short_words) != hipSuccess ||
            hipMalloc(&w.counts, (1 + kClasses) * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&w.skips, sizeof(uint4) * (2 * n / kSkipMin + 1)) != hipSuccess ||
            hipMalloc(&w.skip_count, sizeof(uint32_t)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "pipeline workspace");
        // CU partition between the halves (env SG_FRONT_EIGHTHS = k: the front half gets CUs i with i % 8 < k,
        // the walkers the rest; 0 = no masks, both halves on every CU)
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
        int k8 = h->front_eighths;
        if (const char* e = std::getenv("SG_FRONT_EIGHTHS")) k8 = std::atoi(e);
        // env SG_CU_BLOCKED=1 (tuning): the front half gets CUs i with i / (cus / 8) < k (contiguous eighths)
        const bool blocked = std::getenv("SG_CU_BLOCKED") && std::atoi(std::getenv("SG_CU_BLOCKED")) == 1;
        if (k8 > 0 && k8 < 8 && cus >= 8) {
            std::vector<uint32_t> fm((cus + 31) / 32, 0u), bm((cus + 31) / 32, 0u);
            int nb = 0;
            for (int i = 0; i < cus; ++i) {
                if ((blocked ? i / (cus / 8) : i % 8) < k8) fm[i / 32] |= 1u << (i % 32);
                else {
                    bm[i / 32] |= 1u << (i % 32);
                    ++nb;
                }
            }
            HIP_TRY(h, hipExtStreamCreateWithCUMask(&h->s_front, (uint32_t)fm.size(), fm.data()));
            HIP_TRY(h, hipExtStreamCreateWithCUMask(&h->s_back, (uint32_t)bm.size(), bm.data()));
            HIP_TRY(h, hipExtStreamCreateWithCUMask(&h->s_aux2, (uint32_t)bm.size(), bm.data()));
            HIP_TRY(h, hipExtStreamCreateWithCUMask(&h->s_aux3, (uint32_t)bm.size(), bm.data()));
            h->walk_cus = nb;
        } else {
            HIP_TRY(h, hipStreamCreateWithFlags(&h->s_front, hipStreamNonBlocking));
            HIP_TRY(h, hipStreamCreateWithFlags(&h->s_back, hipStreamNonBlocking));
            HIP_TRY(h, hipStreamCreateWithFlags(&h->s_aux2, hipStreamNonBlocking));
            HIP_TRY(h, hipStreamCreateWithFlags(&h->s_aux3, hipStreamNonBlocking));
        }
        HIP_TRY(h, hipEventCreateWithFlags(&h->tjoin, hipEventDisableTiming));
        for (int x = 0; x < 2; ++x) {
            HIP_TRY(h, hipEventCreateWithFlags(&h->front_done[x], hipEventDisableTiming));
            HIP_TRY(h, hipEventCreateWithFlags(&h->back_done[x], hipEventDisableTiming));
        }
        HIP_TRY(h, hipEventCreateWithFlags(&h->pfork, hipEventDisableTiming));
        HIP_TRY(h, hipEventCreateWithFlags(&h->pjoin, hipEventDisableTiming));
    }
    if (h->pws_segcap < h->K) {
        dfree(w.seg_end);
        if (hipMalloc(&w.seg_end, sizeof(uint32_t) * 2 * (h->K + 1)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "pipeline workspace");
        h->pws_segcap = h->K + 1;
        HIP_TRY(h, hipMemset(w.seg_end, 0, sizeof(uint32_t) * h->pws_segcap));
        HIP_TRY(h, hipMemset(w.seg_end + h->pws_segcap, 0xFF, sizeof(uint32_t) * h->pws_segcap));
    }
    w.seg_start = w.seg_end + h->pws_segcap;
    return SG_OK;
}

BatchArgs flow_args(sg_handle* h, const sg_handle::FlowWs& w, const sg_req* req, uint64_t n, sg_result* out) {
    BatchArgs a{};
    a.req = req;
    a.out = out;
    a.n = n;
    a.rec = w.rec;
    a.rec_sorted = w.rec_sorted;
    a.hist0 = h->n_lim > 0 ? nullptr : w.hist;  // the limiter pre-pass rewrites records after k_prep
    a.hist0_bits = radix_digit_bits(h->kbits);
    a.kshift = 64 - h->kbits;
    a.hist0_shift = a.kshift;
    a.abits = h->abits;
    a.imask = (h->ibits >= 64) ? ~0ull : ((1ull << h->ibits) - 1);
    a.amask = (1ull << h->abits) - 1;
    a.aesc = (1ull << (h->abits - 1)) - 1;
    a.K = h->K;
    a.rules = h->d_rules;
    a.ring = h->d_ring;
    a.hot = h->d_hot;
    a.occ = h->d_occ;
    a.seg_end = w.seg_end;
    a.seg_start = w.seg_start;
    a.short_end = w.short_end;
    a.stride = h->stride;
    a.max_occ_ratio = h->cfg.max_occupy_ratio;
    a.n_wl = h->n_wl;
    std::memcpy(a.wl, h->wl, sizeof(a.wl));
    a.bnd = w.bnd;
    a.p0 = w.p0;
    a.np = w.np;
    a.err = w.err;
    a.last_ts = h->d_last_ts;
    a.check_last = 1;
    a.walk_cus = 0;
    a.long_list = w.long_list;
    a.long_count = w.counts;
    a.short_list = w.short_list;
    a.short_key = w.short_key;
    a.long_key = w.long_key;
    a.long_end = w.long_end;
    a.long_pend = w.long_pend;
    a.short_count = w.counts + 1;
    for (int c = 0; c < kClasses; ++c) a.class_off[c] = h->class_off[c];
    a.skips = w.skips;
    a.skip_count = w.skip_count;
    a.dbg = h->dbg;
    a.generic_walker = (h->cfg.flags & SG_FLAG_RING_REREAD) != 0;
    a.narrow = h->wide_seen ? 0 : 1;
    a.dbg_ctr = h->d_dbg;
    a.skip_cap = (uint32_t)(2 * h->cfg.max_batch / kSkipMin + 1);
    a.short_max = (h->cfg.flags & SG_FLAG_WAVE_ONLY) ? 0u
                  : (h->cfg.flags & SG_FLAG_SERIAL_ONLY) ? 0xFFFFFFFFu : h->short_max;
    a.tiny = tiny_walker_enabled(a) ? 1 : 0;
    return a;
}

// Front half of a batch on `stream`: validation and packed records (k_prep), the namespace limiter pre-pass,
// the stable sort by flowId and the segment lists. Touches only the workspace, the caller's output (default
// results) and the limiter state.
// The namespace limiter pre-pass over a batch's records (after k_prep): TOO_MANY_REQUEST results, sentinel records.
int flow_limiter(sg_handle* h, BatchArgs& a, hipStream_t stream) {
    if (h->n_lim > 0) {
        LimArgs L{};
        L.n_lim = h->n_lim;
        L.wl_idx = h->lim_wl_idx;
        std::memcpy(L.qps, h->lim_qps, sizeof(L.qps));
        L.rule_lim = h->d_rule_lim;
        L.slot = h->d_lim_slot;
        const uint64_t tiles = a.n / 4096 + 1;
        L.tile_tot = h->d_lim_tile;
        L.tile_off = h->d_lim_tile + tiles * kMaxLim;
        L.arrivals = h->d_lim_period;
        L.prefix = h->d_lim_period + (size_t)kMaxLim * kMaxPeriods;
        L.quota = h->d_lim_period + (size_t)2 * kMaxLim * kMaxPeriods;
        L.ring = h->d_lim_ring;
        if (h->lim_x_armed) {
            L.xg = h->lim_xg;
            L.ts = &a.req[0].ts_ms;
            L.ts_stride = sizeof(sg_req) / sizeof(int64_t);
            L.t_base = h->lim_xt;
            L.n_ms = h->lim_xn;
            L.world = h->shard_world;
            L.rank = h->shard_rank;
        }
        HIP_TRY(h, launch_limiter(a, L, stream));
    }
    return SG_OK;
}

// The binned front half (engine.hip k_bin_sort) for a flow batch of workspace w when the handle's records allow it:
// >= 2^14 flowIds (SG_BIN=2: any), at most 2^20 (a regular bin holds <= 2048 flowIds), kBinDigit free middle bits,
// no namespace limiter (its pre-pass rewrites records after k_prep). Sets a's bin fields; false: the two-pass sort.
bool bin_setup(sg_handle* h, sg_handle::FlowWs& w, BatchArgs& a, hipStream_t stream) {
    if (h->bin_mode == 0 || h->n_lim > 0 || !a.hist0 || a.n == 0 || h->K == 0) return false;
    if (h->bin_mode == 1 && h->K < (1u << 14)) return false;
    if (64 - h->kbits - h->ibits - h->abits < kBinDigit) return false;
    const int kb = h->K > 1 ? bits_for((uint64_t)h->K - 1) : 1;
    const int bsh = std::max(0, kb - 9);
    if (bsh > kBinMaxBsh || (((h->K - 1) >> bsh) + 1) > kBinRegular) return false;
    if (!h->d_hot_key) {
        if (hipMalloc(&h->d_hot_key, sizeof(uint32_t) * (kBinHot + 1) + sizeof(uint2) * kHotTab) != hipSuccess)
            return false;
        h->hot_gen = ~0ull;
    }
    uint2* tab = reinterpret_cast<uint2*>(h->d_hot_key + kBinHot + 1);
    if (!w.bin_buf) {
        if (hipMalloc(&w.bin_buf, (h->cfg.max_batch + kRecW) * 8) != hipSuccess) return false;
        if (w.rec == h->d_rec) h->d_bin_buf = w.bin_buf;
        else h->pws.bin_buf = w.bin_buf;
    }
    if (h->hot_gen != h->rules_gen) {  // flowIds renumbered: no hot flowIds yet (stream-ordered before k_prep)
        if (launch_hot_reset(tab, stream) != hipSuccess) return false;
        h->hot_gen = h->rules_gen;
    }
    a.bin_on = 1;
    a.prep_tiles = h->prep_tiles;
    a.bin_dshift = h->abits + h->ibits;
    a.bin_bsh = bsh;
    a.bin_R = ((h->K - 1) >> bsh) + 1;
    a.hot_tab = tab;
    a.hot_key = h->d_hot_key;
    a.bin_buf = w.bin_buf;
    a.hist0_bits = kBinDigit;
    a.hist0_shift = a.bin_dshift;
    return true;
}

int flow_front(sg_handle* h, BatchArgs& a, uint32_t* hist, hipStream_t stream, bool stats) {
    if (stats) HIP_TRY(h, hipEventRecord(h->ev[0], stream));
    HIP_TRY(h, hipMemsetAsync(a.err, 0, sizeof(int), stream));
    HIP_TRY(h, hipMemsetAsync(a.long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream));
    HIP_TRY(h, hipMemsetAsync(a.skip_count, 0, sizeof(uint32_t), stream));
    a.csum0 = nullptr;
    if (a.hist0 && radix_csum_atomic()) {
        a.csum0 = radix_csum(a.hist0, a.n, a.hist0_bits);
        HIP_TRY(h, hipMemsetAsync(a.csum0, 0, radix_csum_bytes(a.n, a.hist0_bits), stream));
    }
    HIP_TRY(h, launch_prep(a, stream));
    const int lrc = flow_limiter(h, a, stream);
    if (lrc) return lrc;
    if (a.front_ts) HIP_TRY(h, launch_front_ts(a, stream));
    if (stats) HIP_TRY(h, hipEventRecord(h->ev[1], stream));
    if (a.bin_on) {  // one scatter pass by bin digit, the regular bins sorted and every segment listed in LDS
        HIP_TRY(h, launch_bin_front(a, hist, true, a.csum0 != nullptr, stream));
        if (a.rec == h->d_rec) h->last_sorted = a.rec_sorted;
        if (stats) HIP_TRY(h, hipEventRecord(h->ev[2], stream));
        return SG_OK;
    }
    {
        uint64_t* sorted = nullptr;
        // segment marks: k_seg_mark after the sort, or (SG_SEG_MARK=0) fused into the last scatter pass
        const SegMark mk{a.seg_start, a.seg_end, a.K, a.kshift};
        a.seg_marked = (a.seg_start && a.seg_end && a.long_end && !h->seg_mark_pass) ? 1 : 0;
        HIP_TRY(h, radix_sort_records(a.rec, a.rec_sorted, a.n, a.kshift, hist, &sorted, stream, 64, a.hist0 != nullptr,
                                      a.seg_marked ? &mk : nullptr, a.csum0 != nullptr));
        a.rec_sorted = sorted;
        if (a.rec == h->d_rec) h->last_sorted = sorted;
    }
    if (stats) HIP_TRY(h, hipEventRecord(h->ev[2], stream));
    HIP_TRY(h, launch_seg_flow(a, stream));
    return SG_OK;
}

// Back half on `stream` (after the front half and after the previous batch's back half): the cross-batch time
// check (when the front half skipped it), both walkers (long segments on `aux`), skipped BLOCK counts, the
// handle's last timestamp; the error word lands in the pinned err_dst.
int flow_back(sg_handle* h, const BatchArgs& a, hipStream_t stream, hipStream_t aux, hipEvent_t fork, hipEvent_t join,
              int* err_dst, bool stats) {
    if (!a.check_last) HIP_TRY(h, launch_check_last(a, stream));
    if (h->dbg & 2) {
        HIP_TRY(h, launch_walk_long(a, stream));
        HIP_TRY(h, launch_walk_short(a, stream));
        HIP_TRY(h, launch_walk_tiny(a, stream));
    } else {
        HIP_TRY(h, hipEventRecord(fork, stream));
        HIP_TRY(h, hipStreamWaitEvent(aux, fork, 0));
        HIP_TRY(h, launch_walk_long(a, aux));
        // the length-class-0 walker on a third stream beside the other two (pipelined flow path), else after the
        // short walker
        const bool third = a.tiny && aux == h->s_aux2 && h->s_aux3;
        if (third) {
            HIP_TRY(h, hipStreamWaitEvent(h->s_aux3, fork, 0));
            HIP_TRY(h, launch_walk_tiny(a, h->s_aux3));
            HIP_TRY(h, hipEventRecord(h->tjoin, h->s_aux3));
        }
        HIP_TRY(h, launch_walk_short(a, stream));
        if (!third) HIP_TRY(h, launch_walk_tiny(a, stream));
        HIP_TRY(h, hipEventRecord(join, aux));
        HIP_TRY(h, hipStreamWaitEvent(stream, join, 0));
        if (third) HIP_TRY(h, hipStreamWaitEvent(stream, h->tjoin, 0));
    }
    HIP_TRY(h, launch_skip_apply(a, stream));
    if (stats) HIP_TRY(h, hipEventRecord(h->ev[3], stream));
    HIP_TRY(h, launch_finish(a, stream));
    HIP_TRY(h, hipMemcpyAsync(err_dst, a.err, sizeof(int), hipMemcpyDeviceToHost, stream));
    if (stats) {
        HIP_TRY(h, hipMemcpyAsync(h->h_long, a.long_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipMemcpyAsync(h->h_long + 1, a.skip_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipEventRecord(h->ev[4], stream));
    }
    return SG_OK;
}

int ensure_layout(sg_handle* h) {
    if (h->K == 0 && h->kbits == 0) return layout_records(h);
    return SG_OK;
}

// Enqueue one batch's whole pipeline on `stream` with workspace 0 (req/out device-resident); its error flags
// land in the pinned word err_dst when the stream reaches the end. Stats events only for the synchronous call.
int enqueue_flow(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, hipStream_t stream, int* err_dst,
                 bool stats) {
    int rc = ensure_layout(h);
    if (rc) return rc;
    sg_handle::FlowWs w;
    main_ws(h, w);
    BatchArgs a = flow_args(h, w, req, n, out);
    bin_setup(h, w, a, stream);
    rc = flow_front(h, a, w.hist, stream, stats);
    if (rc) return rc;
    return flow_back(h, a, stream, h->aux, h->fork, h->join, err_dst, stats);
}

// Enqueue one batch on the pipeline: its front half waits for `after` (its input's arrival, may be null) and for
// the walkers of the batch two back (same workspace); its back half follows its front half and the previous
// batch's back half. With namespace limiters the front half also waits for the previous back half (the limiter
// pre-pass must see only accepted batches, so the cross-batch time check stays in k_prep). Returns the event
// that marks the batch's completion through *done (the back half's end, recorded on s_back).
int enqueue_flow_pipelined(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, hipEvent_t after, int* err_dst,
                           hipEvent_t done) {
    int rc = ensure_layout(h);
    if (rc) return rc;
    rc = pipe_setup(h);
    if (rc) return rc;
    const int x = (int)(h->pipe_seq & 1);
    const int xp = x ^ 1;
    const bool first = h->pipe_seq == 0;
    sg_handle::FlowWs w = h->pws;
    if (x == 0) main_ws(h, w);
    // sharded namespace limiter: the armed exchange is copied into workspace x's own buffer now (the caller's
    // buffer is free again when this returns); the batch two back, which read that buffer, has finished its
    // front half by then
    const bool xshard = h->shard_world > 1 && h->n_lim > 0;
    if (xshard) {
        const uint64_t words = (uint64_t)h->shard_world * h->n_lim * h->lim_xn;
        if (words > h->xg_ws_cap) {
            (void)hipDeviceSynchronize();
            dfree(h->d_xg_ws[0]);
            dfree(h->d_xg_ws[1]);
            if (hipMalloc(&h->d_xg_ws[0], 4 * words) != hipSuccess || hipMalloc(&h->d_xg_ws[1], 4 * words) != hipSuccess)
                return fail(h, SG_E_NOMEM, "exchange buffers");
            h->xg_ws_cap = words;
        } else if (h->pipe_seq >= 2) {
            HIP_TRY(h, hipEventSynchronize(h->front_done[x]));
        }
        // complete before returning (the caller may free or refill its buffer then): a device-to-device hipMemcpy
        // may return before the copy has run, and the front half on s_front could read a half-copied exchange
        if (!h->s_xcopy) {
            HIP_TRY(h, hipStreamCreateWithFlags(&h->s_xcopy, hipStreamNonBlocking));
            HIP_TRY(h, hipEventCreateWithFlags(&h->xcopy_done, hipEventDisableTiming));
        }
        HIP_TRY(h, hipMemcpyAsync(h->d_xg_ws[x], h->lim_xg, 4 * words, hipMemcpyDeviceToDevice, h->s_xcopy));
        HIP_TRY(h, hipEventRecord(h->xcopy_done, h->s_xcopy));
        HIP_TRY(h, hipEventSynchronize(h->xcopy_done));
    }
    BatchArgs a = flow_args(h, w, req, n, out);
    bin_setup(h, w, a, h->s_front);
    if (after) HIP_TRY(h, hipStreamWaitEvent(h->s_front, after, 0));
    if (h->pipe_seq >= 2) HIP_TRY(h, hipStreamWaitEvent(h->s_front, h->back_done[x], 0));
    if (h->n_lim > 0) {
        // the limiter pre-pass must see only accepted batches: k_prep checks the time order against the previous
        // front half's last timestamp (front_ts, advanced once a batch passed validation) as well as last_ts, so
        // this front half need not wait for the previous batch's walkers (env SG_LIM_PIPE=0: it waits, as before).
        // A batch the back half later refuses has still advanced front_ts: the next batch is checked against its
        // timestamps too (a batch must be time-ordered after every batch submitted before it, accepted or not).
        if (!h->lim_pipe) {
            if (!first) HIP_TRY(h, hipStreamWaitEvent(h->s_front, h->back_done[xp], 0));
        } else {
            a.front_ts = h->d_front_ts;
        }
    } else {
        a.check_last = 0;  // checked by the back half, after the previous batch has advanced last_ts
    }
    if (xshard) {
        h->lim_xg = h->d_xg_ws[x];
        h->lim_x_armed = true;  // read by flow_front
    }
    rc = flow_front(h, a, w.hist, h->s_front, false);
    h->lim_x_armed = false;
    if (rc) return rc;
    HIP_TRY(h, hipEventRecord(h->front_done[x], h->s_front));
    HIP_TRY(h, hipStreamWaitEvent(h->s_back, h->front_done[x], 0));
    a.walk_cus = h->walk_cus;
    rc = flow_back(h, a, h->s_back, h->s_aux2, h->pfork, h->pjoin, err_dst, false);
    if (rc) return rc;
    HIP_TRY(h, hipEventRecord(h->back_done[x], h->s_back));
    if (done) HIP_TRY(h, hipEventRecord(done, h->s_back));
    h->pipe_seq++;
    return SG_OK;
}

// Completes every batch of the host pipeline (their statuses are kept for sg_flow_poll / sg_flow_wait): the
// synchronous entry points and every state-changing call start from a drained handle.
int drain_async(sg_handle* h) {
    for (auto& sl : h->slots) {
        if (!sl.ticket) continue;
        hipError_t e = hipEventSynchronize(sl.d2h);
        h->finished[sl.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : flow_status(h, *sl.h_err);
        sl.ticket = 0;
    }
    for (auto& d : h->dev) {
        if (!d.ticket) continue;
        hipError_t e = hipEventSynchronize(d.done);
        h->finished[d.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : ticket_status(h, d);
        d.ticket = 0;
    }
    if (h->s_back) (void)hipStreamSynchronize(h->s_back);  // workspace 0 is the synchronous path's too
    return SG_OK;
}

// The sharded limiter's plan over the armed exchange alone (no local batch): every shard's replica of the namespace
// windows walks the same node arrivals.
int lim_plan_only(sg_handle* h, hipStream_t stream) {
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int rc = ensure_layout(h);
    if (rc) return rc;
    BatchArgs a{};
    a.err = h->d_err;
    LimArgs L{};
    L.n_lim = h->n_lim;
    std::memcpy(L.qps, h->lim_qps, sizeof(L.qps));
    L.arrivals = h->d_lim_period;
    L.prefix = h->d_lim_period + (size_t)kMaxLim * kMaxPeriods;
    L.quota = h->d_lim_period + (size_t)2 * kMaxLim * kMaxPeriods;
    L.ring = h->d_lim_ring;
    L.xg = h->lim_xg;
    L.t_base = h->lim_xt;
    L.n_ms = h->lim_xn;
    L.world = h->shard_world;
    L.rank = h->shard_rank;
    HIP_TRY(h, hipMemsetAsync(a.err, 0, sizeof(int), stream));
    HIP_TRY(h, launch_limiter_plan_only(a, L, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    return SG_OK;
}

}  // namespace

int sg_flow_decide_batch(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, void* stream_) {
    if (!h) return SG_E_INVAL;
    const bool xshard = h->shard_world > 1 && h->n_lim > 0;
    if (xshard && !h->lim_x_armed)
        return fail(h, SG_E_UNSUPPORTED, "sharded namespace limiter: sg_lim_exchange must precede every flow batch");
    const bool armed = h->lim_x_armed;
    h->lim_x_armed = false;  // the exchange is consumed by this call, whatever its outcome
    if (n == 0 && !armed) return SG_OK;
    hipStream_t stream = (hipStream_t)stream_;
    // no requests on this shard, or a batch rejected before the device sees it: the shard's replica of the
    // namespace windows still walks the node's gathered arrivals (the other shards charge them too)
    const char* early = n == 0 ? "" : (!req || !out) ? "null buffer" : n > h->cfg.max_batch ? "batch larger than max_batch" : nullptr;
    if (early) {
        if (armed) {
            int rc = lim_plan_only(h, stream);
            if (rc) return rc;
        }
        if (n == 0) return SG_OK;
        return fail(h, (!req || !out) ? SG_E_INVAL : SG_E_CAPACITY, early);
    }
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    h->lim_x_armed = armed;  // read by flow_front
    int rc = enqueue_flow(h, req, n, out, stream, h->h_err, h->stats_on);
    h->lim_x_armed = false;
    if (rc) return rc;
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (h->stats_on) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[4]);
        h->stats.total_ms = ms;
        (void)hipEventElapsedTime(&ms, h->ev[1], h->ev[2]);
        h->stats.sort_ms = ms;
        (void)hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
        h->stats.walk_ms = ms;
        h->stats.long_segments = h->h_long[0];
        h->stats.skipped_ranges = h->h_long[1];
    }
    return flow_status(h, *h->h_err);
}

void* sg_host_alloc(sg_handle* h, uint64_t bytes) {
    if (!h || bytes == 0) return nullptr;
    if (hipSetDevice(h->device) != hipSuccess) return nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        fail(h, SG_E_NOMEM, "pinned host allocation");
        return nullptr;
    }
    return p;
}

void sg_host_free(sg_handle* h, void* p) {
    if (!h || !p) return;
    (void)hipSetDevice(h->device);
    (void)hipHostFree(p);
}

// A pipelined batch of a shard with a namespace limiter consumes the armed exchange (sg_lim_exchange before every
// batch, as for sg_flow_decide_batch); an empty or refused batch walks it at once (the replica advances).
static int xshard_gate(sg_handle* h, uint64_t n, const char* early) {
    if (!(h->shard_world > 1 && h->n_lim > 0)) return early ? (n == 0 ? 1 : fail(h, SG_E_INVAL, early)) : SG_OK;
    if (!h->lim_x_armed)
        return fail(h, SG_E_UNSUPPORTED, "sharded namespace limiter: sg_lim_exchange must precede every flow batch");
    if (!early) return SG_OK;
    h->lim_x_armed = false;
    int rc = lim_plan_only(h, nullptr);
    if (rc) return rc;
    return n == 0 ? 1 : fail(h, n > h->cfg.max_batch ? SG_E_CAPACITY : SG_E_INVAL, early);
}

int sg_flow_submit(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket) {
    if (!h || !ticket) return SG_E_INVAL;
    *ticket = 0;
    {
        const char* early = n == 0 ? "" : (!req || !out) ? "null buffer"
                            : n > h->cfg.max_batch ? "batch larger than max_batch" : nullptr;
        const int g = xshard_gate(h, n, early);
        if (g) return g == 1 ? SG_OK : g;
    }
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->s_comp) {  // first use: streams, per-slot device buffers, events, pinned error words
        HIP_TRY(h, hipStreamCreateWithFlags(&h->s_in, hipStreamNonBlocking));
        HIP_TRY(h, hipStreamCreateWithFlags(&h->s_comp, hipStreamNonBlocking));
        HIP_TRY(h, hipStreamCreateWithFlags(&h->s_out, hipStreamNonBlocking));
        for (auto& sl : h->slots) {
            if (hipMalloc(&sl.d_req, sizeof(sg_req) * h->cfg.max_batch) != hipSuccess ||
                hipMalloc(&sl.d_out, sizeof(sg_result) * h->cfg.max_batch) != hipSuccess ||
                hipHostMalloc(&sl.h_err, sizeof(int)) != hipSuccess)
                return fail(h, SG_E_NOMEM, "host pipeline buffers");
            HIP_TRY(h, hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming));
            HIP_TRY(h, hipEventCreateWithFlags(&sl.comp, hipEventDisableTiming));
            HIP_TRY(h, hipEventCreateWithFlags(&sl.d2h, hipEventDisableTiming));
        }
    }
    sg_handle::Slot& sl = h->slots[h->next_ticket % kAsyncSlots];
    if (sl.ticket) {  // all slots in flight: complete the oldest (its status waits in `finished`)
        hipError_t e = hipEventSynchronize(sl.d2h);
        h->finished[sl.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : flow_status(h, *sl.h_err);
        sl.ticket = 0;
    }
    // H2D of this batch overlaps the previous batches' compute; the batch's front half (sort) overlaps the
    // previous batch's walkers, the walkers stay in submission order (the batches are time-ordered and share the
    // window state); D2H overlaps the next batch's compute
    HIP_TRY(h, hipMemcpyAsync(sl.d_req, req, sizeof(sg_req) * n, hipMemcpyHostToDevice, h->s_in));
    HIP_TRY(h, hipEventRecord(sl.h2d, h->s_in));
    int rc = enqueue_flow_pipelined(h, sl.d_req, n, sl.d_out, sl.h2d, sl.h_err, sl.comp);
    if (rc) return rc;
    HIP_TRY(h, hipStreamWaitEvent(h->s_out, sl.comp, 0));
    // results back on the copy engine (both directions of the link overlap: H2D of the next batch on s_in), or with
    // SG_D2H=1 by a copy kernel when `out` is pinned host memory the device can address
    void* out_dev = nullptr;
    if (h->d2h_kernel) {
        hipPointerAttribute_t pa{};
        if (hipPointerGetAttributes(&pa, out) == hipSuccess && pa.type == hipMemoryTypeHost && pa.devicePointer &&
            ((uintptr_t)pa.devicePointer & 15) == 0)
            out_dev = pa.devicePointer;
        else
            (void)hipGetLastError();  // pageable memory: not an error, the copy engine takes it
    }
    if (out_dev) HIP_TRY(h, launch_copy_out(sl.d_out, out_dev, sizeof(sg_result) * n, h->d2h_blocks, h->s_out));
    else HIP_TRY(h, hipMemcpyAsync(out, sl.d_out, sizeof(sg_result) * n, hipMemcpyDeviceToHost, h->s_out));
    HIP_TRY(h, hipEventRecord(sl.d2h, h->s_out));
    // (a slot is reused only after its batch completed: above, or when its ticket was collected)
    sl.ticket = h->next_ticket++;
    *ticket = sl.ticket;
    return SG_OK;
}

int sg_flow_enqueue(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket) {
    if (!h || !ticket) return SG_E_INVAL;
    *ticket = 0;
    {
        const char* early = n == 0 ? "" : (!req || !out) ? "null buffer"
                            : n > h->cfg.max_batch ? "batch larger than max_batch" : nullptr;
        const int g = xshard_gate(h, n, early);
        if (g) return g == 1 ? SG_OK : g;
    }
    HIP_TRY(h, hipSetDevice(h->device));
    sg_handle::DevTicket& d = h->dev[h->next_ticket % kDevSlots];
    if (!d.done) {
        if (hipHostMalloc(&d.h_err, sizeof(int)) != hipSuccess) return fail(h, SG_E_NOMEM, "pinned error word");
        HIP_TRY(h, hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    }
    if (d.ticket) {  // every slot in flight: complete the oldest (its status waits in `finished`)
        hipError_t e = hipEventSynchronize(d.done);
        h->finished[d.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : ticket_status(h, d);
        d.ticket = 0;
    }
    int rc = enqueue_flow_pipelined(h, req, n, out, nullptr, d.h_err, d.done);
    if (rc) return rc;
    d.local = false;
    d.ticket = h->next_ticket++;
    *ticket = d.ticket;
    return SG_OK;
}

static int collect(sg_handle* h, uint64_t ticket, bool block) {
    if (!h) return SG_E_INVAL;
    if (ticket == 0) return 1;
    auto it = h->finished.find(ticket);
    if (it != h->finished.end()) {
        const int st = it->second;
        h->finished.erase(it);
        return st == SG_OK ? 1 : st;
    }
    for (auto& sl : h->slots) {
        if (sl.ticket != ticket) continue;
        hipError_t e = block ? hipEventSynchronize(sl.d2h) : hipEventQuery(sl.d2h);
        if (e == hipErrorNotReady) return 0;
        sl.ticket = 0;
        if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
        const int st = flow_status(h, *sl.h_err);
        return st == SG_OK ? 1 : st;
    }
    for (auto& d : h->dev) {
        if (d.ticket != ticket) continue;
        hipError_t e = block ? hipEventSynchronize(d.done) : hipEventQuery(d.done);
        if (e == hipErrorNotReady) return 0;
        d.ticket = 0;
        if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
        const int st = ticket_status(h, d);
        return st == SG_OK ? 1 : st;
    }
    return fail(h, SG_E_INVAL, "unknown or already collected ticket");
}

int sg_flow_poll(sg_handle* h, uint64_t ticket) { return collect(h, ticket, false); }

int sg_flow_wait(sg_handle* h, uint64_t ticket) {
    const int r = collect(h, ticket, true);
    return r == 1 ? SG_OK : r;
}

int sg_flow_decide_batch_host(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out) {
    if (!h) return SG_E_INVAL;
    // empty or refused before the device: the device entry point answers (and walks an armed exchange)
    if (n == 0 || n > h->cfg.max_batch || !req || !out) return sg_flow_decide_batch(h, n ? req : nullptr, n, out, nullptr);
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_req_h) {
        if (hipMalloc(&h->d_req_h, sizeof(sg_req) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_out_h, sizeof(sg_result) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    HIP_TRY(h, hipMemcpy(h->d_req_h, req, sizeof(sg_req) * n, hipMemcpyHostToDevice));
    int rc = sg_flow_decide_batch(h, h->d_req_h, n, h->d_out_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(out, h->d_out_h, sizeof(sg_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

// Envoy RLS (SentinelEnvoyRlsServiceImpl.shouldRateLimit, service/v3/SentinelEnvoyRlsServiceImpl.java:34-85): every
// descriptor of the batch one token request of one device batch (at most max_batch of them), then the per-request codes.
int sg_rls_should_rate_limit(sg_handle* h, const sg_rls_request* req, uint32_t n, const int32_t* desc_rule,
                             uint64_t n_desc, int32_t* overall, sg_rls_status* status) {
    if (!h) return SG_E_INVAL;
    if (n && (!req || !overall)) return fail(h, SG_E_INVAL, "null buffer");
    if (n_desc && (!desc_rule || !status)) return fail(h, SG_E_INVAL, "null buffer");
    for (uint32_t j = 0; j < n; ++j)
        if ((uint64_t)req[j].desc_begin + req[j].desc_count > n_desc)
            return fail(h, SG_E_INVAL, "a request's descriptors lie outside desc_rule");
    // SimpleClusterFlowChecker (flow/SimpleClusterFlowChecker.java:33-65) reads count * exceedCount and has neither a
    // namespace limiter nor AVG_LOCAL thresholds: refuse rules the cluster path would treat differently, and a batch
    // that would need several device batches (no partial commit), before any state changes
    uint64_t n_tok = 0;
    for (uint32_t j = 0; j < n; ++j) {
        if (req[j].hits_addend < 0) continue;
        n_tok += req[j].desc_count;
        for (uint32_t x = 0; x < req[j].desc_count; ++x) {
            const int32_t r = desc_rule[(uint64_t)req[j].desc_begin + x];
            if (r < 0 || (uint32_t)r >= h->K) continue;
            const sg_flow_rule& fr = h->rules[r];
            const int ns = fr.namespace_id;
            if (fr.threshold_type != SG_THRESHOLD_GLOBAL ||
                (ns >= 0 && (size_t)ns < h->ns_slot.size() && h->ns_slot[ns] >= 0))
                return fail(h, SG_E_UNSUPPORTED, "RLS rules are loaded GLOBAL in namespaces without a limiter "
                                                 "(SimpleClusterFlowChecker reads count * exceedCount only)");
        }
    }
    if (n_tok > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "more descriptors than max_batch");
    std::vector<sg_req> batch;
    std::vector<uint64_t> owner;  // descriptor of each token request
    batch.reserve(n_desc);
    owner.reserve(n_desc);
    for (uint64_t d = 0; d < n_desc; ++d) status[d] = sg_rls_status{0, 0, 0, 0};
    for (uint32_t j = 0; j < n; ++j) {
        const sg_rls_request& q = req[j];
        if (q.hits_addend < 0) {  // "acquireCount should be positive": onError, no token requests (:36-40)
            overall[j] = SG_RLS_ERROR;
            continue;
        }
        overall[j] = SG_RLS_OK;
        const int32_t acquire = q.hits_addend == 0 ? 1 : q.hits_addend;  // :41-44
        for (uint32_t x = 0; x < q.desc_count; ++x) {
            const uint64_t d = (uint64_t)q.desc_begin + x;
            const int32_t r = desc_rule[d];
            sg_req t{};
            t.ts_ms = q.ts_ms;
            t.key = (r < 0 || (uint32_t)r >= h->K) ? SG_KEY_NO_RULE : (uint32_t)r;  // checkToken: no rule
            t.acquire = acquire;
            batch.push_back(t);
            owner.push_back(d);
        }
    }
    std::vector<sg_result> res(batch.size());
    if (!batch.empty()) {
        const int rc = sg_flow_decide_batch_host(h, batch.data(), batch.size(), res.data());
        if (rc) return rc;
    }
    for (uint64_t x = 0; x < batch.size(); ++x) {
        const uint64_t d = owner[x];
        int32_t st = res[x].status;
        if (st == SG_STATUS_NO_RULE_EXISTS) st = SG_STATUS_OK;  // a descriptor without a rule passes (:55-58)
        sg_rls_status& o = status[d];
        o.code = st == SG_STATUS_OK ? SG_RLS_OK : SG_RLS_OVER_LIMIT;
        if (batch[x].key != SG_KEY_NO_RULE) {
            const double c = h->rules[batch[x].key].count;  // (int) rule.getCount(), JLS narrowing
            o.requests_per_unit = c >= 2147483647.0 ? INT32_MAX : (int32_t)c;
            o.limit_remaining = res[x].remaining;
            o.has_rule = 1;
        }
    }
    for (uint32_t j = 0; j < n; ++j) {
        if (overall[j] == SG_RLS_ERROR) continue;
        for (uint32_t x = 0; x < req[j].desc_count; ++x)
            if (status[(uint64_t)req[j].desc_begin + x].code != SG_RLS_OK) overall[j] = SG_RLS_OVER_LIMIT;
    }
    return SG_OK;
}

int sg_flow_read_state(sg_handle* h, uint32_t key, int64_t* starts, int64_t* counters, int64_t* occupy) {
    if (!h || key >= h->K || !starts || !counters || !occupy) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    const int S = h->rule_tab[key].S;
    std::vector<Bucket> b(S);
    HIP_TRY(h, hipMemcpy(b.data(), h->d_ring + (size_t)key * h->stride, sizeof(Bucket) * S, hipMemcpyDeviceToHost));
    Occ o;
    HIP_TRY(h, hipMemcpy(&o, h->d_occ + key, sizeof(Occ), hipMemcpyDeviceToHost));
    for (int j = 0; j < S; ++j) {
        starts[j] = b[j].start;
        for (int e = 0; e < SG_NUM_EVENTS; ++e) counters[j * SG_NUM_EVENTS + e] = b[j].start == INT64_MIN ? 0 : b[j].c[e];
    }
    occupy[0] = o.pass;
    occupy[1] = o.pass_req;
    return SG_OK;
}

int sg_flow_export_state(sg_handle* h, int64_t* ring, uint64_t ring_words, int64_t* occ, uint64_t occ_words,
                         int32_t* stride) {
    if (!h || !stride) return SG_E_INVAL;
    *stride = h->stride;
    if (!ring) return SG_OK;
    const uint64_t rw = (uint64_t)h->K * h->stride * 8, ow = 2ull * h->K;
    if (ring_words < rw || !occ || occ_words < ow) return fail(h, SG_E_INVAL, "export buffers too small");
    if (h->K == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    static_assert(sizeof(Bucket) == 64 && sizeof(Occ) == 16, "export layout");
    HIP_TRY(h, hipMemcpy(ring, h->d_ring, rw * 8, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemcpy(occ, h->d_occ, ow * 8, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_flow_import_state(sg_handle* h, const int64_t* ring, uint64_t ring_words, const int64_t* occ,
                         uint64_t occ_words) {
    if (!h || !ring || !occ) return SG_E_INVAL;
    const uint64_t rw = (uint64_t)h->K * h->stride * 8, ow = 2ull * h->K;
    if (ring_words != rw || occ_words != ow) return fail(h, SG_E_INVAL, "import size does not match the loaded rules");
    if (h->K == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    HIP_TRY(h, hipMemcpy(h->d_ring, ring, rw * 8, hipMemcpyHostToDevice));
    HIP_TRY(h, launch_hot_sync(h->d_ring, h->d_hot, (uint64_t)h->K * h->stride, 0));
    HIP_TRY(h, hipDeviceSynchronize());
    HIP_TRY(h, hipMemcpy(h->d_occ, occ, ow * 8, hipMemcpyHostToDevice));
    return SG_OK;
}

int sg_snapshot_metrics(sg_handle* h, int64_t now_ms, double* out, uint64_t cap) {
    if (!h || !out || cap < 2ull * h->K) return SG_E_INVAL;
    if (h->K == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    double* d_out = nullptr;
    HIP_TRY(h, hipMalloc(&d_out, sizeof(double) * 2 * h->K));
    hipError_t e1 = launch_snapshot(h->d_rules, h->d_ring, h->d_occ, h->K, h->stride, now_ms, d_out, 0);
    hipError_t e2 = e1 == hipSuccess ? hipMemcpy(out, d_out, sizeof(double) * 2 * h->K, hipMemcpyDeviceToHost) : e1;
    (void)hipFree(d_out);
    if (e2 != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e2));
    return SG_OK;
}

int sg_snapshot_metrics_device(sg_handle* h, int64_t now_ms, double* out_dev, uint64_t cap, void* stream) {
    if (!h || !out_dev || cap < 2ull * h->K) return SG_E_INVAL;
    if (h->K == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    HIP_TRY(h, launch_snapshot(h->d_rules, h->d_ring, h->d_occ, h->K, h->stride, now_ms, out_dev, (hipStream_t)stream));
    return SG_OK;
}

// The same snapshot ordered on the pipeline after every batch enqueued so far (sg_flow_enqueue / submit): the
// node-wide rollup of one simulated second can run while the next second's batches are being decided.
int sg_snapshot_metrics_enqueue(sg_handle* h, int64_t now_ms, double* out_dev, uint64_t cap, uint64_t* ticket) {
    if (!h || !out_dev || !ticket || cap < 2ull * h->K) return SG_E_INVAL;
    *ticket = 0;
    if (h->K == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    int rc = pipe_setup(h);
    if (rc) return rc;
    sg_handle::DevTicket& d = h->dev[h->next_ticket % kDevSlots];
    if (!d.done) {
        if (hipHostMalloc(&d.h_err, sizeof(int)) != hipSuccess) return fail(h, SG_E_NOMEM, "pinned error word");
        HIP_TRY(h, hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    }
    if (d.ticket) {
        hipError_t e = hipEventSynchronize(d.done);
        h->finished[d.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : ticket_status(h, d);
        d.ticket = 0;
    }
    *d.h_err = 0;
    HIP_TRY(h, launch_snapshot(h->d_rules, h->d_ring, h->d_occ, h->K, h->stride, now_ms, out_dev, h->s_back));
    HIP_TRY(h, hipEventRecord(d.done, h->s_back));
    d.local = false;
    d.ticket = h->next_ticket++;
    *ticket = d.ticket;
    return SG_OK;
}

// ParamFlowRuleManager.loadRules (…/param/ParamFlowRuleManager.java) → fresh ParameterMetric maps.
int sg_param_load_rules(sg_handle* h, const sg_param_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                        uint32_t n_hot) {
    if (!h || (!rules && n) || (!hot && n_hot)) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<PRule> tab(n);
    std::vector<sg_param_hot_item> hot_sorted(hot, hot + n_hot);
    uint64_t base = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_param_rule& r = rules[i];
        if (!(r.count >= 0) || r.duration_sec <= 0) return fail(h, SG_E_INVAL, "invalid param rule");
        if ((uint64_t)r.hot_begin + r.hot_count > n_hot) return fail(h, SG_E_INVAL, "hot item range out of bounds");
        const int lg = r.capacity_log2 ? r.capacity_log2 : 20;
        if (lg < 1 || lg > 30) return fail(h, SG_E_INVAL, "capacity_log2 must be in [1, 30]");
        PRule& R = tab[i];
        R.token_count = (int64_t)r.count;  // (long) rule.getCount(); count is finite and >= 0 here
        if (r.count >= 9.2e18) R.token_count = INT64_MAX;
        R.duration_sec = r.duration_sec;
        R.burst = r.burst;
        R.behavior = r.behavior;
        R.max_queueing_ms = r.max_queueing_ms;
        R.hot_begin = r.hot_begin;
        R.hot_count = r.hot_count;
        R.table_base = base;
        R.table_mask = (1ull << lg) - 1;
        base += (1ull << lg) + 1;  // + the side slot for the value ~0
        std::sort(hot_sorted.begin() + r.hot_begin, hot_sorted.begin() + r.hot_begin + r.hot_count,
                  [](const sg_param_hot_item& x, const sg_param_hot_item& y) { return x.value < y.value; });
    }
    if (base >= (1ull << 32)) return fail(h, SG_E_UNSUPPORTED, "param tables larger than 2^32 slots");
    dfree(h->d_prules);
    dfree(h->d_phot);
    dfree(h->d_ptable);
    h->ptotal = 0;
    if (n) {
        if (hipMalloc(&h->d_prules, sizeof(PRule) * n) != hipSuccess ||
            hipMalloc(&h->d_ptable, sizeof(PSlot) * base) != hipSuccess)
            return fail(h, SG_E_NOMEM, "param table allocation");
        if (n_hot && hipMalloc(&h->d_phot, sizeof(sg_param_hot_item) * n_hot) != hipSuccess)
            return fail(h, SG_E_NOMEM, "param hot items");
        HIP_TRY(h, hipMemcpy(h->d_prules, tab.data(), sizeof(PRule) * n, hipMemcpyHostToDevice));
        if (n_hot)
            HIP_TRY(h, hipMemcpy(h->d_phot, hot_sorted.data(), sizeof(sg_param_hot_item) * n_hot, hipMemcpyHostToDevice));
        HIP_TRY(h, launch_param_clear(h->d_ptable, base, 0));
        HIP_TRY(h, hipDeviceSynchronize());
    }
    h->prules.assign(rules, rules + n);
    h->ptab = tab;
    h->ptotal = base;
    return SG_OK;
}

int sg_param_decide_batch(sg_handle* h, const sg_param_req* req, uint64_t n, int32_t* pass, void* stream_) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !pass) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);  // the main workspace's segment lists may belong to an enqueued flow batch
    PArgs p{};
    p.req = req;
    p.out = pass;
    p.n = n;
    p.rec = h->d_rec;
    p.rec_sorted = h->d_rec_sorted;
    p.ibits = bits_for(h->cfg.max_batch > 1 ? h->cfg.max_batch - 1 : 1);
    p.imask = (1ull << p.ibits) - 1;
    p.rules = h->d_prules;
    p.n_rules = (uint32_t)h->ptab.size();
    p.hot = h->d_phot;
    p.table = h->d_ptable;
    p.total_slots = h->ptotal;
    p.err = h->d_err;
    p.last_ts = h->d_plast_ts;
    p.long_list = h->d_long_list;
    p.long_count = h->d_long_count;
    uint32_t psplit = 64u;  // lane / wave walker split of the hot-parameter walkers (SG_PARAM_SHORT_MAX: tuning; r04: 64 < 32 by 2%)
    if (const char* e = std::getenv("SG_PARAM_SHORT_MAX")) psplit = (uint32_t)std::strtoul(e, nullptr, 10);
    p.short_max = (h->cfg.flags & SG_FLAG_WAVE_ONLY) ? 0u : (h->cfg.flags & SG_FLAG_SERIAL_ONLY) ? 0xFFFFFFFFu : psplit;
    const int gbits = bits_for(h->ptotal + 1);
    p.gshift = p.ibits + 8;  // {slot | acquire code : 8 | request index}
    if (p.gshift + gbits > 64) return fail(h, SG_E_UNSUPPORTED, "param tables x max_batch too large for 64-bit records");
    if (!h->d_p_msb && (hipMalloc(&h->d_p_msb, sizeof(uint32_t) * kMaxPeriods) != hipSuccess ||
                        hipMalloc(&h->d_p_mt, 2 * sizeof(int64_t)) != hipSuccess))  // {t0, {np, zero word}}
        return fail(h, SG_E_NOMEM, "param millisecond table");
    p.msb = h->d_p_msb;
    p.mt0 = h->d_p_mt;
    p.mnp = reinterpret_cast<uint32_t*>(h->d_p_mt + 1);
    if (!h->d_p_mbk && hipMalloc(&h->d_p_mbk, sizeof(uint16_t) * kPcBuckets) != hipSuccess)
        return fail(h, SG_E_NOMEM, "param millisecond buckets");
    p.mbk = h->d_p_mbk;
    p.bshift = 0;
    while ((((uint64_t)n - 1) >> p.bshift) >= kPcBuckets) ++p.bshift;
    BatchArgs sg{};  // k_seg's lists in the main workspace; its error word: a zero word (the param flags are no errors)
    sg.err = reinterpret_cast<int*>(h->d_p_mt) + 3;
    sg.short_list = h->d_short_list;
    sg.short_count = h->d_long_count + 1;
    for (int c = 0; c < kClasses; ++c) sg.class_off[c] = h->class_off[c];
    HIP_TRY(h, hipMemsetAsync(h->d_err, 0, sizeof(int), stream));
    HIP_TRY(h, hipMemsetAsync(h->d_long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream));
    HIP_TRY(h, hipMemsetAsync(sg.err, 0, sizeof(int), stream));
    uint64_t* sorted = nullptr;
    HIP_TRY(h, launch_param_batch(p, sg, h->d_rec, h->d_rec_sorted, h->d_hist, p.gshift, p.gshift + gbits, &sorted, stream,
                                  h->aux, h->fork, h->join));
    h->last_sorted = sorted;
    HIP_TRY(h, hipMemcpyAsync(h->h_err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    const int err = *h->h_err & ~kErrNonPositive;
    if (err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (err & kErrTableFull) return fail(h, SG_E_CAPACITY, "a param rule's value table is full");
    return SG_OK;
}

int sg_param_decide_batch_host(sg_handle* h, const sg_param_req* req, uint64_t n, int32_t* pass) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_preq_h) {
        if (hipMalloc(&h->d_preq_h, sizeof(sg_param_req) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_pout_h, sizeof(int32_t) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    HIP_TRY(h, hipMemcpy(h->d_preq_h, req, sizeof(sg_param_req) * n, hipMemcpyHostToDevice));
    int rc = sg_param_decide_batch(h, h->d_preq_h, n, h->d_pout_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(pass, h->d_pout_h, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_param_read_state(sg_handle* h, uint32_t rule, uint64_t value, int64_t* last_time, int64_t* tokens) {
    if (!h || rule >= h->ptab.size() || !last_time || !tokens) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    const PRule& R = h->ptab[rule];
    PSlot found{};
    bool hit = false;
    if (value == ~0ull) {  // the side slot
        HIP_TRY(h, hipMemcpy(&found, h->d_ptable + R.table_base + R.table_mask + 1, sizeof(PSlot), hipMemcpyDeviceToHost));
        hit = true;
    } else {
        // the probe sequence of param.hip's param_slot, read in chunks of 64 slots
        uint64_t x = value + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        x ^= x >> 31;
        uint64_t i = x & R.table_mask, seen = 0;
        PSlot chunk[64];
        while (!hit && seen <= R.table_mask) {
            const uint64_t m = std::min<uint64_t>(64, R.table_mask + 1 - i);  // up to the table's end
            HIP_TRY(h, hipMemcpy(chunk, h->d_ptable + R.table_base + i, sizeof(PSlot) * m, hipMemcpyDeviceToHost));
            bool empty = false;
            for (uint64_t j = 0; j < m && !hit && !empty; ++j) {
                if (chunk[j].value == value) {
                    found = chunk[j];
                    hit = true;
                } else if (chunk[j].value == ~0ull) {
                    empty = true;
                }
            }
            if (empty) break;
            seen += m;
            i = (i + m) & R.table_mask;
        }
    }
    if (!hit || !found.flags) return 0;
    *last_time = found.time;
    *tokens = found.tokens;
    return (int)found.flags;
}

// --------------------------------------------------------------------- pace controller
// FlowRuleUtil.generateRater (core/.../flow/FlowRuleUtil.java:132-145) builds one RateLimiterController per
// CONTROL_BEHAVIOR_RATE_LIMITER rule; a rebuild starts every latestPassedTime at -1
// (RateLimiterController.java:33). FlowRuleUtil.isValidRule (:167-175) requires count >= 0.
int sg_pace_load_rules(sg_handle* h, const sg_pace_rule* rules, uint32_t n) {
    if (!h || (!rules && n)) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<PaceRule> tab(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!(rules[i].count >= 0)) return fail(h, SG_E_INVAL, "invalid pace rule: count must be >= 0");
        tab[i].count = rules[i].count;
        tab[i].max_queueing_ms = rules[i].max_queueing_ms;
        tab[i].pad = 0;
    }
    dfree(h->d_pace_rules);
    dfree(h->d_pace_latest);
    h->pace_tab.clear();
    if (!h->d_pace_last_ts) {
        const int64_t neg = INT64_MIN;
        if (hipMalloc(&h->d_pace_last_ts, sizeof(int64_t)) != hipSuccess) return fail(h, SG_E_NOMEM, "pace state");
        HIP_TRY(h, hipMemcpy(h->d_pace_last_ts, &neg, sizeof(neg), hipMemcpyHostToDevice));
    }
    if (n) {
        if (hipMalloc(&h->d_pace_rules, sizeof(PaceRule) * n) != hipSuccess ||
            hipMalloc(&h->d_pace_latest, sizeof(int64_t) * n) != hipSuccess)
            return fail(h, SG_E_NOMEM, "pace rule allocation");
        std::vector<int64_t> init(n, -1);
        HIP_TRY(h, hipMemcpy(h->d_pace_rules, tab.data(), sizeof(PaceRule) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_pace_latest, init.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
    }
    h->pace_tab = tab;
    return SG_OK;
}

int sg_pace_decide_batch(sg_handle* h, const sg_pace_req* req, uint64_t n, int32_t* wait, void* stream_) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !wait) return fail(h, SG_E_INVAL, "null buffer");
    if (!h->d_pace_last_ts) return fail(h, SG_E_INVAL, "sg_pace_load_rules first");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(h, hipSetDevice(h->device));
    PaceArgs p{};
    p.req = req;
    p.out = wait;
    p.n = n;
    p.rec = h->d_rec;
    p.rec_sorted = h->d_rec_sorted;
    p.ibits = bits_for(h->cfg.max_batch > 1 ? h->cfg.max_batch - 1 : 1);
    p.imask = (1ull << p.ibits) - 1;
    p.rules = h->d_pace_rules;
    p.n_rules = (uint32_t)h->pace_tab.size();
    p.latest = h->d_pace_latest;
    p.err = h->d_err;
    p.last_ts = h->d_pace_last_ts;
    p.long_list = h->d_long_list;
    p.long_count = h->d_long_count;
    p.short_list = h->d_short_list;
    uint32_t psplit = 128u;  // lane / wave walker split of the pace walkers (SG_PACE_SHORT_MAX: tuning; 1M rules,
                             // 16M canPass: 32 → 1.31, 64 → 1.24, 96..256 → 1.21-1.22, 512 → 1.34 ms/step)
    if (const char* e = std::getenv("SG_PACE_SHORT_MAX")) psplit = (uint32_t)std::strtoul(e, nullptr, 10);
    p.short_max = (h->cfg.flags & SG_FLAG_WAVE_ONLY) ? 0u : (h->cfg.flags & SG_FLAG_SERIAL_ONLY) ? 0xFFFFFFFFu : psplit;
    const int gbits = bits_for((uint64_t)p.n_rules + 1);
    p.gshift = p.ibits + 8;  // {rule | acquire code : 8 | request index}
    if (p.gshift + gbits > 64) return fail(h, SG_E_UNSUPPORTED, "pace rules x max_batch too large for 64-bit records");
    // the millisecond table (shared with the hot-parameter path: both are synchronous calls of this handle)
    if (!h->d_p_msb && (hipMalloc(&h->d_p_msb, sizeof(uint32_t) * kMaxPeriods) != hipSuccess ||
                        hipMalloc(&h->d_p_mt, 2 * sizeof(int64_t)) != hipSuccess))
        return fail(h, SG_E_NOMEM, "pace millisecond table");
    p.msb = h->d_p_msb;
    p.mt0 = h->d_p_mt;
    p.mnp = reinterpret_cast<uint32_t*>(h->d_p_mt + 1);
    if (!h->d_p_mbk && hipMalloc(&h->d_p_mbk, sizeof(uint16_t) * kPcBuckets) != hipSuccess)
        return fail(h, SG_E_NOMEM, "pace millisecond buckets");
    p.mbk = h->d_p_mbk;
    p.bshift = 0;
    while ((((uint64_t)n - 1) >> p.bshift) >= kPcBuckets) ++p.bshift;
    HIP_TRY(h, hipMemsetAsync(h->d_err, 0, sizeof(int), stream));
    for (int c = 0; c < kClasses; ++c) p.class_off[c] = h->class_off[c];
    HIP_TRY(h, hipMemsetAsync(h->d_long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream));
    uint64_t* sorted = nullptr;
    HIP_TRY(h, launch_pace_batch(p, h->d_rec, h->d_rec_sorted, h->d_hist, p.gshift, p.gshift + gbits, &sorted, stream,
                                 h->aux, h->fork, h->join));
    h->last_sorted = sorted;
    HIP_TRY(h, hipMemcpyAsync(h->h_err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (*h->h_err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    return SG_OK;
}

int sg_pace_decide_batch_host(sg_handle* h, const sg_pace_req* req, uint64_t n, int32_t* wait) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !wait) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_pace_req_h) {
        if (hipMalloc(&h->d_pace_req_h, sizeof(sg_pace_req) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_pace_out_h, sizeof(int32_t) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    HIP_TRY(h, hipMemcpy(h->d_pace_req_h, req, sizeof(sg_pace_req) * n, hipMemcpyHostToDevice));
    int rc = sg_pace_decide_batch(h, h->d_pace_req_h, n, h->d_pace_out_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(wait, h->d_pace_out_h, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_pace_read_state(sg_handle* h, uint32_t rule, int64_t* latest_passed_time) {
    if (!h || rule >= h->pace_tab.size() || !latest_passed_time) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipMemcpy(latest_passed_time, h->d_pace_latest + rule, sizeof(int64_t), hipMemcpyDeviceToHost));
    return SG_OK;
}

// --------------------------------------------------------------------- cluster hot-parameter tokens

// ClusterParamFlowRuleManager.loadRules → applyClusterParamRules (…/ClusterParamFlowRuleManager.java:337-360):
// a flowId that survives keeps its metric (and its window shape), the others start empty.
int sg_cparam_load_rules(sg_handle* h, const sg_cparam_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                         uint32_t n_hot, int32_t capacity_log2) {
    if (!h || (!rules && n) || (!hot && n_hot)) return SG_E_INVAL;
    if (n >= SG_KEY_BAD) return fail(h, SG_E_INVAL, "too many rules");
    const int lg = capacity_log2 ? capacity_log2 : 16;
    if (lg < 1 || lg > 28) return fail(h, SG_E_INVAL, "capacity_log2 must be in [1, 28]");
    HIP_TRY(h, hipSetDevice(h->device));
    std::unordered_map<int64_t, uint32_t> seen, old_index;
    for (uint32_t k = 0; k < h->cprules.size(); ++k) old_index.emplace(h->cprules[k].flow_id, k);
    std::vector<CPRule> tab(n);
    std::vector<int32_t> wls;  // distinct window lengths (the batch's period tables)
    std::vector<sg_param_hot_item> hs(hot, hot + n_hot);
    int stride = 1;
    uint64_t base = 0;
    const uint64_t per = (1ull << lg) + 1;  // + the side slot
    for (uint32_t i = 0; i < n; ++i) {
        const sg_cparam_rule& r = rules[i];
        if (r.flow_id <= 0 || !(r.count >= 0)) return fail(h, SG_E_INVAL, "invalid param rule");
        if (r.sample_count <= 0 || r.window_interval_ms <= 0 || r.window_interval_ms % r.sample_count != 0)
            return fail(h, SG_E_INVAL, "invalid window config");
        if (r.namespace_id < 0 || (size_t)r.namespace_id >= h->ns.size()) return fail(h, SG_E_INVAL, "unknown namespace");
        if ((uint64_t)r.hot_begin + r.hot_count > n_hot) return fail(h, SG_E_INVAL, "hot item range out of bounds");
        if (!seen.emplace(r.flow_id, i).second) return fail(h, SG_E_INVAL, "duplicate flowId");
        int S = r.sample_count, interval = r.window_interval_ms;
        auto it = old_index.find(r.flow_id);
        if (it != old_index.end()) {  // the existing metric keeps its window shape
            S = h->cptab[it->second].S;
            interval = h->cptab[it->second].S * h->cptab[it->second].wl;
        }
        if (S > SG_MAX_SAMPLE_COUNT) return fail(h, SG_E_UNSUPPORTED, "sampleCount > 64");
        CPRule& R = tab[i];
        R.count = r.count;
        R.isec = interval / 1000.0;
        R.S = S;
        R.wl = interval / S;
        R.global = r.threshold_type == SG_THRESHOLD_GLOBAL;
        R.connected = h->ns[r.namespace_id].connected_count;
        R.hot_begin = r.hot_begin;
        R.hot_count = r.hot_count;
        R.table_base = base;
        R.table_mask = (1ull << lg) - 1;
        {
            auto wit = std::find(wls.begin(), wls.end(), R.wl);
            if (wit == wls.end()) {
                if ((int)wls.size() == kMaxWl) return fail(h, SG_E_UNSUPPORTED, "more than 8 distinct param window lengths");
                wls.push_back(R.wl);
                wit = wls.end() - 1;
            }
            R.wl_idx = (int32_t)(wit - wls.begin());
            R.pad = 0;
        }
        base += per;
        stride = std::max(stride, S);
        std::sort(hs.begin() + r.hot_begin, hs.begin() + r.hot_begin + r.hot_count,
                  [](const sg_param_hot_item& x, const sg_param_hot_item& y) { return x.value < y.value; });
    }
    if (base >= (1ull << 32)) return fail(h, SG_E_UNSUPPORTED, "param tables larger than 2^32 slots");
    CPRule* d_rules = nullptr;
    sg_param_hot_item* d_hot = nullptr;
    uint64_t* d_keys = nullptr;
    CPBucket* d_ring = nullptr;
    if (n) {
        if (hipMalloc(&d_rules, sizeof(CPRule) * n) != hipSuccess || hipMalloc(&d_keys, 8 * base) != hipSuccess ||
            hipMalloc(&d_ring, sizeof(CPBucket) * base * stride) != hipSuccess ||
            (n_hot && hipMalloc(&d_hot, sizeof(sg_param_hot_item) * n_hot) != hipSuccess)) {
            dfree(d_rules);
            dfree(d_keys);
            dfree(d_ring);
            dfree(d_hot);
            return fail(h, SG_E_NOMEM, "param table allocation");
        }
        HIP_TRY(h, hipMemcpy(d_rules, tab.data(), sizeof(CPRule) * n, hipMemcpyHostToDevice));
        if (n_hot) HIP_TRY(h, hipMemcpy(d_hot, hs.data(), sizeof(sg_param_hot_item) * n_hot, hipMemcpyHostToDevice));
        HIP_TRY(h, launch_cp_clear(d_keys, d_ring, base, stride, 0));
        for (uint32_t i = 0; i < n; ++i) {  // surviving flowIds: move their sub-tables
            auto it = old_index.find(rules[i].flow_id);
            if (it == old_index.end()) continue;
            const CPRule& O = h->cptab[it->second];
            const uint64_t slots = std::min(O.table_mask, tab[i].table_mask) + 2;
            if (O.table_mask != tab[i].table_mask) return fail(h, SG_E_UNSUPPORTED, "capacity change of a live param rule");
            HIP_TRY(h, launch_cp_copy(h->d_cpkeys, h->d_cpring, O.table_base, h->cpstride, d_keys, d_ring, tab[i].table_base,
                                      stride, slots, O.S, 0));
        }
        HIP_TRY(h, hipDeviceSynchronize());
    }
    dfree(h->d_cprules);
    dfree(h->d_cphot);
    dfree(h->d_cpkeys);
    dfree(h->d_cpring);
    h->d_cprules = d_rules;
    h->d_cphot = d_hot;
    h->d_cpkeys = d_keys;
    h->d_cpring = d_ring;
    h->cprules.assign(rules, rules + n);
    h->cptab = tab;
    h->l_groups_stale = true;  // cluster-mode param rules group by these rules' flowIds and namespaces
    h->ps_groups_stale = true;
    h->cp_wls = wls;
    h->cptotal = base;
    h->cpstride = stride;
    if (!h->d_cplast_ts) {
        if (hipMalloc(&h->d_cplast_ts, sizeof(int64_t)) != hipSuccess) return fail(h, SG_E_NOMEM, "ts");
        const int64_t neg = -1;
        HIP_TRY(h, hipMemcpy(h->d_cplast_ts, &neg, sizeof(neg), hipMemcpyHostToDevice));
    }
    return SG_OK;
}

static CPArgs cp_args(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values, uint64_t n_values,
                      sg_result* out) {
    CPArgs c{};
    c.req = req;
    c.values = values;
    c.n_values = n_values;
    c.out = out;
    c.n = n;
    c.ibits = bits_for(h->cfg.max_batch > 1 ? h->cfg.max_batch - 1 : 1);
    c.imask = (1ull << c.ibits) - 1;
    c.rules = h->d_cprules;
    c.n_rules = (uint32_t)h->cptab.size();
    c.hot = h->d_cphot;
    c.keys = h->d_cpkeys;
    c.ring = h->d_cpring;
    c.stride = h->cpstride;
    c.total_slots = h->cptotal;
    c.per = h->cptab.empty() ? 1 : h->cptab[0].table_mask + 2;
    c.err = h->d_err;
    c.last_ts = h->d_cplast_ts;
    return c;
}

namespace {

// allowProceed → GlobalRequestLimiter.tryPass for the namespaces with a limiter (state shared with flow tokens):
// the limiter slot of every cluster param rule's namespace on the device (h->cp_any_lim: some rule has one)
int cp_rule_limiters(sg_handle* h, hipStream_t stream) {
    const uint32_t R = (uint32_t)h->cprules.size();
    std::vector<uint8_t> rl(R ? R : 1, 0xFF);
    bool any_lim = false;
    for (uint32_t k = 0; k < R; ++k) {
        const int ns = h->cprules[k].namespace_id;
        if (ns >= 0 && (size_t)ns < h->ns_slot.size() && h->ns_slot[ns] >= 0) {
            rl[k] = (uint8_t)h->ns_slot[ns];
            any_lim = true;
        }
    }
    h->cp_any_lim = any_lim;
    if (any_lim && (rl != h->cp_rule_lim_host || !h->d_cp_rule_lim)) {
        dfree(h->d_cp_rule_lim);
        if (hipMalloc(&h->d_cp_rule_lim, rl.size()) != hipSuccess) return fail(h, SG_E_NOMEM, "cparam limiter table");
        HIP_TRY(h, hipMemcpyAsync(h->d_cp_rule_lim, rl.data(), rl.size(), hipMemcpyHostToDevice, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        h->cp_rule_lim_host = rl;
    }
    return SG_OK;
}

int cparam_batch(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values, uint64_t n_values,
                 sg_result* out, hipStream_t stream);

}  // namespace

// With a sharded namespace limiter (sg_set_shard, world > 1) every batch consumes an armed sg_lim_exchange over the
// node's param requests (sg_lim_arrivals_param); a batch rejected on the device, an empty one or one refused
// before the device still walks the armed arrivals (the shard's replica of the namespace windows advances).
int sg_cparam_decide_batch(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                           uint64_t n_values, sg_result* out, void* stream_) {
    if (!h) return SG_E_INVAL;
    const bool xshard = h->shard_world > 1 && h->n_lim > 0;
    if (xshard && !h->lim_x_armed)
        return fail(h, SG_E_UNSUPPORTED, "sharded namespace limiter: sg_lim_exchange must precede every param batch");
    const bool armed = h->lim_x_armed;
    h->lim_x_armed = false;  // consumed by this call, whatever its outcome
    hipStream_t stream = (hipStream_t)stream_;
    const char* early = n == 0 ? "" : (!req || !out || (!values && n_values)) ? "null buffer"
                        : n > h->cfg.max_batch ? "batch larger than max_batch"
                        : !h->d_cplast_ts ? "sg_cparam_load_rules first" : nullptr;
    if (early) {
        if (armed) {
            int rc = lim_plan_only(h, stream);
            if (rc) return rc;
        }
        if (n == 0) return SG_OK;
        return fail(h, n > h->cfg.max_batch ? SG_E_CAPACITY : SG_E_INVAL, early);
    }
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    h->lim_x_armed = armed;  // read by cparam_batch's limiter step
    const int rc = cparam_batch(h, req, n, values, n_values, out, stream);
    const bool unused = h->lim_x_armed;  // still set: the batch stopped before its limiter step
    h->lim_x_armed = false;
    if (unused && armed) {
        const int rc2 = lim_plan_only(h, stream);
        if (rc2 && !rc) return rc2;
    }
    return rc;
}

namespace {

int cparam_batch(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values, uint64_t n_values,
                 sg_result* out, hipStream_t stream) {
    CPArgs c = cp_args(h, req, n, values, n_values, out);
    const uint64_t nv = n_values ? n_values : 1;
    const int gbits = bits_for(h->cptotal + 1);
    // value records {slot : gbits | multi : 1 | acquire code : 7 | request index or value position : idbits}
    const int pbits = 64 - gbits;
    const int idbits = pbits - 8;
    if (gbits > 32 || idbits < std::max(bits_for(nv), bits_for(n)))
        return fail(h, SG_E_UNSUPPORTED, "param tables x values too large for 64-bit records");
    // scratch sized for the batch's value positions
    if (nv > h->cp_val_cap) {
        dfree(h->d_cp_owner);
        dfree(h->d_cp_pslot);
        dfree(h->d_cp_long);
        dfree(h->d_cp_short);
        dfree(h->d_cp_chk);
        dfree(h->d_cp_rec);
        dfree(h->d_cp_rec2);
        dfree(h->d_cp_hist);
        dfree(h->d_cp_items);
        if (hipMalloc(&h->d_cp_items, sizeof(uint32_t) * 9 * nv) != hipSuccess ||
            hipMalloc(&h->d_cp_owner, sizeof(uint32_t) * nv) != hipSuccess ||
            hipMalloc(&h->d_cp_pslot, sizeof(uint32_t) * nv) != hipSuccess || hipMalloc(&h->d_cp_chk, nv) != hipSuccess ||
            hipMalloc(&h->d_cp_rec, 8 * nv) != hipSuccess || hipMalloc(&h->d_cp_rec2, 8 * nv) != hipSuccess ||
            hipMalloc(&h->d_cp_hist, sizeof(uint32_t) * radix_hist_words(nv)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "cparam batch scratch");
        uint64_t off = 0;  // k_seg's class slices for nv records (as sg_create sizes them for max_batch)
        for (int c = 0; c < kClasses; ++c) {
            h->cp_class_off[c] = off;
            off += (c == 0 ? nv : nv / (kClassMax[c - 1] + 1)) + 1;
        }
        if (hipMalloc(&h->d_cp_long, sizeof(uint32_t) * (nv + 1)) != hipSuccess ||
            hipMalloc(&h->d_cp_short, sizeof(uint32_t) * off) != hipSuccess)
            return fail(h, SG_E_NOMEM, "cparam segment lists");
        h->cp_val_cap = nv;
    }
    if (h->cptotal > h->cp_slot_item_cap) {
        dfree(h->d_cp_slot_item);
        if (hipMalloc(&h->d_cp_slot_item, sizeof(uint32_t) * h->cptotal) != hipSuccess)
            return fail(h, SG_E_NOMEM, "cparam slot items");
        h->cp_slot_item_cap = h->cptotal;
    }
    if (!h->d_cp_counts && (hipMalloc(&h->d_cp_counts, 8 * sizeof(uint32_t)) != hipSuccess ||
                            hipMalloc(&h->d_cp_mlist, sizeof(uint32_t) * h->cfg.max_batch) != hipSuccess))
        return fail(h, SG_E_NOMEM, "cparam batch scratch");
    if (!h->d_cp_assume && (hipMalloc(&h->d_cp_assume, h->cfg.max_batch) != hipSuccess ||
                            hipMalloc(&h->d_cp_changed, sizeof(int) * (2 + (size_t)h->cp_max_rounds)) != hipSuccess))
        return fail(h, SG_E_NOMEM, "cparam batch scratch");
    int rc = cp_rule_limiters(h, stream);
    if (rc) return rc;
    const bool any_lim = h->cp_any_lim;
    const uint32_t R = (uint32_t)h->cprules.size();
    HIP_TRY(h, hipMemsetAsync(h->d_err, 0, sizeof(int), stream));
    CPBatch b{};
    b.owner = h->d_cp_owner;
    b.chk = h->d_cp_chk;
    b.assume = h->d_cp_assume;
    b.rec = h->d_cp_rec;
    b.pbits = pbits;
    b.pmask = (1ull << pbits) - 1;
    b.idbits = idbits;
    b.idmask = (1ull << idbits) - 1;
    b.n_wl = (int)h->cp_wls.size();
    for (int w = 0; w < b.n_wl; ++w) b.wl[w] = h->cp_wls[w];
    if (!h->d_cp_bnd && (hipMalloc(&h->d_cp_bnd, sizeof(uint32_t) * kMaxWl * kMaxPeriods) != hipSuccess ||
                         hipMalloc(&h->d_cp_p0, sizeof(int64_t) * kMaxWl) != hipSuccess ||
                         hipMalloc(&h->d_cp_np, sizeof(uint32_t) * kMaxWl) != hipSuccess))
        return fail(h, SG_E_NOMEM, "cparam period tables");
    b.bnd = h->d_cp_bnd;
    b.p0 = h->d_cp_p0;
    b.np = h->d_cp_np;
    b.changed = h->d_cp_changed;
    b.pslot = h->d_cp_pslot;
    b.dflag = h->d_cp_items;                      // [nv] (items <= value positions)
    b.item_start = h->d_cp_items + nv;           // [nv]
    b.slot_item = h->d_cp_slot_item;
    b.item_end = h->d_cp_items + 6 * nv;         // [nv]
    b.item_slot = h->d_cp_items + 7 * nv;        // [nv]
    b.dq = h->d_cp_items + 8 * nv;               // [nv]
    b.dcap = (uint32_t)nv;                       // re-walk lists: 2 buffers x {long, short} x nv
    b.mlist = h->d_cp_mlist;
    b.mcount = h->d_cp_counts + 4;
    b.lim = any_lim ? 1 : 0;
    HIP_TRY(h, hipMemsetAsync(h->d_cp_changed, 0, sizeof(int), stream));
    HIP_TRY(h, hipMemsetAsync(b.mcount, 0, sizeof(uint32_t), stream));
    HIP_TRY(h, launch_cp_prep2(c, b, stream));  // sets *changed iff a request has several values, lists them
    if (n_values == 0) {  // every request is BAD_REQUEST, NO_RULE_EXISTS or out of bounds (none reaches the limiter)
        HIP_TRY(h, launch_cp_finish_batch(c, stream));
        int err = 0;
        HIP_TRY(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        h->cp_rounds = 0;
        if (err & kErrTime) return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
        if (err & kErrBounds) return fail(h, SG_E_INVAL, "a request's values lie outside the value array");
        if (err & kErrPeriods) return fail(h, SG_E_UNSUPPORTED, "batch spans more than 65536 window or limiter periods");
        return SG_OK;
    }
    uint64_t* sorted = nullptr;
    HIP_TRY(h, radix_sort_records(h->d_cp_rec, h->d_cp_rec2, nv, pbits, h->d_cp_hist, &sorted, stream, 64));
    HIP_TRY(h, launch_cp_order(c, b, sorted, nv, stream));
    if (any_lim) {  // after validation: a rejected batch leaves the limiter untouched
        BatchArgs a{};
        int kb = bits_for((uint64_t)R);
        if (kb < 1) kb = 1;
        a.n = n;
        a.rec = h->d_rec;
        a.kshift = 64 - kb;
        a.K = R;
        a.bnd = h->d_bnd;
        a.np = h->d_np;
        a.p0 = h->d_p0;
        a.out = out;
        a.err = h->d_err;
        HIP_TRY(h, launch_cp_limprep(c, a, stream));
        LimArgs L{};
        L.n_lim = h->n_lim;
        L.wl_idx = 0;  // the cparam batch's 100 ms periods are row 0
        std::memcpy(L.qps, h->lim_qps, sizeof(L.qps));
        L.rule_lim = h->d_cp_rule_lim;
        L.slot = h->d_lim_slot;
        const uint64_t tiles = n / 4096 + 1;
        L.tile_tot = h->d_lim_tile;
        L.tile_off = h->d_lim_tile + tiles * kMaxLim;
        L.arrivals = h->d_lim_period;
        L.prefix = h->d_lim_period + (size_t)kMaxLim * kMaxPeriods;
        L.quota = h->d_lim_period + (size_t)2 * kMaxLim * kMaxPeriods;
        L.ring = h->d_lim_ring;
        if (h->lim_x_armed) {  // sharded: the node's gathered param arrivals (sg_lim_exchange)
            L.xg = h->lim_xg;
            L.ts = &req[0].ts_ms;
            L.ts_stride = sizeof(sg_cparam_req) / sizeof(int64_t);
            L.t_base = h->lim_xt;
            L.n_ms = h->lim_xn;
            L.world = h->shard_world;
            L.rank = h->shard_rank;
            h->lim_x_armed = false;
        }
        HIP_TRY(h, launch_limiter(a, L, stream));
    }
    // one lane per (rule, value) slot: k_seg's lists over the sorted value records
    BatchArgs sgm{};
    sgm.n = nv;
    sgm.rec_sorted = sorted;
    sgm.kshift = pbits;
    sgm.K = (uint32_t)h->cptotal;
    sgm.err = h->d_err;
    sgm.long_list = h->d_cp_long;
    sgm.long_count = h->d_long_count;
    sgm.short_list = h->d_cp_short;
    sgm.short_count = h->d_long_count + 1;
    for (int cl = 0; cl < kClasses; ++cl) sgm.class_off[cl] = h->cp_class_off[cl];
    uint32_t csplit = 64u;  // lane / wave walker split of the cluster param walkers (SG_CPARAM_SHORT_MAX: tuning; r04: 64 < 32 by 5%)
    if (const char* e = std::getenv("SG_CPARAM_SHORT_MAX")) csplit = (uint32_t)std::strtoul(e, nullptr, 10);
    sgm.short_max = (h->cfg.flags & SG_FLAG_WAVE_ONLY) ? 0u : (h->cfg.flags & SG_FLAG_SERIAL_ONLY) ? 0xFFFFFFFFu : csplit;
    HIP_TRY(h, hipMemsetAsync(h->d_long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream));
    HIP_TRY(h, launch_seg(sgm, stream));
    // are there multi-value requests? (then the first walk saves the touched rings for the re-walks)
    uint32_t counts[1 + kClasses], np[kMaxWl] = {};
    int err = 0, has_multi = 0;
    HIP_TRY(h, hipMemcpyAsync(counts, h->d_long_count, sizeof(counts), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipMemcpyAsync(np, b.np, sizeof(uint32_t) * b.n_wl, hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipMemcpyAsync(&has_multi, h->d_cp_changed, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    uint64_t touched = 0;
    for (uint32_t x : counts) touched += x;
    // work items: segment bounds and each touched slot's item (the walkers need the bounds in every round)
    if (!err && touched > 0) HIP_TRY(h, launch_cp_items(b, sgm, touched, stream));
    if (!err && has_multi && touched > 0) {
        // re-walk flags clear, the multi-value requests' list
        HIP_TRY(h, hipMemsetAsync(b.dflag, 0, sizeof(uint32_t) * touched, stream));
        HIP_TRY(h, launch_cp_mlist(c, b, stream));
        if (touched * h->cpstride > h->cp_save_cap) {
            dfree(h->d_cp_save);
            if (hipMalloc(&h->d_cp_save, sizeof(CPBucket) * touched * h->cpstride) != hipSuccess)
                return fail(h, SG_E_NOMEM, "cparam ring save area");
            h->cp_save_cap = touched * h->cpstride;
        }
        b.save = h->d_cp_save;  // the first walk saves the touched rings, re-walks restore the dirty ones
        // hot slots' ring at the opening of every window period, so a re-walk resumes at the first period a changed
        // outcome touches (batches of <= kCkMaxPeriods periods, within a memory cap)
        constexpr uint32_t kCkMaxPeriods = 64;
        constexpr uint64_t kCkMaxBytes = 1ull << 30;
        uint32_t ck_np = 0;
        for (int w = 0; w < b.n_wl; ++w) ck_np = std::max(ck_np, np[w]);
        const uint64_t ck = (uint64_t)counts[0] * ck_np * h->cpstride;
        if (counts[0] > 0 && ck_np <= kCkMaxPeriods && ck * sizeof(CPBucket) <= kCkMaxBytes &&
            !std::getenv("SG_CP_NO_CKPT")) {
            if (ck > h->cp_ckpt_cap) {
                dfree(h->d_cp_ckpt);
                if (hipMalloc(&h->d_cp_ckpt, sizeof(CPBucket) * ck) != hipSuccess)
                    return fail(h, SG_E_NOMEM, "cparam ring checkpoints");
                h->cp_ckpt_cap = ck;
            }
            b.ckpt = h->d_cp_ckpt;
            b.ck_np = ck_np;
            HIP_TRY(h, hipMemsetAsync(b.dq, 0xFF, sizeof(uint32_t) * touched, stream));
        }
    }
    // saturated ranges of hot slots (pieces of <= 4096 records, each >= 256: at most 2 nv / 256 + 1)
    {
        const uint64_t cap = 2 * nv / 256 + 1;
        if (cap > h->cp_skip_cap) {
            dfree(h->d_cp_skips);
            if (hipMalloc(&h->d_cp_skips, sizeof(uint2) * cap) != hipSuccess ||
                (!h->d_cp_skip_count && hipMalloc(&h->d_cp_skip_count, sizeof(uint32_t)) != hipSuccess))
                return fail(h, SG_E_NOMEM, "cparam skip list");
            h->cp_skip_cap = cap;
        }
        b.skips = h->d_cp_skips;
        b.skip_count = h->d_cp_skip_count;
        b.skip_cap = (uint32_t)cap;
    }
    // rounds: walk every slot under the assumed multi-value outcomes, then recompute the outcomes
    const uint32_t kMaxRounds = h->cp_max_rounds;
    uint32_t round = 0;
    bool converged = false;
    if (!err && !has_multi) {  // single-value requests only: the slots are independent, one walk is exact
        HIP_TRY(h, hipMemsetAsync(b.skip_count, 0, sizeof(uint32_t), stream));
        HIP_TRY(h, launch_cp_walk2(c, b, sgm, stream, h->aux, h->fork, h->join));
        converged = true;
    }
    // Rounds are enqueued kChain at a time and the host reads their flags once per chain (a host round trip costs
    // ~90 us between rounds): round r's combine sets flag r (d_cp_changed[1 + r]) iff an outcome changed, and a round
    // after one that changed nothing returns at once (its lists are empty, combine and relist check the flags).
    // Each round's counters are zeroed on the device: dout_count by combine, skip_count by relist.
    constexpr uint32_t kChain = 3;
    if (!err && !converged) {
        HIP_TRY(h, hipMemsetAsync(h->d_cp_changed + 1, 0, sizeof(int) * (1 + (size_t)kMaxRounds), stream));
        HIP_TRY(h, hipMemsetAsync(b.skip_count, 0, sizeof(uint32_t), stream));
    }
    while (!err && !converged && round < kMaxRounds) {
        const uint32_t r0 = round, r1 = std::min(round + kChain, kMaxRounds);
        for (uint32_t r = r0; r < r1; ++r) {
            b.round = (int)r;
            // this round walks the lists the previous combine filled (buffer r & 1), and combine fills the other
            b.din = h->d_cp_items + (size_t)(2 + 2 * (r & 1)) * nv;
            b.din_count = h->d_cp_counts + 2 * (r & 1);
            b.dout = h->d_cp_items + (size_t)(2 + 2 * ((r + 1) & 1)) * nv;
            b.dout_count = h->d_cp_counts + 2 * ((r + 1) & 1);
            b.changed = h->d_cp_changed + 1 + r;
            b.changed_prev = r > 0 ? h->d_cp_changed + r : nullptr;
            HIP_TRY(h, launch_cp_walk2(c, b, sgm, stream, h->aux, h->fork, h->join));
            HIP_TRY(h, launch_cp_combine(c, b, sgm, touched, stream));
        }
        int changed[kChain] = {0, 0, 0};
        HIP_TRY(h, hipMemcpyAsync(changed, h->d_cp_changed + 1 + r0, sizeof(int) * (r1 - r0), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        round = r1;
        for (uint32_t r = r0; r < r1; ++r) {
            if (!changed[r - r0]) {
                converged = true;
                round = r + 1;
                break;
            }
        }
    }
    if (!err && !converged) {  // rare: replay the groups of linked slots, each in arrival order, from the saved rings
        CPGroups g{};
        g.items = (uint32_t)touched;
        g.label = h->d_cp_items + 2 * nv;  // the re-walk lists are done with (the flags [0, nv) mark moving groups)
        g.flag = h->d_cp_items + 3 * nv;
        g.heads = h->d_cp_items + 4 * nv;
        g.changed = h->d_cp_changed;
        g.ent = h->d_cp_rec;               // the sorted value records are done with too
        g.ent_count = h->d_cp_counts + 5;
        g.head_count = h->d_cp_counts + 6;
        g.ibits = bits_for(n);
        g.all = round == 0 ? 1 : 0;
        uint32_t mreq = 0;
        HIP_TRY(h, hipMemcpyAsync(&mreq, b.mcount, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, launch_cpfb(c, b, g, 0, 0, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        for (int moved = 1; moved;) {  // labels strictly decrease: terminates
            HIP_TRY(h, hipMemsetAsync(g.changed, 0, sizeof(int), stream));
            HIP_TRY(h, launch_cpfb(c, b, g, 1, mreq, stream));
            HIP_TRY(h, hipMemcpyAsync(&moved, g.changed, sizeof(int), hipMemcpyDeviceToHost, stream));
            HIP_TRY(h, hipStreamSynchronize(stream));
        }
        HIP_TRY(h, hipMemsetAsync(g.ent_count, 0, 2 * sizeof(uint32_t), stream));
        HIP_TRY(h, launch_cpfb(c, b, g, 2, mreq, stream));
        uint32_t m = 0;
        HIP_TRY(h, hipMemcpyAsync(&m, g.ent_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        HIP_TRY(h, radix_sort_records(h->d_cp_rec, h->d_cp_rec2, m, 0, h->d_cp_hist, &g.ent_sorted, stream,
                                      g.ibits + bits_for(touched)));
        HIP_TRY(h, launch_cpfb(c, b, g, 3, m, stream));
    }
    h->cp_rounds = converged ? (round ? round : 1) : kMaxRounds + 1;
    HIP_TRY(h, launch_cp_finish_batch(c, stream));
    HIP_TRY(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (err & kErrTime) return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (err & kErrBounds)
        return fail(h, SG_E_INVAL, "a request's values lie outside the value array, overlap another's or go backwards");
    if (err & kErrTableFull) return fail(h, SG_E_CAPACITY, "a param rule's value table is full");
    if (err & kErrPeriods) return fail(h, SG_E_UNSUPPORTED, "batch spans more than 65536 window or limiter periods");
    return SG_OK;
}

}  // namespace

int sg_cparam_last_rounds(const sg_handle* h, uint32_t* rounds) {
    if (!h || !rounds) return SG_E_INVAL;
    *rounds = h->cp_rounds;
    return SG_OK;
}

int sg_cparam_decide_batch_host(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                uint64_t n_values, sg_result* out) {
    if (!h) return SG_E_INVAL;
    // empty or refused before the device: the device entry point answers (and walks an armed exchange)
    if (n == 0 || n > h->cfg.max_batch || !req || !out || (!values && n_values))
        return sg_cparam_decide_batch(h, n ? req : nullptr, n, values, n_values, out, nullptr);
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_cpreq_h) {
        if (hipMalloc(&h->d_cpreq_h, sizeof(sg_cparam_req) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_cpout_h, sizeof(sg_result) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    if (n_values > h->cpval_cap) {
        dfree(h->d_cpval_h);
        if (hipMalloc(&h->d_cpval_h, 8 * n_values) != hipSuccess) return fail(h, SG_E_NOMEM, "host-path values");
        h->cpval_cap = n_values;
    }
    HIP_TRY(h, hipMemcpy(h->d_cpreq_h, req, sizeof(sg_cparam_req) * n, hipMemcpyHostToDevice));
    if (n_values) HIP_TRY(h, hipMemcpy(h->d_cpval_h, values, 8 * n_values, hipMemcpyHostToDevice));
    int rc = sg_cparam_decide_batch(h, h->d_cpreq_h, n, h->d_cpval_h, n_values, h->d_cpout_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(out, h->d_cpout_h, sizeof(sg_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_cparam_read_sum(sg_handle* h, uint32_t rule, uint64_t value, int64_t now_ms, int64_t* sum) {
    if (!h || !sum || rule >= h->cptab.size()) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    int64_t* d = nullptr;
    HIP_TRY(h, hipMalloc(&d, sizeof(int64_t)));
    CPArgs c = cp_args(h, nullptr, 0, nullptr, 0, nullptr);
    hipError_t e = launch_cp_read(c, rule, value, now_ms, d, 0);
    if (e == hipSuccess) e = hipMemcpy(sum, d, sizeof(int64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    return SG_OK;
}

int sg_cparam_top_values(sg_handle* h, int64_t now_ms, uint32_t number, uint64_t* values, double* qps, uint32_t* counts) {
    if (!h || number == 0 || (!h->cptab.empty() && (!values || !qps || !counts))) return SG_E_INVAL;
    const uint32_t R = (uint32_t)h->cptab.size();
    if (R == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    CPArgs c = cp_args(h, nullptr, 0, nullptr, 0, nullptr);
    const uint64_t per = h->cptotal / R;
    CPTop* d_top = nullptr;
    unsigned long long* d_cnt = nullptr;
    if (hipMalloc(&d_top, sizeof(CPTop) * h->cptotal) != hipSuccess || hipMalloc(&d_cnt, sizeof(unsigned long long)) != hipSuccess) {
        dfree(d_top);
        return fail(h, SG_E_NOMEM, "top values buffer");
    }
    unsigned long long cnt = 0;
    hipError_t e = hipMemset(d_cnt, 0, sizeof(cnt));
    if (e == hipSuccess) e = launch_cp_top(c, now_ms, per, d_top, d_cnt, 0);
    if (e == hipSuccess) e = hipMemcpy(&cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost);
    std::vector<CPTop> top(cnt);
    if (e == hipSuccess && cnt) e = hipMemcpy(top.data(), d_top, sizeof(CPTop) * cnt, hipMemcpyDeviceToHost);
    (void)hipFree(d_top);
    (void)hipFree(d_cnt);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    // per rule: count descending (the reference compares (int) casts of the counts), ties by value
    std::sort(top.begin(), top.end(), [](const CPTop& a, const CPTop& b) {
        if (a.rule != b.rule) return a.rule < b.rule;
        const int32_t ca = (int32_t)a.sum, cb = (int32_t)b.sum;
        if (ca != cb) return ca > cb;
        return a.value < b.value;
    });
    std::fill(counts, counts + R, 0u);
    for (const CPTop& t : top) {
        uint32_t& k = counts[t.rule];
        if (k >= number) continue;
        values[(size_t)t.rule * number + k] = t.value;
        qps[(size_t)t.rule * number + k] = (double)t.sum / h->cptab[t.rule].isec;  // count / getIntervalInSecond
        ++k;
    }
    return SG_OK;
}

// ------------------------------------------------------------------------------ local slot chain

int sg_local_load_rules(sg_handle* h, const sg_local_config* cfg, const sg_local_rule* rules, uint32_t n) {
    if (!h || !cfg || (!rules && n)) return SG_E_INVAL;
    if (n >= SG_KEY_BAD) return fail(h, SG_E_INVAL, "too many resources");
    if (cfg->sample_count <= 0 || cfg->interval_ms <= 0 || cfg->interval_ms % cfg->sample_count != 0)
        return fail(h, SG_E_INVAL, "invalid statistic window (SAMPLE_COUNT / INTERVAL)");
    if (cfg->sample_count > kMinuteS) return fail(h, SG_E_UNSUPPORTED, "SAMPLE_COUNT > 60");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    std::vector<LRule> tab(n);
    for (uint32_t i = 0; i < n; ++i) {
        const sg_local_rule& r = rules[i];
        if (r.flow_grade < -1 || r.flow_grade > 1) return fail(h, SG_E_INVAL, "flow grade");
        if (r.flow_grade >= 0 && !(r.flow_count >= 0)) return fail(h, SG_E_INVAL, "flow count must be >= 0");
        if (r.n_breakers < 0 || r.n_breakers > 2) return fail(h, SG_E_INVAL, "at most two degrade rules");
        LRule& L = tab[i];
        L = LRule{};
        L.flow_count = r.flow_count;
        L.flow_grade = r.flow_grade;
        L.nb = r.n_breakers;
        for (int j = 0; j < 2; ++j) {
            LBreakerRule& b = L.b[j];
            b = LBreakerRule{};
            b.stat_ms = 1;
            if (j >= r.n_breakers) continue;
            const sg_degrade_rule& d = r.breakers[j];
            if (d.grade < SG_DEGRADE_RT || d.grade > SG_DEGRADE_EXCEPTION_COUNT || d.stat_interval_ms <= 0 ||
                !(d.count >= 0))
                return fail(h, SG_E_INVAL, "invalid degrade rule");
            b.grade = d.grade;
            b.count = d.count;
            b.slow_ratio = d.slow_ratio_threshold;
            b.max_rt = java_math_round(d.count);  // ResponseTimeCircuitBreaker.java:52
            b.min_request = d.min_request_amount;
            b.recovery_ms = (int32_t)((uint32_t)d.time_window_sec * 1000u);  // int arithmetic, wraps
            b.stat_ms = d.stat_interval_ms;
        }
    }
    // window lengths of the period tables: the second window's bucket and the minute window's 1000 ms
    h->l_n_wl = 0;
    const int32_t wl2 = cfg->interval_ms / cfg->sample_count;
    h->l_wl[h->l_n_wl++] = wl2;
    h->l_wsec = 0;
    h->l_wmin = (wl2 == kMinuteWl) ? 0 : h->l_n_wl;
    if (wl2 != kMinuteWl) h->l_wl[h->l_n_wl++] = kMinuteWl;

    dfree(h->d_lrules);
    dfree(h->d_lfrules);
    dfree(h->d_lctl);
    dfree(h->d_lhead);
    dfree(h->d_lsec);
    dfree(h->d_lbor);
    dfree(h->d_lmin);
    h->l_nodes = n;
    h->l_n_origins = 0;
    h->l_n_contexts = 0;
    h->l_has_cx = false;
    h->l_cluster_rules = false;
    h->l_base_cx.clear();
    h->l_relate.clear();
    h->l_cluster_refs.clear();
    h->l_groups_stale = false;
    h->l_rule_slot.clear();
    dfree(h->d_lnkeys);
    dfree(h->d_lnvals);
    dfree(h->d_ldyn);
    h->l_nmap_cap = 0;
    h->l_pool_cap = h->l_pool_used = 0;
    h->l_epoch = 0;
    h->l_batches = 0;
    dfree(h->d_lgkey);
    dfree(h->d_linbound);  // every resource's entries EntryType.OUT until sg_local_set_entry_types
    h->l_ps_applied = 0;
    if (!h->d_lentry_fetch && (hipMalloc(&h->d_lentry_fetch, sizeof(int64_t)) != hipSuccess ||
                               hipMalloc(&h->d_lentry_acc, sizeof(LBucket) * kMinuteS) != hipSuccess))
        return fail(h, SG_E_NOMEM, "ENTRY_NODE state");
    {
        const int64_t neg1 = -1;  // StatisticNode.lastFetchTime of Constants.ENTRY_NODE
        HIP_TRY(h, hipMemcpy(h->d_lentry_fetch, &neg1, sizeof(neg1), hipMemcpyHostToDevice));
    }
    if (!h->d_llast_ts && hipMalloc(&h->d_llast_ts, sizeof(int64_t)) != hipSuccess) return fail(h, SG_E_NOMEM, "ts");
    const int64_t neg = -1;
    HIP_TRY(h, hipMemcpy(h->d_llast_ts, &neg, sizeof(neg), hipMemcpyHostToDevice));
    h->lcfg = *cfg;
    h->ltab = tab;
    if (n) {
        if (hipMalloc(&h->d_lrules, sizeof(LRule) * n) != hipSuccess || hipMalloc(&h->d_lhead, sizeof(LHead) * n) != hipSuccess ||
            hipMalloc(&h->d_lsec, sizeof(LBucket) * (size_t)n * cfg->sample_count) != hipSuccess ||
            hipMalloc(&h->d_lbor, sizeof(LFuture) * (size_t)n * cfg->sample_count) != hipSuccess ||
            hipMalloc(&h->d_lmin, sizeof(LBucket) * (size_t)n * kMinuteS) != hipSuccess)
            return fail(h, SG_E_NOMEM, "local state allocation");
        HIP_TRY(h, hipMemcpy(h->d_lrules, tab.data(), sizeof(LRule) * n, hipMemcpyHostToDevice));
        LArgs L{};
        L.K = n;
        L.N = n;
        L.S = cfg->sample_count;
        L.head = h->d_lhead;
        L.sec = h->d_lsec;
        L.bor = h->d_lbor;
        L.minute = h->d_lmin;
        HIP_TRY(h, launch_local_init(L, 0));
        dfree(h->d_llast_fetch);
        if (hipMalloc(&h->d_llast_fetch, sizeof(int64_t) * n) != hipSuccess) return fail(h, SG_E_NOMEM, "lastFetchTime");
        std::vector<int64_t> neg1(n, -1);  // StatisticNode.lastFetchTime = -1
        HIP_TRY(h, hipMemcpy(h->d_llast_fetch, neg1.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipDeviceSynchronize());
    }
    return SG_OK;
}

int sg_local_set_entry_types(sg_handle* h, const uint8_t* inbound, uint32_t n) {
    if (!h || (!inbound && n)) return SG_E_INVAL;
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    if (n != h->ltab.size()) return fail(h, SG_E_INVAL, "one entry type per resource");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    std::vector<uint8_t> v(n);
    for (uint32_t k = 0; k < n; ++k) v[k] = inbound[k] ? 1 : 0;
    dfree(h->d_linbound);
    if (n && hipMalloc(&h->d_linbound, n) != hipSuccess) return fail(h, SG_E_NOMEM, "entry types");
    if (n) HIP_TRY(h, hipMemcpy(h->d_linbound, v.data(), n, hipMemcpyHostToDevice));
    return SG_OK;
}

namespace {
int local_metrics(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows, int raw,
                  bool device_out = false);
void local_group_keys(sg_handle* h, std::vector<uint32_t>& gkey);
}

int sg_local_metrics(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows) {
    return local_metrics(h, now_ms, out, cap, n_rows, 0);
}

int sg_local_metrics_raw(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows) {
    return local_metrics(h, now_ms, out, cap, n_rows, 1);
}

int sg_local_metrics_raw_device(sg_handle* h, int64_t now_ms, sg_metric_node* d_out, uint64_t cap, uint64_t* n_rows) {
    return local_metrics(h, now_ms, d_out, cap, n_rows, 1, true);
}

int sg_local_metrics_raw_enqueue(sg_handle* h, int64_t now_ms, sg_metric_node* d_out, uint64_t cap, uint64_t* d_count,
                                 void* stream_) {
    if (!h || !d_count || (!d_out && cap)) return SG_E_INVAL;
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t stream = (hipStream_t)stream_;
    if (h->ltab.empty()) {
        HIP_TRY(h, hipMemsetAsync(d_count, 0, sizeof(uint64_t), stream));
        return SG_OK;
    }
    int rc = pipe_setup(h);
    if (rc) return rc;
    if (!h->lm_done) {
        HIP_TRY(h, hipEventCreateWithFlags(&h->lm_in, hipEventDisableTiming));
        HIP_TRY(h, hipEventCreateWithFlags(&h->lm_done, hipEventDisableTiming));
    }
    if ((!h->d_lm_cnt && hipMalloc(&h->d_lm_cnt, sizeof(unsigned long long)) != hipSuccess) ||
        (!h->d_lm_gate && hipMalloc(&h->d_lm_gate, sizeof(int)) != hipSuccess))
        return fail(h, SG_E_NOMEM, "metric row counter");
    LArgs L{};
    L.K = (uint32_t)h->ltab.size();
    L.minute = h->d_lmin;
    L.last_fetch = h->d_llast_fetch;
    L.inbound = h->d_linbound;
    L.entry_acc = h->d_lentry_acc;
    L.entry_fetch = h->d_lentry_fetch;
    // after the batches already enqueued (their back halves on s_back) and the caller's earlier work on `stream`
    // (e.g. the rollup still reading a previous call's rows); before every batch enqueued later
    hipStream_t s = h->s_back;
    HIP_TRY(h, hipEventRecord(h->lm_in, stream));
    HIP_TRY(h, hipStreamWaitEvent(s, h->lm_in, 0));
    // a capacity that covers every possible row (59 per resource, 60 of the ENTRY_NODE) needs no count pass: the
    // emit pass alone, its counter copied out
    const bool worst = cap >= (uint64_t)L.K * (kMinuteS - 1) + kMinuteS;
    for (int emit = worst ? 1 : 0; emit < 2; ++emit) {
        HIP_TRY(h, launch_entry_acc_reset(h->d_lentry_acc, s));
        HIP_TRY(h, hipMemsetAsync(h->d_lm_cnt, 0, sizeof(unsigned long long), s));
        const int* gate = emit && !worst ? h->d_lm_gate : nullptr;
        HIP_TRY(h, launch_local_metrics(L, now_ms, emit ? d_out : nullptr, h->d_lm_cnt, emit, 1, s, gate));
        if (h->d_linbound)
            HIP_TRY(h, launch_local_entry_rows(L, now_ms, emit ? d_out : nullptr, h->d_lm_cnt, emit, 1, s, gate));
        if (!emit) HIP_TRY(h, launch_metrics_gate(h->d_lm_cnt, cap, (unsigned long long*)d_count, h->d_lm_gate, s));
    }
    if (worst) HIP_TRY(h, hipMemcpyAsync(d_count, h->d_lm_cnt, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    HIP_TRY(h, hipEventRecord(h->lm_done, s));
    HIP_TRY(h, hipStreamWaitEvent(stream, h->lm_done, 0));
    return SG_OK;
}

int sg_local_owners(sg_handle* h, uint32_t world, uint32_t* owner, uint32_t n) {
    if (!h || world == 0 || (!owner && n)) return SG_E_INVAL;
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    const uint32_t K = (uint32_t)h->ltab.size();
    if (n != K) return fail(h, SG_E_INVAL, "owner buffer must hold one entry per resource");
    if (world > 1 && h->l_cluster_state == SG_CLUSTER_SERVER && h->n_lim > 0 && (h->l_cluster_rules || h->ps_cluster))
        return fail(h, SG_E_UNSUPPORTED, "an embedded token server with namespace limiters serves the node from one GPU");
    std::vector<uint32_t> gkey;
    local_group_keys(h, gkey);
    for (uint32_t k = 0; k < K; ++k) {  // splitmix64(group key) mod world (sentinel_amd/cluster.py local_owners)
        uint64_t z = (uint64_t)gkey[k] + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        owner[k] = (uint32_t)(z % world);
    }
    return SG_OK;
}

namespace {
int local_metrics(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows, int raw,
                  bool device_out) {
    if (!h || !n_rows || (!out && cap)) return SG_E_INVAL;
    *n_rows = 0;
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    if (h->ltab.empty()) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    LArgs L{};
    L.K = (uint32_t)h->ltab.size();
    L.minute = h->d_lmin;
    L.last_fetch = h->d_llast_fetch;
    L.inbound = h->d_linbound;
    L.entry_acc = h->d_lentry_acc;
    L.entry_fetch = h->d_lentry_fetch;
    // MetricTimerListener.run: the resources' rows, then the ENTRY_NODE's (counted first, then emitted: the emit
    // pass has the side effects)
    auto pass = [&](sg_metric_node* dst, unsigned long long* d_cnt, int emit) -> hipError_t {
        hipError_t e = launch_entry_acc_reset(h->d_lentry_acc, 0);
        if (e == hipSuccess) e = hipMemsetAsync(d_cnt, 0, sizeof(unsigned long long), 0);
        if (e == hipSuccess) e = launch_local_metrics(L, now_ms, dst, d_cnt, emit, raw, 0);
        if (e == hipSuccess && h->d_linbound) e = launch_local_entry_rows(L, now_ms, dst, d_cnt, emit, raw, 0);
        return e;
    };
    if (!h->d_lm_cnt && hipMalloc(&h->d_lm_cnt, sizeof(unsigned long long)) != hipSuccess)
        return fail(h, SG_E_NOMEM, "metric row counter");
    unsigned long long* d_cnt = h->d_lm_cnt;
    unsigned long long cnt = 0;
    hipError_t e = pass(nullptr, d_cnt, 0);
    if (e == hipSuccess) e = hipMemcpy(&cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    *n_rows = cnt;
    if (cnt > cap) return fail(h, SG_E_CAPACITY, "metric row buffer too small (*n_rows rows)");
    if (device_out) {  // the rows straight into the caller's device buffer, unsorted (the node rollup sorts)
        e = pass(out, d_cnt, 1);
        if (e == hipSuccess) e = hipStreamSynchronize(0);
        if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
        return SG_OK;
    }
    sg_metric_node* d_out = nullptr;
    if (cnt && hipMalloc(&d_out, sizeof(sg_metric_node) * cnt) != hipSuccess) return fail(h, SG_E_NOMEM, "metric rows");
    e = pass(d_out, d_cnt, 1);
    if (e == hipSuccess && cnt) e = hipMemcpy(out, d_out, sizeof(sg_metric_node) * cnt, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipStreamSynchronize(0);
    if (d_out) (void)hipFree(d_out);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    std::sort(out, out + cnt, [](const sg_metric_node& a, const sg_metric_node& b) {  // the listener's TreeMap by time
        return a.timestamp != b.timestamp ? a.timestamp < b.timestamp : a.resource < b.resource;
    });
    return SG_OK;
}
}  // namespace

namespace {

// The ParamFlowSlot flags of the resources (LRule.ps: rules loaded by sg_pslot_load_rules for the resource) on the
// device rule image: a resource with param rules is walked by the full-chain walker.
int local_apply_params(sg_handle* h) {
    const uint64_t want = h->ps_loaded ? h->ps_gen : 0;
    if (h->l_ps_applied == want) return SG_OK;
    const uint32_t K = (uint32_t)h->ltab.size();
    std::vector<LRule> tab = h->ltab;
    bool any = false;
    for (uint32_t k = 0; k < K && h->ps_loaded && k < h->ps_res_rules.size(); ++k) {
        if (!h->ps_res_rules[k]) continue;
        tab[k].ps = 1;
        tab[k].cx = 1;
        any = true;
    }
    if (K) HIP_TRY(h, hipMemcpy(h->d_lrules, tab.data(), sizeof(LRule) * K, hipMemcpyHostToDevice));
    h->l_has_cx_ps = any;
    h->l_ps_applied = want;
    return SG_OK;
}

// Node pool: a map with room for every key a batch of n events may add at load <= 1/2 (host rehash when it
// grows), the per-event slot buffer and the per-resource epochs.
int lnode_prepare(sg_handle* h, uint64_t n) {
    const uint32_t K = (uint32_t)h->ltab.size();
    if (!h->d_lev_node) {
        if (hipMalloc(&h->d_lev_node, sizeof(uint2) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_lnode_new, sizeof(uint32_t)) != hipSuccess ||
            hipHostMalloc(&h->h_lnode_new, sizeof(uint32_t)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "node pool workspace");
    }
    if (!h->d_ldyn) {
        if (hipMalloc(&h->d_ldyn, sizeof(uint32_t) * (K ? K : 1)) != hipSuccess) return fail(h, SG_E_NOMEM, "node pool");
        HIP_TRY(h, hipMemset(h->d_ldyn, 0, sizeof(uint32_t) * (K ? K : 1)));
        h->l_epoch = 0;
    }
    const uint64_t keys_per_event = (h->l_n_origins > 0 ? 1 : 0) + (h->l_n_contexts > 0 ? 1 : 0);
    const uint64_t need = 2 * ((uint64_t)h->l_pool_used + n * keys_per_event);
    if (h->d_lnkeys && need <= h->l_nmap_cap) return SG_OK;
    uint64_t cap = h->l_nmap_cap ? h->l_nmap_cap : (1ull << 12);
    while (cap < need) cap <<= 1;
    std::vector<uint64_t> ok, nk(cap, 0);
    std::vector<uint32_t> ov, nv(cap, kNoNode);
    if (h->d_lnkeys) {  // rehash the existing keys
        ok.resize(h->l_nmap_cap);
        ov.resize(h->l_nmap_cap);
        HIP_TRY(h, hipDeviceSynchronize());
        HIP_TRY(h, hipMemcpy(ok.data(), h->d_lnkeys, sizeof(uint64_t) * ok.size(), hipMemcpyDeviceToHost));
        HIP_TRY(h, hipMemcpy(ov.data(), h->d_lnvals, sizeof(uint32_t) * ov.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < ok.size(); ++i) {
            if (!ok[i]) continue;
            uint64_t j = lnode_hash(ok[i]) & (cap - 1);
            while (nk[j]) j = (j + 1) & (cap - 1);
            nk[j] = ok[i];
            nv[j] = ov[i];
        }
    }
    uint64_t* dk = nullptr;
    uint32_t* dv = nullptr;
    if (hipMalloc(&dk, sizeof(uint64_t) * cap) != hipSuccess || hipMalloc(&dv, sizeof(uint32_t) * cap) != hipSuccess) {
        dfree(dk);
        dfree(dv);
        return fail(h, SG_E_NOMEM, "node pool map");
    }
    hipError_t e = hipMemcpy(dk, nk.data(), sizeof(uint64_t) * cap, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dv, nv.data(), sizeof(uint32_t) * cap, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        dfree(dk);
        dfree(dv);
        return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    }
    dfree(h->d_lnkeys);
    dfree(h->d_lnvals);
    h->d_lnkeys = dk;
    h->d_lnvals = dv;
    h->l_nmap_cap = cap;
    return SG_OK;
}

// Pool capacity >= used nodes: new node arrays (the resources, the old pool, empty nodes), geometric growth. Every
// growth copies the resources' nodes too (~4.2 KB each: 4 GB at 1M resources), so the pool starts at K / 16 nodes
// (~260 MB at 1M resources) and grows fourfold with room for twice the nodes in use.
int lnode_grow(sg_handle* h, uint64_t used) {
    if (used <= h->l_pool_cap) return SG_OK;
    if (const char* f = std::getenv("SG_TEST_POOL_FAIL"))  // test aid: a failed growth (tests/test_local_rules_gpu.py)
        if (std::atoi(f)) return fail(h, SG_E_NOMEM, "node pool (SG_TEST_POOL_FAIL)");
    const uint64_t K = h->ltab.size();
    uint64_t cap = std::max<uint64_t>({2ull * used, 4ull * h->l_pool_cap, 1024ull, K / 16});
    if (K + cap >= SG_KEY_BAD) cap = SG_KEY_BAD - 1 - K;
    if (K + used >= SG_KEY_BAD || cap < used) return fail(h, SG_E_CAPACITY, "too many origin / context nodes");
    const uint64_t N = K + cap, old = h->l_nodes;
    const int S = h->lcfg.sample_count;
    LHead* hd = nullptr;
    LBucket *sec = nullptr, *mnt = nullptr;
    LFuture* bor = nullptr;
    if (hipMalloc(&hd, sizeof(LHead) * N) != hipSuccess || hipMalloc(&sec, sizeof(LBucket) * N * S) != hipSuccess ||
        hipMalloc(&bor, sizeof(LFuture) * N * S) != hipSuccess || hipMalloc(&mnt, sizeof(LBucket) * N * kMinuteS) != hipSuccess) {
        dfree(hd);
        dfree(sec);
        dfree(bor);
        dfree(mnt);
        return fail(h, SG_E_NOMEM, "node pool");
    }
    hipError_t e = hipMemcpy(hd, h->d_lhead, sizeof(LHead) * old, hipMemcpyDeviceToDevice);
    if (e == hipSuccess) e = hipMemcpy(sec, h->d_lsec, sizeof(LBucket) * old * S, hipMemcpyDeviceToDevice);
    if (e == hipSuccess) e = hipMemcpy(bor, h->d_lbor, sizeof(LFuture) * old * S, hipMemcpyDeviceToDevice);
    if (e == hipSuccess) e = hipMemcpy(mnt, h->d_lmin, sizeof(LBucket) * old * kMinuteS, hipMemcpyDeviceToDevice);
    if (e == hipSuccess) {
        LArgs L{};
        L.S = S;
        L.head = hd;
        L.sec = sec;
        L.bor = bor;
        L.minute = mnt;
        e = launch_local_init_range(L, old, N, 0);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        dfree(hd);
        dfree(sec);
        dfree(bor);
        dfree(mnt);
        return fail(h, SG_E_DEVICE, std::string("node pool growth: ") + hipGetErrorString(e));
    }
    dfree(h->d_lhead);
    dfree(h->d_lsec);
    dfree(h->d_lbor);
    dfree(h->d_lmin);
    h->d_lhead = hd;
    h->d_lsec = sec;
    h->d_lbor = bor;
    h->d_lmin = mnt;
    h->l_nodes = (uint32_t)N;
    h->l_pool_cap = (uint32_t)cap;
    return SG_OK;
}

// The local path's batch buffers of one pipeline workspace: 0 the handle's own (every synchronous batch), 1 the
// flow pipeline's second workspace plus lws[1] (every other sg_local_enqueue batch).
struct LocalBufs {
    uint64_t* rec;
    uint64_t* rec_sorted;
    uint32_t* hist;
    uint32_t* bnd;
    int64_t* p0;
    uint32_t* np;
    int* err;
    uint32_t* long_list;
    uint32_t* counts;  // [1 + kClasses]: long count, short counts per class
    uint32_t* short_list;
    sg_handle::LocalWs* lw;
};

int local_bufs(sg_handle* h, int x, LocalBufs& b) {
    if (x == 0) {
        b = LocalBufs{h->d_rec, h->d_rec_sorted, h->d_hist, h->d_bnd, h->d_p0, h->d_np, h->d_err, h->d_long_list,
                      h->d_long_count, h->d_short_list, &h->lws[0]};
    } else {
        const auto& w = h->pws;
        b = LocalBufs{w.rec, w.rec_sorted, w.hist, w.bnd, w.p0, w.np, w.err, w.long_list, w.counts, w.short_list, &h->lws[1]};
    }
    sg_handle::LocalWs& lw = h->lws[x];
    if (!lw.flags) {  // the local path's own buffers of the workspace (sized for max_batch)
        const uint64_t mb = h->cfg.max_batch;
        h->lskip_cap = (uint32_t)(2 * mb / kSkipMin + 1);
        if (hipMalloc(&lw.flags, sizeof(int)) != hipSuccess ||
            hipMalloc(&lw.exit_pos, sizeof(uint32_t) * (mb + 1)) != hipSuccess ||
            hipMalloc(&lw.exit_cnt, sizeof(uint32_t) * (mb / kLTile + 2)) != hipSuccess ||
            hipMalloc(&lw.skips, sizeof(LSkip) * h->lskip_cap) != hipSuccess ||
            hipMalloc(&lw.skip_count, sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&lw.cxw_next, sizeof(uint32_t)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "local batch workspace");
    }
    return SG_OK;
}

// The kernels' arguments of a local batch on workspace buffers b (node tracking set up by the caller).
int local_args(sg_handle* h, const LocalBufs& b, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
               const sg_pslot_arg* args, uint64_t n_args, const uint64_t* values, uint64_t n_values, sg_local_result* out,
               bool emb, LArgs& L, BatchArgs& sgm) {
    const uint32_t K = (uint32_t)h->ltab.size();
    int kbits = bits_for((uint64_t)K);
    if (kbits < 1) kbits = 1;
    const int ibits = bits_for(h->cfg.max_batch > 1 ? h->cfg.max_batch - 1 : 1);
    const int abits = 64 - kbits - ibits;
    if (abits < 4) return fail(h, SG_E_UNSUPPORTED, "resources x max_batch too large for 64-bit records");

    L = LArgs{};
    L.ev = ev;
    L.out = out;
    L.cxw = h->l_cxw;
    // the short classes whose segments all have >= l_cxw_min records: one lane walking a few hundred records event by
    // event outlasts a wave that decides their dead periods 64 at a time
    L.cxw_cls = kClasses;
    for (int c = kClasses - 1; c >= 0 && (c == 0 ? 1u : kClassMax[c - 1] + 1u) >= h->l_cxw_min; --c) L.cxw_cls = c;
    L.n = n;
    L.rec = b.rec;
    L.rec_sorted = b.rec_sorted;
    L.kshift = 64 - kbits;
    L.abits = abits;
    L.imask = (ibits >= 64) ? ~0ull : ((1ull << ibits) - 1);
    L.amask = (1ull << abits) - 1;
    L.aesc = (1ull << (abits - 3)) - 1;
    L.K = K;
    L.N = h->l_nodes;
    L.rules = h->d_lrules;
    L.frules = h->d_lfrules;
    L.ctl = h->d_lctl;
    L.n_origins = h->l_n_origins;
    L.head = h->d_lhead;
    L.sec = h->d_lsec;
    L.bor = h->d_lbor;
    L.minute = h->d_lmin;
    L.S = h->lcfg.sample_count;
    L.wl2 = h->lcfg.interval_ms / h->lcfg.sample_count;
    L.interval = h->lcfg.interval_ms;
    L.isec = h->lcfg.interval_ms / 1000.0;
    L.occupy_timeout = h->lcfg.occupy_timeout_ms;
    L.wsec = h->l_wsec;
    L.wmin = h->l_wmin;
    L.n_wl = h->l_n_wl;
    std::memcpy(L.wl, h->l_wl, sizeof(L.wl));
    L.bnd = b.bnd;
    L.p0 = b.p0;
    L.np = b.np;
    L.err = b.err;
    L.last_ts = h->d_llast_ts;
    L.ext = ext;
    L.n_contexts = h->l_n_contexts;
    L.gkey = h->d_lgkey;
    L.has_ps = h->ps_loaded ? 1 : 0;
    if (h->ps_loaded) {
        L.ps = pslot_args(h);
        L.ps.args = args;
        L.ps.n_args = args ? n_args : 0;
        L.ps.values = values;
        L.ps.n_values = values ? n_values : 0;
        const int prc = pslot_embed(h, L.ps, 0);  // cluster-mode param rules on the embedded token server
        if (prc) return prc;
        if (h->l_cxw) {
            if (!b.lw->pslot && hipMalloc(&b.lw->pslot, sizeof(uint64_t) * h->cfg.max_batch) != hipSuccess)
                return fail(h, SG_E_NOMEM, "param lookups of the local batch");
            L.pslot = b.lw->pslot;
        }
    }
    if (emb) {  // the embedded token server: this handle's cluster flow state
        L.emb = 1;
        L.c3_rules = h->d_rules;
        L.c3_ring = h->d_ring;
        L.c3_hot = h->d_hot;
        L.c3_occ = h->d_occ;
        L.c3_stride = h->stride;
        L.c3_K = h->K;
        L.max_occ_ratio = h->cfg.max_occupy_ratio;
        L.c3_rule_lim = h->d_rule_lim;
        L.lim_ring = h->d_lim_ring;
        for (int j = 0; j < kMaxLim; ++j) L.lim_qps[j] = h->lim_qps[j];
        L.c3_last_ts = h->d_last_ts;
    }
    L.flags = b.lw->flags;
    L.cxw_next = b.lw->cxw_next;
    if (h->l_cxw && (h->l_has_cx || h->l_has_cx_ps)) {  // the cx wave walker's sorted-order side words
        if (!b.lw->cxside && hipMalloc(&b.lw->cxside, sizeof(CxSide) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "side words of the local batch");
        L.cxside = b.lw->cxside;
    }
    if (h->l_has_cx || h->l_has_cx_ps || h->l_n_contexts > 0) {
        if (!b.lw->cx_list && hipMalloc(&b.lw->cx_list, sizeof(uint32_t) * (h->cfg.max_batch + 1)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "cx segment list of the local batch");
        L.cx_list = b.lw->cx_list;
        L.cx_count = b.lw->cx_list + h->cfg.max_batch;
    }
    L.exit_pos = b.lw->exit_pos;
    L.exit_cnt = b.lw->exit_cnt;
    L.skips = b.lw->skips;
    L.skip_count = b.lw->skip_count;
    L.skip_cap = h->lskip_cap;
    L.hist0 = b.hist;
    L.hist0_bits = radix_digit_bits(64 - L.kshift);

    sgm = BatchArgs{};  // segment lists (k_seg)
    sgm.dbg = h->dbg;
    sgm.dbg_ctr = h->d_dbg;
    sgm.n = n;
    sgm.rec_sorted = b.rec_sorted;
    sgm.kshift = L.kshift;
    sgm.K = K;
    sgm.err = b.err;
    sgm.long_list = b.long_list;
    sgm.long_count = b.counts;
    sgm.short_list = b.short_list;
    sgm.short_count = b.counts + 1;
    for (int c = 0; c < kClasses; ++c) sgm.class_off[c] = h->class_off[c];
    // Lane / wave walker split: with many events per resource (n >= 256 K) the lanes' longest class (65..256 events)
    // sets the lane walker's end and the wave walker takes those segments sooner (C2, 10k resources: 0.88 → 0.82
    // ms/step); with few (C5, 1M resources) 256 stays best (1.97 against 2.28 ms at 64). SG_SHORT_MAX overrides.
    const uint32_t lsplit = (!h->short_max_env && (uint64_t)n >= 256ull * K) ? 64u : h->short_max;
    sgm.short_max = (h->cfg.flags & SG_FLAG_WAVE_ONLY) ? 0u : (h->cfg.flags & SG_FLAG_SERIAL_ONLY) ? 0xFFFFFFFFu : lsplit;

    return SG_OK;
}

// Front half of a local batch on `stream`: validation, default results and packed records (k_local_prep, with the
// first sort digit's histogram), the stable sort by resource, the segment lists and the exit positions. Reads no
// state a walker writes (with L.defer_last the first timestamp's check waits for the back half).
int local_front(sg_handle* h, LArgs& L, BatchArgs& sgm, hipStream_t stream) {
    HIP_TRY(h, hipMemsetAsync(L.err, 0, sizeof(int), stream));
    HIP_TRY(h, hipMemsetAsync(sgm.long_count, 0, (1 + kClasses) * sizeof(uint32_t), stream));
    HIP_TRY(h, hipMemsetAsync(L.flags, 0, sizeof(int), stream));
    HIP_TRY(h, hipMemsetAsync(L.skip_count, 0, sizeof(uint32_t), stream));
    L.csum0 = nullptr;
    if (radix_csum_atomic()) {
        L.csum0 = radix_csum(L.hist0, L.n, L.hist0_bits);
        HIP_TRY(h, hipMemsetAsync(L.csum0, 0, radix_csum_bytes(L.n, L.hist0_bits), stream));
    }
    HIP_TRY(h, launch_local_prep(L, stream));
    return SG_OK;
}

// count_exits: k_seg also counts the exit records per exit tile (k_lexit_count's pass, pipelined path)
int local_sort(sg_handle* h, LArgs& L, BatchArgs& sgm, uint64_t* spare, hipStream_t stream, bool count_exits = false) {
    uint64_t* sorted = nullptr;
    HIP_TRY(h, radix_sort_records(L.rec, spare, L.n, L.kshift, L.hist0, &sorted, stream, 64, true, nullptr,
                                  L.csum0 != nullptr));
    L.rec_sorted = sorted;
    sgm.rec_sorted = sorted;
    if (count_exits) {
        HIP_TRY(h, hipMemsetAsync(L.exit_cnt, 0, sizeof(uint32_t) * (L.n / kLTile + 2), stream));
        sgm.exit_cnt = L.exit_cnt;
        sgm.exit_amask = L.amask;
    }
    HIP_TRY(h, launch_seg(sgm, stream));
    return SG_OK;
}

// StatisticSlot around ParamFlowSlot → FlowSlot → DegradeSlot for a time-ordered batch (ext nullable).
int local_decide(sg_handle* h, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n, const sg_pslot_arg* args,
                 uint64_t n_args, const uint64_t* values, uint64_t n_values, sg_local_result* out, void* stream_) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!ev || !out) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    hipStream_t stream = (hipStream_t)stream_;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    if (h->l_groups_stale && (h->l_cluster_rules || h->ps_cluster)) {
        const int grc = local_apply_groups(h);
        if (grc) return grc;
    }
    int prc = local_apply_params(h);
    if (prc) return prc;
    const bool emb = h->l_cluster_state == SG_CLUSTER_SERVER && h->l_cluster_rules;
    if (emb && h->shard_world > 1 && h->n_lim > 0)
        return fail(h, SG_E_UNSUPPORTED, "an embedded token server on a sharded handle with namespace limiters: the "
                                         "limiter exchange covers flow and param batches only");
    LocalBufs b;
    int rc = local_bufs(h, 0, b);
    if (rc) return rc;
    LArgs L;
    BatchArgs sgm;
    rc = local_args(h, b, ev, ext, n, args, n_args, values, n_values, out, emb, L, sgm);
    if (rc) return rc;
    const uint32_t K = L.K;
    const bool track = h->l_n_origins > 0 || h->l_n_contexts > 0;
    if (track) {
        const int rc = lnode_prepare(h, n);
        if (rc) return rc;
        L.nkeys = h->d_lnkeys;
        L.nvals = h->d_lnvals;
        L.nmask = h->l_nmap_cap - 1;
        L.node_base = K + h->l_pool_used;
        L.node_new = h->d_lnode_new;
        L.ev_node = h->d_lev_node;
        L.dyn = h->d_ldyn;
        if (++h->l_epoch == 0) {  // the epochs wrapped: no resource may match a stale one
            HIP_TRY(h, hipMemset(h->d_ldyn, 0, sizeof(uint32_t) * (K ? K : 1)));
            h->l_epoch = 1;
        }
        L.epoch = h->l_epoch;
        L.track_ctx = h->l_n_contexts > 0 ? 1 : 0;
    }

    if (h->stats_on) HIP_TRY(h, hipEventRecord(h->ev[0], stream));
    rc = local_front(h, L, sgm, stream);
    if (rc) return rc;
    if (track) {  // the batch's new pool nodes (only for a batch that passed validation), then room for them
        HIP_TRY(h, hipMemsetAsync(h->d_lnode_new, 0, sizeof(uint32_t), stream));
        HIP_TRY(h, launch_lnode_assign(L, stream));
        HIP_TRY(h, hipMemcpyAsync(h->h_lnode_new, h->d_lnode_new, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipStreamSynchronize(stream));
        const uint64_t used = (uint64_t)h->l_pool_used + *h->h_lnode_new;
        // The map now holds the batch's new nodes (indices below K + used), so the allocator moves past them even
        // when the pool cannot grow now: this batch is then refused, and the next one grows the pool before any
        // walker reads a node. Nodes a refused batch created stay, with zero counts (NodeSelectorSlot and
        // ClusterBuilderSlot create them at entry, before any rule is checked).
        const int rc = lnode_grow(h, used);
        h->l_pool_used = (uint32_t)used;
        if (rc) return rc;
        L.N = h->l_nodes;
        L.head = h->d_lhead;
        L.sec = h->d_lsec;
        L.bor = h->d_lbor;
        L.minute = h->d_lmin;
    }
    if (h->stats_on) HIP_TRY(h, hipEventRecord(h->ev[1], stream));
    rc = local_sort(h, L, sgm, b.rec_sorted, stream);
    if (rc) return rc;
    h->last_sorted = L.rec_sorted;
    if (h->stats_on) HIP_TRY(h, hipEventRecord(h->ev[2], stream));
    HIP_TRY(h, launch_local_walk(L, sgm, h->l_has_cx || h->l_has_cx_ps || track, h->aux, stream, h->fork, h->join));
    if (h->stats_on) HIP_TRY(h, hipEventRecord(h->ev[3], stream));
    HIP_TRY(h, hipMemcpyAsync(h->h_err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    if (h->stats_on) {
        HIP_TRY(h, hipMemcpyAsync(h->h_long, h->d_long_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipMemcpyAsync(h->h_long + 1, L.skip_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(h, hipEventRecord(h->ev[4], stream));
    }
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (h->stats_on) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[4]);
        h->stats.total_ms = ms;
        (void)hipEventElapsedTime(&ms, h->ev[1], h->ev[2]);
        h->stats.sort_ms = ms;
        (void)hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
        h->stats.walk_ms = ms;
        h->stats.long_segments = h->h_long[0];
        h->stats.skipped_ranges = h->h_long[1];
    }
    rc = local_status(h, *h->h_err);
    if (rc) return rc;
    ++h->l_batches;
    return SG_OK;
}

// Whether a local batch may go on the pipeline: no node tracking (the pool grows with a host round trip inside the
// batch), no embedded token server (it shares the cluster flow state and its last timestamp), no rule tables
// waiting to be uploaded, no per-batch phase timing. Other batches drain the pipeline and run synchronously.
bool local_pipelinable(sg_handle* h) {
    const uint64_t want = h->ps_loaded ? h->ps_gen : 0;
    return h->l_n_origins == 0 && h->l_n_contexts == 0 && h->l_cluster_state != SG_CLUSTER_SERVER &&
           !(h->l_groups_stale && (h->l_cluster_rules || h->ps_cluster)) && h->l_ps_applied == want && !h->stats_on;
}

// One local batch on the pipeline, as enqueue_flow_pipelined: its front half (validation, sort, segments, exit
// positions) on s_front waits for the back half of the batch two back (same workspace) and runs beside the previous
// batch's walkers; its back half on s_back follows its front half and the previous batch's back half (the batches
// share the window state), and checks the first timestamp against last_ts once that batch has advanced it.
int enqueue_local_pipelined(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out, int* err_dst,
                            hipEvent_t done) {
    int rc = pipe_setup(h);
    if (rc) return rc;
    const int x = (int)(h->pipe_seq & 1);
    LocalBufs b;
    rc = local_bufs(h, x, b);
    if (rc) return rc;
    LArgs L;
    BatchArgs sgm;
    rc = local_args(h, b, ev, nullptr, n, nullptr, 0, nullptr, 0, out, false, L, sgm);
    if (rc) return rc;
    L.defer_last = 1;
    if (h->pipe_seq >= 2) HIP_TRY(h, hipStreamWaitEvent(h->s_front, h->back_done[x], 0));
    rc = local_front(h, L, sgm, h->s_front);
    if (rc) return rc;
    rc = local_sort(h, L, sgm, b.rec_sorted, h->s_front, true);
    if (rc) return rc;
    HIP_TRY(h, launch_local_exits(L, h->s_front, true));
    HIP_TRY(h, hipEventRecord(h->front_done[x], h->s_front));
    HIP_TRY(h, hipStreamWaitEvent(h->s_back, h->front_done[x], 0));
    HIP_TRY(h, launch_local_back(L, sgm, h->l_has_cx || h->l_has_cx_ps, h->s_aux2, h->s_back, h->pfork, h->pjoin));
    HIP_TRY(h, hipMemcpyAsync(err_dst, L.err, sizeof(int), hipMemcpyDeviceToHost, h->s_back));
    HIP_TRY(h, hipEventRecord(h->back_done[x], h->s_back));
    if (done) HIP_TRY(h, hipEventRecord(done, h->s_back));
    h->pipe_seq++;
    ++h->l_batches;
    return SG_OK;
}

}  // namespace

int sg_local_decide_batch(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out, void* stream) {
    return local_decide(h, ev, nullptr, n, nullptr, 0, nullptr, 0, out, stream);
}

int sg_slot_decide_batch(sg_handle* h, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
                         const sg_pslot_arg* args, uint64_t n_args, const uint64_t* values, uint64_t n_values,
                         sg_local_result* out, void* stream) {
    return local_decide(h, ev, ext, n, args, n_args, values, n_values, out, stream);
}

int sg_local_enqueue(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out, uint64_t* ticket) {
    if (!h || !ticket) return SG_E_INVAL;
    *ticket = 0;
    if (n == 0) return SG_OK;
    if (!ev || !out) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!local_pipelinable(h)) {  // the synchronous path (after the pipeline drained); its status waits for the ticket
        const int rc = local_decide(h, ev, nullptr, n, nullptr, 0, nullptr, 0, out, nullptr);
        if (rc == SG_E_DEVICE) return rc;
        *ticket = h->next_ticket++;
        h->finished[*ticket] = rc;
        return SG_OK;
    }
    sg_handle::DevTicket& d = h->dev[h->next_ticket % kDevSlots];
    if (!d.done) {
        if (hipHostMalloc(&d.h_err, sizeof(int)) != hipSuccess) return fail(h, SG_E_NOMEM, "pinned error word");
        HIP_TRY(h, hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    }
    if (d.ticket) {  // every slot in flight: complete the oldest (its status waits in `finished`)
        hipError_t e = hipEventSynchronize(d.done);
        h->finished[d.ticket] = e != hipSuccess ? fail(h, SG_E_DEVICE, hipGetErrorString(e)) : ticket_status(h, d);
        d.ticket = 0;
    }
    const int rc = enqueue_local_pipelined(h, ev, n, out, d.h_err, d.done);
    if (rc) return rc;
    d.local = true;
    d.ticket = h->next_ticket++;
    *ticket = d.ticket;
    return SG_OK;
}

int sg_local_poll(sg_handle* h, uint64_t ticket) { return sg_flow_poll(h, ticket); }

int sg_local_wait(sg_handle* h, uint64_t ticket) { return sg_flow_wait(h, ticket); }

int sg_slot_decide_batch_host(sg_handle* h, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
                              const sg_pslot_arg* args, uint64_t n_args, const uint64_t* values, uint64_t n_values,
                              sg_local_result* out) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!ev || !out) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_lev_h) {
        if (hipMalloc(&h->d_lev_h, sizeof(sg_local_event) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_lout_h, sizeof(sg_local_result) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    if (ext && !h->d_lext_h && hipMalloc(&h->d_lext_h, sizeof(sg_slot_ext) * h->cfg.max_batch) != hipSuccess)
        return fail(h, SG_E_NOMEM, "host-path buffers");
    sg_pslot_arg* d_args = nullptr;
    uint64_t* d_vals = nullptr;
    hipError_t e = hipMemcpy(h->d_lev_h, ev, sizeof(sg_local_event) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && ext) e = hipMemcpy(h->d_lext_h, ext, sizeof(sg_slot_ext) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && args && n_args) {
        e = hipMalloc(&d_args, sizeof(sg_pslot_arg) * n_args);
        if (e == hipSuccess) e = hipMemcpy(d_args, args, sizeof(sg_pslot_arg) * n_args, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && values && n_values) {
        e = hipMalloc(&d_vals, sizeof(uint64_t) * n_values);
        if (e == hipSuccess) e = hipMemcpy(d_vals, values, sizeof(uint64_t) * n_values, hipMemcpyHostToDevice);
    }
    int rc = SG_E_DEVICE;
    if (e == hipSuccess) {
        rc = local_decide(h, h->d_lev_h, ext ? h->d_lext_h : nullptr, n, d_args, d_args ? n_args : 0, d_vals,
                          d_vals ? n_values : 0, h->d_lout_h, nullptr);
        if (rc == SG_OK) e = hipMemcpy(out, h->d_lout_h, sizeof(sg_local_result) * n, hipMemcpyDeviceToHost);
    }
    if (d_args) (void)hipFree(d_args);
    if (d_vals) (void)hipFree(d_vals);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    return rc;
}

int sg_local_decide_batch_host(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_lev_h) {
        if (hipMalloc(&h->d_lev_h, sizeof(sg_local_event) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_lout_h, sizeof(sg_local_result) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    HIP_TRY(h, hipMemcpy(h->d_lev_h, ev, sizeof(sg_local_event) * n, hipMemcpyHostToDevice));
    int rc = sg_local_decide_batch(h, h->d_lev_h, n, h->d_lout_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(out, h->d_lout_h, sizeof(sg_local_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

namespace {

// One node's windows (resource or origin node) in the sg_local_read_state layout.
int local_read_node(sg_handle* h, uint32_t node, int64_t* second, int64_t* borrow, int64_t* minute, int64_t* head) {
    if ((uint64_t)node >= h->l_nodes) return fail(h, SG_E_INVAL, "node index past the node arrays");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    const int S = h->lcfg.sample_count;
    std::vector<LBucket> sb(S), mb(kMinuteS);
    std::vector<LFuture> fb(S);
    LHead hd;
    HIP_TRY(h, hipMemcpy(sb.data(), h->d_lsec + (size_t)node * S, sizeof(LBucket) * S, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemcpy(fb.data(), h->d_lbor + (size_t)node * S, sizeof(LFuture) * S, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemcpy(mb.data(), h->d_lmin + (size_t)node * kMinuteS, sizeof(LBucket) * kMinuteS, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemcpy(&hd, h->d_lhead + node, sizeof(LHead), hipMemcpyDeviceToHost));
    auto dump = [](const LBucket& b, int64_t* o) {
        const bool p = b.start != INT64_MIN;
        o[0] = b.start;
        for (int e = 0; e < kLEv; ++e) o[1 + e] = p ? b.c[e] : 0;
        o[7] = p ? b.min_rt : 0;
    };
    for (int j = 0; j < S; ++j) {
        dump(sb[j], second + 8 * j);
        borrow[2 * j] = fb[j].start;
        borrow[2 * j + 1] = fb[j].start != INT64_MIN ? fb[j].pass : 0;
    }
    for (int j = 0; j < kMinuteS; ++j) dump(mb[j], minute + 8 * j);
    head[0] = hd.threads;
    for (int j = 0; j < 2; ++j) {
        int64_t* o = head + 1 + 6 * j;
        o[0] = hd.cb[j].state;
        o[1] = hd.cb[j].next_retry;
        o[2] = hd.cb[j].stat_start;
        o[3] = hd.cb[j].stat_start != INT64_MIN ? hd.cb[j].bad : 0;
        o[4] = hd.cb[j].stat_start != INT64_MIN ? hd.cb[j].total : 0;
        o[5] = 0;
    }
    head[13] = 0;
    return SG_OK;
}

// A pool node's windows (sg_local_read_state layout): 1 when the node exists, 0 when no event created it yet (the
// dumps of an empty node: null slots, zero counters and threads).
int local_read_pool_node(sg_handle* h, uint64_t key, int64_t* second, int64_t* borrow, int64_t* minute, int64_t* head) {
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    uint32_t node = kNoNode;
    if (h->d_lnkeys) {
        HIP_TRY(h, hipDeviceSynchronize());
        HIP_TRY(h, launch_lnode_find(h->d_lnkeys, h->d_lnvals, h->l_nmap_cap - 1, key, h->d_lnode_new, 0));
        HIP_TRY(h, hipMemcpy(&node, h->d_lnode_new, sizeof(node), hipMemcpyDeviceToHost));
    }
    // A node a refused batch created past the pool's capacity (lnode_grow failed, l_pool_used moved past it) has
    // no storage yet: it exists with zero counts, which is what the empty dumps below say.
    const bool stored = node != kNoNode && (uint64_t)node < h->l_nodes;
    if (stored) {
        const int rc = local_read_node(h, node, second, borrow, minute, head);
        return rc ? rc : 1;
    }
    const int S = h->lcfg.sample_count;
    for (int j = 0; j < S; ++j) {
        for (int e = 0; e < 8; ++e) second[8 * j + e] = e == 0 ? INT64_MIN : 0;
        borrow[2 * j] = INT64_MIN;
        borrow[2 * j + 1] = 0;
    }
    for (int j = 0; j < kMinuteS; ++j)
        for (int e = 0; e < 8; ++e) minute[8 * j + e] = e == 0 ? INT64_MIN : 0;
    std::fill(head, head + 14, 0);
    head[3] = head[9] = INT64_MIN;  // the breakers' stat buckets of a fresh node: never created
    return node != kNoNode ? 1 : 0;
}

// FlowRuleUtil.isValidRule (:167-251) for local rules: count >= 0, grade / strategy / behaviour >= 0; QPS rules:
// checkClusterField (an invalid ClusterFlowConfig), checkStrategyField (RELATE / CHAIN need a refResource) and
// checkControlBehaviorField (warm-up period > 0, queueing time > 0); THREAD rules: checkClusterConcurrentField
bool local_flow_rule_valid(const sg_local_flow_rule& r) {
    if (!(r.count >= 0) || r.grade < 0 || r.strategy < 0 || r.control_behavior < 0) return false;
    if (r.cluster_mode == SG_CLUSTER_MODE_INVALID) return false;
    if (r.grade == 0) return true;
    if (r.grade != 1) return false;
    if ((r.strategy == SG_STRATEGY_RELATE || r.strategy == SG_STRATEGY_CHAIN) && r.ref_resource < 0) return false;
    switch (r.control_behavior) {
    case SG_CONTROL_WARM_UP: return r.warm_up_period_sec > 0;
    case SG_CONTROL_RATE_LIMITER: return r.max_queueing_ms > 0;
    case SG_CONTROL_WARM_UP_RATE_LIMITER: return r.warm_up_period_sec > 0 && r.max_queueing_ms > 0;
    default: return true;
    }
}

// FlowRule.equals (FlowRule.java, AbstractRule.equals): Double.compare on count, refResource, clusterMode and the
// ClusterFlowConfig (its caller-given id)
bool local_flow_rule_same(const sg_local_flow_rule& a, const sg_local_flow_rule& b) {
    return a.resource == b.resource && a.grade == b.grade && std::memcmp(&a.count, &b.count, sizeof(double)) == 0 &&
           a.control_behavior == b.control_behavior && a.limit_app == b.limit_app && a.strategy == b.strategy &&
           a.warm_up_period_sec == b.warm_up_period_sec && a.max_queueing_ms == b.max_queueing_ms &&
           (a.ref_resource < 0 ? b.ref_resource < 0 : a.ref_resource == b.ref_resource) &&
           (a.cluster_mode != 0) == (b.cluster_mode != 0) &&
           (a.cluster_mode == 0 || (a.cluster_mode == b.cluster_mode && a.cluster_config == b.cluster_config));
}

int32_t d2i_host(double x) {  // (int) double
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

// The controller constants of one flow rule (FlowRuleUtil.generateRater; WarmUpController.construct :83-106 in
// Java int arithmetic).
LFlowRule make_flow_rule(const sg_local_flow_rule& r, int cold) {
    LFlowRule f{};
    f.count = r.count;
    f.grade = r.grade;
    f.behavior = (r.grade == 1 && r.control_behavior >= SG_CONTROL_WARM_UP &&
                  r.control_behavior <= SG_CONTROL_WARM_UP_RATE_LIMITER) ? r.control_behavior : SG_CONTROL_DEFAULT;
    f.limit_app = r.limit_app;
    f.max_queue_ms = r.max_queueing_ms;
    f.cold = cold;
    f.strategy = r.strategy;
    f.ref = r.ref_resource < 0 ? -1 : r.ref_resource;
    f.cluster_mode = r.cluster_mode;
    f.cluster_key = r.cluster_key;
    if (f.behavior == SG_CONTROL_WARM_UP || f.behavior == SG_CONTROL_WARM_UP_RATE_LIMITER) {
        f.warning_token = d2i_host(r.warm_up_period_sec * r.count) / (cold - 1);
        const int32_t two_w = (int32_t)(2u * (uint32_t)r.warm_up_period_sec);  // 2 * warmUpPeriodInSec: int
        f.max_token = (int32_t)((uint32_t)f.warning_token + (uint32_t)d2i_host(two_w * r.count / (1.0 + cold)));
        f.slope = (cold - 1.0) / r.count / (double)(int32_t)((uint32_t)f.max_token - (uint32_t)f.warning_token);
    }
    return f;
}

}  // namespace

int sg_local_read_state(sg_handle* h, uint32_t res, int64_t* second, int64_t* borrow, int64_t* minute, int64_t* head) {
    if (!h || res >= h->ltab.size() || !second || !borrow || !minute || !head) return SG_E_INVAL;
    return local_read_node(h, res, second, borrow, minute, head);
}

int sg_local_read_origin_state(sg_handle* h, uint32_t res, int32_t origin, int64_t* second, int64_t* borrow,
                               int64_t* minute, int64_t* head) {
    if (!h || res >= h->ltab.size() || !second || !borrow || !minute || !head) return SG_E_INVAL;
    if (origin <= 0 || origin > h->l_n_origins) return fail(h, SG_E_INVAL, "origin id outside 1..n_origins");
    return local_read_pool_node(h, lnode_key(res, 0, (uint32_t)origin), second, borrow, minute, head);
}

int sg_local_read_context_state(sg_handle* h, uint32_t res, int32_t context, int64_t* second, int64_t* borrow,
                                int64_t* minute, int64_t* head) {
    if (!h || res >= h->ltab.size() || !second || !borrow || !minute || !head) return SG_E_INVAL;
    if (context < 0 || context >= h->l_n_contexts) return fail(h, SG_E_INVAL, "context id outside 0..n_contexts-1");
    return local_read_pool_node(h, lnode_key(res, kLNodeCtx, (uint32_t)context), second, borrow, minute, head);
}

int sg_local_read_controller(sg_handle* h, uint32_t rule, int64_t* state3) {
    if (!h || !state3 || rule >= h->l_rule_slot.size() || h->l_rule_slot[rule] == -1) return SG_E_INVAL;
    const int64_t slot = h->l_rule_slot[rule];
    if (slot == -2) {  // a DefaultController keeps no state
        state3[0] = 0;
        state3[1] = 0;
        state3[2] = -1;
        return SG_OK;
    }
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    LCtl c;
    HIP_TRY(h, hipMemcpy(&c, h->d_lctl + slot, sizeof(LCtl), hipMemcpyDeviceToHost));
    state3[0] = c.stored;
    state3[1] = c.last_filled;
    state3[2] = c.latest;
    return SG_OK;
}

int sg_local_set_cluster_state(sg_handle* h, int32_t state) {
    if (!h) return SG_E_INVAL;
    if (state != SG_CLUSTER_CLIENT && state != SG_CLUSTER_SERVER && state != SG_CLUSTER_NOT_STARTED)
        return fail(h, SG_E_INVAL, "cluster state: CLIENT 0, SERVER 1 or NOT_STARTED -1");
    if (state == SG_CLUSTER_CLIENT && (h->l_cluster_rules || h->ps_cluster))
        return fail(h, SG_E_UNSUPPORTED, "cluster-mode flow / param rules on a token client: the tokens come over the "
                                         "network, not in event order (INTEGRATION.md §8)");
    if (state != h->l_cluster_state) h->l_groups_stale = h->ps_groups_stale = true;  // key groups follow the state
    h->l_cluster_state = state;
    return SG_OK;
}

namespace {

// The embedded token server's sharing among the cluster-mode param rules (ParamFlowChecker.passClusterCheck →
// requestParamToken): rules naming one cluster param rule share its ClusterParamMetric, rules whose cluster param rule
// lies in a limiter-enabled namespace share its GlobalRequestLimiter (by_slot: a resource per limiter slot, shared with
// the flow rules' groups). unite(a, b) joins two resources.
void ps_cluster_unions(sg_handle* h, const std::function<void(uint32_t, uint32_t)>& unite, int* by_slot) {
    std::unordered_map<uint32_t, uint32_t> by_key;
    for (const auto& cr : h->ps_cluster_refs) {
        const uint32_t key = cr.second & SG_KEY_INDEX;
        if (key >= h->cprules.size()) continue;  // NO_RULE_EXISTS / BAD_REQUEST: no shared state
        auto it = by_key.emplace(key, cr.first).first;
        unite(cr.first, it->second);
        const int ns = h->cprules[key].namespace_id;
        const int sl = (ns >= 0 && (size_t)ns < h->ns_slot.size()) ? h->ns_slot[ns] : -1;
        if (sl >= 0) {
            if (by_slot[sl] < 0) by_slot[sl] = (int)cr.first;
            unite(cr.first, (uint32_t)by_slot[sl]);
        }
    }
}

// Key groups of the local chain (union-find, smallest resource first): a RELATE rule reads another resource's
// ClusterNode (FlowRuleChecker.selectReferenceNode :96-112); on an embedded token server the resources whose
// cluster-mode rules share a flowId share its ClusterMetric, and those naming flowIds of one limiter-enabled
// namespace share its GlobalRequestLimiter — each group walks in event order on one lane. Sets LRule.grp / cx and
// uploads the rule image and the record keys.
// The key groups of the local chain (resources whose decisions read each other's state): RELATE references and, on
// an embedded token server, resources sharing a flowId's ClusterMetric or a limited namespace. gkey[k] = the smallest
// resource of k's group.
void local_group_keys(sg_handle* h, std::vector<uint32_t>& gkey) {
    const uint32_t K = (uint32_t)h->ltab.size();
    std::vector<uint32_t> parent(K);
    for (uint32_t k = 0; k < K; ++k) parent[k] = k;
    auto find = [&](uint32_t x) {
        while (parent[x] != x) x = parent[x] = parent[parent[x]];
        return x;
    };
    auto unite = [&](uint32_t a, uint32_t b) {
        if (a >= K || b >= K) return;  // param rules of resources the chain does not have
        const uint32_t x = find(a), y = find(b);
        if (x != y) parent[std::max(x, y)] = std::min(x, y);
    };
    for (const auto& pr : h->l_relate) unite(pr.first, pr.second);
    if (h->l_cluster_state == SG_CLUSTER_SERVER) {
        std::unordered_map<uint32_t, uint32_t> by_key;
        int by_slot[kMaxLim];
        for (int j = 0; j < kMaxLim; ++j) by_slot[j] = -1;
        if (h->ps_loaded && h->ps_cluster) ps_cluster_unions(h, unite, by_slot);
        for (const auto& cr : h->l_cluster_refs) {
            const uint32_t key = cr.second & SG_KEY_INDEX;
            if (key >= h->K) continue;  // NO_RULE_EXISTS / BAD_REQUEST: no shared state
            auto it = by_key.emplace(key, cr.first).first;
            unite(cr.first, it->second);
            const int ns = h->rules[key].namespace_id;
            const int sl = (ns >= 0 && (size_t)ns < h->ns_slot.size()) ? h->ns_slot[ns] : -1;
            if (sl >= 0) {
                if (by_slot[sl] < 0) by_slot[sl] = (int)cr.first;
                unite(cr.first, (uint32_t)by_slot[sl]);
            }
        }
    }
    gkey.resize(K);
    for (uint32_t k = 0; k < K; ++k) gkey[k] = find(k);
}

int local_apply_groups(sg_handle* h) {
    const uint32_t K = (uint32_t)h->ltab.size();
    std::vector<uint32_t> gkey, gsize(K, 0);
    local_group_keys(h, gkey);
    for (uint32_t k = 0; k < K; ++k) ++gsize[gkey[k]];
    bool groups = false, has_cx = false;
    for (uint32_t k = 0; k < K; ++k) {
        LRule& L = h->ltab[k];
        L.grp = gsize[gkey[k]] > 1 ? 1 : 0;
        L.cx = (h->l_base_cx.size() == K && h->l_base_cx[k]) || L.grp ? 1 : 0;
        groups = groups || L.grp;
        has_cx = has_cx || L.cx;
    }
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipDeviceSynchronize());
    dfree(h->d_lgkey);
    if (groups) {
        if (hipMalloc(&h->d_lgkey, sizeof(uint32_t) * K) != hipSuccess) return fail(h, SG_E_NOMEM, "key groups");
        HIP_TRY(h, hipMemcpy(h->d_lgkey, gkey.data(), sizeof(uint32_t) * K, hipMemcpyHostToDevice));
    }
    if (K) HIP_TRY(h, hipMemcpy(h->d_lrules, h->ltab.data(), sizeof(LRule) * K, hipMemcpyHostToDevice));
    h->l_has_cx = has_cx;
    h->l_ps_applied = 0;  // param flags are re-applied to the new rule image by the next batch
    h->l_groups_stale = false;
    return SG_OK;
}

}  // namespace

int sg_local_load_flow_rules(sg_handle* h, const sg_local_flow_rule* rules, uint32_t n, int32_t n_origins,
                             int32_t n_contexts) {
    if (!h || (!rules && n)) return SG_E_INVAL;
    if (!h->d_llast_ts) return fail(h, SG_E_INVAL, "sg_local_load_rules first");
    if (n_origins < 0 || n_contexts < 0) return fail(h, SG_E_INVAL, "n_origins / n_contexts < 0");
    if (n_origins < h->l_n_origins || n_contexts < h->l_n_contexts)
        return fail(h, SG_E_INVAL, "origin / context ids keep their meaning across loads: the counts cannot shrink");
    drain_async(h);  // batches on the pipeline decide under the rules they were enqueued with (and settle l_batches)
    if (n_contexts > 0 && h->l_n_contexts == 0 && h->l_batches > 0)
        return fail(h, SG_E_UNSUPPORTED, "context tracking (n_contexts >= 1) starts before the first batch: a DefaultNode "
                                         "holds every entry of its context since the resource's first one");
    const bool track_ctx = n_contexts > 0;
    const uint32_t K = (uint32_t)h->ltab.size();
    const int cold = h->lcfg.cold_factor > 1 ? h->lcfg.cold_factor : 3;
    // FlowRuleUtil.buildFlowRuleMap (:83-130): drop invalid rules and duplicates (its HashSet), group by resource
    std::vector<int64_t> slot(n, -1);
    std::vector<std::vector<uint32_t>> by_res(K);
    bool cluster_rules = false;
    for (uint32_t i = 0; i < n; ++i) {
        const sg_local_flow_rule& r = rules[i];
        if (r.resource >= K || !local_flow_rule_valid(r)) continue;
        if (r.limit_app > n_origins || r.limit_app < SG_LIMIT_APP_OTHER)
            return fail(h, SG_E_INVAL, "limit_app names an origin id outside 1..n_origins");
        if (r.strategy == SG_STRATEGY_CHAIN && r.ref_resource >= n_contexts)
            return fail(h, SG_E_INVAL, "a CHAIN rule names a context id outside 0..n_contexts-1");
        if (r.cluster_mode != SG_CLUSTER_MODE_OFF && r.cluster_mode != SG_CLUSTER_MODE_FALLBACK &&
            r.cluster_mode != SG_CLUSTER_MODE_NO_FALLBACK)
            return fail(h, SG_E_INVAL, "cluster_mode");
        if (r.cluster_mode != SG_CLUSTER_MODE_OFF && h->l_cluster_state == SG_CLUSTER_CLIENT)
            return fail(h, SG_E_UNSUPPORTED, "cluster-mode flow rules on a token client (INTEGRATION.md §8)");
        bool dup = false;
        for (uint32_t j : by_res[r.resource]) dup = dup || local_flow_rule_same(rules[j], r);
        if (!dup) by_res[r.resource].push_back(i);
        cluster_rules = cluster_rules || r.cluster_mode != SG_CLUSTER_MODE_OFF;
    }
    std::vector<std::pair<uint32_t, uint32_t>> relate, cluster_refs;
    std::vector<uint8_t> base_cx(K, 0);
    std::vector<LRule> tab = h->ltab;
    std::vector<LFlowRule> fr;
    for (uint32_t k = 0; k < K; ++k) {
        std::vector<uint32_t>& v = by_res[k];
        // Collections.sort(FlowRuleComparator) (:30-55): stable; cluster-mode rules last, then limitApp "default" last
        auto key = [&](uint32_t x) {
            return (rules[x].cluster_mode != SG_CLUSTER_MODE_OFF ? 2 : 0) + (rules[x].limit_app == SG_LIMIT_APP_DEFAULT ? 1 : 0);
        };
        std::stable_sort(v.begin(), v.end(), [&](uint32_t x, uint32_t y) { return key(x) < key(y); });
        for (uint32_t i : v) {
            const sg_local_flow_rule& r = rules[i];
            if (r.strategy == SG_STRATEGY_RELATE && r.ref_resource >= 0 && (uint32_t)r.ref_resource < K &&
                (uint32_t)r.ref_resource != k)
                relate.emplace_back(k, (uint32_t)r.ref_resource);
            if (r.cluster_mode != SG_CLUSTER_MODE_OFF) cluster_refs.emplace_back(k, r.cluster_key);
        }
        LRule& L = tab[k];
        L.fr_begin = L.fr_n = 0;
        L.cx = 0;
        L.ps = 0;
        L.grp = 0;
        L.flow_grade = -1;
        L.flow_count = 0;
        // (with context tracking every event also updates its context's DefaultNode: the cx walker; a fast resource
        // that lands in a key group is walked there too, its one rule read from flow_grade / flow_count)
        const bool fast = v.size() == 1 && !track_ctx && rules[v[0]].limit_app == SG_LIMIT_APP_DEFAULT &&
                          rules[v[0]].strategy == SG_STRATEGY_DIRECT && rules[v[0]].cluster_mode == SG_CLUSTER_MODE_OFF &&
                          make_flow_rule(rules[v[0]], cold).behavior == SG_CONTROL_DEFAULT;
        if (fast) {  // the fast walkers' one DefaultController rule on the ClusterNode
            L.flow_grade = rules[v[0]].grade;
            L.flow_count = rules[v[0]].count;
            slot[v[0]] = -2;
            continue;
        }
        if (v.empty() && !track_ctx) continue;
        base_cx[k] = 1;
        L.fr_begin = (uint32_t)fr.size();
        L.fr_n = (uint32_t)v.size();
        for (uint32_t i : v) {
            slot[i] = (int64_t)fr.size();
            fr.push_back(make_flow_rule(rules[i], cold));
        }
    }
    // the nodes (ClusterNodes and the pool) are untouched: statistics outlive the reload
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipDeviceSynchronize());
    LFlowRule* d_fr = nullptr;
    LCtl* d_ctl = nullptr;
    auto release = [&]() {
        dfree(d_fr);
        dfree(d_ctl);
    };
    if (!fr.empty() && (hipMalloc(&d_fr, sizeof(LFlowRule) * fr.size()) != hipSuccess ||
                        hipMalloc(&d_ctl, sizeof(LCtl) * fr.size()) != hipSuccess)) {
        release();
        return fail(h, SG_E_NOMEM, "local flow rule allocation");
    }
    hipError_t e = hipSuccess;
    if (!fr.empty()) {
        e = hipMemcpy(d_fr, fr.data(), sizeof(LFlowRule) * fr.size(), hipMemcpyHostToDevice);
        std::vector<LCtl> c(fr.size(), LCtl{0, 0, -1, 0});  // storedTokens 0, lastFilledTime 0, latestPassedTime -1
        if (e == hipSuccess) e = hipMemcpy(d_ctl, c.data(), sizeof(LCtl) * c.size(), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        release();
        return fail(h, SG_E_DEVICE, std::string("local flow rule upload: ") + hipGetErrorString(e));
    }
    dfree(h->d_lfrules);
    dfree(h->d_lctl);
    h->d_lfrules = d_fr;
    h->d_lctl = d_ctl;
    h->ltab = tab;
    h->l_base_cx = base_cx;
    h->l_relate = relate;
    h->l_cluster_refs = cluster_refs;
    h->l_n_origins = n_origins;
    h->l_n_contexts = n_contexts;
    h->l_cluster_rules = cluster_rules;
    h->l_rule_slot = slot;
    const int rc = local_apply_groups(h);
    if (rc) return rc;
    int kept = 0;
    for (int64_t x : slot) kept += x != -1;
    return kept;
}

// ------------------------------------------------------------------------ concurrent cluster tokens

namespace {

// Upload what the concurrency kernels read (thresholds, timeouts, flowIds, counters) after rules / namespaces /
// timeouts changed; first use allocates the token table and the per-batch buffers.
int conc_prepare(sg_handle* h) {
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_ctok) {
        h->ctok_slots = 1ull << 20;
        if (hipMalloc(&h->d_ctok, sizeof(CTok) * h->ctok_slots) != hipSuccess ||
            hipMalloc(&h->d_calive, h->cfg.max_batch) != hipSuccess || hipMalloc(&h->d_clast_ts, sizeof(int64_t)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "concurrent token table");
        HIP_TRY(h, hipMemset(h->d_ctok, 0, sizeof(CTok) * h->ctok_slots));
        const int64_t neg = -1;
        HIP_TRY(h, hipMemcpy(h->d_clast_ts, &neg, sizeof(neg), hipMemcpyHostToDevice));
        h->ctok_used = 0;
    }
    if (!h->conc_dirty) return SG_OK;
    const uint32_t K = h->K;
    if (h->c_off.size() != K) {
        h->c_off.assign(K, 2000);
        h->c_res.assign(K, 2000);
    }
    std::vector<double> thr(K);
    std::vector<int64_t> fid(K);
    for (uint32_t k = 0; k < K; ++k) {  // ConcurrentClusterFlowChecker.calcGlobalThreshold (:36-46)
        const sg_flow_rule& r = h->rules[k];
        const int connected = (r.namespace_id >= 0 && (size_t)r.namespace_id < h->ns.size())
                                  ? h->ns[r.namespace_id].connected_count : 0;
        thr[k] = r.threshold_type == SG_THRESHOLD_GLOBAL ? r.count : r.count * connected;
        fid[k] = r.flow_id;
    }
    std::vector<int32_t> now = h->cnow_pending ? h->cnow_host : std::vector<int32_t>(K, 0);
    if (!h->cnow_pending && h->d_cnow && now.size() == K) {  // unchanged rules: keep the device counters
        HIP_TRY(h, hipMemcpy(now.data(), h->d_cnow, sizeof(int32_t) * K, hipMemcpyDeviceToHost));
    }
    dfree(h->d_cnow);
    dfree(h->d_cthr);
    dfree(h->d_coff);
    dfree(h->d_cres);
    dfree(h->d_cfid);
    const size_t k1 = K ? K : 1;
    if (hipMalloc(&h->d_cnow, sizeof(int32_t) * k1) != hipSuccess || hipMalloc(&h->d_cthr, sizeof(double) * k1) != hipSuccess ||
        hipMalloc(&h->d_coff, sizeof(int64_t) * k1) != hipSuccess || hipMalloc(&h->d_cres, sizeof(int64_t) * k1) != hipSuccess ||
        hipMalloc(&h->d_cfid, sizeof(int64_t) * k1) != hipSuccess)
        return fail(h, SG_E_NOMEM, "concurrency rule state");
    if (K) {
        HIP_TRY(h, hipMemcpy(h->d_cnow, now.data(), sizeof(int32_t) * K, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_cthr, thr.data(), sizeof(double) * K, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_coff, h->c_off.data(), sizeof(int64_t) * K, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_cres, h->c_res.data(), sizeof(int64_t) * K, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_cfid, fid.data(), sizeof(int64_t) * K, hipMemcpyHostToDevice));
    }
    if (!h->d_fid) {
        int rc = upload_fid_table(h);
        if (rc) return rc;
    }
    h->cnow_pending = false;
    h->conc_dirty = false;
    return SG_OK;
}

ConcArgs conc_args(sg_handle* h) {
    ConcArgs c{};
    c.base = h->conc_seq;
    c.K = h->K;
    c.thr = h->d_cthr;
    c.now = h->d_cnow;
    c.client_off = h->d_coff;
    c.res_to = h->d_cres;
    c.flow_id = h->d_cfid;
    c.tab = h->d_ctok;
    c.tmask = h->ctok_slots - 1;
    c.fid = h->d_fid;
    c.fid_mask = h->fid_mask;
    c.alive = h->d_calive;
    c.err = h->d_err;
    c.last_ts = h->d_clast_ts;
    return c;
}

// Keeps the token table at most half full: a rehash into a larger table when the batch could overflow it.
int conc_reserve(sg_handle* h, uint64_t n) {
    if (h->ctok_used + n <= h->ctok_slots / 2) return SG_OK;
    ConcArgs c = conc_args(h);
    unsigned long long* d_live = nullptr;
    HIP_TRY(h, hipMalloc(&d_live, sizeof(unsigned long long)));
    HIP_TRY(h, hipMemset(d_live, 0, sizeof(unsigned long long)));
    HIP_TRY(h, launch_conc_count(c, d_live, 0));
    unsigned long long live = 0;
    HIP_TRY(h, hipMemcpy(&live, d_live, sizeof(live), hipMemcpyDeviceToHost));
    (void)hipFree(d_live);
    uint64_t slots = 1ull << 20;
    while (slots < 4 * (live + n)) slots <<= 1;
    CTok* t = nullptr;
    if (hipMalloc(&t, sizeof(CTok) * slots) != hipSuccess) return fail(h, SG_E_NOMEM, "concurrent token table");
    HIP_TRY(h, hipMemset(t, 0, sizeof(CTok) * slots));
    HIP_TRY(h, hipMemset(h->d_err, 0, sizeof(int)));
    HIP_TRY(h, launch_conc_rehash(h->d_ctok, h->ctok_slots, t, slots - 1, h->d_err, 0));
    HIP_TRY(h, hipDeviceSynchronize());
    dfree(h->d_ctok);
    h->d_ctok = t;
    h->ctok_slots = slots;
    h->ctok_used = live;
    return SG_OK;
}

}  // namespace

int sg_conc_set_rule_timeouts(sg_handle* h, const int64_t* client_offline_ms, const int64_t* resource_timeout_ms,
                              uint32_t n) {
    if (!h || (n && (!client_offline_ms || !resource_timeout_ms))) return SG_E_INVAL;
    if (n != h->K) return fail(h, SG_E_INVAL, "one timeout pair per loaded rule");
    drain_async(h);
    h->c_off.assign(client_offline_ms, client_offline_ms + n);
    h->c_res.assign(resource_timeout_ms, resource_timeout_ms + n);
    h->conc_dirty = true;
    return SG_OK;
}

int sg_conc_decide_batch(sg_handle* h, const sg_conc_req* req, uint64_t n, sg_conc_result* out, void* stream_) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out) return fail(h, SG_E_INVAL, "null buffer");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int rc = conc_prepare(h);
    if (rc) return rc;
    rc = conc_reserve(h, n);
    if (rc) return rc;
    hipStream_t stream = (hipStream_t)stream_;
    int kbits = bits_for((uint64_t)h->K);
    if (kbits < 1) kbits = 1;
    if (kbits + bits_for(h->cfg.max_batch) > 64) return fail(h, SG_E_UNSUPPORTED, "rules x max_batch too large");
    ConcArgs c = conc_args(h);
    c.req = req;
    c.out = out;
    c.n = n;
    c.rec = h->d_rec;
    c.kshift = 64 - kbits;
    c.imask = (1ull << c.kshift) - 1;
    HIP_TRY(h, hipMemsetAsync(h->d_err, 0, sizeof(int), stream));
    HIP_TRY(h, launch_conc_batch(c, h->d_rec_sorted, h->d_hist, stream));
    HIP_TRY(h, hipMemcpyAsync(h->h_err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (*h->h_err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (*h->h_err & kErrTableFull) return fail(h, SG_E_CAPACITY, "concurrent token table full");
    h->conc_seq += n;
    h->ctok_used += n;
    return SG_OK;
}

int sg_conc_decide_batch_host(sg_handle* h, const sg_conc_req* req, uint64_t n, sg_conc_result* out) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->d_creq_h) {
        if (hipMalloc(&h->d_creq_h, sizeof(sg_conc_req) * h->cfg.max_batch) != hipSuccess ||
            hipMalloc(&h->d_cout_h, sizeof(sg_conc_result) * h->cfg.max_batch) != hipSuccess)
            return fail(h, SG_E_NOMEM, "host-path buffers");
    }
    HIP_TRY(h, hipMemcpy(h->d_creq_h, req, sizeof(sg_conc_req) * n, hipMemcpyHostToDevice));
    int rc = sg_conc_decide_batch(h, h->d_creq_h, n, h->d_cout_h, nullptr);
    if (rc) return rc;
    HIP_TRY(h, hipMemcpy(out, h->d_cout_h, sizeof(sg_conc_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_conc_expire(sg_handle* h, int64_t now_ms, const uint8_t* client_online, uint32_t n_clients, uint64_t* removed) {
    if (!h || (n_clients && !client_online)) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int rc = conc_prepare(h);
    if (rc) return rc;
    uint8_t* d_on = nullptr;
    unsigned long long* d_rm = nullptr;
    HIP_TRY(h, hipMalloc(&d_on, n_clients ? n_clients : 1));
    HIP_TRY(h, hipMalloc(&d_rm, sizeof(unsigned long long)));
    hipError_t e = n_clients ? hipMemcpy(d_on, client_online, n_clients, hipMemcpyHostToDevice) : hipSuccess;
    if (e == hipSuccess) e = hipMemset(d_rm, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = launch_conc_expire(conc_args(h), now_ms, d_on, n_clients, d_rm, 0);
    unsigned long long rm = 0;
    if (e == hipSuccess) e = hipMemcpy(&rm, d_rm, sizeof(rm), hipMemcpyDeviceToHost);
    (void)hipFree(d_on);
    (void)hipFree(d_rm);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    if (removed) *removed = rm;
    return SG_OK;
}

int sg_conc_read_state(sg_handle* h, uint32_t key, int32_t* now_calls, uint64_t* live_tokens) {
    if (!h || key >= h->K) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int rc = conc_prepare(h);
    if (rc) return rc;
    if (now_calls) HIP_TRY(h, hipMemcpy(now_calls, h->d_cnow + key, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (live_tokens) {
        unsigned long long* d = nullptr;
        HIP_TRY(h, hipMalloc(&d, sizeof(unsigned long long)));
        hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
        if (e == hipSuccess) e = launch_conc_count(conc_args(h), d, 0);
        unsigned long long v = 0;
        if (e == hipSuccess) e = hipMemcpy(&v, d, sizeof(v), hipMemcpyDeviceToHost);
        (void)hipFree(d);
        if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
        *live_tokens = v;
    }
    return SG_OK;
}

// ------------------------------------------------------------------------------ ParamFlowSlot chain

namespace {

PSArgs pslot_args(sg_handle* h) {
    PSArgs s{};
    s.cmode = h->d_ps_cmode;
    s.ckey = h->d_ps_ckey;
    s.p.rules = h->d_prules;
    s.p.n_rules = (uint32_t)h->ptab.size();
    s.p.hot = h->d_phot;
    s.p.table = h->d_ptable;
    s.p.total_slots = h->ptotal;
    s.p.err = h->d_err;
    s.n_res = h->ps_nres;
    s.res_begin = h->d_ps_begin;
    s.res_rules = h->d_ps_rules;
    s.grade = h->d_ps_grade;
    s.cur_idx = h->d_ps_idx;
    s.inited = h->d_ps_init;
    s.tc = h->d_ps_tc;
    s.tc_mask = h->ps_tc_slots - 1;
    s.err = h->d_err;
    s.last_ts = h->d_ps_last_ts;
    return s;
}

// The embedded token server of the cluster-mode param rules (ClusterStateManager SERVER with cluster rules loaded):
// this handle's cluster param state (sg_cparam_load_rules), its namespace limiters and the param batches' last
// timestamp. Without cluster param rules every token would be NO_RULE_EXISTS, which falls back as NOT_STARTED does.
int pslot_embed(sg_handle* h, PSArgs& s, hipStream_t stream) {
    s.emb = 0;
    if (!(h->l_cluster_state == SG_CLUSTER_SERVER && h->ps_cluster && h->d_cplast_ts)) return SG_OK;
    if (h->shard_world > 1 && h->n_lim > 0)
        return fail(h, SG_E_UNSUPPORTED, "an embedded token server on a sharded handle with namespace limiters: the "
                                         "limiter exchange covers flow and param batches only");
    const int rc = cp_rule_limiters(h, stream);
    if (rc) return rc;
    s.emb = 1;
    s.cp = cp_args(h, nullptr, 0, nullptr, 0, nullptr);
    s.cp_rule_lim = h->cp_any_lim ? h->d_cp_rule_lim : nullptr;
    s.lim_ring = h->d_lim_ring;
    for (int j = 0; j < kMaxLim; ++j) s.lim_qps[j] = h->lim_qps[j];
    s.cp_last_ts = h->d_cplast_ts;
    return SG_OK;
}

// Key groups of sg_pslot_decide_batch on an embedded token server (ps_cluster_unions): the record key of each resource.
int pslot_apply_groups(sg_handle* h) {
    if (!h->ps_groups_stale) return SG_OK;
    const uint32_t R = h->ps_nres;
    std::vector<uint32_t> parent(R);
    for (uint32_t k = 0; k < R; ++k) parent[k] = k;
    auto find = [&](uint32_t x) {
        while (parent[x] != x) x = parent[x] = parent[parent[x]];
        return x;
    };
    auto unite = [&](uint32_t a, uint32_t b) {
        const uint32_t x = find(a), y = find(b);
        if (x != y) parent[std::max(x, y)] = std::min(x, y);
    };
    int by_slot[kMaxLim];
    for (int j = 0; j < kMaxLim; ++j) by_slot[j] = -1;
    if (h->l_cluster_state == SG_CLUSTER_SERVER && h->ps_cluster) ps_cluster_unions(h, unite, by_slot);
    std::vector<uint32_t> gkey(R);
    bool groups = false;
    for (uint32_t k = 0; k < R; ++k) groups = (gkey[k] = find(k)) != k || groups;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipDeviceSynchronize());
    dfree(h->d_ps_gkey);
    if (groups) {
        if (hipMalloc(&h->d_ps_gkey, sizeof(uint32_t) * R) != hipSuccess) return fail(h, SG_E_NOMEM, "key groups");
        HIP_TRY(h, hipMemcpy(h->d_ps_gkey, gkey.data(), sizeof(uint32_t) * R, hipMemcpyHostToDevice));
    }
    h->ps_groups_stale = false;
    return SG_OK;
}

}  // namespace

int sg_pslot_load_rules(sg_handle* h, const sg_pslot_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                        uint32_t n_hot, uint32_t n_resources) {
    if (!h || (!rules && n)) return SG_E_INVAL;
    drain_async(h);
    std::vector<sg_param_rule> pr(n);
    std::vector<std::vector<uint32_t>> per(n_resources);
    std::vector<int32_t> grade(n), idx(n), zero(n, 0), cmode(n);
    std::vector<uint32_t> ckey(n);
    std::vector<std::pair<uint32_t, uint32_t>> cluster_refs;
    for (uint32_t i = 0; i < n; ++i) {
        if (rules[i].resource >= n_resources) return fail(h, SG_E_INVAL, "rule resource >= n_resources");
        if (rules[i].grade != 0 && rules[i].grade != 1) return fail(h, SG_E_INVAL, "grade must be THREAD or QPS");
        const int32_t cm = rules[i].cluster_mode;
        if (cm != SG_CLUSTER_MODE_OFF && cm != SG_CLUSTER_MODE_FALLBACK && cm != SG_CLUSTER_MODE_NO_FALLBACK &&
            cm != SG_CLUSTER_MODE_INVALID)
            return fail(h, SG_E_INVAL, "cluster_mode must be SG_CLUSTER_MODE_*");
        pr[i] = rules[i].rule;
        // ParamFlowRuleManager keeps the valid rules only (ParamFlowRuleUtil.isValidRule → checkCluster :54-66), per
        // resource in load order (getRulesOfResource)
        if (cm != SG_CLUSTER_MODE_INVALID) per[rules[i].resource].push_back(i);
        grade[i] = rules[i].grade;
        idx[i] = rules[i].param_idx;
        cmode[i] = cm;
        ckey[i] = rules[i].cluster_key;
        if ((cm == SG_CLUSTER_MODE_FALLBACK || cm == SG_CLUSTER_MODE_NO_FALLBACK) && rules[i].grade == 1)
            cluster_refs.emplace_back(rules[i].resource, rules[i].cluster_key);  // passCheck → passClusterCheck
    }
    if (!cluster_refs.empty() && h->l_cluster_state == SG_CLUSTER_CLIENT)
        return fail(h, SG_E_UNSUPPORTED, "cluster-mode param rules on a token client: the tokens come over the network, "
                                         "not in event order (INTEGRATION.md §8)");
    int rc = sg_param_load_rules(h, pr.data(), n, hot, n_hot);
    if (rc) return rc;
    std::vector<uint32_t> begin(n_resources + 1, 0), list;
    for (uint32_t r = 0; r < n_resources; ++r) {
        begin[r] = (uint32_t)list.size();
        list.insert(list.end(), per[r].begin(), per[r].end());
    }
    begin[n_resources] = (uint32_t)list.size();
    HIP_TRY(h, hipSetDevice(h->device));
    dfree(h->d_ps_begin);
    dfree(h->d_ps_rules);
    dfree(h->d_ps_grade);
    dfree(h->d_ps_idx);
    dfree(h->d_ps_init);
    dfree(h->d_ps_cmode);
    dfree(h->d_ps_ckey);
    const size_t n1 = n ? n : 1;
    if (hipMalloc(&h->d_ps_begin, sizeof(uint32_t) * (n_resources + 1)) != hipSuccess ||
        hipMalloc(&h->d_ps_rules, sizeof(uint32_t) * n1) != hipSuccess ||
        hipMalloc(&h->d_ps_grade, sizeof(int32_t) * n1) != hipSuccess ||
        hipMalloc(&h->d_ps_idx, sizeof(int32_t) * n1) != hipSuccess || hipMalloc(&h->d_ps_init, sizeof(int32_t) * n1) != hipSuccess ||
        hipMalloc(&h->d_ps_cmode, sizeof(int32_t) * n1) != hipSuccess || hipMalloc(&h->d_ps_ckey, sizeof(uint32_t) * n1) != hipSuccess)
        return fail(h, SG_E_NOMEM, "param slot rules");
    HIP_TRY(h, hipMemcpy(h->d_ps_begin, begin.data(), sizeof(uint32_t) * (n_resources + 1), hipMemcpyHostToDevice));
    if (!list.empty()) HIP_TRY(h, hipMemcpy(h->d_ps_rules, list.data(), sizeof(uint32_t) * list.size(), hipMemcpyHostToDevice));
    if (n) {
        HIP_TRY(h, hipMemcpy(h->d_ps_cmode, cmode.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_ps_ckey, ckey.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_ps_grade, grade.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_ps_idx, idx.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
        HIP_TRY(h, hipMemcpy(h->d_ps_init, zero.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
    }
    if (!h->d_ps_tc) {
        h->ps_tc_slots = 1ull << 20;
        if (hipMalloc(&h->d_ps_tc, sizeof(PSThread) * h->ps_tc_slots) != hipSuccess ||
            hipMalloc(&h->d_ps_last_ts, sizeof(int64_t)) != hipSuccess)
            return fail(h, SG_E_NOMEM, "thread count table");
    }
    HIP_TRY(h, launch_pslot_clear(h->d_ps_tc, h->ps_tc_slots, 0));
    const int64_t neg = -1;
    HIP_TRY(h, hipMemcpy(h->d_ps_last_ts, &neg, sizeof(neg), hipMemcpyHostToDevice));
    HIP_TRY(h, hipDeviceSynchronize());
    h->ps_nres = n_resources;
    h->ps_loaded = true;
    h->ps_cluster = !cluster_refs.empty();
    h->ps_cluster_refs = cluster_refs;
    h->ps_groups_stale = true;
    h->l_groups_stale = true;  // the slot chain's key groups include the cluster-mode param rules
    h->ps_res_rules.assign(n_resources, 0);
    for (uint32_t r = 0; r < n_resources; ++r) h->ps_res_rules[r] = (uint32_t)per[r].size();
    ++h->ps_gen;
    return SG_OK;
}

int sg_pslot_decide_batch(sg_handle* h, const sg_pslot_event* ev, uint64_t n, const sg_pslot_arg* args, uint64_t n_args,
                          const uint64_t* values, uint64_t n_values, sg_pslot_result* out, void* stream_) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!ev || !out) return fail(h, SG_E_INVAL, "null buffer");
    if (!h->ps_loaded) return fail(h, SG_E_INVAL, "sg_pslot_load_rules first");
    if (n > h->cfg.max_batch) return fail(h, SG_E_CAPACITY, "batch larger than max_batch");
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int kbits = bits_for((uint64_t)h->ps_nres);
    if (kbits < 1) kbits = 1;
    if (kbits + bits_for(h->cfg.max_batch) > 64) return fail(h, SG_E_UNSUPPORTED, "resources x max_batch too large");
    hipStream_t stream = (hipStream_t)stream_;
    int rc = pslot_apply_groups(h);
    if (rc) return rc;
    PSArgs s = pslot_args(h);
    rc = pslot_embed(h, s, stream);
    if (rc) return rc;
    s.gkey = s.emb ? h->d_ps_gkey : nullptr;
    s.ev = ev;
    s.args = args;
    s.n_args = n_args;
    s.values = values;
    s.n_values = n_values;
    s.out = out;
    s.n = n;
    s.rec = h->d_rec;
    s.kshift = 64 - kbits;
    s.imask = (1ull << s.kshift) - 1;
    HIP_TRY(h, hipMemsetAsync(h->d_err, 0, sizeof(int), stream));
    HIP_TRY(h, launch_pslot_batch(s, h->d_rec_sorted, h->d_hist, stream));
    HIP_TRY(h, hipMemcpyAsync(h->h_err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_TRY(h, hipStreamSynchronize(stream));
    if (*h->h_err & kErrTime)
        return fail(h, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than earlier batches");
    if (*h->h_err & kErrBounds) return fail(h, SG_E_INVAL, "an event's arguments lie outside the arg / value arrays");
    if (*h->h_err & kErrTableFull) return fail(h, SG_E_CAPACITY, "a param or thread-count table is full");
    return SG_OK;
}

int sg_pslot_decide_batch_host(sg_handle* h, const sg_pslot_event* ev, uint64_t n, const sg_pslot_arg* args,
                               uint64_t n_args, const uint64_t* values, uint64_t n_values, sg_pslot_result* out) {
    if (!h) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    sg_pslot_event* d_ev = nullptr;
    sg_pslot_arg* d_args = nullptr;
    uint64_t* d_vals = nullptr;
    sg_pslot_result* d_out = nullptr;
    hipError_t e = hipMalloc(&d_ev, sizeof(sg_pslot_event) * n);
    if (e == hipSuccess) e = hipMalloc(&d_args, sizeof(sg_pslot_arg) * (n_args ? n_args : 1));
    if (e == hipSuccess) e = hipMalloc(&d_vals, sizeof(uint64_t) * (n_values ? n_values : 1));
    if (e == hipSuccess) e = hipMalloc(&d_out, sizeof(sg_pslot_result) * n);
    if (e == hipSuccess) e = hipMemcpy(d_ev, ev, sizeof(sg_pslot_event) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && n_args) e = hipMemcpy(d_args, args, sizeof(sg_pslot_arg) * n_args, hipMemcpyHostToDevice);
    if (e == hipSuccess && n_values) e = hipMemcpy(d_vals, values, sizeof(uint64_t) * n_values, hipMemcpyHostToDevice);
    int rc = SG_E_DEVICE;
    if (e == hipSuccess) {
        rc = sg_pslot_decide_batch(h, d_ev, n, d_args, n_args, d_vals, n_values, d_out, nullptr);
        if (rc == SG_OK) e = hipMemcpy(out, d_out, sizeof(sg_pslot_result) * n, hipMemcpyDeviceToHost);
    }
    (void)hipFree(d_ev);
    (void)hipFree(d_args);
    (void)hipFree(d_vals);
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    return rc;
}

int sg_pslot_thread_count(sg_handle* h, uint32_t resource, int32_t param_idx, uint64_t value, int64_t* count) {
    if (!h || !count || !h->ps_loaded || resource >= h->ps_nres || param_idx < 0) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    int64_t* d = nullptr;
    HIP_TRY(h, hipMalloc(&d, sizeof(int64_t)));
    hipError_t e = launch_pslot_thread_read(pslot_args(h), resource, param_idx, value, d, 0);
    if (e == hipSuccess) e = hipMemcpy(count, d, sizeof(int64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(h, SG_E_DEVICE, hipGetErrorString(e));
    return SG_OK;
}

int sg_pslot_param_idx(sg_handle* h, uint32_t rule, int32_t* param_idx) {
    if (!h || !param_idx || !h->ps_loaded || rule >= h->ptab.size()) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    drain_async(h);
    HIP_TRY(h, hipMemcpy(param_idx, h->d_ps_idx + rule, sizeof(int32_t), hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_debug_copy(sg_handle* h, int what, void* dst, uint64_t bytes) {
    if (!h || !dst) return SG_E_INVAL;
    const void* src = nullptr;
    uint64_t cap = 0;
    switch (what) {
    case 0: src = (h->last_sorted == h->d_rec) ? h->d_rec_sorted : h->d_rec; cap = h->cfg.max_batch * 8; break;
    case 1: src = h->last_sorted ? h->last_sorted : h->d_rec_sorted; cap = h->cfg.max_batch * 8; break;
    case 2: src = h->d_bnd; cap = sizeof(uint32_t) * kMaxWl * kMaxPeriods; break;
    case 3: src = h->d_p0; cap = sizeof(int64_t) * kMaxWl; break;
    case 4: src = h->d_np; cap = sizeof(uint32_t) * kMaxWl; break;
    case 5: src = h->d_dbg; cap = 128 * 8; break;
    default: return SG_E_INVAL;
    }
    if (bytes > cap) return SG_E_INVAL;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return SG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------ node handle
//
// One token server over G shard handles (include/sentinel_gpu.h, sg_node_*): the reference's single TokenService
// (DefaultTokenService.java:39-50) serving every flowId, with the flowIds hashed over the shards (SURVEY §8(b)
// "multi-GPU fan-out is internal to the handle", §8(e)). A batch in caller order goes to the front handle (on the
// first shard's device: validation and the namespace limiter over the whole batch in caller order — the node's
// exact arrival order), then is split by owner (node.hip), decided by every shard concurrently on its own stream
// (peer copies for shards on other devices), and gathered back into caller order.

struct sg_node {
    std::string err;
    sg_config cfg{};
    std::vector<int32_t> devices;       // device of each shard
    sg_handle* front = nullptr;         // devices[0]: validation + namespace limiter over the node batch
    std::vector<sg_handle*> shards;
    std::vector<hipStream_t> streams;   // one per shard, on its device
    std::vector<hipEvent_t> done;       // per shard: its slice decided (and copied back)
    std::vector<int*> h_err;            // pinned, per shard
    hipStream_t s0 = nullptr;           // devices[0]
    hipEvent_t routed = nullptr;
    std::vector<sg_flow_rule> rules;
    std::vector<uint8_t> shard_of;
    std::vector<uint32_t> local_of;
    uint8_t* d_shard_of = nullptr;
    uint32_t* d_local_of = nullptr;
    uint32_t* d_tile_cnt = nullptr;
    uint32_t* d_base = nullptr;         // [kMaxShards + 1] bases, then [kMaxShards] totals
    uint32_t* h_base = nullptr;         // pinned copy
    int* h_front_err = nullptr;         // pinned
    sg_req* d_sub_req = nullptr;
    uint32_t* d_sub_pos = nullptr;
    sg_result* d_sub_out = nullptr;
    std::vector<sg_req*> r_req;         // per shard on another device: its slice there
    std::vector<sg_result*> r_out;
    sg_req* d_req_h = nullptr;          // host path
    sg_result* d_out_h = nullptr;
    // every shard on the front's device with the front's request-index / acquire layout: the records path (the
    // shards start at the sort, on the front's period tables, and write the caller's results in place)
    bool rec_path = false;
    uint64_t* d_sub_rec = nullptr;      // [max_batch] the shards' record slices
    std::vector<sg_namespace> ns;       // the node's namespaces (rollback of a failed sg_node_set_namespaces)
    // pipelined node batches (sg_node_flow_enqueue, records path): two workspaces alternating, as the single
    // handle's pipeline — the front's k_prep / limiter / routing of batch i+1 and the shards' sorts beside the
    // shards' walkers of batch i
    struct PipeSlot {
        uint64_t ticket = 0;
        hipEvent_t done = nullptr;   // every shard's back half of the slot's batch (recorded on s0)
        int* h_err = nullptr;        // pinned [kMaxShards]: each shard's error word
        uint32_t* h_base = nullptr;  // pinned [2 * kMaxShards + 1]: slice bases and counts
        uint32_t G_used = 0;         // shards the batch went to
    };
    PipeSlot pipe[2];
    hipEvent_t fdone[2] = {nullptr, nullptr};  // the front's part of the slot's batch
    uint64_t* d_sub_rec2 = nullptr;            // workspace 1's record slices
    uint64_t pseq = 0, next_ticket = 1;
    std::unordered_map<uint64_t, int> finished;  // tickets completed while making room, not yet collected
    // cluster param and concurrent tokens over the node (sg_node_cparam_*, sg_node_conc_*): a param rule lives on the
    // shard owning its flowId; a concurrent token on the shard owning its flow rule's flowId
    std::vector<sg_cparam_rule> cp_rules;
    std::vector<uint8_t> cp_shard_of;
    std::vector<uint32_t> cp_local_of;
    uint8_t* d_cp_shard_of = nullptr;
    uint32_t* d_cp_local_of = nullptr;
    uint64_t* d_nrec = nullptr;        // [max_batch] owner records, then the sort's other buffer
    uint64_t* d_nrec2 = nullptr;
    uint32_t* d_nhist = nullptr;
    uint32_t* d_nvals = nullptr;       // [max_batch]
    uint32_t* d_ncnt = nullptr;        // [3 * kMaxShards]: requests, values, value bases per shard
    uint32_t* d_ntsum = nullptr;       // [tiles]
    int* d_nerr = nullptr;
    void* d_sub_nreq = nullptr;        // [max_batch] slices (sg_cparam_req / sg_conc_req: 24 B / 32 B each)
    void* d_sub_nout = nullptr;        // [max_batch] slice results (sg_result / sg_conc_result)
    uint64_t* d_sub_vals = nullptr;    // the param slices' values
    uint64_t sub_vals_cap = 0;
    std::vector<void*> r_nreq, r_nout; // shards on other devices: their slices there
    std::vector<uint64_t*> r_vals;
    std::vector<uint64_t> r_vals_cap;
    int64_t cp_last_ts = -1, cc_last_ts = -1;  // the node's previous param / concurrent batch (time order)
    // host-path staging
    void* d_nreq_h = nullptr;
    void* d_nout_h = nullptr;
    uint64_t* d_nvals_h = nullptr;
    uint64_t nvals_h_cap = 0;
    // node snapshot on the device: each shard's part gathered into the front's buffer in node rule order
    std::vector<uint32_t*> d_node_key;  // per shard (on the front's device): node rule of each local rule
    double* d_snap = nullptr;
    uint64_t snap_cap = 0;
    bool node_key_stale = true;         // the flow rules changed since d_node_key was built
    std::vector<double*> r_snap;        // per shard on another device: its part there
};

namespace {

int nfail(sg_node* nd, int code, const std::string& msg) {
    if (nd) nd->err = msg;
    return code;
}

#define NHIP(nd, expr)                                                                          \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return nfail((nd), SG_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e));   \
    } while (0)

// splitmix64(flowId) mod G: the owner shard (sentinel_amd/cluster.py shard_of)
uint32_t node_owner(int64_t flow_id, uint32_t G) {
    uint64_t z = (uint64_t)flow_id + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z % G);
}

// A shard's error, in the node's words.
int node_child(sg_node* nd, sg_handle* h, int rc) {
    if (rc < 0) nd->err = h->err;
    return rc;
}

// The shards' rules indexed into the front's window-length table (a superset: the front holds every node rule, and the
// limiter's 100 ms), so that a shard walks the node batch's period tables as the front's k_prep built them; and
// whether the records path applies (every shard on the front's device, the same record layout below the key).
int node_sync_layout(sg_node* nd) {
    sg_handle* f = nd->front;
    int rc = ensure_layout(f);
    if (rc) return node_child(nd, f, rc);
    bool same = true;
    for (size_t g = 0; g < nd->shards.size(); ++g) {
        sg_handle* h = nd->shards[g];
        rc = ensure_layout(h);
        if (rc) return node_child(nd, h, rc);
        same = same && nd->devices[g] == nd->devices[0] && h->ibits == f->ibits && h->abits == f->abits;
        if (!h->K) continue;
        for (uint32_t k = 0; k < h->K; ++k) {
            Rule& R = h->rule_tab[k];
            int w = 0;
            while (w < f->n_wl && f->wl[w] != R.wl) ++w;
            if (w == f->n_wl) return nfail(nd, SG_E_DEVICE, "a shard window length missing at the front");
            R.wl_idx = w;
        }
        h->n_wl = f->n_wl;
        std::memcpy(h->wl, f->wl, sizeof(h->wl));
        NHIP(nd, hipSetDevice(h->device));
        NHIP(nd, hipMemcpy(h->d_rules, h->rule_tab.data(), sizeof(Rule) * h->K, hipMemcpyHostToDevice));
    }
    nd->rec_path = same && std::getenv("SG_NODE_LEGACY") == nullptr;
    if (nd->rec_path && !nd->d_sub_rec) {
        NHIP(nd, hipSetDevice(nd->devices[0]));
        if (hipMalloc(&nd->d_sub_rec, sizeof(uint64_t) * (nd->cfg.max_batch + kRecW)) != hipSuccess)
            return nfail(nd, SG_E_NOMEM, "shard record slices");
    }
    return SG_OK;
}

// The walker CUs of shard g: its device's share when several shards of the node live on one device (each shard's
// persistent walker grids were sized for the whole CU set, and G of them contended for it: round 5's G = 4 step took
// 5x one handle's). `cus` is the CU set the walkers' streams may use (0: the whole device).
int node_walk_cus(const sg_node* nd, uint32_t g, int cus) {
    int same = 0;
    for (int32_t d : nd->devices) same += d == nd->devices[g] ? 1 : 0;
    if (same <= 1) return cus;
    if (cus <= 0) {
        int all = 0;
        (void)hipDeviceGetAttribute(&all, hipDeviceAttributeMultiprocessorCount, nd->devices[g]);
        cus = all > 0 ? all : 256;
    }
    return std::max(1, cus / same);
}

// Waits for the shard streams [0, g) (an early return must not leave slices in flight).
void node_sync_shards(sg_node* nd, uint32_t g) {
    for (uint32_t x = 0; x < g && x < nd->streams.size(); ++x) {
        (void)hipSetDevice(nd->devices[x]);
        (void)hipStreamSynchronize(nd->streams[x]);
    }
    (void)hipSetDevice(nd->devices[0]);
}

// One shard's slice of a node batch on the records path: the sort of its records (node request indices), its
// segments, both walkers and the skipped BLOCK counts, its error word into err_dst. `front` carries the sort and
// segments, `back` the walkers (the same stream for a synchronous node batch); front_done (may be null) joins them.
int node_shard_rec(sg_handle* h, BatchArgs b, uint64_t cnt, uint32_t* hist, hipStream_t front, hipStream_t back,
                   hipStream_t aux, hipEvent_t fork, hipEvent_t join, hipEvent_t front_done, int* err_dst) {
    HIP_TRY(h, hipMemsetAsync(b.err, 0, sizeof(int), front));
    HIP_TRY(h, hipMemsetAsync(b.long_count, 0, (1 + kClasses) * sizeof(uint32_t), front));
    HIP_TRY(h, hipMemsetAsync(b.skip_count, 0, sizeof(uint32_t), front));
    uint64_t* sorted = nullptr;
    const SegMark mk{b.seg_start, b.seg_end, b.K, b.kshift};
    b.seg_marked = (b.seg_start && b.seg_end && b.long_end && !h->seg_mark_pass) ? 1 : 0;
    HIP_TRY(h, radix_sort_records(b.rec, b.rec_sorted, cnt, b.kshift, hist, &sorted, front, 64, b.hist0 != nullptr,
                                  b.seg_marked ? &mk : nullptr, b.csum0 != nullptr));
    b.rec_sorted = sorted;
    HIP_TRY(h, launch_seg_flow(b, front));
    if (front_done) {
        HIP_TRY(h, hipEventRecord(front_done, front));
        HIP_TRY(h, hipStreamWaitEvent(back, front_done, 0));
    }
    HIP_TRY(h, hipEventRecord(fork, back));
    HIP_TRY(h, hipStreamWaitEvent(aux, fork, 0));
    HIP_TRY(h, launch_walk_long(b, aux));
    HIP_TRY(h, launch_walk_short(b, back));
    HIP_TRY(h, launch_walk_tiny(b, back));
    HIP_TRY(h, hipEventRecord(join, aux));
    HIP_TRY(h, hipStreamWaitEvent(back, join, 0));
    HIP_TRY(h, launch_skip_apply(b, back));
    HIP_TRY(h, hipMemcpyAsync(err_dst, b.err, sizeof(int), hipMemcpyDeviceToHost, back));
    return SG_OK;
}

// A completed pipelined node batch's status: the first shard error (the front's was answered at enqueue).
int node_slot_status(sg_node* nd, const sg_node::PipeSlot& sl) {
    for (uint32_t g = 0; g < sl.G_used; ++g)
        if (sl.h_err[g]) return node_child(nd, nd->shards[g], flow_status(nd->shards[g], sl.h_err[g]));
    return SG_OK;
}

// Completes the node's pipelined batches (their statuses wait for sg_node_flow_poll / _wait): every other node call
// starts from a drained node, and the synchronous path uses workspace 0.
int node_drain(sg_node* nd) {
    for (auto& sl : nd->pipe) {
        if (!sl.ticket) continue;
        (void)hipSetDevice(nd->devices[0]);
        const hipError_t e = hipEventSynchronize(sl.done);
        nd->finished[sl.ticket] = e != hipSuccess ? nfail(nd, SG_E_DEVICE, hipGetErrorString(e)) : node_slot_status(nd, sl);
        sl.ticket = 0;
    }
    for (sg_handle* h : nd->shards) drain_async(h);
    if (nd->front) drain_async(nd->front);
    if (!nd->devices.empty()) (void)hipSetDevice(nd->devices[0]);
    return SG_OK;
}

}  // namespace

extern "C" {

void sg_node_destroy(sg_node* nd) {
    if (!nd) return;
    node_drain(nd);
    for (size_t g = 0; g < nd->shards.size(); ++g) {
        (void)hipSetDevice(nd->devices[g]);
        if (g < nd->streams.size() && nd->streams[g]) (void)hipStreamDestroy(nd->streams[g]);
        if (g < nd->done.size() && nd->done[g]) (void)hipEventDestroy(nd->done[g]);
        if (g < nd->h_err.size() && nd->h_err[g]) (void)hipHostFree(nd->h_err[g]);
        if (g < nd->r_req.size()) dfree(nd->r_req[g]);
        if (g < nd->r_out.size()) dfree(nd->r_out[g]);
        sg_destroy(nd->shards[g]);
    }
    if (!nd->devices.empty()) (void)hipSetDevice(nd->devices[0]);
    if (nd->s0) (void)hipStreamDestroy(nd->s0);
    if (nd->routed) (void)hipEventDestroy(nd->routed);
    dfree(nd->d_shard_of);
    dfree(nd->d_local_of);
    dfree(nd->d_tile_cnt);
    dfree(nd->d_base);
    dfree(nd->d_sub_req);
    dfree(nd->d_sub_pos);
    dfree(nd->d_sub_out);
    dfree(nd->d_req_h);
    dfree(nd->d_out_h);
    dfree(nd->d_sub_rec);
    dfree(nd->d_sub_rec2);
    dfree(nd->d_cp_shard_of);
    dfree(nd->d_cp_local_of);
    dfree(nd->d_nrec);
    dfree(nd->d_nrec2);
    dfree(nd->d_nhist);
    dfree(nd->d_nvals);
    dfree(nd->d_ncnt);
    dfree(nd->d_ntsum);
    dfree(nd->d_nerr);
    dfree(nd->d_sub_nreq);
    dfree(nd->d_sub_nout);
    dfree(nd->d_sub_vals);
    dfree(nd->d_nreq_h);
    dfree(nd->d_nout_h);
    dfree(nd->d_nvals_h);
    dfree(nd->d_snap);
    for (uint32_t* p : nd->d_node_key) dfree(p);
    for (size_t g = 0; g < nd->r_nreq.size(); ++g) {
        (void)hipSetDevice(nd->devices[g]);
        dfree(nd->r_nreq[g]);
        dfree(nd->r_nout[g]);
        dfree(nd->r_vals[g]);
        if (g < nd->r_snap.size()) dfree(nd->r_snap[g]);
    }
    (void)hipSetDevice(nd->devices.empty() ? 0 : nd->devices[0]);
    for (auto& sl : nd->pipe) {
        if (sl.done) (void)hipEventDestroy(sl.done);
        if (sl.h_err) (void)hipHostFree(sl.h_err);
        if (sl.h_base) (void)hipHostFree(sl.h_base);
    }
    for (hipEvent_t e : nd->fdone)
        if (e) (void)hipEventDestroy(e);
    if (nd->h_base) (void)hipHostFree(nd->h_base);
    if (nd->h_front_err) (void)hipHostFree(nd->h_front_err);
    sg_destroy(nd->front);
    delete nd;
}

const char* sg_node_last_error(const sg_node* nd) { return nd ? nd->err.c_str() : "null node"; }

int sg_node_create(const sg_config* cfg, const int32_t* devices, uint32_t n_shards, sg_node** out) {
    if (!cfg || !devices || !out || n_shards == 0 || n_shards > (uint32_t)kMaxShards) return SG_E_INVAL;
    *out = nullptr;
    sg_node* nd = new sg_node();
    nd->cfg = *cfg;
    nd->devices.assign(devices, devices + n_shards);
    auto bail = [&](int rc) {
        sg_node_destroy(nd);
        return rc;
    };
    sg_config c = *cfg;
    c.device = devices[0];
    int rc = sg_create(&c, &nd->front);
    if (rc) return bail(rc);
    nd->front->front_only = true;
    for (uint32_t g = 0; g < n_shards; ++g) {
        c.device = devices[g];
        sg_handle* h = nullptr;
        rc = sg_create(&c, &h);
        if (rc) return bail(rc);
        nd->shards.push_back(h);
        if (hipSetDevice(devices[g]) != hipSuccess) return bail(SG_E_DEVICE);
        hipStream_t st = nullptr;
        hipEvent_t ev = nullptr;
        int* he = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(&he, sizeof(int)) != hipSuccess)
            return bail(SG_E_DEVICE);
        nd->streams.push_back(st);
        nd->done.push_back(ev);
        nd->h_err.push_back(he);
        sg_req* rq = nullptr;
        sg_result* ro = nullptr;
        if (devices[g] != devices[0] &&
            (hipMalloc(&rq, sizeof(sg_req) * cfg->max_batch) != hipSuccess ||
             hipMalloc(&ro, sizeof(sg_result) * cfg->max_batch) != hipSuccess))
            return bail(SG_E_NOMEM);
        nd->r_req.push_back(rq);
        nd->r_out.push_back(ro);
    }
    // shards on other devices: peer access both ways (their slices and results cross xGMI as peer copies)
    for (uint32_t g = 1; g < n_shards; ++g) {
        const int d0 = devices[0], dg = devices[g];
        if (dg == d0) continue;
        int can0 = 0, can1 = 0;
        (void)hipDeviceCanAccessPeer(&can0, d0, dg);
        (void)hipDeviceCanAccessPeer(&can1, dg, d0);
        if (can0) {
            (void)hipSetDevice(d0);
            const hipError_t e = hipDeviceEnablePeerAccess(dg, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return bail(SG_E_DEVICE);
        }
        if (can1) {
            (void)hipSetDevice(dg);
            const hipError_t e = hipDeviceEnablePeerAccess(d0, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return bail(SG_E_DEVICE);
        }
        (void)hipGetLastError();  // an already-enabled peer leaves its error behind
    }
    if (hipSetDevice(devices[0]) != hipSuccess) return bail(SG_E_DEVICE);
    nd->r_nreq.assign(n_shards, nullptr);
    nd->r_nout.assign(n_shards, nullptr);
    nd->r_vals.assign(n_shards, nullptr);
    nd->r_vals_cap.assign(n_shards, 0);
    nd->r_snap.assign(n_shards, nullptr);
    const uint64_t n = cfg->max_batch;
    if (hipStreamCreateWithFlags(&nd->s0, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&nd->routed, hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&nd->d_tile_cnt, sizeof(uint32_t) * kMaxShards * (route_tiles(n) + 1)) != hipSuccess ||
        hipMalloc(&nd->d_base, sizeof(uint32_t) * (2 * kMaxShards + 1)) != hipSuccess ||
        hipMalloc(&nd->d_sub_req, sizeof(sg_req) * n) != hipSuccess ||
        hipMalloc(&nd->d_sub_pos, sizeof(uint32_t) * n) != hipSuccess ||
        hipMalloc(&nd->d_sub_out, sizeof(sg_result) * n) != hipSuccess ||
        hipHostMalloc(&nd->h_base, sizeof(uint32_t) * (2 * kMaxShards + 1)) != hipSuccess ||
        hipHostMalloc(&nd->h_front_err, sizeof(int)) != hipSuccess)
        return bail(SG_E_NOMEM);
    *out = nd;
    return SG_OK;
}

int sg_node_set_namespaces(sg_node* nd, const sg_namespace* ns, uint32_t n) {
    if (!nd || (!ns && n)) return SG_E_INVAL;
    node_drain(nd);
    // the front runs every namespace limiter over the node batch (and validates the set); the shards see only admitted
    // requests. A shard that fails (allocation, device) puts the front and the shards before it back on the node's
    // previous namespaces.
    const std::vector<sg_namespace> old = nd->ns;
    auto limiters_off = [](std::vector<sg_namespace> v) {
        for (auto& x : v) x.limiter_enabled = 0;
        return v;
    };
    int rc = sg_set_namespaces(nd->front, ns, n);
    if (rc) return node_child(nd, nd->front, rc);
    const std::vector<sg_namespace> off = limiters_off(std::vector<sg_namespace>(ns, ns + n));
    for (size_t g = 0; g < nd->shards.size(); ++g) {
        rc = sg_set_namespaces(nd->shards[g], off.data(), n);
        if (rc) {
            rc = node_child(nd, nd->shards[g], rc);
            const std::vector<sg_namespace> old_off = limiters_off(old);
            (void)sg_set_namespaces(nd->front, old.data(), (uint32_t)old.size());
            for (size_t x = 0; x < g; ++x) (void)sg_set_namespaces(nd->shards[x], old_off.data(), (uint32_t)old_off.size());
            (void)node_sync_layout(nd);
            return rc;
        }
    }
    nd->ns.assign(ns, ns + n);
    return node_sync_layout(nd);
}

int sg_node_load_flow_rules(sg_node* nd, const sg_flow_rule* rules, uint32_t n) {
    if (!nd || (!rules && n)) return SG_E_INVAL;
    node_drain(nd);
    // All or nothing: the node's rule set is validated on the front, every shard's part and the front's whole set are
    // prepared beside the live state (surviving flowIds' metrics copied: a surviving flowId keeps its owner, hence its
    // ClusterMetric) together with the routing tables, and only when all of that succeeded is anything committed. A
    // failure (validation, allocation, device) leaves the node deciding with its previous rules.
    sg_handle* f = nd->front;
    NHIP(nd, hipSetDevice(nd->devices[0]));
    drain_async(f);
    int rc = flow_rules_validate(f, rules, n);
    if (rc) return node_child(nd, f, rc);
    const uint32_t G = (uint32_t)nd->shards.size();
    std::vector<std::vector<sg_flow_rule>> part(G);
    std::vector<uint8_t> so(n);
    std::vector<uint32_t> lo(n);
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t g = node_owner(rules[k].flow_id, G);
        so[k] = (uint8_t)g;
        lo[k] = (uint32_t)part[g].size();
        part[g].push_back(rules[k]);
    }
    std::vector<FlowLoad> prep(G + 1);
    uint8_t* d_so = nullptr;
    uint32_t* d_lo = nullptr;
    auto abort_all = [&](uint32_t upto) {  // the prepared shards [0, upto), the front's (index G) and the tables
        for (uint32_t x = 0; x < upto; ++x) {
            (void)hipSetDevice(nd->devices[x]);
            flow_rules_abort(prep[x]);
        }
        (void)hipSetDevice(nd->devices[0]);
        flow_rules_abort(prep[G]);
        dfree(d_so);
        dfree(d_lo);
    };
    // env SG_TEST_NODE_FAIL_SHARD = g (tests): preparing shard g fails as an allocation would
    const char* inj = std::getenv("SG_TEST_NODE_FAIL_SHARD");
    const int fail_g = inj ? std::atoi(inj) : -1;
    for (uint32_t g = 0; g < G; ++g) {
        sg_handle* h = nd->shards[g];
        NHIP(nd, hipSetDevice(h->device));
        drain_async(h);
        rc = (int)g == fail_g ? fail(h, SG_E_NOMEM, "injected shard load failure (SG_TEST_NODE_FAIL_SHARD)")
                              : flow_rules_validate(h, part[g].data(), (uint32_t)part[g].size());
        if (!rc) rc = flow_rules_prepare(h, part[g].data(), (uint32_t)part[g].size(), prep[g]);
        if (rc) {
            rc = node_child(nd, h, rc);
            abort_all(g);
            return rc;
        }
    }
    NHIP(nd, hipSetDevice(nd->devices[0]));
    rc = flow_rules_prepare(f, rules, n, prep[G]);
    if (!rc && n && (hipMalloc(&d_so, n) != hipSuccess || hipMalloc(&d_lo, sizeof(uint32_t) * n) != hipSuccess ||
                     hipMemcpy(d_so, so.data(), n, hipMemcpyHostToDevice) != hipSuccess ||
                     hipMemcpy(d_lo, lo.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess))
        rc = fail(f, SG_E_NOMEM, "routing tables");
    if (rc) {
        rc = node_child(nd, f, rc);
        abort_all(G);
        return rc;
    }
    // commit (host tables and pointer swaps; only the small per-rule uploads can still fail)
    for (uint32_t g = 0; g < G; ++g) {
        NHIP(nd, hipSetDevice(nd->devices[g]));
        rc = flow_rules_commit(nd->shards[g], part[g].data(), (uint32_t)part[g].size(), prep[g]);
        if (rc) return node_child(nd, nd->shards[g], rc);
    }
    NHIP(nd, hipSetDevice(nd->devices[0]));
    rc = flow_rules_commit(f, rules, n, prep[G]);
    if (rc) return node_child(nd, f, rc);
    dfree(nd->d_shard_of);
    dfree(nd->d_local_of);
    nd->d_shard_of = d_so;
    nd->d_local_of = d_lo;
    nd->rules.assign(rules, rules + n);
    nd->shard_of = so;
    nd->local_of = lo;
    nd->node_key_stale = true;
    return node_sync_layout(nd);
}

sg_handle* sg_node_front(sg_node* nd) { return nd ? nd->front : nullptr; }

int sg_node_shard_of(const sg_node* nd, uint32_t key, uint32_t* shard, uint32_t* local_key) {
    if (!nd || !shard || !local_key || key >= nd->shard_of.size()) return SG_E_INVAL;
    *shard = nd->shard_of[key];
    *local_key = nd->local_of[key];
    return SG_OK;
}

int sg_node_flow_decide_batch(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out, void* stream_) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    sg_handle* f = nd->front;
    const uint32_t G = (uint32_t)nd->shards.size();
    hipStream_t user = (hipStream_t)stream_;
    NHIP(nd, hipSetDevice(nd->devices[0]));
    node_drain(nd);
    int rc = ensure_layout(f);
    if (rc) return node_child(nd, f, rc);
    // 1. the front: validation + namespace limiter in caller order, the batch's time check, its last timestamp, the
    // default results in the caller's buffer, the batch's period tables
    NHIP(nd, hipStreamSynchronize(user));  // the caller's batch is in place
    sg_handle::FlowWs w;
    main_ws(f, w);
    BatchArgs a = flow_args(f, w, req, n, out);
    // one shard holding every rule in the front's order (G = 1): the front's records are its records as they are
    const bool direct = nd->rec_path && G == 1 && nd->shards[0]->K == f->K && nd->shards[0]->kbits == f->kbits;
    if (!direct) a.hist0 = nullptr;
    a.csum0 = nullptr;
    NHIP(nd, hipMemsetAsync(a.err, 0, sizeof(int), nd->s0));
    if (a.hist0 && radix_csum_atomic()) {
        a.csum0 = radix_csum(a.hist0, a.n, a.hist0_bits);
        NHIP(nd, hipMemsetAsync(a.csum0, 0, radix_csum_bytes(a.n, a.hist0_bits), nd->s0));
    }
    NHIP(nd, launch_prep(a, nd->s0));
    rc = flow_limiter(f, a, nd->s0);
    if (rc) return node_child(nd, f, rc);
    NHIP(nd, launch_finish(a, nd->s0));
    // 2. routing by owner (not for one shard on the records path)
    RouteArgs r{};
    r.req = req;
    r.rec = a.rec;
    r.n = n;
    r.kshift = a.kshift;
    r.abits = a.abits;
    r.imask = a.imask;
    r.K = f->K;
    r.shard_of = nd->d_shard_of;
    r.local_of = nd->d_local_of;
    r.G = (int)G;
    r.tile_cnt = nd->d_tile_cnt;
    r.shard_base = nd->d_base;
    r.shard_tot = nd->d_base + kMaxShards + 1;
    r.sub_req = nd->d_sub_req;
    r.sub_pos = nd->d_sub_pos;
    if (nd->rec_path) {
        r.sub_rec = nd->d_sub_rec;
        r.low_mask = (1ull << a.kshift) - 1;
        for (uint32_t g = 0; g < G; ++g) r.skshift[g] = 64 - nd->shards[g]->kbits;
    }
    if (!direct) {
        NHIP(nd, launch_route(r, nd->s0));
        NHIP(nd, hipMemcpyAsync(nd->h_base, nd->d_base, sizeof(uint32_t) * (2 * kMaxShards + 1), hipMemcpyDeviceToHost,
                                nd->s0));
    }
    NHIP(nd, hipMemcpyAsync(nd->h_front_err, a.err, sizeof(int), hipMemcpyDeviceToHost, nd->s0));
    NHIP(nd, hipEventRecord(nd->routed, nd->s0));
    NHIP(nd, hipStreamSynchronize(nd->s0));
    if (*nd->h_front_err) return node_child(nd, f, flow_status(f, *nd->h_front_err));
    if (direct) {
        nd->h_base[0] = 0;
        nd->h_base[kMaxShards + 1] = (uint32_t)n;  // the sentinel records of rejected requests sort to the end
    }
    // 3. every shard decides its slice on its own stream
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t base = nd->h_base[g], cnt = nd->h_base[kMaxShards + 1 + g];
        *nd->h_err[g] = 0;
        if (cnt == 0) continue;
        sg_handle* h = nd->shards[g];
        const int dev = nd->devices[g];
        NHIP(nd, hipSetDevice(dev));
        NHIP(nd, hipStreamWaitEvent(nd->streams[g], nd->routed, 0));
        if (nd->rec_path) {
            // the slice's records (node request indices) through the shard's sort and walkers; the period tables,
            // window lengths, requests and results are the node batch's
            sg_handle::FlowWs sw;
            main_ws(h, sw);
            BatchArgs b = flow_args(h, sw, req, cnt, out);
            b.rec = direct ? a.rec : nd->d_sub_rec + base;
            b.rec_sorted = direct ? h->d_rec_sorted : sw.rec;  // the sort's other buffer
            b.hist0 = direct ? a.hist0 : nullptr;
            b.hist0_bits = a.hist0_bits;
            b.csum0 = direct ? a.csum0 : nullptr;
            b.n_wl = a.n_wl;
            std::memcpy(b.wl, a.wl, sizeof(b.wl));
            b.bnd = a.bnd;
            b.p0 = a.p0;
            b.np = a.np;
            b.walk_cus = node_walk_cus(nd, g, 0);
            hipStream_t st = nd->streams[g];
            rc = node_shard_rec(h, b, cnt, direct ? w.hist : sw.hist, st, st, h->aux, h->fork, h->join, nullptr,
                                nd->h_err[g]);
            if (rc) {
                node_sync_shards(nd, g + 1);
                return node_child(nd, h, rc);
            }
        } else {
            const sg_req* sreq = nd->d_sub_req + base;
            sg_result* sout = nd->d_sub_out + base;
            if (dev != nd->devices[0]) {
                NHIP(nd, hipMemcpyPeerAsync(nd->r_req[g], dev, sreq, nd->devices[0], sizeof(sg_req) * cnt, nd->streams[g]));
                sreq = nd->r_req[g];
                sout = nd->r_out[g];
            }
            rc = enqueue_flow(h, sreq, cnt, sout, nd->streams[g], nd->h_err[g], false);
            if (rc) {
                node_sync_shards(nd, g + 1);
                return node_child(nd, h, rc);
            }
            if (dev != nd->devices[0])
                NHIP(nd, hipMemcpyPeerAsync(nd->d_sub_out + base, nd->devices[0], sout, dev, sizeof(sg_result) * cnt,
                                            nd->streams[g]));
        }
        NHIP(nd, hipEventRecord(nd->done[g], nd->streams[g]));
    }
    // 4. back into caller order (the sub_req path; the records path wrote the results in place)
    NHIP(nd, hipSetDevice(nd->devices[0]));
    for (uint32_t g = 0; g < G; ++g)
        if (nd->h_base[kMaxShards + 1 + g]) NHIP(nd, hipStreamWaitEvent(nd->s0, nd->done[g], 0));
    if (!nd->rec_path) NHIP(nd, launch_route_gather(nd->d_sub_out, nd->d_sub_pos, nd->h_base[G], out, nd->s0));
    NHIP(nd, hipEventRecord(nd->routed, nd->s0));
    NHIP(nd, hipStreamWaitEvent(user, nd->routed, 0));
    NHIP(nd, hipStreamSynchronize(nd->s0));
    for (uint32_t g = 0; g < G; ++g) {
        const int e = *nd->h_err[g];
        if (e) return node_child(nd, nd->shards[g], flow_status(nd->shards[g], e));
    }
    return SG_OK;
}

int sg_node_flow_decide_batch_host(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    NHIP(nd, hipSetDevice(nd->devices[0]));
    if (!nd->d_req_h && (hipMalloc(&nd->d_req_h, sizeof(sg_req) * nd->cfg.max_batch) != hipSuccess ||
                         hipMalloc(&nd->d_out_h, sizeof(sg_result) * nd->cfg.max_batch) != hipSuccess))
        return nfail(nd, SG_E_NOMEM, "host-path buffers");
    NHIP(nd, hipMemcpy(nd->d_req_h, req, sizeof(sg_req) * n, hipMemcpyHostToDevice));
    const int rc = sg_node_flow_decide_batch(nd, nd->d_req_h, n, nd->d_out_h, nullptr);
    if (rc) return rc;
    NHIP(nd, hipMemcpy(out, nd->d_out_h, sizeof(sg_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_node_flow_enqueue(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket) {
    if (!nd || !ticket) return SG_E_INVAL;
    *ticket = 0;
    if (n == 0) return SG_OK;
    if (!req || !out) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    sg_handle* f = nd->front;
    const uint32_t G = (uint32_t)nd->shards.size();
    NHIP(nd, hipSetDevice(nd->devices[0]));
    int rc = ensure_layout(f);
    if (rc) return node_child(nd, f, rc);
    if (!nd->rec_path) {  // shards on other devices: the synchronous node batch, its status kept for the ticket
        rc = sg_node_flow_decide_batch(nd, req, n, out, nullptr);
        if (rc == SG_E_DEVICE) return rc;
        *ticket = nd->next_ticket++;
        nd->finished[*ticket] = rc;
        return SG_OK;
    }
    rc = pipe_setup(f);
    if (rc) return node_child(nd, f, rc);
    for (sg_handle* h : nd->shards) {
        rc = pipe_setup(h);
        if (rc) return node_child(nd, h, rc);
    }
    const int x = (int)(nd->pseq & 1);
    sg_node::PipeSlot& sl = nd->pipe[x];
    if (!sl.done) {
        if (hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&nd->fdone[x], hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(&sl.h_err, sizeof(int) * kMaxShards) != hipSuccess ||
            hipHostMalloc(&sl.h_base, sizeof(uint32_t) * (2 * kMaxShards + 1)) != hipSuccess)
            return nfail(nd, SG_E_NOMEM, "node pipeline slot");
    }
    if (x == 1 && !nd->d_sub_rec2 && hipMalloc(&nd->d_sub_rec2, sizeof(uint64_t) * (nd->cfg.max_batch + kRecW)) != hipSuccess)
        return nfail(nd, SG_E_NOMEM, "shard record slices");
    if (sl.ticket) {  // the batch two back used this workspace: complete it (its status waits in `finished`)
        const hipError_t e = hipEventSynchronize(sl.done);
        nd->finished[sl.ticket] = e != hipSuccess ? nfail(nd, SG_E_DEVICE, hipGetErrorString(e)) : node_slot_status(nd, sl);
        sl.ticket = 0;
    }
    // 1. the front on its pipeline stream: validation, the namespace limiter in caller order, the time check against
    // the previous node batch (the front's own last timestamp, in stream order), the period tables, the routing
    sg_handle::FlowWs w = f->pws;
    if (x == 0) main_ws(f, w);
    BatchArgs a = flow_args(f, w, req, n, out);
    const bool direct = G == 1 && nd->shards[0]->K == f->K && nd->shards[0]->kbits == f->kbits;
    if (!direct) a.hist0 = nullptr;
    a.csum0 = nullptr;
    hipStream_t fs = f->s_front;
    if (nd->pseq >= 2) NHIP(nd, hipStreamWaitEvent(fs, sl.done, 0));
    NHIP(nd, hipMemsetAsync(a.err, 0, sizeof(int), fs));
    if (a.hist0 && radix_csum_atomic()) {
        a.csum0 = radix_csum(a.hist0, a.n, a.hist0_bits);
        NHIP(nd, hipMemsetAsync(a.csum0, 0, radix_csum_bytes(a.n, a.hist0_bits), fs));
    }
    NHIP(nd, launch_prep(a, fs));
    rc = flow_limiter(f, a, fs);
    if (rc) return node_child(nd, f, rc);
    NHIP(nd, launch_finish(a, fs));
    uint64_t* sub_rec = x == 0 ? nd->d_sub_rec : nd->d_sub_rec2;
    if (!direct) {
        RouteArgs r{};
        r.req = req;
        r.rec = a.rec;
        r.n = n;
        r.kshift = a.kshift;
        r.abits = a.abits;
        r.imask = a.imask;
        r.K = f->K;
        r.shard_of = nd->d_shard_of;
        r.local_of = nd->d_local_of;
        r.G = (int)G;
        r.tile_cnt = nd->d_tile_cnt;
        r.shard_base = nd->d_base;
        r.shard_tot = nd->d_base + kMaxShards + 1;
        r.sub_req = nd->d_sub_req;
        r.sub_pos = nd->d_sub_pos;
        r.sub_rec = sub_rec;
        r.low_mask = (1ull << a.kshift) - 1;
        for (uint32_t g = 0; g < G; ++g) r.skshift[g] = 64 - nd->shards[g]->kbits;
        NHIP(nd, launch_route(r, fs));
        NHIP(nd, hipMemcpyAsync(sl.h_base, nd->d_base, sizeof(uint32_t) * (2 * kMaxShards + 1), hipMemcpyDeviceToHost, fs));
    }
    NHIP(nd, hipMemcpyAsync(nd->h_front_err, a.err, sizeof(int), hipMemcpyDeviceToHost, fs));
    NHIP(nd, hipEventRecord(nd->fdone[x], fs));
    // the slice sizes are launch parameters of the shards' sorts: wait for the front (the shards' walkers of the
    // previous batch keep the device busy meanwhile)
    NHIP(nd, hipEventSynchronize(nd->fdone[x]));
    const uint64_t t = nd->next_ticket++;
    *ticket = t;
    if (*nd->h_front_err) {  // refused as a whole (nothing reached the shards)
        nd->finished[t] = node_child(nd, f, flow_status(f, *nd->h_front_err));
        NHIP(nd, hipEventRecord(sl.done, fs));
        sl.G_used = 0;
        nd->pseq++;
        return SG_OK;
    }
    if (direct) {
        sl.h_base[0] = 0;
        sl.h_base[kMaxShards + 1] = (uint32_t)n;
    }
    // 2. every shard: its sort on its front stream (beside its walkers of the previous batch), then its walkers, one
    // shard after another from this thread (enqueueing them from one host thread per shard was slower: 3.5 -> 6.0 ms
    // per G = 4 node batch, r06, the HIP runtime serialising the threads' launches)
    std::vector<int> src(G, SG_OK);
    auto enqueue_shard = [&](uint32_t g) {
        sl.h_err[g] = 0;
        const uint32_t base = sl.h_base[g], cnt = sl.h_base[kMaxShards + 1 + g];
        if (cnt == 0) return;
        sg_handle* h = nd->shards[g];
        if (hipSetDevice(h->device) != hipSuccess) {
            src[g] = SG_E_DEVICE;
            return;
        }
        sg_handle::FlowWs sw = h->pws;
        if (x == 0) main_ws(h, sw);
        BatchArgs b = flow_args(h, sw, req, cnt, out);
        b.rec = direct ? a.rec : sub_rec + base;
        b.rec_sorted = direct ? sw.rec_sorted : sw.rec;
        b.hist0 = direct ? a.hist0 : nullptr;
        b.hist0_bits = a.hist0_bits;
        b.csum0 = direct ? a.csum0 : nullptr;
        b.n_wl = a.n_wl;
        std::memcpy(b.wl, a.wl, sizeof(b.wl));
        b.bnd = a.bnd;
        b.p0 = a.p0;
        b.np = a.np;
        b.walk_cus = node_walk_cus(nd, g, h->walk_cus);
        if (hipStreamWaitEvent(h->s_front, nd->fdone[x], 0) != hipSuccess) {
            src[g] = SG_E_DEVICE;
            return;
        }
        src[g] = node_shard_rec(h, b, cnt, direct ? w.hist : sw.hist, h->s_front, h->s_back, h->s_aux2, h->pfork,
                                h->pjoin, h->front_done[x], &sl.h_err[g]);
        if (src[g] == SG_OK && hipEventRecord(h->back_done[x], h->s_back) != hipSuccess) src[g] = SG_E_DEVICE;
    };
    for (uint32_t g = 0; g < G; ++g) {
        enqueue_shard(g);
        if (src[g] != SG_OK) break;
    }
    NHIP(nd, hipSetDevice(nd->devices[0]));
    for (uint32_t g = 0; g < G; ++g) {
        if (src[g] == SG_OK) continue;
        for (uint32_t q = 0; q < G; ++q) {
            (void)hipStreamSynchronize(nd->shards[q]->s_front);
            (void)hipStreamSynchronize(nd->shards[q]->s_back);
        }
        nd->finished.erase(t);
        *ticket = 0;
        return src[g] == SG_E_DEVICE ? nfail(nd, SG_E_DEVICE, "shard enqueue") : node_child(nd, nd->shards[g], src[g]);
    }
    for (uint32_t g = 0; g < G; ++g)
        if (sl.h_base[kMaxShards + 1 + g]) NHIP(nd, hipStreamWaitEvent(nd->s0, nd->shards[g]->back_done[x], 0));
    NHIP(nd, hipEventRecord(sl.done, nd->s0));
    sl.G_used = G;
    sl.ticket = t;
    nd->pseq++;
    return SG_OK;
}

static int node_collect(sg_node* nd, uint64_t ticket, bool block) {
    if (!nd) return SG_E_INVAL;
    if (ticket == 0) return 1;
    auto it = nd->finished.find(ticket);
    if (it != nd->finished.end()) {
        const int st = it->second;
        nd->finished.erase(it);
        return st == SG_OK ? 1 : st;
    }
    for (auto& sl : nd->pipe) {
        if (sl.ticket != ticket) continue;
        (void)hipSetDevice(nd->devices[0]);
        const hipError_t e = block ? hipEventSynchronize(sl.done) : hipEventQuery(sl.done);
        if (e == hipErrorNotReady) return 0;
        sl.ticket = 0;
        if (e != hipSuccess) return nfail(nd, SG_E_DEVICE, hipGetErrorString(e));
        const int st = node_slot_status(nd, sl);
        return st == SG_OK ? 1 : st;
    }
    return nfail(nd, SG_E_INVAL, "unknown or already collected ticket");
}

int sg_node_flow_poll(sg_node* nd, uint64_t ticket) { return node_collect(nd, ticket, false); }

int sg_node_flow_wait(sg_node* nd, uint64_t ticket) {
    const int r = node_collect(nd, ticket, true);
    return r == 1 ? SG_OK : r;
}

int sg_node_flow_read_state(sg_node* nd, uint32_t key, int64_t* starts, int64_t* counters, int64_t* occupy) {
    if (!nd || key >= nd->shard_of.size()) return SG_E_INVAL;
    node_drain(nd);
    sg_handle* h = nd->shards[nd->shard_of[key]];
    return node_child(nd, h, sg_flow_read_state(h, nd->local_of[key], starts, counters, occupy));
}

int sg_node_snapshot_metrics(sg_node* nd, int64_t now_ms, double* out, uint64_t cap) {
    if (!nd || (!out && cap)) return SG_E_INVAL;
    node_drain(nd);
    const uint64_t K = nd->shard_of.size();
    if (cap < 2 * K) return nfail(nd, SG_E_CAPACITY, "snapshot buffer smaller than 2 * rules");
    if (K == 0) return SG_OK;
    // ClusterMetricNodeGenerator.generateCurrentNodeMap (ClusterMetricNodeGenerator.java:39-61) over the node: every
    // shard's {passQps, blockQps} computed on its device, moved to the front's device (peer copies), scattered into
    // node rule order there, one copy to the host
    const uint32_t G = (uint32_t)nd->shards.size();
    NHIP(nd, hipSetDevice(nd->devices[0]));
    if (nd->node_key_stale || nd->d_node_key.size() != G) {
        for (uint32_t* p : nd->d_node_key) dfree(p);
        nd->d_node_key.assign(G, nullptr);
        std::vector<std::vector<uint32_t>> keys(G);
        for (uint64_t k = 0; k < K; ++k) {
            auto& v = keys[nd->shard_of[k]];
            if (v.size() <= nd->local_of[k]) v.resize(nd->local_of[k] + 1);
            v[nd->local_of[k]] = (uint32_t)k;
        }
        for (uint32_t g = 0; g < G; ++g) {
            if (keys[g].empty()) continue;
            if (hipMalloc(&nd->d_node_key[g], sizeof(uint32_t) * keys[g].size()) != hipSuccess)
                return nfail(nd, SG_E_NOMEM, "node snapshot keys");
            NHIP(nd, hipMemcpy(nd->d_node_key[g], keys[g].data(), sizeof(uint32_t) * keys[g].size(), hipMemcpyHostToDevice));
        }
        nd->node_key_stale = false;
    }
    uint64_t part_max = 0;
    for (sg_handle* h : nd->shards) part_max = std::max<uint64_t>(part_max, h->K);
    const uint64_t need = 2 * K + 2 * part_max;  // the node's rows, then one shard part staged on the front
    if (need > nd->snap_cap) {
        dfree(nd->d_snap);
        if (hipMalloc(&nd->d_snap, sizeof(double) * need) != hipSuccess) return nfail(nd, SG_E_NOMEM, "node snapshot");
        nd->snap_cap = need;
    }
    double* stage = nd->d_snap + 2 * K;
    for (uint32_t g = 0; g < G; ++g) {
        sg_handle* h = nd->shards[g];
        if (h->K == 0) continue;
        const int dev = nd->devices[g];
        double* part = stage;
        if (dev != nd->devices[0]) {  // computed on its device, then copied over xGMI
            NHIP(nd, hipSetDevice(dev));
            if (!nd->r_snap[g] && hipMalloc(&nd->r_snap[g], sizeof(double) * 2 * part_max) != hipSuccess)
                return nfail(nd, SG_E_NOMEM, "node snapshot part");
            part = nd->r_snap[g];
        }
        NHIP(nd, launch_snapshot(h->d_rules, h->d_ring, h->d_occ, h->K, h->stride, now_ms, part, nd->streams[g]));
        NHIP(nd, hipStreamSynchronize(nd->streams[g]));
        NHIP(nd, hipSetDevice(nd->devices[0]));
        if (dev != nd->devices[0])
            NHIP(nd, hipMemcpyPeerAsync(stage, nd->devices[0], part, dev, sizeof(double) * 2 * h->K, nd->s0));
        NHIP(nd, launch_nsnap_scatter(stage, nd->d_node_key[g], h->K, nd->d_snap, nd->s0));
        NHIP(nd, hipStreamSynchronize(nd->s0));  // the stage is reused by the next shard
    }
    NHIP(nd, hipMemcpy(out, nd->d_snap, sizeof(double) * 2 * K, hipMemcpyDeviceToHost));
    return SG_OK;
}

// ---- cluster param and concurrent tokens over the node ----

int sg_node_cparam_load_rules(sg_node* nd, const sg_cparam_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                              uint32_t n_hot, int32_t capacity_log2) {
    if (!nd || (!rules && n) || (!hot && n_hot)) return SG_E_INVAL;
    node_drain(nd);
    // ClusterParamFlowRuleManager over the node: a rule (and its hot items) lives on the shard owning its flowId. The
    // shards' loads are validated by each shard; a failing one leaves the earlier shards on the new rules (node-wide
    // all-or-nothing is the flow rules' contract, not this one's: reload after a failure)
    const uint32_t G = (uint32_t)nd->shards.size();
    for (uint32_t i = 0; i < n; ++i)
        if ((uint64_t)rules[i].hot_begin + rules[i].hot_count > n_hot) return nfail(nd, SG_E_INVAL, "hot item range out of bounds");
    std::vector<std::vector<sg_cparam_rule>> part(G);
    std::vector<std::vector<sg_param_hot_item>> hp(G);
    std::vector<uint8_t> so(n);
    std::vector<uint32_t> lo(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t g = node_owner(rules[i].flow_id, G);
        so[i] = (uint8_t)g;
        lo[i] = (uint32_t)part[g].size();
        sg_cparam_rule r = rules[i];
        r.hot_begin = (uint32_t)hp[g].size();
        hp[g].insert(hp[g].end(), hot + rules[i].hot_begin, hot + rules[i].hot_begin + rules[i].hot_count);
        part[g].push_back(r);
    }
    for (uint32_t g = 0; g < G; ++g) {
        sg_handle* h = nd->shards[g];
        NHIP(nd, hipSetDevice(h->device));
        const int rc = sg_cparam_load_rules(h, part[g].data(), (uint32_t)part[g].size(), hp[g].data(),
                                            (uint32_t)hp[g].size(), capacity_log2);
        if (rc) return node_child(nd, h, rc);
    }
    NHIP(nd, hipSetDevice(nd->devices[0]));
    dfree(nd->d_cp_shard_of);
    dfree(nd->d_cp_local_of);
    if (n && (hipMalloc(&nd->d_cp_shard_of, n) != hipSuccess || hipMalloc(&nd->d_cp_local_of, sizeof(uint32_t) * n) != hipSuccess))
        return nfail(nd, SG_E_NOMEM, "param routing tables");
    if (n) {
        NHIP(nd, hipMemcpy(nd->d_cp_shard_of, so.data(), n, hipMemcpyHostToDevice));
        NHIP(nd, hipMemcpy(nd->d_cp_local_of, lo.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    }
    nd->cp_rules.assign(rules, rules + n);
    nd->cp_shard_of = so;
    nd->cp_local_of = lo;
    return SG_OK;
}

}  // extern "C"

namespace {

// Scratch of the node's param / concurrent routing, sized for max_batch requests (values: n_values).
int node_nreq_scratch(sg_node* nd, uint64_t n_values) {
    const uint64_t n = nd->cfg.max_batch;
    NHIP(nd, hipSetDevice(nd->devices[0]));
    if (!nd->d_nrec) {
        if (hipMalloc(&nd->d_nrec, 8 * n) != hipSuccess || hipMalloc(&nd->d_nrec2, 8 * n) != hipSuccess ||
            hipMalloc(&nd->d_nhist, sizeof(uint32_t) * radix_hist_words(n)) != hipSuccess ||
            hipMalloc(&nd->d_nvals, sizeof(uint32_t) * n) != hipSuccess ||
            hipMalloc(&nd->d_ncnt, sizeof(uint32_t) * 3 * kMaxShards) != hipSuccess ||
            hipMalloc(&nd->d_ntsum, sizeof(uint32_t) * (nreq_tiles(n) + 1)) != hipSuccess ||
            hipMalloc(&nd->d_nerr, sizeof(int)) != hipSuccess ||
            hipMalloc(&nd->d_sub_nreq, std::max(sizeof(sg_cparam_req), sizeof(sg_conc_req)) * n) != hipSuccess ||
            hipMalloc(&nd->d_sub_nout, std::max(sizeof(sg_result), sizeof(sg_conc_result)) * n) != hipSuccess)
            return nfail(nd, SG_E_NOMEM, "node token routing scratch");
    }
    if (n_values > nd->sub_vals_cap) {
        dfree(nd->d_sub_vals);
        if (hipMalloc(&nd->d_sub_vals, 8 * n_values) != hipSuccess) return nfail(nd, SG_E_NOMEM, "node param values");
        nd->sub_vals_cap = n_values;
    }
    return SG_OK;
}

// The node batch's slices (stable by owner): per-shard request bases / counts and value bases / counts on the host.
int node_nreq_route(sg_node* nd, NodeReqArgs q, std::vector<uint64_t>& base, std::vector<uint64_t>& cnt,
                    std::vector<uint64_t>& vbase, std::vector<uint64_t>& vcnt) {
    const uint32_t G = (uint32_t)nd->shards.size();
    hipStream_t st = nd->s0;
    q.G = (int)G;
    q.rec = nd->d_nrec;
    q.nvals = nd->d_nvals;
    q.cnt = nd->d_ncnt;
    q.vcnt = nd->d_ncnt + kMaxShards;
    q.tsum = nd->d_ntsum;
    q.vbase = nd->d_ncnt + 2 * kMaxShards;
    q.sub_vals = nd->d_sub_vals;
    q.sub_pos = nd->d_sub_pos;
    q.err = nd->d_nerr;
    NHIP(nd, hipMemsetAsync(nd->d_ncnt, 0, sizeof(uint32_t) * 2 * kMaxShards, st));
    NHIP(nd, hipMemsetAsync(nd->d_nerr, 0, sizeof(int), st));
    NHIP(nd, launch_nreq_keys(q, st));
    uint32_t h_cnt[2 * kMaxShards];
    int err = 0;
    NHIP(nd, hipMemcpyAsync(h_cnt, nd->d_ncnt, sizeof(h_cnt), hipMemcpyDeviceToHost, st));
    NHIP(nd, hipMemcpyAsync(&err, nd->d_nerr, sizeof(int), hipMemcpyDeviceToHost, st));
    NHIP(nd, hipStreamSynchronize(st));
    if (err & kErrTime)
        return nfail(nd, SG_E_TIME, "timestamps must be >= 0, non-decreasing, and not older than the node's earlier batches");
    if (err & kErrBounds) return nfail(nd, SG_E_INVAL, "a request's values lie outside the value array");
    base.assign(G, 0);
    cnt.assign(G, 0);
    vbase.assign(G, 0);
    vcnt.assign(G, 0);
    uint32_t vb[kMaxShards] = {};
    uint64_t b = 0, v = 0;
    for (uint32_t g = 0; g < G; ++g) {
        base[g] = b;
        cnt[g] = h_cnt[g];
        vbase[g] = v;
        vcnt[g] = h_cnt[kMaxShards + g];
        vb[g] = (uint32_t)v;
        b += cnt[g];
        v += vcnt[g];
    }
    NHIP(nd, hipMemcpyAsync(nd->d_ncnt + 2 * kMaxShards, vb, sizeof(vb), hipMemcpyHostToDevice, st));
    uint64_t* sorted = nullptr;
    NHIP(nd, radix_sort_records(nd->d_nrec, nd->d_nrec2, q.n, 56, nd->d_nhist, &sorted, st, 64));
    NHIP(nd, launch_nreq_gather(q, sorted, st));
    NHIP(nd, hipStreamSynchronize(st));
    return SG_OK;
}

// Buffers for shard g's slice on its own device (shards off the front's device; grown as needed): requests,
// results, values.
int node_slice_alloc(sg_node* nd, uint32_t g, uint64_t nv) {
    const int dev = nd->devices[g];
    if (dev == nd->devices[0]) return SG_OK;
    NHIP(nd, hipSetDevice(dev));
    const uint64_t n = nd->cfg.max_batch;
    if (!nd->r_nreq[g] && (hipMalloc(&nd->r_nreq[g], std::max(sizeof(sg_cparam_req), sizeof(sg_conc_req)) * n) != hipSuccess ||
                           hipMalloc(&nd->r_nout[g], std::max(sizeof(sg_result), sizeof(sg_conc_result)) * n) != hipSuccess))
        return nfail(nd, SG_E_NOMEM, "shard slice buffers");
    if (nv > nd->r_vals_cap[g]) {
        dfree(nd->r_vals[g]);
        if (hipMalloc(&nd->r_vals[g], 8 * nv) != hipSuccess) return nfail(nd, SG_E_NOMEM, "shard values");
        nd->r_vals_cap[g] = nv;
    }
    return SG_OK;
}

// Shard g's part of a node token batch, run by `decide(h, req, vals, out, stream)` on the shard's slice [base, base +
// cnt) of the routed requests (req_b / out_b bytes each; nv values from svals): peer copies in and out for a shard
// off the front's device. Every shard with work runs in its own host thread — a shard's call waits on the host
// between its own kernels (the param fixed point's rounds, the concurrent batch's error check), so the shards overlap
// whether they share a device or not. The first failure is reported after all have finished.
template <class Decide>
int node_run_shards(sg_node* nd, const std::vector<uint64_t>& base, const std::vector<uint64_t>& cnt,
                    const std::vector<uint64_t>& vbase, const std::vector<uint64_t>& vcnt, size_t req_b, size_t out_b,
                    const void* sub_req, void* sub_out, Decide decide) {
    const uint32_t G = (uint32_t)nd->shards.size();
    for (uint32_t g = 0; g < G; ++g)
        if (cnt[g]) {
            const int rc = node_slice_alloc(nd, g, vcnt[g]);
            if (rc) return rc;
        }
    std::vector<int> rc(G, SG_OK);
    std::vector<char> child(G, 0);
    std::vector<std::string> msg(G);
    auto run = [&](uint32_t g) {
        sg_handle* h = nd->shards[g];
        const int dev = h->device;
        const bool remote = dev != nd->devices[0];
        const char* sreq = static_cast<const char*>(sub_req) + req_b * base[g];
        const uint64_t* svals = nd->d_sub_vals + vbase[g];
        char* sout = static_cast<char*>(sub_out) + out_b * base[g];
        hipError_t e = hipSetDevice(dev);
        const void* req = sreq;
        const uint64_t* vals = svals;
        void* out = sout;
        if (remote) {
            if (e == hipSuccess) e = hipMemcpyPeer(nd->r_nreq[g], dev, sreq, nd->devices[0], req_b * cnt[g]);
            if (e == hipSuccess && vcnt[g]) e = hipMemcpyPeer(nd->r_vals[g], dev, svals, nd->devices[0], 8 * vcnt[g]);
            req = nd->r_nreq[g];
            vals = nd->r_vals[g];
            out = nd->r_nout[g];
        }
        if (e != hipSuccess) {
            rc[g] = SG_E_DEVICE;
            msg[g] = hipGetErrorString(e);
            return;
        }
        const int r = decide(h, req, vcnt[g] ? vals : nullptr, vcnt[g], cnt[g], out, nd->streams[g]);
        if (r) {
            rc[g] = r;
            child[g] = 1;
            return;
        }
        e = hipStreamSynchronize(nd->streams[g]);
        if (e == hipSuccess && remote) e = hipMemcpyPeer(sout, nd->devices[0], out, dev, out_b * cnt[g]);
        if (e != hipSuccess) {
            rc[g] = SG_E_DEVICE;
            msg[g] = hipGetErrorString(e);
        }
    };
    std::vector<uint32_t> work;
    for (uint32_t g = 0; g < G; ++g)
        if (cnt[g]) work.push_back(g);
    if (work.size() == 1) {
        run(work[0]);
    } else {
        std::vector<std::thread> th;
        th.reserve(work.size());
        for (uint32_t g : work) th.emplace_back(run, g);
        for (auto& t : th) t.join();
    }
    (void)hipSetDevice(nd->devices[0]);
    for (uint32_t g : work) {
        if (!rc[g]) continue;
        if (child[g]) return node_child(nd, nd->shards[g], rc[g]);
        return nfail(nd, rc[g], msg[g].c_str());
    }
    return SG_OK;
}

}  // namespace

extern "C" {

int sg_node_cparam_decide_batch(sg_node* nd, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                uint64_t n_values, sg_result* out, void* stream) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out || (!values && n_values)) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    if (n_values >= (1ull << 32)) return nfail(nd, SG_E_CAPACITY, "more than 2^32 values");
    node_drain(nd);
    // allowProceed (ClusterParamFlowChecker.java:43-45) needs the namespace's limiter in the node's caller order: the
    // node's param path serves namespaces without one
    for (const auto& r : nd->cp_rules)
        if (r.namespace_id >= 0 && (size_t)r.namespace_id < nd->ns.size() && nd->ns[r.namespace_id].limiter_enabled)
            return nfail(nd, SG_E_UNSUPPORTED, "node param tokens with a namespace limiter (use one handle, or the "
                                               "sharded limiter exchange)");
    int rc = node_nreq_scratch(nd, n_values ? n_values : 1);
    if (rc) return rc;
    NodeReqArgs q{};
    q.n = n;
    q.cp = req;
    q.values = values;
    q.n_values = n_values;
    q.K = (uint32_t)nd->cp_rules.size();
    q.shard_of = nd->d_cp_shard_of;
    q.local_of = nd->d_cp_local_of;
    q.sub_cp = static_cast<sg_cparam_req*>(nd->d_sub_nreq);
    q.last_ts = nd->cp_last_ts;
    NHIP(nd, hipStreamSynchronize((hipStream_t)stream));  // the caller's batch is in place (synchronous call)
    std::vector<uint64_t> base, cnt, vbase, vcnt;
    rc = node_nreq_route(nd, q, base, cnt, vbase, vcnt);
    if (rc) return rc;
    sg_result* sub_out = static_cast<sg_result*>(nd->d_sub_nout);
    rc = node_run_shards(nd, base, cnt, vbase, vcnt, sizeof(sg_cparam_req), sizeof(sg_result), q.sub_cp, sub_out,
                         [](sg_handle* h, const void* r, const uint64_t* v, uint64_t nv, uint64_t c, void* o, hipStream_t st) {
                             return sg_cparam_decide_batch(h, static_cast<const sg_cparam_req*>(r), c, v, nv,
                                                           static_cast<sg_result*>(o), st);
                         });
    if (rc) return rc;
    NHIP(nd, hipSetDevice(nd->devices[0]));
    NHIP(nd, launch_route_gather(sub_out, nd->d_sub_pos, n, out, nd->s0));
    int64_t last = 0;
    NHIP(nd, hipMemcpyAsync(&last, &req[n - 1].ts_ms, sizeof(int64_t), hipMemcpyDeviceToHost, nd->s0));
    NHIP(nd, hipStreamSynchronize(nd->s0));
    nd->cp_last_ts = last;
    return SG_OK;
}

int sg_node_cparam_decide_batch_host(sg_node* nd, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                     uint64_t n_values, sg_result* out) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out || (!values && n_values)) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    NHIP(nd, hipSetDevice(nd->devices[0]));
    node_drain(nd);
    if (!nd->d_nreq_h && (hipMalloc(&nd->d_nreq_h, sizeof(sg_conc_req) * nd->cfg.max_batch) != hipSuccess ||
                          hipMalloc(&nd->d_nout_h, sizeof(sg_conc_result) * nd->cfg.max_batch) != hipSuccess))
        return nfail(nd, SG_E_NOMEM, "node host-path buffers");
    if (n_values > nd->nvals_h_cap) {
        dfree(nd->d_nvals_h);
        if (hipMalloc(&nd->d_nvals_h, 8 * n_values) != hipSuccess) return nfail(nd, SG_E_NOMEM, "node host-path values");
        nd->nvals_h_cap = n_values;
    }
    NHIP(nd, hipMemcpy(nd->d_nreq_h, req, sizeof(sg_cparam_req) * n, hipMemcpyHostToDevice));
    if (n_values) NHIP(nd, hipMemcpy(nd->d_nvals_h, values, 8 * n_values, hipMemcpyHostToDevice));
    const int rc = sg_node_cparam_decide_batch(nd, static_cast<const sg_cparam_req*>(nd->d_nreq_h), n,
                                               n_values ? nd->d_nvals_h : nullptr, n_values,
                                               static_cast<sg_result*>(nd->d_nout_h), nullptr);
    if (rc) return rc;
    NHIP(nd, hipMemcpy(out, nd->d_nout_h, sizeof(sg_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_node_cparam_read_sum(sg_node* nd, uint32_t rule, uint64_t value, int64_t now_ms, int64_t* sum) {
    if (!nd || !sum || rule >= nd->cp_rules.size()) return SG_E_INVAL;
    node_drain(nd);
    sg_handle* h = nd->shards[nd->cp_shard_of[rule]];
    return node_child(nd, h, sg_cparam_read_sum(h, nd->cp_local_of[rule], value, now_ms, sum));
}

// ClusterParamMetric.getTopValues per node rule (ClusterMetricNodeGenerator.paramToMetricNode :88-104): each rule's
// values come from its owner (its metric lives there), laid out in node rule order as sg_cparam_top_values does.
int sg_node_cparam_top_values(sg_node* nd, int64_t now_ms, uint32_t number, uint64_t* values, double* qps,
                              uint32_t* counts) {
    const uint64_t R = nd ? nd->cp_rules.size() : 0;
    if (!nd || (R && (!values || !qps || !counts))) return SG_E_INVAL;
    node_drain(nd);
    const uint32_t G = (uint32_t)nd->shards.size();
    for (uint32_t g = 0; g < G; ++g) {
        sg_handle* h = nd->shards[g];
        const uint64_t r = h->cprules.size();
        if (!r) continue;
        std::vector<uint64_t> v(r * number);
        std::vector<double> q(r * number);
        std::vector<uint32_t> c(r);
        const int rc = sg_cparam_top_values(h, now_ms, number, v.data(), q.data(), c.data());
        if (rc) return node_child(nd, h, rc);
        for (uint64_t k = 0; k < R; ++k) {
            if (nd->cp_shard_of[k] != g) continue;
            const uint32_t l = nd->cp_local_of[k];
            counts[k] = c[l];
            for (uint32_t j = 0; j < number; ++j) {
                values[k * number + j] = v[(uint64_t)l * number + j];
                qps[k * number + j] = q[(uint64_t)l * number + j];
            }
        }
    }
    return SG_OK;
}

int sg_node_conc_decide_batch(sg_node* nd, const sg_conc_req* req, uint64_t n, sg_conc_result* out, void* stream) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    node_drain(nd);
    int rc = node_nreq_scratch(nd, 1);
    if (rc) return rc;
    const uint32_t G = (uint32_t)nd->shards.size();
    NodeReqArgs q{};
    q.n = n;
    q.cc = req;
    q.K = (uint32_t)nd->shard_of.size();
    q.shard_of = nd->d_shard_of;
    q.local_of = nd->d_local_of;
    q.sub_cc = static_cast<sg_conc_req*>(nd->d_sub_nreq);
    q.last_ts = nd->cc_last_ts;
    NHIP(nd, hipStreamSynchronize((hipStream_t)stream));  // the caller's batch is in place (synchronous call)
    std::vector<uint64_t> base, cnt, vbase, vcnt;
    rc = node_nreq_route(nd, q, base, cnt, vbase, vcnt);
    if (rc) return rc;
    sg_conc_result* sub_out = static_cast<sg_conc_result*>(nd->d_sub_nout);
    rc = node_run_shards(nd, base, cnt, vbase, vcnt, sizeof(sg_conc_req), sizeof(sg_conc_result), q.sub_cc, sub_out,
                         [](sg_handle* h, const void* r, const uint64_t*, uint64_t, uint64_t c, void* o, hipStream_t st) {
                             return sg_conc_decide_batch(h, static_cast<const sg_conc_req*>(r), c,
                                                         static_cast<sg_conc_result*>(o), st);
                         });
    if (rc) return rc;
    NHIP(nd, hipSetDevice(nd->devices[0]));
    for (uint32_t g = 0; g < G; ++g)
        NHIP(nd, launch_nconc_scatter(sub_out, nd->d_sub_pos, q.sub_cc, base[g], cnt[g], g, G, out, nd->s0));
    int64_t last = 0;
    NHIP(nd, hipMemcpyAsync(&last, &req[n - 1].ts_ms, sizeof(int64_t), hipMemcpyDeviceToHost, nd->s0));
    NHIP(nd, hipStreamSynchronize(nd->s0));
    nd->cc_last_ts = last;
    return SG_OK;
}

int sg_node_conc_decide_batch_host(sg_node* nd, const sg_conc_req* req, uint64_t n, sg_conc_result* out) {
    if (!nd) return SG_E_INVAL;
    if (n == 0) return SG_OK;
    if (!req || !out) return nfail(nd, SG_E_INVAL, "null buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, SG_E_CAPACITY, "batch larger than max_batch");
    NHIP(nd, hipSetDevice(nd->devices[0]));
    node_drain(nd);
    if (!nd->d_nreq_h && (hipMalloc(&nd->d_nreq_h, sizeof(sg_conc_req) * nd->cfg.max_batch) != hipSuccess ||
                          hipMalloc(&nd->d_nout_h, sizeof(sg_conc_result) * nd->cfg.max_batch) != hipSuccess))
        return nfail(nd, SG_E_NOMEM, "node host-path buffers");
    NHIP(nd, hipMemcpy(nd->d_nreq_h, req, sizeof(sg_conc_req) * n, hipMemcpyHostToDevice));
    const int rc = sg_node_conc_decide_batch(nd, static_cast<const sg_conc_req*>(nd->d_nreq_h), n,
                                             static_cast<sg_conc_result*>(nd->d_nout_h), nullptr);
    if (rc) return rc;
    NHIP(nd, hipMemcpy(out, nd->d_nout_h, sizeof(sg_conc_result) * n, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_node_conc_set_rule_timeouts(sg_node* nd, const int64_t* client_offline_ms, const int64_t* resource_timeout_ms,
                                   uint32_t n) {
    if (!nd || (n && (!client_offline_ms || !resource_timeout_ms))) return SG_E_INVAL;
    if (n != nd->shard_of.size()) return nfail(nd, SG_E_INVAL, "one timeout pair per loaded rule");
    node_drain(nd);
    const uint32_t G = (uint32_t)nd->shards.size();
    std::vector<std::vector<int64_t>> off(G), res(G);
    for (uint32_t g = 0; g < G; ++g) {
        off[g].resize(nd->shards[g]->K);
        res[g].resize(nd->shards[g]->K);
    }
    for (uint32_t k = 0; k < n; ++k) {
        off[nd->shard_of[k]][nd->local_of[k]] = client_offline_ms[k];
        res[nd->shard_of[k]][nd->local_of[k]] = resource_timeout_ms[k];
    }
    for (uint32_t g = 0; g < G; ++g) {
        sg_handle* h = nd->shards[g];
        const int rc = sg_conc_set_rule_timeouts(h, off[g].data(), res[g].data(), (uint32_t)off[g].size());
        if (rc) return node_child(nd, h, rc);
    }
    return SG_OK;
}

int sg_node_conc_expire(sg_node* nd, int64_t now_ms, const uint8_t* client_online, uint32_t n_clients, uint64_t* removed) {
    if (!nd || !removed) return SG_E_INVAL;
    node_drain(nd);
    uint64_t total = 0;
    for (sg_handle* h : nd->shards) {
        uint64_t r = 0;
        const int rc = sg_conc_expire(h, now_ms, client_online, n_clients, &r);
        if (rc) return node_child(nd, h, rc);
        total += r;
    }
    *removed = total;
    return SG_OK;
}

int sg_node_conc_read_state(sg_node* nd, uint32_t key, int32_t* now_calls, uint64_t* live_tokens) {
    if (!nd || !now_calls || !live_tokens || key >= nd->shard_of.size()) return SG_E_INVAL;
    node_drain(nd);
    uint64_t live = 0;
    for (uint32_t g = 0; g < (uint32_t)nd->shards.size(); ++g) {
        int32_t nc = 0;
        uint64_t l = 0;
        sg_handle* h = nd->shards[g];
        const bool owner = g == nd->shard_of[key];
        if (!owner && h->K == 0) continue;
        const int rc = sg_conc_read_state(h, owner ? nd->local_of[key] : 0u, &nc, &l);
        if (rc) return node_child(nd, h, rc);
        if (owner) *now_calls = nc;
        live += l;
    }
    *live_tokens = live;
    return SG_OK;
}

}  // extern "C"
