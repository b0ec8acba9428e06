/*
 * sentinel_gpu.h — C ABI of the MI355X batched flow-decision engine.
 *
 * This is the drop-in boundary for Sentinel's cluster token service hot path.
 * Every entry point below replaces a piece of the Java reference
 * (paths relative to /root/reference; see INTEGRATION.md for the JNI / Panama
 * bindings a Sentinel maintainer would add):
 *
 *   sg_flow_decide_batch      ← TokenService.requestToken(Long,int,boolean)
 *                               sentinel-core/.../cluster/TokenService.java:36, implemented by
 *                               DefaultTokenService.requestToken
 *                               sentinel-cluster/sentinel-cluster-server-default/.../flow/DefaultTokenService.java:39-50
 *                               → ClusterFlowChecker.acquireClusterToken (…/flow/ClusterFlowChecker.java:55-112),
 *                               evaluated for a whole batch of requests in (timestamp, arrival) order.
 *   sg_load_flow_rules        ← ClusterFlowRuleManager.loadRules / applyClusterFlowRule
 *                               (…/flow/rule/ClusterFlowRuleManager.java:254-260, 325-375); metrics of a
 *                               flowId that survives a reload are kept (putMetricIfAbsent :361).
 *   sg_set_namespaces         ← ClusterServerConfigManager (exceedCount / maxOccupyRatio / maxAllowedQps,
 *                               …/server/config/ClusterServerConfigManager.java:303-346) +
 *                               GlobalRequestLimiter.initIfAbsent (…/statistic/limit/GlobalRequestLimiter.java:32-37)
 *                               + ConnectionManager.getConnectedCount (…/server/connection/ConnectionManager.java:47-51)
 *   sg_flow_read_state        ← ClusterMetric window contents (…/statistic/metric/ClusterMetric.java) — read back
 *                               for parity checks and the metric snapshot.
 *   sg_snapshot_metrics       ← ClusterMetricNodeGenerator.generateCurrentNodeMap passQps/blockQps per flowId
 *                               (…/flow/statistic/ClusterMetricNodeGenerator.java:39-105).
 *
 * Conventions: plain C types only, no exceptions across the ABI, 0 = success, negative SG_E* on error
 * (the Java shim then answers TokenResult(FAIL) so FlowRuleChecker.fallbackToLocalOrPass applies,
 * sentinel-core/.../slots/block/flow/FlowRuleChecker.java:166-209). One handle = one submitter.
 */
#ifndef SENTINEL_GPU_H
#define SENTINEL_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---- */
#define SG_OK              0
#define SG_E_INVAL        -1   /* bad argument / invalid rule / bad request record layout          */
#define SG_E_DEVICE       -2   /* HIP runtime error                                               */
#define SG_E_NOMEM        -3   /* device allocation failed                                        */
#define SG_E_UNSUPPORTED  -4   /* configuration outside the device path (e.g. sampleCount > 64)   */
#define SG_E_TIME         -5   /* timestamps negative or not non-decreasing (batch or vs. state)  */
#define SG_E_CAPACITY     -6   /* batch larger than sg_config.max_batch                           */

/* ---- TokenResultStatus (sentinel-core/.../cluster/TokenResultStatus.java:27-53) ---- */
#define SG_STATUS_BAD_REQUEST      (-4)
#define SG_STATUS_TOO_MANY_REQUEST (-2)
#define SG_STATUS_FAIL             (-1)
#define SG_STATUS_OK                 0
#define SG_STATUS_BLOCKED            1
#define SG_STATUS_SHOULD_WAIT        2
#define SG_STATUS_NO_RULE_EXISTS     3

/* ---- ClusterRuleConstant (sentinel-core/.../slots/block/ClusterRuleConstant.java:27-28) ---- */
#define SG_THRESHOLD_AVG_LOCAL 0
#define SG_THRESHOLD_GLOBAL    1

/* ---- ClusterFlowEvent ordinals (…/flow/statistic/data/ClusterFlowEvent.java:22-52) ---- */
#define SG_EV_PASS           0
#define SG_EV_BLOCK          1
#define SG_EV_PASS_REQUEST   2
#define SG_EV_BLOCK_REQUEST  3
#define SG_EV_OCCUPIED_PASS  4
#define SG_EV_OCCUPIED_BLOCK 5
#define SG_EV_WAITING        6
#define SG_NUM_EVENTS        7

/* ---- request key encoding ----
 * key = dense rule index assigned by sg_load_flow_rules (position in the rule array),
 * OR-ed with SG_KEY_PRIO for prioritized requests. Two reserved values let the host shim
 * submit requests it has already classified without splitting the batch:
 *   SG_KEY_BAD     → BAD_REQUEST   (DefaultTokenService.notValidRequest, id null/<=0, :87-89)
 *   SG_KEY_NO_RULE → NO_RULE_EXISTS (rule lookup miss, DefaultTokenService.java:44-47)
 * Any other index >= number of loaded rules also answers NO_RULE_EXISTS. */
#define SG_KEY_PRIO    0x80000000u
#define SG_KEY_INDEX   0x7FFFFFFFu
#define SG_KEY_NO_RULE 0x7FFFFFFFu
#define SG_KEY_BAD     0x7FFFFFFEu

/* sg_config.flags: force one walker for every flowId segment (testing both walkers on any trace). */
#define SG_FLAG_SERIAL_ONLY 1   /* one lane per flowId, however long its segment */
#define SG_FLAG_WAVE_ONLY   2   /* one wave per flowId, however short its segment */
#define SG_FLAG_RING_REREAD 4   /* short walker without the register ring snapshot (re-reads the ring)   */

/* Largest sampleCount the device walker keeps in a wave (one bucket per lane). */
#define SG_MAX_SAMPLE_COUNT 64

typedef struct sg_handle sg_handle;

typedef struct sg_config {
    int32_t  device;            /* HIP device ordinal                                   */
    int32_t  flags;             /* SG_FLAG_* (0 = default walker selection)             */
    double   exceed_count;      /* ServerFlowConfig.exceedCount, default 1.0 (:26)      */
    double   max_occupy_ratio;  /* ServerFlowConfig.maxOccupyRatio, default 1.0 (:27)  */
    uint64_t max_batch;         /* largest n accepted by sg_flow_decide_batch           */
} sg_config;

/* One cluster-mode QPS FlowRule with its ClusterFlowConfig
 * (FlowRule.java:52-95, ClusterFlowConfig.java:29-74). */
typedef struct sg_flow_rule {
    int64_t flow_id;            /* ClusterFlowConfig.flowId (must be > 0)                      */
    double  count;              /* FlowRule.count (threshold, >= 0)                            */
    int32_t threshold_type;     /* SG_THRESHOLD_AVG_LOCAL / SG_THRESHOLD_GLOBAL                */
    int32_t sample_count;       /* ClusterFlowConfig.sampleCount, default 10                   */
    int32_t window_interval_ms; /* ClusterFlowConfig.windowIntervalMs, default 1000            */
    int32_t namespace_id;       /* index into the sg_set_namespaces array                      */
} sg_flow_rule;

/* Per-namespace server settings. */
typedef struct sg_namespace {
    int32_t limiter_enabled;    /* GlobalRequestLimiter has a RequestLimiter for this namespace */
    int32_t connected_count;    /* ConnectionManager.getConnectedCount(namespace)               */
    double  max_allowed_qps;    /* ServerFlowConfig.maxAllowedQps, default 30000 (:31)          */
} sg_namespace;

/* One token request: requestToken(flowId→key, acquireCount, prioritized) at time ts_ms. */
typedef struct sg_req {
    int64_t  ts_ms;             /* explicit TimeUtil.currentTimeMillis() of the call          */
    uint32_t key;               /* rule index | SG_KEY_PRIO, or SG_KEY_BAD / SG_KEY_NO_RULE     */
    int32_t  acquire;           /* acquireCount; <= 0 → BAD_REQUEST                            */
} sg_req;

/* TokenResult (sentinel-core/.../cluster/TokenResult.java:26-35) minus tokenId/attachments. */
typedef struct sg_result {
    int32_t status;
    int32_t remaining;
    int32_t wait_ms;
} sg_result;

/* ---- hot-parameter flow control (ParamFlowChecker, sentinel-extension/sentinel-parameter-flow-control) ---- */

/* One QPS ParamFlowRule (ParamFlowRule.java:45-83). The parameter value itself is a u64 chosen by the
 * caller (a Long argument as is, other types through the shim's value dictionary). */
typedef struct sg_param_rule {
    double   count;             /* ParamFlowRule.count (token count per duration)                 */
    int64_t  duration_sec;      /* durationInSec, default 1                                       */
    int32_t  burst;             /* burstCount, default 0                                          */
    int32_t  behavior;          /* CONTROL_BEHAVIOR_DEFAULT 0 (token bucket) / RATE_LIMITER 2      */
    int32_t  max_queueing_ms;   /* maxQueueingTimeMs (throttle), default 0                        */
    uint32_t hot_begin;         /* this rule's hot items: hot[hot_begin .. hot_begin + hot_count) */
    uint32_t hot_count;
    int32_t  capacity_log2;     /* device table: 2^capacity_log2 distinct values (0 = 2^20)        */
} sg_param_rule;

/* ParamFlowItem → parsed hot item: value-specific threshold (ParamFlowRuleUtil.parseHotItems :188-209). */
typedef struct sg_param_hot_item {
    uint64_t value;
    int32_t  threshold;
    int32_t  reserved;
} sg_param_hot_item;

/* One single-value check: passSingleValueCheck(rule, acquireCount, value) at ts_ms. */
typedef struct sg_param_req {
    int64_t  ts_ms;
    uint64_t value;
    uint32_t rule;              /* index into the loaded param rules                               */
    int32_t  acquire;           /* acquireCount                                                    */
} sg_param_req;

/* ---- ParamFlowSlot: every param rule of a resource, collection/array arguments, THREAD grade ----
 * SphU.entry(resource, count, args...) through ParamFlowSlot.checkFlow (ParamFlowSlot.java:66-93): the resource's
 * rules in load order (the first failing one throws ParamFlowException), each on args[paramIdx]
 * (ParamFlowChecker.passCheck :48-73): no argument or a null one passes, a collection / array is checked element by
 * element in order with the state changes of the elements before a failing one kept (passLocalCheck :75-104),
 * QPS rules through the token bucket / throttle of sg_param_*, THREAD rules against the per-(resource, paramIdx,
 * value) thread counts (passSingleValueCheck :114-122) that ParamFlowStatisticEntryCallback / ExitCallback keep
 * (ParameterMetric.addThreadCount / decreaseThreadCount :125-239). Rules are sg_param_rule plus the fields below;
 * a negative paramIdx is resolved against the first call's argument count and then kept (applyRealParamIdx
 * :57-64). Resources with several rules and collection arguments are walked one event at a time per resource. */
#define SG_ARG_NULL        0
#define SG_ARG_VALUE       1
#define SG_ARG_COLLECTION  2
/* ParamFlowRule.clusterMode with its ParamFlowClusterConfig (cluster_mode: SG_CLUSTER_MODE_* as for flow rules,
 * below). passCheck sends a clusterMode QPS rule to passClusterCheck (ParamFlowChecker.java:71-73, :278-303): on a
 * node that is neither token client nor server (sg_local_set_cluster_state, NOT_STARTED the default) pickClusterService
 * is null and fallbackToLocalOrPass (:305-313) applies — SG_CLUSTER_MODE_FALLBACK checks the rule locally,
 * SG_CLUSTER_MODE_NO_FALLBACK passes it. On a node whose embedded token server runs on this handle (SERVER) the rule
 * requests a param token for all of the argument's values (toCollection) from the handle's cluster param state
 * (sg_cparam_load_rules, the namespace limiter included: DefaultTokenService.requestParamToken →
 * ClusterParamFlowChecker.acquireClusterToken) in event order: OK passes, BLOCKED throws ParamFlowException,
 * NO_RULE_EXISTS / BAD_REQUEST / TOO_MANY_REQUEST go to fallbackToLocalOrPass. THREAD-grade cluster rules are checked
 * locally (passCheck's condition). SG_CLUSTER_MODE_INVALID (ParamFlowRuleUtil.checkCluster :54-66 failed: no config,
 * an invalid window or flowId <= 0) drops the rule at load, as ParamFlowRuleManager does. A token client (CLIENT)
 * with cluster-mode QPS rules loaded is SG_E_UNSUPPORTED. */
typedef struct sg_pslot_rule {
    sg_param_rule rule;          /* token bucket / throttle parameters, hot items                          */
    uint32_t      resource;      /* resource index                                                         */
    int32_t       param_idx;     /* ParamFlowRule.paramIdx                                                 */
    int32_t       grade;         /* 0 FLOW_GRADE_THREAD, 1 FLOW_GRADE_QPS                                 */
    int32_t       cluster_mode;  /* SG_CLUSTER_MODE_* (0: a local rule)                                     */
    uint32_t      cluster_key;   /* SERVER: ParamFlowClusterConfig.flowId as a rule index of this handle's
                                    sg_cparam_load_rules (SG_KEY_NO_RULE: the server has no rule for it)     */
    int32_t       reserved;
} sg_pslot_rule;
typedef struct sg_pslot_arg {    /* one argument: null, a value, or a collection / array of values        */
    uint32_t value_begin;
    uint32_t value_count;
    int32_t  kind;               /* SG_ARG_*                                                              */
    int32_t  reserved;
} sg_pslot_arg;
typedef struct sg_pslot_event {  /* an entry (SphU.entry) or the exit of a passed entry (its own arguments) */
    int64_t  ts_ms;
    uint32_t resource;
    int32_t  count;              /* acquireCount                                                          */
    int32_t  kind;               /* SG_LOCAL_ENTRY / SG_LOCAL_EXIT                                         */
    uint32_t arg_begin;          /* args[arg_begin .. + arg_count)                                         */
    uint32_t arg_count;
    int32_t  args_null;          /* 1: the Object[] args itself is null (checkFlow returns at once)         */
} sg_pslot_event;
typedef struct sg_pslot_result {
    int32_t pass;                /* entries: 1 pass / 0 ParamFlowException; exits: 1                       */
    int32_t rule;                /* the rule that threw (index into the loaded rules), else -1              */
} sg_pslot_result;
/* Loads the rules (state of sg_param_* starts empty, as for sg_param_load_rules). */
int sg_pslot_load_rules(sg_handle* h, const sg_pslot_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                        uint32_t n_hot, uint32_t n_resources);
/* A time-ordered batch; events, args, values and results are DEVICE pointers (asynchronous on stream). */
int sg_pslot_decide_batch(sg_handle* h, const sg_pslot_event* ev, uint64_t n, const sg_pslot_arg* args,
                          uint64_t n_args, const uint64_t* values, uint64_t n_values, sg_pslot_result* out, void* stream);
int sg_pslot_decide_batch_host(sg_handle* h, const sg_pslot_event* ev, uint64_t n, const sg_pslot_arg* args,
                               uint64_t n_args, const uint64_t* values, uint64_t n_values, sg_pslot_result* out);
/* ParameterMetric.getThreadCount(paramIdx, value) of a resource, and a rule's current paramIdx. */
int sg_pslot_thread_count(sg_handle* h, uint32_t resource, int32_t param_idx, uint64_t value, int64_t* count);
int sg_pslot_param_idx(sg_handle* h, uint32_t rule, int32_t* param_idx);

/* ---- pace controller: FlowRule with CONTROL_BEHAVIOR_RATE_LIMITER (RateLimiterController) ---- */

/* One FlowRule whose controller is RateLimiterController(maxQueueingTimeMs, count)
 * (sentinel-core/.../slots/block/flow/controller/RateLimiterController.java:35-38). Each rule owns one
 * latestPassedTime, initially -1. */
typedef struct sg_pace_rule {
    double   count;             /* FlowRule.count (requests per second), >= 0                      */
    int32_t  max_queueing_ms;   /* FlowRule.maxQueueingTimeMs, default 500                         */
    int32_t  reserved;
} sg_pace_rule;

/* canPass(node, acquireCount) at ts_ms (RateLimiterController.java:46-91). */
typedef struct sg_pace_req {
    int64_t  ts_ms;
    uint32_t rule;              /* index into the loaded pace rules; >= n passes (no rule)         */
    int32_t  acquire;           /* acquireCount                                                    */
} sg_pace_req;

#define SG_PACE_BLOCKED (-1)    /* result: canPass false; >= 0: passes after sleeping that many ms */

/* ---- cluster hot-parameter tokens (TokenService.requestParamToken → ClusterParamFlowChecker) ---- */

/* One cluster-mode ParamFlowRule with its ParamFlowClusterConfig (ParamFlowRule.java, ParamFlowClusterConfig.java). */
typedef struct sg_cparam_rule {
    int64_t  flow_id;            /* ParamFlowClusterConfig.flowId (> 0)                                   */
    double   count;              /* ParamFlowRule.count (threshold of values without a hot item)         */
    int32_t  threshold_type;     /* SG_THRESHOLD_AVG_LOCAL / SG_THRESHOLD_GLOBAL                           */
    int32_t  sample_count;       /* ParamFlowClusterConfig.sampleCount, default 10                         */
    int32_t  window_interval_ms; /* windowIntervalMs, default 1000                                         */
    int32_t  namespace_id;       /* index into the sg_set_namespaces array                                 */
    uint32_t hot_begin;          /* this rule's hot items (exclusive item counts): hot[hot_begin ..)     */
    uint32_t hot_count;
} sg_cparam_rule;

/* requestParamToken(ruleId→key, acquireCount, params) at ts_ms; the parameter values are
 * values[value_begin .. value_begin + value_count) of the batch's u64 value array. */
typedef struct sg_cparam_req {
    int64_t  ts_ms;
    uint32_t key;                /* rule index, or SG_KEY_BAD / SG_KEY_NO_RULE                             */
    int32_t  acquire;
    uint32_t value_begin;
    uint32_t value_count;        /* 0 → BAD_REQUEST (params empty, DefaultTokenService.java:54)            */
} sg_cparam_req;

/* ---- concurrent (thread-grade) cluster tokens: TokenService.requestConcurrentToken / releaseConcurrentToken ----
 * DefaultTokenService.java:66-85 → ConcurrentClusterFlowChecker.acquireConcurrentToken / releaseConcurrentToken
 * (srv/flow/ConcurrentClusterFlowChecker.java:48-101) over the loaded cluster flow rules: one nowCalls counter per
 * flowId (CurrentConcurrencyManager; kept for flowIds that survive a rule reload, ClusterFlowRuleManager.java:
 * 356-358) and a token table (TokenCacheNodeManager). Token ids are deterministic instead of UUID bits: an acquire
 * that passes gets id 1 + (number of concurrent requests this handle decided before it). */
#define SG_CONC_ACQUIRE 0
#define SG_CONC_RELEASE 1
#define SG_STATUS_RELEASE_OK      6   /* TokenResultStatus.RELEASE_OK      */
#define SG_STATUS_ALREADY_RELEASE 7   /* TokenResultStatus.ALREADY_RELEASE */
typedef struct sg_conc_req {
    int64_t  ts_ms;
    uint64_t token_id;           /* release: the token (0 = null → BAD_REQUEST); acquire: ignored          */
    uint32_t key;                /* acquire: rule index (or SG_KEY_BAD / SG_KEY_NO_RULE); release: ignored   */
    int32_t  acquire;            /* acquire: acquireCount (<= 0 → BAD_REQUEST)                              */
    uint32_t client;             /* acquire: client address id, 0 = null / "" (→ BAD_REQUEST)               */
    int32_t  kind;               /* SG_CONC_*                                                              */
} sg_conc_req;
typedef struct sg_conc_result {
    int32_t  status;             /* OK / BLOCKED / BAD_REQUEST / NO_RULE_EXISTS / RELEASE_OK / ALREADY_RELEASE */
    int32_t  reserved;
    uint64_t token_id;           /* acquire OK: the new token                                               */
} sg_conc_result;

/* Per-rule ClusterFlowConfig.clientOfflineTime / resourceTimeout (ms) for the token expiry, rule index order;
 * defaults 2000 / 2000 (ClusterFlowConfig.java); reset to the defaults by sg_load_flow_rules. */
int sg_conc_set_rule_timeouts(sg_handle* h, const int64_t* client_offline_ms, const int64_t* resource_timeout_ms,
                              uint32_t n);
/* A time-ordered batch of acquires and releases (DEVICE pointers; asynchronous on stream). */
int sg_conc_decide_batch(sg_handle* h, const sg_conc_req* req, uint64_t n, sg_conc_result* out, void* stream);
int sg_conc_decide_batch_host(sg_handle* h, const sg_conc_req* req, uint64_t n, sg_conc_result* out);
/* RegularExpireStrategy.clearToken (…/statistic/concurrent/expire/RegularExpireStrategy.java:94-123) at now_ms:
 * removes tokens whose client is offline past clientOfflineTime, or held more than 2 x resourceTimeout, and gives
 * their counts back. client_online[c] = ConnectionManager.isClientOnline(client c) (ids >= n_clients: offline).
 * Every token is examined (the reference stops after 1000 keys in ConcurrentHashMap order). *removed = count. */
int sg_conc_expire(sg_handle* h, int64_t now_ms, const uint8_t* client_online, uint32_t n_clients, uint64_t* removed);
/* nowCalls of rule `key` and the number of live tokens. */
int sg_conc_read_state(sg_handle* h, uint32_t key, int32_t* now_calls, uint64_t* live_tokens);

/* ---- local slot chain: StatisticSlot → FlowSlot (DefaultController) → DegradeSlot (circuit breakers) ---- */

/* DegradeRule (sentinel-core/.../slots/block/degrade/DegradeRule.java). */
#define SG_DEGRADE_RT              0
#define SG_DEGRADE_EXCEPTION_RATIO 1
#define SG_DEGRADE_EXCEPTION_COUNT 2
typedef struct sg_degrade_rule {
    int32_t grade;                /* SG_DEGRADE_*                                            */
    int32_t time_window_sec;      /* timeWindow: recovery timeout in seconds                  */
    double  count;                /* RT: max allowed RT (rounded); else ratio / count         */
    double  slow_ratio_threshold; /* RT only (default 1.0)                                    */
    int32_t min_request_amount;   /* default 5                                               */
    int32_t stat_interval_ms;     /* default 1000                                            */
} sg_degrade_rule;

/* One resource: its FlowRule with the default controller (limitApp "default", DIRECT strategy, read
 * from the resource's ClusterNode) and up to two DegradeRules, checked in order. sg_local_load_flow_rules
 * below replaces the flow rules with any number per resource. */
typedef struct sg_local_rule {
    double  flow_count;           /* FlowRule.count                                           */
    int32_t flow_grade;           /* 0 FLOW_GRADE_THREAD, 1 FLOW_GRADE_QPS, -1 no flow rule    */
    int32_t n_breakers;           /* 0..2                                                     */
    sg_degrade_rule breakers[2];
} sg_local_rule;

#define SG_LOCAL_ENTRY      0     /* SphU.entry(resource, count, prioritized)                 */
#define SG_LOCAL_EXIT       1     /* Entry.exit() of a passed entry                           */
#define SG_LOCAL_EXIT_ERROR 2     /* Entry.exit() after Tracer.traceEntry(business exception) */
typedef struct sg_local_event {
    int64_t  ts_ms;               /* TimeUtil time of the entry or exit                        */
    int64_t  create_ts;           /* exit: the entry's createTimestamp                         */
    uint32_t resource;            /* resource index | SG_KEY_PRIO (prioritized entry)          */
    int32_t  count;               /* acquireCount of the entry (also the exit's batchCount)    */
    int32_t  kind;                /* SG_LOCAL_*                                               */
    int32_t  origin;              /* Context origin: 0 = none (""), 1..n_origins = an origin id   */
} sg_local_event;

#define SG_LOCAL_PASS          0  /* passes; wait_ms > 0: after the rate limiter's sleep        */
#define SG_LOCAL_BLOCK_FLOW    1  /* FlowException                                            */
#define SG_LOCAL_BLOCK_DEGRADE 2  /* DegradeException                                         */
#define SG_LOCAL_PASS_WAIT     3  /* PriorityWaitException: passes after wait_ms              */
                                  /* 4: SG_LOCAL_BLOCK_PARAM (sg_slot_decide_batch, below)     */
typedef struct sg_local_result {
    int32_t status;               /* entries: SG_LOCAL_*; exits: 0                            */
    int32_t wait_ms;
} sg_local_result;

/* Node-wide statistic settings of the local chain (static properties in the reference). */
typedef struct sg_local_config {
    int32_t sample_count;         /* SampleCountProperty.SAMPLE_COUNT, default 2 (1..60)          */
    int32_t interval_ms;          /* IntervalProperty.INTERVAL, default 1000                      */
    int32_t occupy_timeout_ms;    /* OccupyTimeoutProperty.occupyTimeout, default 500              */
    int32_t cold_factor;          /* ColdFactorProperty.coldFactor (SentinelConfig, default 3; <= 1 → 3) */
} sg_local_config;

/* ---- the flow rules of the local chain: FlowRuleManager.loadRules → FlowRuleChecker.checkFlow ----
 * FlowRule (core/.../slots/block/flow/FlowRule.java) of one resource, with its traffic-shaping controller
 * (FlowRuleUtil.generateRater, FlowRuleUtil.java:132-149) and limitApp node selection
 * (FlowRuleChecker.selectNodeByRequesterAndStrategy, FlowRuleChecker.java:115-145). Origins are the caller's
 * dense ids for the Context origin strings (never "default" / "other"). */
#define SG_CONTROL_DEFAULT               0  /* DefaultController (THREAD rules always use it)        */
#define SG_CONTROL_WARM_UP               1  /* WarmUpController                                       */
#define SG_CONTROL_RATE_LIMITER          2  /* RateLimiterController                                  */
#define SG_CONTROL_WARM_UP_RATE_LIMITER  3  /* WarmUpRateLimiterController                            */
#define SG_LIMIT_APP_DEFAULT   0            /* limitApp "default": the resource's ClusterNode         */
#define SG_LIMIT_APP_OTHER   (-1)           /* limitApp "other": origins no rule of the resource names */
#define SG_STRATEGY_DIRECT     0            /* RuleConstant.STRATEGY_DIRECT: the node limitApp selects      */
#define SG_STRATEGY_RELATE     1            /* STRATEGY_RELATE: the ClusterNode of resource ref_resource     */
#define SG_STRATEGY_CHAIN      2            /* STRATEGY_CHAIN: the resource's DefaultNode of context ref_resource,
                                               only for entries in that context                             */
/* FlowRule.clusterMode with its ClusterFlowConfig (FlowRuleChecker.passClusterCheck :147-164). On a node that is
 * neither token client nor server (CLUSTER_NOT_STARTED, the default) pickClusterService() is null, so
 * fallbackToLocalOrPass (:166-175) applies. On a node whose embedded token server runs on this handle
 * (sg_local_set_cluster_state(SERVER), DefaultEmbeddedTokenServer.requestToken → DefaultTokenService, :46-51) a
 * cluster-mode rule requests a token for its flowId from the handle's own cluster flow state (sg_load_flow_rules,
 * the namespace limiter included) in the batch's event order, and applyTokenResult (:186-209) maps the answer: OK
 * passes, SHOULD_WAIT passes after wait_ms (added to the entry's wait), BLOCKED throws FlowException, and
 * NO_RULE_EXISTS / BAD_REQUEST / FAIL / TOO_MANY_REQUEST go to fallbackToLocalOrPass. */
#define SG_CLUSTER_MODE_OFF         0       /* a local rule                                                 */
#define SG_CLUSTER_MODE_FALLBACK    1       /* clusterMode, fallbackToLocalWhenFail: checked as a local rule  */
#define SG_CLUSTER_MODE_NO_FALLBACK 2       /* clusterMode without fallback: the rule is not activated (pass) */
#define SG_CLUSTER_MODE_INVALID   (-1)      /* clusterMode with an invalid ClusterFlowConfig
                                               (FlowRuleUtil.checkClusterField :197-215): ignored at load   */
typedef struct sg_local_flow_rule {
    uint32_t resource;            /* resource index (sg_local_load_rules order)                    */
    int32_t  grade;               /* 0 FLOW_GRADE_THREAD, 1 FLOW_GRADE_QPS                        */
    double   count;
    int32_t  control_behavior;    /* SG_CONTROL_*                                                 */
    int32_t  limit_app;           /* SG_LIMIT_APP_DEFAULT, SG_LIMIT_APP_OTHER or an origin id > 0   */
    int32_t  strategy;            /* SG_STRATEGY_*                                                */
    int32_t  warm_up_period_sec;  /* warmUpPeriodSec, default 10                                  */
    int32_t  max_queueing_ms;     /* maxQueueingTimeMs, default 500                               */
    int32_t  ref_resource;        /* RELATE: resource index; CHAIN: context id; < 0: refResource blank */
    int32_t  cluster_mode;        /* SG_CLUSTER_MODE_*                                            */
    int32_t  cluster_config;      /* the caller's id of the ClusterFlowConfig value (FlowRule.equals
                                     compares it; 0 = none)                                       */
    uint32_t cluster_key;         /* cluster mode on an embedded server: ClusterFlowConfig.flowId as a rule
                                     index of this handle's sg_load_flow_rules (SG_KEY_NO_RULE: the server
                                     has no rule for it, as sg_req.key)                           */
} sg_local_flow_rule;

/* ClusterStateManager state of the node (ClusterStateManager.java: CLUSTER_CLIENT 0, CLUSTER_SERVER 1,
 * CLUSTER_NOT_STARTED -1). NOT_STARTED and SERVER (the embedded token server on this handle, see above) are
 * decided on the device. In SERVER state the resources whose cluster-mode rules share a flowId, or name flowIds of
 * one limiter-enabled namespace, walk together in event order (one key group), and a local batch with such rules
 * must not precede the handle's flow batches in time (SG_E_TIME), nor they it. CLIENT sends tokens over the
 * network, which a batch cannot call in order: loading cluster-mode rules in CLIENT state (or entering it while they
 * are loaded) is SG_E_UNSUPPORTED, as is SERVER on a sharded handle (sg_set_shard) whose cluster
 * rules name a limiter-enabled namespace. The state is the handle's (one ClusterStateManager per node): it also decides
 * the cluster-mode ParamFlowRules of sg_pslot_load_rules, in sg_pslot_decide_batch and in the slot chain
 * (sg_slot_decide_batch). In SERVER state the resources whose cluster-mode param rules share a flowId (a cluster param
 * rule of sg_cparam_load_rules) or a limiter-enabled namespace walk as one key group, and the batch's events may not
 * precede the handle's cluster param batches in time (SG_E_TIME), nor they it. */
#define SG_CLUSTER_CLIENT        0
#define SG_CLUSTER_SERVER        1
#define SG_CLUSTER_NOT_STARTED (-1)
int sg_local_set_cluster_state(sg_handle* h, int32_t state);

/* Per-call timing of the last sg_flow_decide_batch (device time, HIP events on the call's stream). */
typedef struct sg_batch_stats {
    float    total_ms;          /* whole pipeline                                         */
    float    walk_ms;           /* per-flowId walk kernels                                */
    float    sort_ms;           /* key partition (radix sort)                             */
    uint64_t touched_keys;      /* distinct flowIds that received >= 1 request            */
    uint64_t long_segments;     /* flowIds walked by a whole wave                         */
    uint64_t skipped_ranges;    /* all-BLOCKED period tails the wave walker jumped over   */
} sg_batch_stats;

int         sg_create(const sg_config* cfg, sg_handle** out);
void        sg_destroy(sg_handle* h);
const char* sg_last_error(const sg_handle* h);

int sg_set_namespaces(sg_handle* h, const sg_namespace* ns, uint32_t n);

/* Marks the handle as one of `world` shards of a node's flowIds (flowIds hashed over the GPUs,
 * no collective on the decision path). GlobalRequestLimiter's per-namespace QPS limiter counts every request of
 * the namespace in node order (GlobalRequestLimiter.java:46-55, ClusterFlowChecker.allowProceed :45-51), which a
 * shard does not see on its own: with world > 1 and limiter-enabled namespaces every flow batch of the shard goes
 * through the exchange below — synchronous, pipelined (sg_flow_enqueue) and host-pipelined (sg_flow_submit) flow
 * batches and cluster param batches (sg_cparam_decide_batch) alike; a batch without an armed exchange is refused
 * with SG_E_UNSUPPORTED. */
int sg_set_shard(sg_handle* h, int32_t rank, int32_t world);

/* Sharded namespace limiter exchange (replaces GlobalRequestLimiter.tryPass's node-wide counting):
 *   1. sg_lim_arrivals (flow batches) / sg_lim_arrivals_param (cluster param batches, ClusterParamFlowChecker
 *      .java:43-45 shares the limiter): this shard's valid requests of limited namespaces per (limiter slot,
 *      millisecond), counts_out[slot * n_ms + (ts_ms - t_base)] (DEVICE, n_lim * n_ms uint32; slots = the
 *      limiter-enabled namespaces in sg_set_namespaces order). [t_base, t_base + n_ms) is node-wide and must hold
 *      every shard's limited requests of the node batch (SG_E_INVAL otherwise); n_ms <= 65536. `req` is device
 *      memory (or pinned host memory the device can read). Synchronous on `stream`; batches in flight on the
 *      pipeline go on.
 *   2. the node all-gathers the counts of its `world` shards (RCCL) into gathered[world][n_lim][n_ms] (DEVICE);
 *   3. sg_lim_exchange arms the handle's next flow or param batch with them: sg_flow_decide_batch / _host,
 *      sg_flow_enqueue, sg_flow_submit or sg_cparam_decide_batch / _host consumes it. The buffer must stay valid
 *      until that call returns (the pipelined calls copy it before returning).
 * The node's arrival order is (ts_ms, shard rank, position in the shard's batch). Every shard walks the same
 * per-100 ms node arrivals, so each keeps an identical replica of the namespace windows, and admits its request
 * iff its node-wide rank in the period is below the period's quota: the results equal one handle deciding the
 * merged batch. A shard with no requests in a node batch still calls sg_lim_exchange and sg_flow_decide_batch
 * with n = 0 (its replica advances). A shard batch rejected by an error (SG_E_TIME, SG_E_INVAL, SG_E_CAPACITY …)
 * still walks the armed node arrivals, so its replica stays equal to the other shards' (the node counted that shard's
 * requests as limiter arrivals; their flow decisions did not happen). */
int sg_lim_arrivals(sg_handle* h, const sg_req* req, uint64_t n, int64_t t_base, uint32_t n_ms, uint32_t* counts_out,
                    uint64_t counts_words, void* stream);
int sg_lim_arrivals_param(sg_handle* h, const sg_cparam_req* req, uint64_t n, int64_t t_base, uint32_t n_ms,
                          uint32_t* counts_out, uint64_t counts_words, void* stream);
int sg_lim_exchange(sg_handle* h, const uint32_t* gathered, uint64_t gathered_words, int64_t t_base, uint32_t n_ms);
/* The handle's limiter-slot count n_lim (limiter-enabled namespaces of sg_set_namespaces): counts_words of
 * sg_lim_arrivals must equal n_lim * n_ms and gathered_words of sg_lim_exchange world * n_lim * n_ms (SG_E_INVAL). */
int sg_lim_slots(const sg_handle* h, uint32_t* n_lim);
int sg_load_flow_rules(sg_handle* h, const sg_flow_rule* rules, uint32_t n);

/* Decide a batch. req/out are DEVICE pointers (HBM-resident); stream is a hipStream_t (NULL = default).
 * Requests must be ordered by (ts_ms, arrival); ts_ms must be >= 0 and >= every ts of earlier batches. */
int sg_flow_decide_batch(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, void* stream);

/* Same with HOST buffers (H2D + D2H included; synchronous). */
int sg_flow_decide_batch_host(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out);

/* Asynchronous host pipeline — what a token server's request loop calls: sg_flow_submit
 * enqueues H2D of req, the decision pipeline and D2H into out, and returns at once with a ticket; up to 3
 * batches are in flight (H2D of batch i+1 and D2H of batch i-1 overlap the compute of batch i; compute runs in
 * submission order, so batches must still be time-ordered). A 4th submit first completes the oldest batch.
 * req/out are HOST memory and must stay untouched until the ticket completes; allocate them with sg_host_alloc
 * (pinned) for the copies to run asynchronously. sg_flow_poll: 1 done and OK, 0 still running, < 0 that batch's
 * error (the batch was rejected, as sg_flow_decide_batch would); sg_flow_wait blocks and returns SG_OK or that
 * error. Every other call on the handle first completes the batches in flight. Ticket 0 (empty batch) is done.
 * Batches in flight are pipelined on the device: the front half of batch i+1 (validation, sort by flowId,
 * segment lists) runs beside the walkers of batch i, two batch workspaces alternating; a batch that fails the
 * cross-batch time check is still rejected as a whole (checked before its walkers). */
int   sg_flow_submit(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket);
/* The same pipeline for DEVICE buffers (ClusterFlowChecker over HBM-resident batches back to back: the
 * DefaultTokenService request loop at full rate): enqueues the batch and returns a ticket for
 * sg_flow_poll / sg_flow_wait. req/out must stay allocated and untouched until the ticket completes (each batch
 * in flight needs its own out buffer); up to 4 batches in flight (a 5th enqueue first completes the oldest). */
int   sg_flow_enqueue(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket);
int   sg_flow_poll(sg_handle* h, uint64_t ticket);
int   sg_flow_wait(sg_handle* h, uint64_t ticket);
void* sg_host_alloc(sg_handle* h, uint64_t bytes);   /* pinned (page-locked) host memory, NULL on failure */
void  sg_host_free(sg_handle* h, void* p);

/* Opt-in per-call timing (adds HIP events; off by default). */
int sg_enable_stats(sg_handle* h, int on);
int sg_get_stats(const sg_handle* h, sg_batch_stats* out);

/* Read one flowId's window: starts[sample_count] (INT64_MIN = never-created bucket),
 * counters[sample_count * SG_NUM_EVENTS], occupy[2] = {occupied PASS, occupied PASS_REQUEST}. */
int sg_flow_read_state(sg_handle* h, uint32_t key, int64_t* starts, int64_t* counters, int64_t* occupy);

/* Bulk copy of every flowId's window to / from HOST memory — the checkpoint of the cluster flow state (the
 * reference keeps it only in memory; SURVEY §5 "checkpoint / resume") and the parity harness's state dump.
 * ring: n_rules * stride * 8 int64 = per flowId `stride` buckets {start, PASS, BLOCK, PASS_REQUEST,
 * BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING} (start INT64_MIN = never-created slot; slots >= the
 * flow's sampleCount are unused and stay INT64_MIN), occ: n_rules * 2 int64 = {occupied PASS, occupied
 * PASS_REQUEST} (ClusterMetricLeapArray.occupyCounter). stride = the largest sampleCount of the loaded rules
 * (written to *stride; with ring == NULL only *stride is written). Import expects the same layout and the same
 * loaded rules; it is synchronous. */
int sg_flow_export_state(sg_handle* h, int64_t* ring, uint64_t ring_words, int64_t* occ, uint64_t occ_words,
                         int32_t* stride);
int sg_flow_import_state(sg_handle* h, const int64_t* ring, uint64_t ring_words, const int64_t* occ,
                         uint64_t occ_words);

/* Per-flowId {passQps, blockQps} at time now_ms (ClusterMetric.getAvg(PASS/BLOCK) without the
 * currentWindow side effect); out has 2*n_rules doubles, HOST memory. */
int sg_snapshot_metrics(sg_handle* h, int64_t now_ms, double* out, uint64_t cap);

/* Same into DEVICE memory (2*n_rules doubles, {passQps, blockQps} per flowId), asynchronous on `stream`:
 * the per-GPU input of the node-wide RCCL metric rollup. */
int sg_snapshot_metrics_device(sg_handle* h, int64_t now_ms, double* out_dev, uint64_t cap, void* stream);
/* sg_snapshot_metrics_device ordered after every batch enqueued so far on the pipeline (sg_flow_enqueue /
 * sg_flow_submit), without draining it: completes with the returned ticket (sg_flow_poll / sg_flow_wait). */
int sg_snapshot_metrics_enqueue(sg_handle* h, int64_t now_ms, double* out_dev, uint64_t cap, uint64_t* ticket);

/* Hot-parameter rules (replaces ParamFlowRuleManager.loadRules → ParameterMetric maps). A reload starts
 * every rule's value table empty. Hot items of a rule may be given in any order. */
int sg_param_load_rules(sg_handle* h, const sg_param_rule* rules, uint32_t n,
                        const sg_param_hot_item* hot, uint32_t n_hot);
/* passSingleValueCheck for a time-ordered batch: pass[i] = 1 admitted / 0 blocked. req/pass are DEVICE
 * pointers. Requests naming a rule index >= n pass (no rule). */
int sg_param_decide_batch(sg_handle* h, const sg_param_req* req, uint64_t n, int32_t* pass, void* stream);
int sg_param_decide_batch_host(sg_handle* h, const sg_param_req* req, uint64_t n, int32_t* pass);
/* State of (rule, value): returns flags (bit0 time counter, bit1 token counter; 0 = absent) or < 0. */
int sg_param_read_state(sg_handle* h, uint32_t rule, uint64_t value, int64_t* last_time, int64_t* tokens);

/* ---- pace controller ----
 *   sg_pace_load_rules    ← FlowRuleUtil.generateRater for CONTROL_BEHAVIOR_RATE_LIMITER rules
 *                           (core/.../flow/FlowRuleUtil.java:132-145): fresh controllers, latestPassedTime -1.
 *   sg_pace_decide_batch  ← RateLimiterController.canPass (RateLimiterController.java:46-91) for a
 *                           time-ordered batch; wait[i] = SG_PACE_BLOCKED or the sleep in ms (the caller
 *                           sleeps; the reference sleeps inside canPass). req/wait are DEVICE pointers.
 *   sg_pace_read_state    ← latestPassedTime.get() of a rule's controller. */
int sg_pace_load_rules(sg_handle* h, const sg_pace_rule* rules, uint32_t n);
int sg_pace_decide_batch(sg_handle* h, const sg_pace_req* req, uint64_t n, int32_t* wait, void* stream);
int sg_pace_decide_batch_host(sg_handle* h, const sg_pace_req* req, uint64_t n, int32_t* wait);
int sg_pace_read_state(sg_handle* h, uint32_t rule, int64_t* latest_passed_time);

/* ---- cluster hot-parameter tokens ----
 *   sg_cparam_load_rules    ← ClusterParamFlowRuleManager.loadRules → applyClusterParamRules
 *                             (…/flow/rule/ClusterParamFlowRuleManager.java:337-360): a surviving flowId keeps its
 *                             ClusterParamMetric; each rule owns an exact 2^capacity_log2 value table (0 = 2^16).
 *   sg_cparam_decide_batch  ← TokenService.requestParamToken(Long, int, Collection<Object>)
 *                             (DefaultTokenService.java:53-64 → ClusterParamFlowChecker.acquireClusterToken,
 *                             ClusterParamFlowChecker.java:42-87), time-ordered; values[] holds every request's
 *                             parameter values (u64; other types through the shim's value dictionary). Request i's
 *                             values are values[value_begin, value_begin + value_count): the ranges of the valid
 *                             requests must not overlap and must follow request order (value_begin increasing with
 *                             i, as a packer appending each request's values produces) — else SG_E_INVAL.
 *                             allowProceed goes through the namespace's QPS limiter, the same state the flow-token
 *                             path uses (GlobalRequestLimiter is per namespace): keep flow and param batches that
 *                             share a limiter in time order. A rejected batch changes no state.
 *   sg_cparam_last_rounds   fixed-point rounds the last batch needed (1 = single pass; requests with several values
 *                           may need more; max_rounds + 1 = it was decided serially). Tuning / tests.
 *   sg_cparam_read_sum      ← ClusterParamMetric.getSum(value) at now_ms (without currentWindow's side effect). */
int sg_cparam_load_rules(sg_handle* h, const sg_cparam_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                         uint32_t n_hot, int32_t capacity_log2);
int sg_cparam_decide_batch(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                           uint64_t n_values, sg_result* out, void* stream);
int sg_cparam_decide_batch_host(sg_handle* h, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                uint64_t n_values, sg_result* out);
int sg_cparam_read_sum(sg_handle* h, uint32_t rule, uint64_t value, int64_t now_ms, int64_t* sum);
int sg_cparam_last_rounds(const sg_handle* h, uint32_t* rounds);
/*   sg_cparam_top_values ← ClusterParamMetric.getTopValues(number) (…/metric/ClusterParamMetric.java:90-133), the
 *                          topParams of ClusterMetricNodeGenerator.paramToMetricNode (:88-104): per rule up to
 *                          `number` values with the largest window sums at now_ms (count / intervalSec), zero sums
 *                          excluded; ties by ascending value (the reference's order among equal counts is HashMap
 *                          order). values / qps: n_rules * number entries, HOST memory; counts[r] = entries of rule
 *                          r. Without currentWindow's side effect. Like sg_cparam_read_sum, exact for now_ms at or
 *                          after the latest decided request (the metricList task's current time): the device keeps a
 *                          ring per (rule, value), which equals the reference's bucket maps from that time on. */
int sg_cparam_top_values(sg_handle* h, int64_t now_ms, uint32_t number, uint64_t* values, double* qps, uint32_t* counts);

/* ---- local slot chain (the ProcessorSlot chain's statistic / flow / degrade slots, batched) ----
 *   sg_local_load_rules    ← FlowRuleManager.loadRules + DegradeRuleManager.loadRules for one resource each
 *                            (one DefaultController QPS/thread rule per resource, limitApp "default",
 *                            DIRECT strategy; up to two circuit breakers), with fresh StatisticNodes.
 *   sg_local_decide_batch  ← SphU.entry(resource, count, prioritized) → StatisticSlot.entry around
 *                            FlowSlot.checkFlow (DefaultController.canPass, DefaultController.java:49-76) and
 *                            DegradeSlot.performChecking (DegradeSlot.java:43-81); Entry.exit() →
 *                            StatisticSlot.exit (StatisticSlot.java:124-165) + DegradeSlot.exit →
 *                            onRequestComplete. Events in (timestamp, arrival) order; exits only for entries
 *                            that passed (the caller holds no Entry for a blocked one).
 * Event/result types: sg_local_event / sg_local_result above. */
int sg_local_load_rules(sg_handle* h, const sg_local_config* cfg, const sg_local_rule* rules, uint32_t n);
int sg_local_decide_batch(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out, void* stream);
int sg_local_decide_batch_host(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out);
/* sg_local_decide_batch on the device pipeline (DEVICE buffers, like sg_flow_enqueue): enqueues the batch and
 * returns at once with a ticket for sg_local_poll / sg_local_wait (same meaning as sg_flow_poll / _wait; tickets
 * are shared with the flow pipeline). The front half of batch i+1 (validation, sort by resource, segment and exit
 * lists) runs beside the walkers of batch i; the walkers run in enqueue order, so batches must be time-ordered as
 * for sg_local_decide_batch, and a batch older than the one before is rejected as a whole (checked before its
 * walkers). ev/out must stay allocated and untouched until the ticket completes (each batch in flight needs its
 * own out buffer); up to 4 batches in flight. A batch the pipeline does not take — origin or context nodes tracked,
 * the embedded token server, or rules loaded since the last batch — first completes the batches in flight and is
 * decided synchronously (its status still comes with its ticket). Every other call on the handle first completes
 * the batches in flight. */
int sg_local_enqueue(sg_handle* h, const sg_local_event* ev, uint64_t n, sg_local_result* out, uint64_t* ticket);
int sg_local_poll(sg_handle* h, uint64_t ticket);
int sg_local_wait(sg_handle* h, uint64_t ticket);
/* Resource state: second window [S][8] {start, PASS, BLOCK, EXCEPTION, SUCCESS, RT, OCCUPIED_PASS, minRt},
 * borrow array [S][2] {start, PASS}, minute window [60][8] (start INT64_MIN = never created; counters of
 * such slots read 0), head[14] = {curThreadNum, then per breaker: state, nextRetry, stat start, slow/error
 * count, total count, 0}. */
int sg_local_read_state(sg_handle* h, uint32_t res, int64_t* second, int64_t* borrow, int64_t* minute, int64_t* head);
/*   sg_local_load_flow_rules ← FlowRuleManager.loadRules (FlowRuleManager.java, FlowRuleUtil.buildFlowRuleMap
 *                              :83-130): replaces every resource's flow rules. Invalid rules are ignored as the
 *                              reference ignores them (FlowRuleUtil.isValidRule :167-251), duplicates are dropped
 *                              (its HashSet), and each resource's rules are stably sorted by FlowRuleComparator
 *                              (FlowRuleComparator.java:30-55: local rules before cluster-mode ones, specific /
 *                              other limitApps before "default"). Fresh controllers (warm-up tokens 0,
 *                              latestPassedTime -1); resource statistics are kept. Returns the number of rules kept
 *                              (>= 0) or an error.
 *                              n_origins: the largest origin id events may carry; n_contexts: context ids events may
 *                              carry are 0 .. n_contexts - 1 (sg_slot_ext.context; 0 when no ext). Origin and context
 *                              ids are the caller's dense ids of the Context origin / name strings and must keep
 *                              their meaning across loads (neither count may shrink).
 *                              Nodes besides the ClusterNodes, created at the first event that needs them whatever
 *                              the rules say, as the reference does, and kept for the life of the resources (rule
 *                              reloads keep them): every event from an origin (id > 0) updates the resource's origin
 *                              StatisticNode (ClusterBuilderSlot.java:99-102 → ClusterNode.getOrCreateOriginNode), and,
 *                              with context tracking on (n_contexts >= 1), every event updates the resource's DefaultNode
 *                              of its context (NodeSelectorSlot.java:156-170). Nodes live in a device pool that grows
 *                              with the (resource, origin / context) pairs seen. Context tracking (needed by CHAIN rules,
 *                              whose context ids must be < n_contexts) starts before the first batch: raising n_contexts
 *                              from 0 after a batch is SG_E_UNSUPPORTED (the DefaultNodes would miss earlier entries).
 *                              With it, every resource is walked by the full-chain walker. A RELATE rule joins its
 *                              resource and ref_resource into one key group walked in event order (the read of
 *                              another resource's ClusterNode, FlowRuleChecker.selectReferenceNode :96-112); a
 *                              resource never entered has no ClusterNode yet (ClusterBuilderSlot), and the rule
 *                              then passes.
 *   sg_local_read_origin_state  ← that origin node: same layout as sg_local_read_state (head[0] = curThreadNum);
 *                              returns 1 when the node exists, 0 when no event created it yet (the dumps of an empty
 *                              node).
 *   sg_local_read_context_state ← the DefaultNode of (resource, context): same layout and return values.
 *   sg_local_read_controller   ← the controller of input rule i: {storedTokens, lastFilledTime, latestPassedTime};
 *                              SG_E_INVAL for an ignored rule. */
int sg_local_load_flow_rules(sg_handle* h, const sg_local_flow_rule* rules, uint32_t n, int32_t n_origins,
                             int32_t n_contexts);

/* ---- the whole slot chain in one batch (the ProcessorSlot chain's SPI order, Constants.java:76-83 and
 * ParamFlowSlot @Spi(order = -3000)): StatisticSlot.entry around ParamFlowSlot → FlowSlot → DegradeSlot.
 *   sg_slot_decide_batch ← SphU.entry(resource, count, prioritized, args...) / Entry.exit(count, args...) for a
 *     time-ordered batch. Per entry: ParamFlowSlot.checkFlow (the param rules sg_pslot_load_rules loaded for the
 *     resource, args of the event; args_null or no rules: nothing) — a ParamFlowException ends the chain
 *     (SG_LOCAL_BLOCK_PARAM, wait_ms = the index of the param rule that threw); FlowSlot (the flow rules above);
 *     DegradeSlot; then StatisticSlot (StatisticSlot.java:55-122): a pass raises curThreadNum and PASS on the
 *     ClusterNode, the origin node and the DefaultNode and runs ParamFlowStatisticEntryCallback.onPass (the param
 *     thread counts of the args, ParameterMetric.addThreadCount); a PriorityWaitException raises the thread counts
 *     and runs onPass; any BlockException — ParamFlowException included — adds BLOCK to those nodes. Exit
 *     (StatisticSlot.exit :124-165, passed entries only): RT / success / exception and curThreadNum on the nodes,
 *     ParamFlowStatisticExitCallback (decreaseThreadCount of the exit's args), DegradeSlot.exit.
 *     ext[i] (nullable: every event in context 0 with null args) carries the event's context and arguments; args,
 *     values and ext are DEVICE pointers like ev and out. sg_local_decide_batch = this call with ext = NULL. */
typedef struct sg_slot_ext {
    uint32_t context;             /* Context name id (0 .. n_contexts - 1); CHAIN rules select by it              */
    uint32_t arg_begin;           /* the event's args: args[arg_begin .. + arg_count)                           */
    uint32_t arg_count;
    int32_t  args_null;           /* 1: Object[] args is null (ParamFlowSlot.checkFlow returns at once)          */
} sg_slot_ext;
#define SG_LOCAL_BLOCK_PARAM   4  /* ParamFlowException (result wait_ms: the index of the param rule that threw) */
int sg_slot_decide_batch(sg_handle* h, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
                         const sg_pslot_arg* args, uint64_t n_args, const uint64_t* values, uint64_t n_values,
                         sg_local_result* out, void* stream);
int sg_slot_decide_batch_host(sg_handle* h, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
                              const sg_pslot_arg* args, uint64_t n_args, const uint64_t* values, uint64_t n_values,
                              sg_local_result* out);
int sg_local_read_context_state(sg_handle* h, uint32_t res, int32_t context, int64_t* second, int64_t* borrow,
                                int64_t* minute, int64_t* head);

/* ---- metric snapshots ----
 *   sg_local_metrics ← MetricTimerListener.run (core/.../node/metric/MetricTimerListener.java:40-69) over every
 *                      resource's ClusterNode: StatisticNode.metrics() (StatisticNode.java:116-133) at now_ms — the
 *                      minute window's buckets (ArrayMetric.details, :156-204, with currentWindow's side effect) newer
 *                      than the node's lastFetchTime and older than now's second, non-empty; lastFetchTime advances.
 *                      Rows sorted by (timestamp, resource) into HOST memory; *n_rows = the number of rows (with
 *                      SG_E_CAPACITY and no side effect when cap is too small). The host formats them as metrics.log
 *                      lines (MetricNode.toFatString, MetricNode.java:213-229; sentinel_amd/metrics.py). After
 *                      the resources, Constants.ENTRY_NODE (__total_inbound_traffic__, MetricTimerListener.java:46):
 *                      rows with resource = SG_ENTRY_NODE_RESOURCE, the sums of the inbound resources' buckets of each
 *                      second (StatisticSlot adds every EntryType.IN entry / exit to it, StatisticSlot.java:71-75,
 *                      :139-141) less their occupied passes (StatisticNode.addOccupiedPass raises only the selected
 *                      node's PASS, StatisticNode.java:333-336), occupied_pass_qps 0, with the ENTRY_NODE's own
 *                      lastFetchTime. Exact when rows are fetched at least once a minute and at a time not behind the
 *                      latest decided event, as MetricTimerListener does (a resource's bucket of a second outlives
 *                      the ENTRY_NODE's by up to the minute window).
 *   sg_local_set_entry_types ← the EntryType of each resource's SphU.entry calls (1 = IN; default OUT, as
 *                      SphU.entry(name)). */
#define SG_ENTRY_NODE_RESOURCE 0xFFFFFFFFu
typedef struct sg_metric_node {
    int64_t  timestamp;
    int64_t  pass_qps, block_qps, success_qps, exception_qps;
    int64_t  rt;                  /* rt / success when success != 0, else the raw rt sum (ArrayMetric.fromBucket) */
    int64_t  occupied_pass_qps;
    uint32_t resource;
    int32_t  concurrency;         /* 0, as fromBucket leaves it */
} sg_metric_node;
int sg_local_metrics(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows);
/* sg_local_metrics with `rt` as the bucket's raw sum in every row (not divided by success): one GPU's share of a node's
 * rows, which the node's rollup merges (sentinel_amd/cluster.py LocalMetricRollup: the ENTRY_NODE rows of the same
 * second are summed over the GPUs, then rt = Σrt / Σsuccess), with the same side effects as sg_local_metrics. */
int sg_local_metrics_raw(sg_handle* h, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n_rows);
/* sg_local_metrics_raw into DEVICE memory (d_out on the handle's device), rows unsorted, complete on return: the
 * node's device rollup (cluster.DeviceLocalMetricRollup: RCCL all_gather of the rows, ENTRY_NODE sums and the
 * (timestamp, resource) order on the GPU). Same side effects, same SG_E_CAPACITY contract. */
int sg_local_metrics_raw_device(sg_handle* h, int64_t now_ms, sg_metric_node* d_out, uint64_t cap, uint64_t* n_rows);
/* sg_local_metrics_raw_device enqueued, no host wait: the rows of now_ms after every local batch enqueued so far
 * (sg_local_enqueue) and after the caller's earlier work on `stream`, before every batch enqueued later; `stream` is
 * made to wait for them. *d_count (DEVICE memory) receives the row count; when it exceeds cap, no row is written and
 * nothing changes (the listener's state included). A cap of at least 59 rows per resource + 60 skips the counting
 * pass. Rows unsorted, as sg_local_metrics_raw_device. */
int sg_local_metrics_raw_enqueue(sg_handle* h, int64_t now_ms, sg_metric_node* d_out, uint64_t cap, uint64_t* d_count,
                                 void* stream);
/* The local chain sharded over a node's GPUs (one process per GPU): every GPU loads the same rules and
 * decides the entries and exits of the resources it owns — owner[r] = splitmix64(g(r)) mod world, g(r) the smallest
 * resource of r's key group (RELATE references; on an embedded token server also the resources sharing a flowId or
 * a limited namespace), so every state a decision reads (ClusterNode, origin and context nodes, breakers, flow
 * controllers, param tables) lives on one GPU. The caller routes each event to owner[event.resource] in arrival order;
 * the per-GPU metric rows merge by sg_local_metrics_raw. SG_E_UNSUPPORTED: an embedded token server with namespace
 * limiters (its GlobalRequestLimiter sees the whole node). Replaces nothing in the reference (one JVM, one chain):
 * the node-level deployment of StatisticSlot / FlowSlot / DegradeSlot. */
int sg_local_owners(sg_handle* h, uint32_t world, uint32_t* owner, uint32_t n);
int sg_local_set_entry_types(sg_handle* h, const uint8_t* inbound, uint32_t n);
int sg_local_read_origin_state(sg_handle* h, uint32_t res, int32_t origin, int64_t* second, int64_t* borrow,
                               int64_t* minute, int64_t* head);
int sg_local_read_controller(sg_handle* h, uint32_t rule, int64_t* state3);

/* ---- the node handle: one token server over G shard handles (SURVEY §8(b) "multi-GPU fan-out is internal to the
 * handle", §8(e) flowIds hashed over the GPUs) ----
 * The reference serves every flowId from one TokenService (DefaultTokenService.requestToken, DefaultTokenService
 * .java:39-50) for all Netty workers (NettyTransportServer.java:53-54). A node handle owns G shard handles (shard g on
 * devices[g]; one device may hold several shards) and a front handle on devices[0]. A node batch in caller order is
 * validated and passed through the namespace limiters by the front (GlobalRequestLimiter over the whole batch in
 * caller order: the node's arrival order), split by owner — splitmix64(flowId) mod G — with a stable device multisplit,
 * decided by every shard concurrently on its own stream (slices copied peer to peer for shards on other devices),
 * and gathered back into caller order: the results equal one handle deciding the batch.
 *   sg_node_create          ← G shards (1..64) on devices[0..G-1], each with cfg (max_batch per shard and node)
 *   sg_node_set_namespaces  ← sg_set_namespaces (the front keeps the limiters)
 *   sg_node_load_flow_rules ← sg_load_flow_rules for the node's rule set (keys = rule indices of this array);
 *                             a surviving flowId keeps its owner, hence its ClusterMetric
 *   sg_node_flow_decide_batch(_host) ← sg_flow_decide_batch over the node (device buffers on devices[0] / host)
 *   sg_node_flow_enqueue / _poll / _wait ← sg_flow_enqueue / _poll / _wait over the node (pipelined)
 *   sg_node_flow_read_state, sg_node_snapshot_metrics ← per node rule, as the single-handle calls
 *   sg_node_shard_of        owner shard and local rule index of node rule `key` */
typedef struct sg_node sg_node;
int         sg_node_create(const sg_config* cfg, const int32_t* devices, uint32_t n_shards, sg_node** out);
void        sg_node_destroy(sg_node* nd);
const char* sg_node_last_error(const sg_node* nd);
int         sg_node_set_namespaces(sg_node* nd, const sg_namespace* ns, uint32_t n);
int         sg_node_load_flow_rules(sg_node* nd, const sg_flow_rule* rules, uint32_t n);
int         sg_node_flow_decide_batch(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out, void* stream);
int         sg_node_flow_decide_batch_host(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out);
/* sg_flow_enqueue / _poll / _wait over the node (DEVICE buffers on devices[0], same ticket meaning): with every shard
 * on devices[0] the node batches are pipelined — the front's validation, limiter and routing of batch i+1 and the
 * shards' sorts run beside the shards' walkers of batch i, two node workspaces alternating; the host waits only for
 * the front of the batch it enqueues (the slice sizes). Batches must be time-ordered; a batch the front refuses
 * (validation, time order) reaches no shard and its ticket carries the error. With shards on other devices a node
 * batch is decided synchronously and its status kept for the ticket. Every other sg_node_* call first completes
 * the batches in flight. */
int         sg_node_flow_enqueue(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket);
int         sg_node_flow_poll(sg_node* nd, uint64_t ticket);
int         sg_node_flow_wait(sg_node* nd, uint64_t ticket);
int         sg_node_flow_read_state(sg_node* nd, uint32_t key, int64_t* starts, int64_t* counters, int64_t* occupy);
int         sg_node_snapshot_metrics(sg_node* nd, int64_t now_ms, double* out, uint64_t cap);
int         sg_node_shard_of(const sg_node* nd, uint32_t key, uint32_t* shard, uint32_t* local_key);
/* The node's front handle (devices[0]; owned by the node, not to be destroyed): it holds the namespace limiters, so
 * cluster param tokens whose rules sit under an enabled GlobalRequestLimiter (ClusterParamFlowChecker.java:43-45
 * shares the limiter in caller order) are decided on it with sg_cparam_*; every other param and concurrent token
 * goes through the sharded sg_node_cparam_* / sg_node_conc_* below. Its own sg_flow_* entry points must not be
 * called. */
sg_handle*  sg_node_front(sg_node* nd);
/* Cluster param and concurrent tokens sharded over the node (DefaultTokenService.requestParamToken /
 * requestConcurrentToken / releaseConcurrentToken, DefaultTokenService.java:53-85): a param rule (with its hot items)
 * lives on the shard owning its flowId; a concurrent acquire goes to the owner of its flow rule's flowId, a release
 * to the shard its token id names (node token id = (shard token id - 1) * G + shard + 1). A node batch in caller order
 * is checked for time order and the value-range contract of sg_cparam_decide_batch over the whole batch (the valid
 * requests' ranges inside the value array, in request order, not overlapping) on devices[0] (refused whole, nothing
 * decided), split stably by owner
 * with one 8-bit radix pass, decided shard by shard in the node's order and gathered back: the statuses, counters and
 * metrics equal one handle deciding the batch; token ids are the node's own (unique, as the reference's are only
 * unique). Param batches whose rules name a namespace with the GlobalRequestLimiter enabled are refused
 * (SG_E_UNSUPPORTED): allowProceed (ClusterParamFlowChecker.java:43-45) takes the limiter in caller order, which the
 * front handle serves (sg_node_front). Device buffers are on devices[0]; the _host forms take host buffers.
 *   sg_node_cparam_load_rules      ← sg_cparam_load_rules for the node's param rule set (rule = index of this array)
 *   sg_node_cparam_read_sum / _top_values ← per node param rule, as the single-handle calls
 *   sg_node_conc_*                 ← sg_conc_* with node flow rule indices (timeouts per node rule) */
int sg_node_cparam_load_rules(sg_node* nd, const sg_cparam_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                              uint32_t n_hot, int32_t capacity_log2);
int sg_node_cparam_decide_batch(sg_node* nd, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                uint64_t n_values, sg_result* out, void* stream);
int sg_node_cparam_decide_batch_host(sg_node* nd, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                     uint64_t n_values, sg_result* out);
int sg_node_cparam_read_sum(sg_node* nd, uint32_t rule, uint64_t value, int64_t now_ms, int64_t* sum);
int sg_node_cparam_top_values(sg_node* nd, int64_t now_ms, uint32_t number, uint64_t* values, double* qps,
                              uint32_t* counts);
int sg_node_conc_set_rule_timeouts(sg_node* nd, const int64_t* client_offline_ms, const int64_t* resource_timeout_ms,
                                   uint32_t n);
int sg_node_conc_decide_batch(sg_node* nd, const sg_conc_req* req, uint64_t n, sg_conc_result* out, void* stream);
int sg_node_conc_decide_batch_host(sg_node* nd, const sg_conc_req* req, uint64_t n, sg_conc_result* out);
int sg_node_conc_expire(sg_node* nd, int64_t now_ms, const uint8_t* client_online, uint32_t n_clients, uint64_t* removed);
int sg_node_conc_read_state(sg_node* nd, uint32_t key, int32_t* now_calls, uint64_t* live_tokens);

/* ---------- token-server wire codec ----------
 * The default token server frames every message with a 2-byte big-endian length
 * (LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) / LengthFieldPrepender(2),
 * srv/server/NettyTransportServer.java:89-92). A request payload is [i32 xid][u8 type][data]
 * (DefaultRequestEntityDecoder.java:36-58); MSG_TYPE_FLOW data is [i64 flowId][i32 count][bool priority?]
 * (FlowRequestDataDecoder.java:31-43). A response frame is [u16 len = 14][i32 xid][u8 type][u8 status]
 * [i32 remaining][i32 waitInMs] (DefaultResponseEntityWriter.java:32-51, FlowResponseDataWriter.java:28-32),
 * all big-endian (Netty ByteBuf). The batching front-end that a Netty handler feeds appends each frame's
 * payload (length prefix stripped) to one buffer and records where it starts.
 *
 * sg_codec_decode_flow: payload bytes + offsets[n + 1] (frame i = [offsets[i], offsets[i+1])) + arrival
 * timestamps → sg_req records for sg_flow_decide_batch (flowId → rule index through the handle's device
 * table: unknown → SG_KEY_NO_RULE, flowId <= 0 → SG_KEY_BAD, as DefaultTokenService.requestToken would
 * answer), the xid of every frame and its kind (SG_FRAME_*). Frames that are not decodable flow requests
 * get key SG_KEY_BAD and acquire 0 (a harmless BAD_REQUEST slot in the batch). All pointers are device
 * memory (payload 4-byte aligned); the call is asynchronous on `stream`. offsets must be non-decreasing and
 * offsets[n] <= the payload's size, and the payload allocation must reach the next 4-byte multiple past offsets[n]
 * (staged loads read whole aligned words; hipMalloc'd buffers always do): the kernel does not know the payload's
 * size, so an offset past it is read as given. A frame whose end lies before its start decodes as SG_FRAME_SHORT.
 * sg_codec_encode_flow: one 16-byte response frame per request at frames_out + 16 * i (zero-filled for
 * frames whose kind is not SG_FRAME_FLOW: the Java server sends nothing for those). */
#define SG_MSG_TYPE_PING       0
#define SG_MSG_TYPE_FLOW       1
#define SG_MSG_TYPE_PARAM_FLOW 2
#define SG_FRAME_FLOW     0   /* a flow token request, decoded                                          */
#define SG_FRAME_SHORT    1   /* fewer than 5 bytes: DefaultRequestEntityDecoder returns null            */
#define SG_FRAME_NO_DATA  2   /* MSG_TYPE_FLOW without a decodable body (fewer than 12 data bytes)       */
#define SG_FRAME_OTHER    3   /* another message type (ping, param, concurrent): the host's own path     */
#define SG_RESPONSE_FRAME_BYTES 16
int sg_codec_decode_flow(sg_handle* h, const uint8_t* payload, const uint32_t* offsets, const int64_t* ts_ms,
                         uint64_t n, sg_req* req_out, int32_t* xid_out, uint8_t* kind_out, void* stream);
int sg_codec_encode_flow(sg_handle* h, const int32_t* xid, const uint8_t* kind, const sg_result* res, uint64_t n,
                         uint8_t* frames_out, void* stream);

/* ---------- Envoy rate-limit service ----------
 * SentinelEnvoyRlsServiceImpl.shouldRateLimit (sentinel-cluster/sentinel-cluster-server-envoy-rls/.../service/v3/
 * SentinelEnvoyRlsServiceImpl.java:34-85) for a time-ordered batch of n RateLimitRequests on a handle whose flow
 * rules were loaded as the RLS checker reads them (SimpleClusterFlowChecker.acquireClusterToken, flow/
 * SimpleClusterFlowChecker.java:33-65: GLOBAL threshold count · exceedCount, no namespace limiter, no prioritized
 * occupy). Request j is served at ts_ms with acquireCount = hits_addend (0 → 1) over its descriptors
 * desc_rule[desc_begin, desc_begin + desc_count): a descriptor's rule index (the caller resolves
 * EnvoySentinelRuleConverter.generateFlowId over domain + entries on its side), or -1 when it has no rule. Every
 * descriptor is one token request, all of a batch in one device batch, in order.
 *   overall[j]  SG_RLS_OK / SG_RLS_OVER_LIMIT (any descriptor not OK), or SG_RLS_ERROR when hits_addend < 0
 *               (responseObserver.onError, :36-40; its descriptors are not requested and get code 0)
 *   status[d]   code (SG_RLS_OK when the result is OK or the rule is missing, :55-58, else SG_RLS_OVER_LIMIT),
 *               and for a descriptor with a rule: limit_remaining = the TokenResult's remaining and
 *               requests_per_unit = (int) rule.getCount() (:67-73), has_rule = 1.
 * A descriptor whose rule is not GLOBAL or lies in a namespace with a limiter (the cluster path would apply them,
 * SimpleClusterFlowChecker does not) is SG_E_UNSUPPORTED, more descriptors than max_batch SG_E_CAPACITY: both
 * before any state change. */
#define SG_RLS_OK          1   /* envoy.service.ratelimit.v3.RateLimitResponse.Code.OK         */
#define SG_RLS_OVER_LIMIT  2   /* ... Code.OVER_LIMIT                                          */
#define SG_RLS_ERROR      (-1) /* hits_addend < 0: the call fails                               */
typedef struct {
    int64_t  ts_ms;        /* TimeUtil.currentTimeMillis() when the call is served */
    int32_t  hits_addend;  /* RateLimitRequest.hits_addend                         */
    uint32_t desc_begin;
    uint32_t desc_count;
    uint32_t pad;
} sg_rls_request;          /* 24 bytes */
typedef struct {
    int32_t code;
    int32_t limit_remaining;
    int32_t requests_per_unit;
    int32_t has_rule;
} sg_rls_status;           /* 16 bytes */
int sg_rls_should_rate_limit(sg_handle* h, const sg_rls_request* req, uint32_t n, const int32_t* desc_rule,
                             uint64_t n_desc, int32_t* overall, sg_rls_status* status);

/* Testing aid: copy an internal buffer of the last batch to host memory.
 * what: 0 = records (request order, u64), 1 = records sorted by flowId, 2 = window-period table
 * (u32 [8][65536]), 3 = first period per window length (i64[8]), 4 = periods per window length (u32[8]). */
int sg_debug_copy(sg_handle* h, int what, void* dst, uint64_t bytes);

/* Library build identification (architecture the kernels were compiled for). */
const char* sg_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* SENTINEL_GPU_H */
