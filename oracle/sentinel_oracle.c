/*
 * sentinel_oracle.c — TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h).
 *
 * Sequential, explicit-time C restatement of Sentinel 1.8.5's sliding-window statistics and
 * cluster flow checks. Every function cites the Java it follows; paths abbreviated as in SURVEY.md:
 *   core/ = sentinel-core/src/main/java/com/alibaba/csp/sentinel/
 *   srv/  = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/
 * Built with -fwrapv so signed overflow wraps exactly like Java long/int arithmetic.
 */
#include "sentinel_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ===================================================================================== */
/* Java numeric semantics                                                                */
/* ===================================================================================== */

/* JLS §5.1.3 narrowing double → int: NaN → 0, saturate at the int range, else truncate. */
int32_t or_d2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

/* JLS §5.1.3 narrowing double → long. */
int64_t or_d2l(double x) {
    if (x != x) return 0;
    if (x >= 9223372036854775807.0) return INT64_MAX;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

/* java.lang.Math.round(double) as implemented since JDK 7u (exact floor(x + 1/2)). */
int64_t or_math_round(double a) {
    int64_t bits;
    memcpy(&bits, &a, 8);
    int64_t biased_exp = (bits & 0x7FF0000000000000LL) >> 52;
    int64_t shift = (52 - 1 + 1023) - biased_exp;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000FFFFFFFFFFFFFLL) | 0x0010000000000000LL;
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return or_d2l(a);
}

/* ===================================================================================== */
/* LeapArray family                                                                      */
/* ===================================================================================== */

#define OR_MAX_EV 7
#define OR_STAT_MAX_RT 5000 /* SentinelConfig.DEFAULT_STATISTIC_MAX_RT, core/config/SentinelConfig.java:69 */

typedef struct or_bucket {
    int64_t start;
    int64_t c[OR_MAX_EV];
    int64_t min_rt;
} or_bucket;

struct or_leap {
    int kind;
    int S, wl, interval;   /* sampleCount, windowLengthInMs, intervalInMs (LeapArray.java:43-46) */
    double isec;           /* intervalInSecond = intervalInMs / 1000.0 (LeapArray.java:68)        */
    uint8_t* present;      /* AtomicReferenceArray slot != null                                   */
    or_bucket* b;
    or_bucket detached;    /* LeapArray.java:197-199: "should not go through here"                */
    struct or_leap* borrow;            /* OccupiableBucketLeapArray.borrowArray                   */
    int64_t occ[OR_MAX_EV];            /* ClusterMetricLeapArray.occupyCounter                    */
    int has_occupied;                  /* ClusterMetricLeapArray.hasOccupied                      */
};

static or_bucket* slot_ptr(or_leap* l, int slot) {
    return slot == -2 ? &l->detached : &l->b[slot];
}
static const or_bucket* slot_cptr(const or_leap* l, int slot) {
    return slot == -2 ? &l->detached : &l->b[slot];
}

or_leap* or_leap_new(int kind, int sample_count, int interval_ms) {
    /* LeapArray(int sampleCount, int intervalInMs), base/LeapArray.java:61-72 */
    if (sample_count <= 0 || interval_ms <= 0 || interval_ms % sample_count != 0) return NULL;
    or_leap* l = (or_leap*)calloc(1, sizeof(or_leap));
    l->kind = kind;
    l->S = sample_count;
    l->wl = interval_ms / sample_count;
    l->interval = interval_ms;
    l->isec = interval_ms / 1000.0;
    l->present = (uint8_t*)calloc((size_t)sample_count, 1);
    l->b = (or_bucket*)calloc((size_t)sample_count, sizeof(or_bucket));
    for (int i = 0; i < sample_count; i++) l->b[i].start = INT64_MIN;
    l->detached.start = INT64_MIN;
    if (kind == OR_LEAP_OCCUPIABLE) {
        /* OccupiableBucketLeapArray.java:33-37 */
        l->borrow = or_leap_new(OR_LEAP_FUTURE, sample_count, interval_ms);
    }
    return l;
}

void or_leap_free(or_leap* l) {
    if (!l) return;
    if (l->borrow) or_leap_free(l->borrow);
    free(l->present);
    free(l->b);
    free(l);
}

or_leap* or_leap_borrow(or_leap* l) { return l->borrow; }
double or_leap_interval_sec(const or_leap* l) { return l->isec; }

/* LeapArray.isWindowDeprecated(long, WindowWrap), base/LeapArray.java:270-272;
 * FutureBucketLeapArray overrides it, metric/occupy/FutureBucketLeapArray.java:49-52. */
static int is_deprecated(const or_leap* l, int64_t t, const or_bucket* w) {
    if (l->kind == OR_LEAP_FUTURE) return t >= w->start;
    return t - w->start > l->interval;
}

/* LeapArray.getWindowValue(long), base/LeapArray.java:244-257 + WindowWrap.isTimeInWindow :87-89 */
int or_leap_window_value(const or_leap* l, int64_t t) {
    if (t < 0) return -1;
    int idx = (int)((t / l->wl) % l->S);
    if (!l->present[idx]) return -1;
    const or_bucket* w = &l->b[idx];
    if (!(w->start <= t && t < w->start + l->wl)) return -1;
    return idx;
}

static void zero_counters(or_bucket* w) {
    for (int e = 0; e < OR_MAX_EV; e++) w->c[e] = 0;
    w->min_rt = OR_STAT_MAX_RT; /* MetricBucket.initMinRt, data/MetricBucket.java:52-54 */
}

/* newEmptyBucket(timeMillis) per subclass. */
static void new_empty_bucket(or_leap* l, or_bucket* w, int64_t t) {
    zero_counters(w);
    if (l->kind == OR_LEAP_OCCUPIABLE) {
        /* OccupiableBucketLeapArray.newEmptyBucket, :40-48: MetricBucket.reset(borrowBucket) copies
         * all 6 counters (data/MetricBucket.java:43-50); minRt re-initialised. */
        int bs = or_leap_window_value(l->borrow, t);
        if (bs >= 0) {
            for (int e = 0; e < OR_M_NUM; e++) w->c[e] = l->borrow->b[bs].c[e];
        }
    }
}

/* ClusterMetricLeapArray.transferOccupyToBucket, srv/flow/statistic/metric/ClusterMetricLeapArray.java:56-71 */
static void cluster_transfer_occupy(or_leap* l, or_bucket* w) {
    if (l->has_occupied) {
        w->c[SG_EV_OCCUPIED_PASS] += l->occ[SG_EV_PASS]; /* transferOccupiedCount (sum, no reset) */
        w->c[SG_EV_PASS] += l->occ[SG_EV_PASS];          /* transferOccupiedThenReset            */
        l->occ[SG_EV_PASS] = 0;
        w->c[SG_EV_PASS_REQUEST] += l->occ[SG_EV_PASS_REQUEST];
        l->occ[SG_EV_PASS_REQUEST] = 0;
        l->has_occupied = 0;
    }
}

/* resetWindowTo(w, startTime) per subclass. */
static void reset_window_to(or_leap* l, or_bucket* w, int64_t start) {
    w->start = start;
    switch (l->kind) {
    case OR_LEAP_OCCUPIABLE: {
        /* OccupiableBucketLeapArray.resetWindowTo, :50-63 */
        int bs = or_leap_window_value(l->borrow, start);
        zero_counters(w);
        if (bs >= 0) {
            /* w.value().addPass((int)borrowBucket.pass()): long → int narrowing keeps the low 32 bits */
            w->c[OR_M_PASS] += (int64_t)(int32_t)l->borrow->b[bs].c[OR_M_PASS];
        }
        break;
    }
    case OR_LEAP_CLUSTER:
        /* ClusterMetricLeapArray.resetWindowTo, :49-54 */
        zero_counters(w);
        cluster_transfer_occupy(l, w);
        break;
    default:
        /* BucketLeapArray / FutureBucketLeapArray / UnaryLeapArray: reset value */
        zero_counters(w);
        break;
    }
}

/* LeapArray.currentWindow(long timeMillis), base/LeapArray.java:116-202 (single-threaded: the CAS /
 * tryLock / yield branches collapse to their successful arm). */
int or_leap_current_window(or_leap* l, int64_t t) {
    if (t < 0) return -1;
    int idx = (int)((t / l->wl) % l->S);                 /* calculateTimeIdx :100-104   */
    int64_t ws = t - t % l->wl;                          /* calculateWindowStart :106-108 */
    if (!l->present[idx]) {                              /* (1) bucket absent → create */
        or_bucket* w = &l->b[idx];
        new_empty_bucket(l, w, t);
        w->start = ws;
        l->present[idx] = 1;
        return idx;
    }
    or_bucket* old = &l->b[idx];
    if (ws == old->start) return idx;                    /* (2) up to date             */
    if (ws > old->start) {                               /* (3) deprecated → reset     */
        reset_window_to(l, old, ws);
        return idx;
    }
    /* ws < old.start: a fresh bucket outside the array; writes to it are lost. */
    new_empty_bucket(l, &l->detached, t);
    l->detached.start = ws;
    return -2;
}

int64_t or_leap_slot_start(const or_leap* l, int slot) {
    if (slot >= 0 && !l->present[slot]) return INT64_MIN;
    return slot_cptr(l, slot)->start;
}
int64_t or_leap_slot_get(const or_leap* l, int slot, int ev) { return slot_cptr(l, slot)->c[ev]; }
void or_leap_slot_add(or_leap* l, int slot, int ev, int64_t n) { slot_ptr(l, slot)->c[ev] += n; }
int64_t or_leap_slot_min_rt(const or_leap* l, int slot) { return slot_cptr(l, slot)->min_rt; }

/* MetricBucket.addRT, data/MetricBucket.java:126-132 */
void or_leap_slot_add_rt(or_leap* l, int slot, int64_t rt) {
    or_bucket* w = slot_ptr(l, slot);
    w->c[OR_M_RT] += rt;
    if (rt < w->min_rt) w->min_rt = rt;
}

void or_leap_add(or_leap* l, int64_t t, int ev, int64_t n) {
    int s = or_leap_current_window(l, t);
    if (s == -1) return; /* Java would NPE; callers never pass t < 0 */
    or_leap_slot_add(l, s, ev, n);
}

/* LeapArray.values(long), base/LeapArray.java:329-344 */
int or_leap_values(const or_leap* l, int64_t t, int* out_slots) {
    if (t < 0) return 0;
    int k = 0;
    for (int i = 0; i < l->S; i++) {
        if (!l->present[i] || is_deprecated(l, t, &l->b[i])) continue;
        if (out_slots) out_slots[k] = i;
        k++;
    }
    return k;
}

/* ArrayMetric/ClusterMetric.getSum: currentWindow(); Σ values() (metric/ArrayMetric.java:301-310,
 * srv/flow/statistic/metric/ClusterMetric.java:53-62). */
int64_t or_leap_get_sum(or_leap* l, int64_t t, int ev) {
    or_leap_current_window(l, t);
    int64_t sum = 0;
    if (t < 0) return 0;
    for (int i = 0; i < l->S; i++) {
        if (!l->present[i] || is_deprecated(l, t, &l->b[i])) continue;
        sum += l->b[i].c[ev];
    }
    return sum;
}

/* LeapArray.getValidHead(long), base/LeapArray.java:353-363; its isWindowDeprecated(wrap) reads
 * TimeUtil.currentTimeMillis(), which in replay is the same t. */
int or_leap_valid_head(const or_leap* l, int64_t t) {
    int idx = (int)(((t + l->wl) / l->wl) % l->S);
    if (!l->present[idx] || is_deprecated(l, t, &l->b[idx])) return -1;
    return idx;
}

/* LeapArray.getPreviousWindow(long), base/LeapArray.java:210-227 (deprecation at the *current*
 * time = the original t in replay, since isWindowDeprecated(wrap) reads TimeUtil). */
int or_leap_previous_window(const or_leap* l, int64_t t) {
    if (t < 0) return -1;
    /* For t < windowLength the Java index (t - wl) / wl % S is <= 0: -1 throws
     * IndexOutOfBoundsException, 0 aliases slot 0. Epoch-time callers never get here. */
    if (t < l->wl) return -1;
    int64_t now = t;
    int idx = (int)(((t - l->wl) / l->wl) % l->S);
    int64_t tp = t - l->wl;
    if (!l->present[idx] || is_deprecated(l, now, &l->b[idx])) return -1;
    if (l->b[idx].start + l->wl < tp) return -1;
    return idx;
}

/* OccupiableBucketLeapArray.currentWaiting, :66-75 */
int64_t or_leap_current_waiting(or_leap* l, int64_t t) {
    or_leap_current_window(l->borrow, t);
    int64_t w = 0;
    for (int i = 0; i < l->borrow->S; i++) {
        if (!l->borrow->present[i] || is_deprecated(l->borrow, t, &l->borrow->b[i])) continue;
        w += l->borrow->b[i].c[OR_M_PASS];
    }
    return w;
}

/* OccupiableBucketLeapArray.addWaiting, :77-81 */
void or_leap_add_waiting(or_leap* l, int64_t t, int acquire) {
    int s = or_leap_current_window(l->borrow, t);
    if (s == -1) return;
    or_leap_slot_add(l->borrow, s, OR_M_PASS, acquire);
}

/* ===================================================================================== */
/* ClusterMetric (srv/flow/statistic/metric/ClusterMetric.java:28-99)                    */
/* ===================================================================================== */

or_leap* or_cluster_metric_new(int sample_count, int interval_ms) {
    return or_leap_new(OR_LEAP_CLUSTER, sample_count, interval_ms);
}

/* ClusterMetric.add, :39-41 */
void or_cluster_metric_add(or_leap* m, int64_t t, int ev, int64_t n) { or_leap_add(m, t, ev, n); }

/* ClusterMetric.getSum, :53-62 */
int64_t or_cluster_metric_get_sum(or_leap* m, int64_t t, int ev) { return or_leap_get_sum(m, t, ev); }

/* ClusterMetric.getAvg, :70-72 (long / double) */
double or_cluster_metric_get_avg(or_leap* m, int64_t t, int ev) {
    return (double)or_leap_get_sum(m, t, ev) / m->isec;
}

/* ClusterMetricLeapArray.getFirstCountOfWindow, ClusterMetricLeapArray.java:83-92 */
static int64_t cluster_first_count_of_window(const or_leap* m, int64_t t, int ev) {
    int h = or_leap_valid_head(m, t);
    if (h < 0) return 0;
    return m->b[h].c[ev];
}

int64_t or_cluster_metric_occupied(const or_leap* m, int ev) { return m->occ[ev]; }

/* ClusterMetric.tryOccupyNext, :79-87, and canOccupy, :89-98 */
int or_cluster_metric_try_occupy_next(or_leap* m, int64_t t, int ev, int acquire, double threshold) {
    double latest_qps = or_cluster_metric_get_avg(m, t, SG_EV_PASS);
    int64_t head_pass = cluster_first_count_of_window(m, t, ev);
    int64_t occupied = m->occ[ev];
    /* latestQps + (acquireCount + occupiedCount) - headPass <= threshold:
     * int + long → long, double + long → double, double - long → double */
    int can = latest_qps + (double)((int64_t)acquire + occupied) - (double)head_pass <= threshold;
    if (!can) return 0;
    /* ClusterMetricLeapArray.addOccupyPass, :73-77 */
    m->occ[SG_EV_PASS] += acquire;
    m->occ[SG_EV_PASS_REQUEST] += 1;
    m->has_occupied = 1;
    or_cluster_metric_add(m, t, SG_EV_WAITING, acquire);
    return 1000 / m->S; /* hard-coded 1000, ClusterMetric.java:86 */
}

/* ===================================================================================== */
/* RequestLimiter (srv/flow/statistic/limit/RequestLimiter.java:29-88)                   */
/* ===================================================================================== */

struct or_limiter {
    double qps_allowed;
    or_leap* data; /* new UnaryLeapArray(10, 1000), :35-37 */
};

or_limiter* or_limiter_new(double qps_allowed) {
    or_limiter* r = (or_limiter*)calloc(1, sizeof(or_limiter));
    r->qps_allowed = qps_allowed;
    r->data = or_leap_new(OR_LEAP_UNARY, 10, 1000);
    return r;
}
void or_limiter_free(or_limiter* r) {
    if (!r) return;
    or_leap_free(r->data);
    free(r);
}
void or_limiter_add(or_limiter* r, int64_t t, int x) { or_leap_add(r->data, t, 0, x); } /* :49-51 */
int64_t or_limiter_get_sum(or_limiter* r, int64_t t) { return or_leap_get_sum(r->data, t, 0); } /* :53-62 */
double or_limiter_get_qps(or_limiter* r, int64_t t) {                                          /* :64-66 */
    return (double)or_limiter_get_sum(r, t) / r->data->isec;
}
int or_limiter_can_pass(or_limiter* r, int64_t t) { return or_limiter_get_qps(r, t) + 1 <= r->qps_allowed; } /* :72-74 */
int or_limiter_try_pass(or_limiter* r, int64_t t) {                                           /* :81-87 */
    if (or_limiter_can_pass(r, t)) {
        or_limiter_add(r, t, 1);
        return 1;
    }
    return 0;
}
void or_limiter_set_qps_allowed(or_limiter* r, double q) { r->qps_allowed = q; }
double or_limiter_get_qps_allowed(const or_limiter* r) { return r->qps_allowed; }

/* ===================================================================================== */
/* Cluster token service: DefaultTokenService.requestToken → ClusterFlowChecker          */
/* ===================================================================================== */

typedef struct or_cts_rule {
    int64_t flow_id;
    double count;
    int32_t threshold_type;
    int32_t ns;
    or_leap* metric; /* ClusterMetricStatistics.METRIC_MAP[flowId] */
} or_cts_rule;

typedef struct or_cpm or_cpm;  /* ClusterParamMetric, below */

typedef struct or_cpr {        /* one cluster ParamFlowRule + its metric */
    sg_cparam_rule rule;
    const sg_param_hot_item* hot;  /* into or_cts.phot */
    or_cpm* metric;            /* ClusterParamMetricStatistics.METRIC_MAP[flowId] */
} or_cpr;

struct or_cts {
    or_cpr* prules;
    uint32_t n_prules;
    sg_param_hot_item* phot;
    double exceed_count;
    double max_occupy_ratio;
    or_cts_rule* rules;
    uint32_t n_rules;
    sg_namespace* ns;
    or_limiter** limiters; /* GlobalRequestLimiter.GLOBAL_QPS_LIMITER_MAP (null = no limiter) */
    uint32_t n_ns;
};

or_cts* or_cts_new(double exceed_count, double max_occupy_ratio) {
    or_cts* s = (or_cts*)calloc(1, sizeof(or_cts));
    s->exceed_count = exceed_count;
    s->max_occupy_ratio = max_occupy_ratio;
    return s;
}

static void cpm_free(or_cpm* m);

void or_cts_free(or_cts* s) {
    if (!s) return;
    for (uint32_t j = 0; j < s->n_prules; j++) cpm_free(s->prules[j].metric);
    free(s->prules);
    free(s->phot);
    for (uint32_t i = 0; i < s->n_rules; i++) or_leap_free(s->rules[i].metric);
    free(s->rules);
    for (uint32_t i = 0; i < s->n_ns; i++) or_limiter_free(s->limiters[i]);
    free(s->limiters);
    free(s->ns);
    free(s);
}

int or_cts_set_namespaces(or_cts* s, const sg_namespace* ns, uint32_t n) {
    /* Limiters persist across config updates (GlobalRequestLimiter.initIfAbsent :32-37,
     * applyMaxQpsChange :73-80); a namespace whose limiter is switched off loses it. */
    or_limiter** lim = (or_limiter**)calloc(n ? n : 1, sizeof(or_limiter*));
    for (uint32_t i = 0; i < n; i++) {
        or_limiter* old = i < s->n_ns ? s->limiters[i] : NULL;
        if (ns[i].limiter_enabled) {
            lim[i] = old ? old : or_limiter_new(ns[i].max_allowed_qps);
            or_limiter_set_qps_allowed(lim[i], ns[i].max_allowed_qps);
            if (old) s->limiters[i] = NULL;
        }
    }
    for (uint32_t i = 0; i < s->n_ns; i++) or_limiter_free(s->limiters[i]);
    free(s->limiters);
    free(s->ns);
    s->ns = (sg_namespace*)calloc(n ? n : 1, sizeof(sg_namespace));
    memcpy(s->ns, ns, n * sizeof(sg_namespace));
    s->limiters = lim;
    s->n_ns = n;
    return 0;
}

/* ClusterFlowRuleManager.applyClusterFlowRule, srv/flow/rule/ClusterFlowRuleManager.java:325-375:
 * a flowId that survives keeps its ClusterMetric (putMetricIfAbsent :361, even if the window
 * config changed); removed flowIds lose theirs (clearAndResetRulesConditional :287-302). */
int or_cts_load_rules(or_cts* s, const sg_flow_rule* rules, uint32_t n) {
    or_cts_rule* nr = (or_cts_rule*)calloc(n ? n : 1, sizeof(or_cts_rule));
    for (uint32_t i = 0; i < n; i++) {
        const sg_flow_rule* r = &rules[i];
        nr[i].flow_id = r->flow_id;
        nr[i].count = r->count;
        nr[i].threshold_type = r->threshold_type;
        nr[i].ns = r->namespace_id;
        for (uint32_t j = 0; j < s->n_rules; j++) {
            if (s->rules[j].metric && s->rules[j].flow_id == r->flow_id) {
                nr[i].metric = s->rules[j].metric;
                s->rules[j].metric = NULL;
                break;
            }
        }
        if (!nr[i].metric) nr[i].metric = or_cluster_metric_new(r->sample_count, r->window_interval_ms);
        if (!nr[i].metric) {
            for (uint32_t k = 0; k <= i; k++) or_leap_free(nr[k].metric);
            free(nr);
            return SG_E_INVAL;
        }
    }
    for (uint32_t j = 0; j < s->n_rules; j++) or_leap_free(s->rules[j].metric);
    free(s->rules);
    s->rules = nr;
    s->n_rules = n;
    return 0;
}

/* ClusterFlowChecker.calcGlobalThreshold, srv/flow/ClusterFlowChecker.java:38-48 */
static double calc_global_threshold(const or_cts* s, const or_cts_rule* r) {
    if (r->threshold_type == SG_THRESHOLD_GLOBAL) return r->count;
    int connected = 0;
    if (r->ns >= 0 && (uint32_t)r->ns < s->n_ns) connected = s->ns[r->ns].connected_count;
    return r->count * connected;
}

static sg_result mk(int32_t status, int32_t remaining, int32_t wait) {
    sg_result x;
    x.status = status;
    x.remaining = remaining;
    x.wait_ms = wait;
    return x;
}

/* ClusterFlowChecker.acquireClusterToken, srv/flow/ClusterFlowChecker.java:55-112 */
static sg_result acquire_cluster_token(or_cts* s, or_cts_rule* r, int64_t t, int acquire, int prio) {
    /* allowProceed → GlobalRequestLimiter.tryPass(namespace), :50-53, GlobalRequestLimiter.java:46-55 */
    if (r->ns < 0 || (uint32_t)r->ns >= s->n_ns) return mk(SG_STATUS_TOO_MANY_REQUEST, 0, 0); /* null ns */
    or_limiter* lim = s->limiters[r->ns];
    if (lim && !or_limiter_try_pass(lim, t)) return mk(SG_STATUS_TOO_MANY_REQUEST, 0, 0);

    or_leap* m = r->metric;
    double latest_qps = or_cluster_metric_get_avg(m, t, SG_EV_PASS);
    double global_threshold = calc_global_threshold(s, r) * s->exceed_count;
    double next_remaining = global_threshold - latest_qps - acquire;

    if (next_remaining >= 0) {
        or_cluster_metric_add(m, t, SG_EV_PASS, acquire);
        or_cluster_metric_add(m, t, SG_EV_PASS_REQUEST, 1);
        if (prio) or_cluster_metric_add(m, t, SG_EV_OCCUPIED_PASS, acquire);
        return mk(SG_STATUS_OK, or_d2i(next_remaining), 0);
    }
    if (prio) {
        double occupy_avg = or_cluster_metric_get_avg(m, t, SG_EV_WAITING);
        if (occupy_avg <= s->max_occupy_ratio * global_threshold) {
            int wait = or_cluster_metric_try_occupy_next(m, t, SG_EV_PASS, acquire, global_threshold);
            if (wait > 0) return mk(SG_STATUS_SHOULD_WAIT, 0, wait);
        }
    }
    or_cluster_metric_add(m, t, SG_EV_BLOCK, acquire);
    or_cluster_metric_add(m, t, SG_EV_BLOCK_REQUEST, 1);
    if (prio) or_cluster_metric_add(m, t, SG_EV_OCCUPIED_BLOCK, acquire);
    return mk(SG_STATUS_BLOCKED, 0, 0);
}

/* DefaultTokenService.requestToken, srv/flow/DefaultTokenService.java:39-50 */
int or_cts_decide(or_cts* s, const sg_req* req, uint64_t n, sg_result* out) {
    for (uint64_t i = 0; i < n; i++) {
        uint32_t key = req[i].key & SG_KEY_INDEX;
        int prio = (req[i].key & SG_KEY_PRIO) != 0;
        if (key == SG_KEY_BAD || req[i].acquire <= 0) {           /* notValidRequest :87-89 */
            out[i] = mk(SG_STATUS_BAD_REQUEST, 0, 0);
            continue;
        }
        if (key >= s->n_rules) {                                    /* rule == null :44-47 */
            out[i] = mk(SG_STATUS_NO_RULE_EXISTS, 0, 0);
            continue;
        }
        out[i] = acquire_cluster_token(s, &s->rules[key], req[i].ts_ms, req[i].acquire, prio);
    }
    return 0;
}

/* ClusterMetric.getAvg(ev) of one flowId at `now` (with its currentWindow side effect, as in Java). */
double or_cts_avg(or_cts* s, uint32_t key, int64_t now, int ev) {
    if (key >= s->n_rules) return 0;
    return or_cluster_metric_get_avg(s->rules[key].metric, now, ev);
}

int or_cts_sample_count(const or_cts* s, uint32_t key) {
    if (key >= s->n_rules) return -1;
    return s->rules[key].metric->S;
}

int or_cts_read_state(const or_cts* s, uint32_t key, int64_t* starts, int64_t* counters, int64_t* occupy) {
    if (key >= s->n_rules) return SG_E_INVAL;
    const or_leap* m = s->rules[key].metric;
    for (int j = 0; j < m->S; j++) {
        starts[j] = m->present[j] ? m->b[j].start : INT64_MIN;
        for (int e = 0; e < SG_NUM_EVENTS; e++) counters[j * SG_NUM_EVENTS + e] = m->present[j] ? m->b[j].c[e] : 0;
    }
    occupy[0] = m->occ[SG_EV_PASS];
    occupy[1] = m->occ[SG_EV_PASS_REQUEST];
    return 0;
}

/* Every flowId's window in the layout of sg_flow_export_state: ring[k][stride][8] = {start, 7 counters}
 * (start INT64_MIN and zero counters for never-created slots and slots >= S), occ[k][2]. */
int or_cts_export_state(const or_cts* s, int stride, int64_t* ring, int64_t* occ) {
    for (uint32_t k = 0; k < s->n_rules; k++) {
        const or_leap* m = s->rules[k].metric;
        if (m->S > stride) return SG_E_INVAL;
        int64_t* o = ring + (size_t)k * stride * 8;
        for (int j = 0; j < stride; j++) {
            const int p = j < m->S && m->present[j];
            o[8 * j] = p ? m->b[j].start : INT64_MIN;
            for (int e = 0; e < SG_NUM_EVENTS; e++) o[8 * j + 1 + e] = p ? m->b[j].c[e] : 0;
        }
        occ[2 * (size_t)k] = m->occ[SG_EV_PASS];
        occ[2 * (size_t)k + 1] = m->occ[SG_EV_PASS_REQUEST];
    }
    return 0;
}

/* ===================================================================================== */
/* Hot-parameter flow control: ParamFlowChecker.passDefaultLocalCheck / passThrottleLocalCheck */
/* (sentinel-extension/sentinel-parameter-flow-control/.../slots/block/flow/param/ParamFlowChecker.java) */
/* ===================================================================================== */
/* The reference keeps per-rule CacheMaps (ConcurrentLinkedHashMap LRU, capacity
 * min(4000 * durationInSec, 200000), ParameterMetric.java:95-122). This restatement keeps exact,
 * unbounded maps: it equals the reference whenever the distinct values per rule stay within that
 * capacity (eviction order is CLHM's and is not pinned by any reference test). */

typedef struct or_pf_slot {
    uint64_t value;
    uint32_t rule;
    uint8_t used, has_time, has_tokens;
    int64_t time;   /* timeCounters[value]  (lastAddTokenTime / last pass time for the throttle) */
    int64_t tokens; /* tokenCounters[value] */
} or_pf_slot;

struct or_pf {
    sg_param_rule* rules;
    uint32_t n_rules;
    sg_param_hot_item* hot;
    uint32_t n_hot;
    or_pf_slot* tab;
    uint64_t cap, size;
};

static uint64_t pf_hash(uint32_t rule, uint64_t v) {
    uint64_t z = v + 0x9E3779B97F4A7C15ULL * (rule + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

or_pf* or_pf_new(void) {
    or_pf* p = (or_pf*)calloc(1, sizeof(or_pf));
    p->cap = 1024;
    p->tab = (or_pf_slot*)calloc(p->cap, sizeof(or_pf_slot));
    return p;
}

void or_pf_free(or_pf* p) {
    if (!p) return;
    free(p->rules);
    free(p->hot);
    free(p->tab);
    free(p);
}

static or_pf_slot* pf_find(const or_pf* p, uint32_t rule, uint64_t v) {
    uint64_t i = pf_hash(rule, v) & (p->cap - 1);
    for (;;) {
        or_pf_slot* s = &p->tab[i];
        if (!s->used) return s;
        if (s->rule == rule && s->value == v) return s;
        i = (i + 1) & (p->cap - 1);
    }
}

static void pf_grow(or_pf* p) {
    or_pf_slot* old = p->tab;
    uint64_t oc = p->cap;
    p->cap *= 2;
    p->tab = (or_pf_slot*)calloc(p->cap, sizeof(or_pf_slot));
    for (uint64_t i = 0; i < oc; i++)
        if (old[i].used) *pf_find(p, old[i].rule, old[i].value) = old[i];
    free(old);
}

static or_pf_slot* pf_get_or_add(or_pf* p, uint32_t rule, uint64_t v) {
    if ((p->size + 1) * 2 > p->cap) pf_grow(p);
    or_pf_slot* s = pf_find(p, rule, v);
    if (!s->used) {
        s->used = 1;
        s->rule = rule;
        s->value = v;
        s->has_time = s->has_tokens = 0;
        p->size++;
    }
    return s;
}

/* A rule reload rebuilds the per-rule maps (ParameterMetricStorage.initParamMetricsFor creates maps for
 * rules not seen before; rules are keyed by equality, so here by position): state is cleared. */
int or_pf_load_rules(or_pf* p, const sg_param_rule* rules, uint32_t n, const sg_param_hot_item* hot, uint32_t n_hot) {
    free(p->rules);
    free(p->hot);
    p->rules = (sg_param_rule*)calloc(n ? n : 1, sizeof(sg_param_rule));
    memcpy(p->rules, rules, n * sizeof(sg_param_rule));
    p->n_rules = n;
    p->hot = (sg_param_hot_item*)calloc(n_hot ? n_hot : 1, sizeof(sg_param_hot_item));
    memcpy(p->hot, hot, n_hot * sizeof(sg_param_hot_item));
    p->n_hot = n_hot;
    memset(p->tab, 0, p->cap * sizeof(or_pf_slot));
    p->size = 0;
    return 0;
}

/* tokenCount: the hot item's threshold when the value is one, else (long) rule.count (:137-141). */
static int64_t pf_token_count(const or_pf* p, const sg_param_rule* r, uint64_t v) {
    for (uint32_t i = 0; i < r->hot_count; i++)
        if (p->hot[r->hot_begin + i].value == v) return p->hot[r->hot_begin + i].threshold;
    return or_d2l(r->count);
}

/* passDefaultLocalCheck, ParamFlowChecker.java:127-202 (single-threaded: CAS retries collapse). */
static int pf_default(or_pf* p, uint32_t ri, uint64_t v, int64_t t, int acquire) {
    const sg_param_rule* r = &p->rules[ri];
    int64_t token_count = pf_token_count(p, r, v);
    if (token_count == 0) return 0;
    int64_t max_count = token_count + r->burst;
    if (acquire > max_count) return 0;
    or_pf_slot* s = pf_get_or_add(p, ri, v);
    if (!s->has_time) {                  /* timeCounters.putIfAbsent → absent */
        s->has_time = 1;
        s->time = t;
        if (!s->has_tokens) {            /* tokenCounters.putIfAbsent keeps existing tokens */
            s->has_tokens = 1;
            s->tokens = max_count - acquire;
        }
        return 1;
    }
    int64_t pass_time = t - s->time;
    if (pass_time > r->duration_sec * 1000) {
        if (!s->has_tokens) {
            s->has_tokens = 1;
            s->tokens = max_count - acquire;
            s->time = t;
            return 1;
        }
        int64_t rest = s->tokens;
        int64_t to_add = (pass_time * token_count) / (r->duration_sec * 1000);
        int64_t new_qps = to_add + rest > max_count ? (max_count - acquire) : (rest + to_add - acquire);
        if (new_qps < 0) return 0;       /* lastAddTokenTime unchanged */
        s->tokens = new_qps;
        s->time = t;
        return 1;
    }
    if (s->has_tokens) {
        if (s->tokens - acquire >= 0) {
            s->tokens -= acquire;
            return 1;
        }
        return 0;
    }
    return 0; /* Java spins (Thread.yield) until tokens appear; unreachable without LRU eviction */
}

/* passThrottleLocalCheck, ParamFlowChecker.java:204-254 (the wait is a sleep; replay skips it). */
static int pf_throttle(or_pf* p, uint32_t ri, uint64_t v, int64_t t, int acquire) {
    const sg_param_rule* r = &p->rules[ri];
    int64_t token_count = pf_token_count(p, r, v);
    if (token_count == 0) return 0;
    int64_t cost = or_math_round(1.0 * 1000 * acquire * (double)r->duration_sec / (double)token_count);
    or_pf_slot* s = pf_get_or_add(p, ri, v);
    if (!s->has_time) {
        s->has_time = 1;
        s->time = t;
        return 1;
    }
    int64_t last = s->time;
    int64_t expected = last + cost;
    if (expected <= t || expected - t < r->max_queueing_ms) {
        s->time = t;
        if (expected - t > 0) s->time = expected;
        return 1;
    }
    return 0;
}

int or_pf_decide(or_pf* p, const sg_param_req* req, uint64_t n, int32_t* out) {
    for (uint64_t i = 0; i < n; i++) {
        uint32_t ri = req[i].rule;
        if (ri >= p->n_rules) { out[i] = 1; continue; } /* no rule for the resource: pass */
        if (p->rules[ri].behavior == 2)                 /* RuleConstant.CONTROL_BEHAVIOR_RATE_LIMITER */
            out[i] = pf_throttle(p, ri, req[i].value, req[i].ts_ms, req[i].acquire);
        else
            out[i] = pf_default(p, ri, req[i].value, req[i].ts_ms, req[i].acquire);
    }
    return 0;
}

int or_pf_read_state(const or_pf* p, uint32_t rule, uint64_t value, int64_t* last_time, int64_t* tokens) {
    or_pf_slot* s = pf_find(p, rule, value);
    if (!s->used) return 0;
    *last_time = s->time;
    *tokens = s->tokens;
    return (s->has_time ? 1 : 0) | (s->has_tokens ? 2 : 0);
}

uint64_t or_pf_size(const or_pf* p) { return p->size; }

/* ===================================================================================== */
/* Pace controller: RateLimiterController.canPass                                          */
/* (sentinel-core/.../slots/block/flow/controller/RateLimiterController.java:46-91)        */
/* ===================================================================================== */
/* One controller per CONTROL_BEHAVIOR_RATE_LIMITER FlowRule (FlowRuleUtil.generateRater,
 * FlowRuleUtil.java:132-145). Single-threaded replay: TimeUtil.currentTimeMillis() is the request's
 * ts for every read inside one call, and Thread.sleep(waitTime) is returned to the caller instead. */

struct or_pace {
    sg_pace_rule* rules;
    int64_t* latest;            /* latestPassedTime, AtomicLong(-1) (:33) */
    uint32_t n;
};

or_pace* or_pace_new(void) { return (or_pace*)calloc(1, sizeof(or_pace)); }

void or_pace_free(or_pace* p) {
    if (!p) return;
    free(p->rules);
    free(p->latest);
    free(p);
}

int or_pace_load_rules(or_pace* p, const sg_pace_rule* rules, uint32_t n) {
    for (uint32_t i = 0; i < n; i++)
        if (!(rules[i].count >= 0)) return -1;   /* FlowRuleUtil.isValidRule: count >= 0 (:167-175) */
    free(p->rules);
    free(p->latest);
    p->rules = (sg_pace_rule*)calloc(n ? n : 1, sizeof(sg_pace_rule));
    memcpy(p->rules, rules, n * sizeof(sg_pace_rule));
    p->latest = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    for (uint32_t i = 0; i < n; i++) p->latest[i] = -1;
    p->n = n;
    return 0;
}

static int32_t pace_can_pass(or_pace* p, uint32_t ri, int64_t now, int acquire) {
    const sg_pace_rule* r = &p->rules[ri];
    if (acquire <= 0) return 0;                                  /* :48-50 */
    if (r->count <= 0) return SG_PACE_BLOCKED;                   /* :53-55 */
    int64_t cost = or_math_round(1.0 * (acquire) / r->count * 1000);   /* :59 */
    int64_t expected = cost + p->latest[ri];                     /* :62 (long wraps: -fwrapv) */
    if (expected <= now) {                                       /* :64-67 */
        p->latest[ri] = now;
        return 0;
    }
    int64_t wait = cost + p->latest[ri] - now;                   /* :70 */
    if (wait > r->max_queueing_ms) return SG_PACE_BLOCKED;       /* :71-72 */
    p->latest[ri] += cost;                                       /* :74 addAndGet */
    int64_t old = p->latest[ri];
    wait = old - now;                                            /* :76 */
    if (wait > r->max_queueing_ms) {                             /* :77-80, unreachable single-threaded */
        p->latest[ri] -= cost;
        return SG_PACE_BLOCKED;
    }
    return wait > 0 ? (int32_t)wait : 0;                         /* :82-85 sleeps waitTime if > 0 */
}

int or_pace_decide(or_pace* p, const sg_pace_req* req, uint64_t n, int32_t* wait) {
    for (uint64_t i = 0; i < n; i++) {
        if (req[i].rule >= p->n) { wait[i] = 0; continue; }      /* no rule for the resource: pass */
        wait[i] = pace_can_pass(p, req[i].rule, req[i].ts_ms, req[i].acquire);
    }
    return 0;
}

int64_t or_pace_latest(const or_pace* p, uint32_t rule) { return rule < p->n ? p->latest[rule] : INT64_MIN; }

/* ===================================================================================== */
/* Local slot chain for one resource per rule: StatisticSlot.entry/exit                   */
/* (core/slots/statistic/StatisticSlot.java:55-165), FlowSlot with DefaultController      */
/* (core/slots/block/flow/controller/DefaultController.java:49-76), DegradeSlot           */
/* (core/slots/block/degrade/DegradeSlot.java:43-81) and the circuit breakers             */
/* (…/degrade/circuitbreaker/{AbstractCircuitBreaker,ResponseTimeCircuitBreaker,ExceptionCircuitBreaker}.java). */
/* One StatisticNode per resource stands for its DefaultNode and ClusterNode (identical for */
/* a single context; FlowRuleChecker reads the ClusterNode for limitApp "default").        */
/* ===================================================================================== */

enum { OR_CB_CLOSED = 0, OR_CB_OPEN = 1, OR_CB_HALF_OPEN = 2 };

typedef struct or_breaker {
    sg_degrade_rule rule;
    int state;
    int64_t next_retry;
    or_leap* stat; /* LeapArray(1, statIntervalMs): c[0] slow / error count, c[1] total count */
} or_breaker;

/* One FlowRule of a resource with its TrafficShapingController (FlowRuleUtil.generateRater, :132-149). */
typedef struct or_ctl {
    sg_local_flow_rule rule;
    int behavior;              /* the controller: THREAD rules and unknown behaviours use DefaultController */
    /* WarmUpController fields (WarmUpController.java:66-73), fixed by construct (:83-106) */
    int32_t warning_token, max_token, cold;
    double slope;
    int64_t stored_tokens, last_filled;   /* AtomicLong(0) each */
    int64_t latest;                       /* RateLimiter / WarmUpRateLimiter latestPassedTime, AtomicLong(-1) */
    int32_t input;                        /* index in the loaded rule array */
} or_ctl;

typedef struct or_node {
    or_leap* second;  /* ArrayMetric(SAMPLE_COUNT, INTERVAL): OccupiableBucketLeapArray (StatisticNode.java:96-97) */
    or_leap* minute;  /* ArrayMetric(60, 60000, false) (:103)                                                   */
    int64_t threads;  /* curThreadNum                                                                            */
    sg_local_rule rule;
    or_breaker cb[2];
    or_ctl* ctl;      /* the resource's flow rules in FlowRuleComparator order */
    uint32_t n_ctl;
    int created;      /* ClusterBuilderSlot created the ClusterNode (the resource's first entry)                 */
    struct or_node** origin;  /* ClusterNode.originCountMap: [n_origins + 1], created on first use, kept across
                                 rule reloads */
    int32_t origin_cap;       /* entries of origin[] */
    struct or_node** ctxn;    /* NodeSelectorSlot's DefaultNode per context id: [ctx_cap], created at the first
                                 event in the context */
    int32_t ctx_cap;
} or_node;

struct or_local {
    int S, interval, occupy_timeout, cold_factor;
    or_node* nodes;
    uint32_t n;
    int64_t* last_fetch;     /* StatisticNode.lastFetchTime per resource (metrics()) */
    int32_t n_origins, n_contexts;
    uint64_t batches;        /* batches decided since or_local_load_rules */
    or_cts* cts;             /* the embedded token server's DefaultTokenService (cluster_state SERVER) */
    int cluster_state;       /* ClusterStateManager: SG_CLUSTER_NOT_STARTED (default), SERVER */
    int64_t* rule_pos;       /* loaded flow rule i → (resource << 32 | position), -1 = ignored */
    uint32_t n_rules;
    struct or_pslot* ps;     /* ParamFlowSlot's rules and metrics (or_local_attach_pslot), NULL = none */
    uint8_t* inbound;        /* per resource: its entries are EntryType.IN (Constants.ENTRY_NODE counts them) */
    or_node* entry;          /* Constants.ENTRY_NODE, the global inbound StatisticNode (created with the resources) */
    int64_t entry_fetch;     /* its lastFetchTime */
};

or_local* or_local_new(int second_sample_count, int second_interval_ms, int occupy_timeout_ms) {
    or_local* l = (or_local*)calloc(1, sizeof(or_local));
    l->S = second_sample_count;            /* SampleCountProperty.SAMPLE_COUNT, default 2   */
    l->interval = second_interval_ms;      /* IntervalProperty.INTERVAL, default 1000        */
    l->occupy_timeout = occupy_timeout_ms; /* OccupyTimeoutProperty.occupyTimeout, 500      */
    l->cold_factor = 3;                    /* ColdFactorProperty.coldFactor (SentinelConfig default 3) */
    l->cluster_state = SG_CLUSTER_NOT_STARTED;
    return l;
}

void or_local_set_cold_factor(or_local* l, int cold_factor) { l->cold_factor = cold_factor > 1 ? cold_factor : 3; }

static or_node* node_new_plain(or_local* l) {
    or_node* o = (or_node*)calloc(1, sizeof(or_node));
    o->second = or_leap_new(OR_LEAP_OCCUPIABLE, l->S, l->interval);
    o->minute = or_leap_new(OR_LEAP_BUCKET, 60, 60 * 1000);
    return o;
}

static void free_plain(or_node* x) {
    if (!x) return;
    or_leap_free(x->second);
    or_leap_free(x->minute);
    free(x);
}

static void free_origins(or_local* l, or_node* nd) {
    (void)l;
    for (int32_t o = 0; o < nd->origin_cap; o++) free_plain(nd->origin[o]);
    free(nd->origin);
    nd->origin = NULL;
    nd->origin_cap = 0;
    for (int32_t c = 0; c < nd->ctx_cap; c++) free_plain(nd->ctxn[c]);
    free(nd->ctxn);
    nd->ctxn = NULL;
    nd->ctx_cap = 0;
}

static void free_nodes(or_local* l) {
    for (uint32_t i = 0; i < l->n; i++) {
        or_leap_free(l->nodes[i].second);
        or_leap_free(l->nodes[i].minute);
        for (int j = 0; j < 2; j++) or_leap_free(l->nodes[i].cb[j].stat);
        free(l->nodes[i].ctl);
        free_origins(l, &l->nodes[i]);
    }
    free(l->nodes);
    free(l->rule_pos);
    free(l->last_fetch);
    free(l->inbound);
    l->inbound = NULL;
    free_plain(l->entry);
    l->entry = NULL;
    l->last_fetch = NULL;
    l->rule_pos = NULL;
    l->n_rules = 0;
    l->nodes = NULL;
    l->n = 0;
}

void or_local_free(or_local* l) {
    if (!l) return;
    free_nodes(l);
    free(l);
}

/* WarmUpController.construct (WarmUpController.java:83-106), int arithmetic as Java's */
static void ctl_init(or_ctl* c, const sg_local_flow_rule* r, int cold, int32_t input) {
    memset(c, 0, sizeof(*c));
    c->rule = *r;
    c->input = input;
    c->behavior = (r->grade == 1 && r->control_behavior >= SG_CONTROL_WARM_UP &&
                   r->control_behavior <= SG_CONTROL_WARM_UP_RATE_LIMITER) ? r->control_behavior : SG_CONTROL_DEFAULT;
    c->latest = -1;
    c->cold = cold;
    if (c->behavior == SG_CONTROL_WARM_UP || c->behavior == SG_CONTROL_WARM_UP_RATE_LIMITER) {
        c->warning_token = or_d2i(r->warm_up_period_sec * r->count) / (cold - 1);
        const int32_t two_w = (int32_t)(2u * (uint32_t)r->warm_up_period_sec);      /* 2 * warmUpPeriodInSec: int */
        c->max_token = (int32_t)((uint32_t)c->warning_token + (uint32_t)or_d2i(two_w * r->count / (1.0 + cold)));
        c->slope = (cold - 1.0) / r->count / (double)(int32_t)((uint32_t)c->max_token - (uint32_t)c->warning_token);
    }
}

/* FlowRuleUtil.isValidRule (:167-251): count >= 0, grade / strategy / behaviour >= 0; QPS rules: checkClusterField
 * (an invalid ClusterFlowConfig), checkStrategyField (RELATE / CHAIN need a refResource) and
 * checkControlBehaviorField; THREAD rules: checkClusterConcurrentField. */
static int flow_rule_valid(const sg_local_flow_rule* r) {
    if (!(r->count >= 0) || r->grade < 0 || r->strategy < 0 || r->control_behavior < 0) return 0;
    if (r->grade == 1) {
        if (r->cluster_mode == SG_CLUSTER_MODE_INVALID) return 0;
        if ((r->strategy == SG_STRATEGY_RELATE || r->strategy == SG_STRATEGY_CHAIN) && r->ref_resource < 0) return 0;
        switch (r->control_behavior) {
        case SG_CONTROL_WARM_UP: return r->warm_up_period_sec > 0;
        case SG_CONTROL_RATE_LIMITER: return r->max_queueing_ms > 0;
        case SG_CONTROL_WARM_UP_RATE_LIMITER: return r->warm_up_period_sec > 0 && r->max_queueing_ms > 0;
        default: return 1;
        }
    }
    return r->grade == 0 && r->cluster_mode != SG_CLUSTER_MODE_INVALID;
}

/* FlowRule.equals (FlowRule.java, AbstractRule.equals) over the fields the ABI carries (the reference's HashSet
 * drops duplicates, FlowRuleUtil.java:109-117); Double.compare on count */
static int flow_rule_same(const sg_local_flow_rule* a, const sg_local_flow_rule* b) {
    return a->resource == b->resource && a->grade == b->grade && memcmp(&a->count, &b->count, sizeof(double)) == 0 &&
           a->control_behavior == b->control_behavior && a->limit_app == b->limit_app && a->strategy == b->strategy &&
           a->warm_up_period_sec == b->warm_up_period_sec && a->max_queueing_ms == b->max_queueing_ms &&
           (a->ref_resource < 0 ? b->ref_resource < 0 : a->ref_resource == b->ref_resource) &&
           (a->cluster_mode != 0) == (b->cluster_mode != 0) &&
           (a->cluster_mode == 0 || (a->cluster_mode == b->cluster_mode && a->cluster_config == b->cluster_config));
}

int or_local_load_flow_rules(or_local* l, const sg_local_flow_rule* rules, uint32_t n, int32_t n_origins,
                             int32_t n_contexts) {
    if (n_origins < l->n_origins || n_contexts < l->n_contexts) return SG_E_INVAL;   /* ids keep their meaning */
    /* the DefaultNodes are kept from the first batch on (NodeSelectorSlot creates one at a context's first entry):
     * context tracking cannot start later */
    if (n_contexts > 0 && l->n_contexts == 0 && l->batches > 0) return SG_E_UNSUPPORTED;
    for (uint32_t k = 0; k < l->n; k++) {   /* the origin / context nodes stay (they outlive rule reloads) */
        free(l->nodes[k].ctl);
        l->nodes[k].ctl = NULL;
        l->nodes[k].n_ctl = 0;
    }
    l->n_origins = n_origins;
    l->n_contexts = n_contexts;
    free(l->rule_pos);
    l->rule_pos = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    l->n_rules = n;
    uint32_t* cnt = (uint32_t*)calloc(l->n ? l->n : 1, sizeof(uint32_t));
    /* the kept rules of each resource as a chain (a duplicate has the same resource): last kept index per resource,
     * previous kept index of the same resource per rule */
    int64_t* last = (int64_t*)malloc((l->n ? l->n : 1) * sizeof(int64_t));
    int64_t* prev = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    for (uint32_t k = 0; k < l->n; k++) last[k] = -1;
    for (uint32_t i = 0; i < n; i++) {
        l->rule_pos[i] = -1;
        const sg_local_flow_rule* r = &rules[i];
        if (r->resource >= l->n || !flow_rule_valid(r)) continue;   /* ignored, as RecordLog.warn + continue */
        if (r->limit_app > n_origins || (r->strategy == SG_STRATEGY_CHAIN && r->ref_resource >= n_contexts)) {
            free(cnt);
            free(last);
            free(prev);
            return SG_E_INVAL;
        }
        int dup = 0;
        for (int64_t j = last[r->resource]; j >= 0 && !dup; j = prev[j]) dup = flow_rule_same(&rules[j], r);
        if (dup) continue;
        l->rule_pos[i] = 0;
        prev[i] = last[r->resource];
        last[r->resource] = i;
        cnt[r->resource]++;
    }
    free(last);
    free(prev);
    for (uint32_t k = 0; k < l->n; k++)
        if (cnt[k]) l->nodes[k].ctl = (or_ctl*)calloc(cnt[k], sizeof(or_ctl));
    /* Collections.sort(rules, FlowRuleComparator): stable; local rules before cluster-mode ones, then non-"default"
     * limitApps before "default" (:30-55) */
    for (int pass = 0; pass < 4; pass++) {
        for (uint32_t i = 0; i < n; i++) {
            if (l->rule_pos[i] < 0) continue;
            const int key = (rules[i].cluster_mode != SG_CLUSTER_MODE_OFF ? 2 : 0) +
                            (rules[i].limit_app == SG_LIMIT_APP_DEFAULT ? 1 : 0);
            if (key != pass) continue;
            or_node* nd = &l->nodes[rules[i].resource];
            ctl_init(&nd->ctl[nd->n_ctl], &rules[i], l->cold_factor, (int32_t)i);
            l->rule_pos[i] = (int64_t)(((uint64_t)rules[i].resource << 32) | (uint32_t)nd->n_ctl);
            nd->n_ctl++;
        }
    }
    free(cnt);
    uint32_t kept = 0;
    for (uint32_t i = 0; i < n; i++) kept += l->rule_pos[i] >= 0;
    return (int)kept;
}

int or_local_load_rules(or_local* l, const sg_local_rule* rules, uint32_t n) {
    free_nodes(l);
    l->nodes = (or_node*)calloc(n ? n : 1, sizeof(or_node));
    l->n = n;
    l->n_origins = 0;
    l->n_contexts = 0;
    l->batches = 0;
    l->inbound = (uint8_t*)calloc(n ? n : 1, 1);   /* SphU.entry's default EntryType.OUT */
    l->entry = node_new_plain(l);
    l->entry_fetch = -1;
    for (uint32_t i = 0; i < n; i++) {
        or_node* nd = &l->nodes[i];
        nd->rule = rules[i];
        nd->second = or_leap_new(OR_LEAP_OCCUPIABLE, l->S, l->interval);
        nd->minute = or_leap_new(OR_LEAP_BUCKET, 60, 60 * 1000);
        for (int j = 0; j < rules[i].n_breakers && j < 2; j++) {
            nd->cb[j].rule = rules[i].breakers[j];
            nd->cb[j].state = OR_CB_CLOSED;
            nd->cb[j].stat = or_leap_new(OR_LEAP_BUCKET, 1, rules[i].breakers[j].stat_interval_ms);
            if (!nd->cb[j].stat) return SG_E_INVAL;
        }
        if (rules[i].flow_grade >= 0) {  /* the one DefaultController rule, limitApp "default" */
            sg_local_flow_rule fr;
            memset(&fr, 0, sizeof(fr));
            fr.resource = i;
            fr.grade = rules[i].flow_grade;
            fr.count = rules[i].flow_count;
            nd->ctl = (or_ctl*)calloc(1, sizeof(or_ctl));
            ctl_init(&nd->ctl[0], &fr, l->cold_factor, -1);
            nd->n_ctl = 1;
        }
    }
    return 0;
}

/* StatisticNode.passQps = rollingCounterInSecond.pass() / getWindowIntervalInSec (StatisticNode.java:200-202) */
static double node_pass_qps(or_node* nd, int64_t t) {
    return (double)or_leap_get_sum(nd->second, t, OR_M_PASS) / nd->second->isec;
}

/* StatisticNode.previousPassQps = rollingCounterInMinute.previousWindowPass() (StatisticNode.java:175-177,
 * ArrayMetric.java:270-277): currentWindow, then getPreviousWindow's PASS */
static double node_previous_pass_qps(or_node* nd, int64_t t) {
    or_leap_current_window(nd->minute, t);
    int s = or_leap_previous_window(nd->minute, t);
    return s < 0 ? 0.0 : (double)nd->minute->b[s].c[OR_M_PASS];
}

/* StatisticNode.tryOccupyNext, StatisticNode.java:288-320 */
static int64_t node_try_occupy_next(or_local* l, or_node* nd, int64_t now, int acquire, double threshold) {
    double max_count = threshold * l->interval / 1000;
    int64_t current_borrow = or_leap_current_waiting(nd->second, now);
    if (current_borrow >= max_count) return l->occupy_timeout;
    int window_length = l->interval / l->S;
    int64_t earliest = now - now % window_length + window_length - l->interval;
    int idx = 0;
    int64_t current_pass = or_leap_get_sum(nd->second, now, OR_M_PASS);
    while (earliest < now) {
        int64_t wait = (int64_t)idx * window_length + window_length - now % window_length;
        if (wait >= l->occupy_timeout) break;
        int wv = or_leap_window_value(nd->second, earliest); /* ArrayMetric.getWindowPass */
        int64_t window_pass = wv >= 0 ? nd->second->b[wv].c[OR_M_PASS] : 0;
        if (current_pass + current_borrow + acquire - window_pass <= max_count) return wait;
        earliest += window_length;
        current_pass -= window_pass;
        idx++;
    }
    return l->occupy_timeout;
}

static void node_add(or_leap* w, int64_t t, int ev, int64_t n) { or_leap_add(w, t, ev, n); }

/* ---- traffic-shaping controllers (core/.../slots/block/flow/controller) ---- */

/* WarmUpController.coolDownTokens (:161-175) */
static int64_t warm_cool_down(const or_ctl* c, int64_t current_time, int64_t pass_qps) {
    int64_t old = c->stored_tokens, nv = old;
    if (old < c->warning_token) {
        nv = or_d2l((double)old + (double)(current_time - c->last_filled) * c->rule.count / 1000);
    } else if (old > c->warning_token) {
        if (pass_qps < or_d2i(c->rule.count) / c->cold)
            nv = or_d2l((double)old + (double)(current_time - c->last_filled) * c->rule.count / 1000);
    }
    return nv < c->max_token ? nv : (int64_t)c->max_token;
}

/* WarmUpController.syncToken (:140-159), single-threaded: the compareAndSet succeeds */
static void warm_sync_token(or_ctl* c, int64_t now, int64_t pass_qps) {
    int64_t current_time = now - now % 1000;
    if (current_time <= c->last_filled) return;
    c->stored_tokens = warm_cool_down(c, current_time, pass_qps);
    int64_t cur = (int64_t)((uint64_t)c->stored_tokens - (uint64_t)pass_qps);   /* addAndGet(0 - passQps) */
    c->stored_tokens = cur < 0 ? 0 : cur;
    c->last_filled = current_time;
}

/* Math.nextUp(1.0 / (aboveToken * slope + 1.0 / count)) */
static double warm_qps(const or_ctl* c, int64_t above) {
    return nextafter(1.0 / ((double)above * c->slope + 1.0 / c->rule.count), INFINITY);
}

/* WarmUpController.canPass (:113-138) with the node's passQps / previousPassQps */
int or_warm_can_pass(or_ctl* c, int64_t now, double pass_qps_d, double prev_qps_d, int acquire) {
    int64_t pass_qps = or_d2l(pass_qps_d);
    int64_t prev = or_d2l(prev_qps_d);
    warm_sync_token(c, now, prev);
    int64_t rest = c->stored_tokens;
    int64_t sum = (int64_t)((uint64_t)pass_qps + (uint64_t)(int64_t)acquire);   /* long + int */
    if (rest >= c->warning_token) return (double)sum <= warm_qps(c, rest - c->warning_token);
    return (double)sum <= c->rule.count;
}

/* WarmUpRateLimiterController.canPass (:43-87): 1 pass (*wait = the sleep), 0 block */
int or_warm_rl_can_pass(or_ctl* c, int64_t now, double prev_qps_d, int acquire, int64_t* wait) {
    *wait = 0;
    warm_sync_token(c, now, or_d2l(prev_qps_d));
    int64_t rest = c->stored_tokens;
    int64_t cost;
    if (rest >= c->warning_token) cost = or_math_round(1.0 * (acquire) / warm_qps(c, rest - c->warning_token) * 1000);
    else cost = or_math_round(1.0 * (acquire) / c->rule.count * 1000);
    int64_t expected = cost + c->latest;
    if (expected <= now) {
        c->latest = now;
        return 1;
    }
    int64_t w = cost + c->latest - now;
    if (w > c->rule.max_queueing_ms) return 0;
    c->latest += cost;
    w = c->latest - now;
    if (w > c->rule.max_queueing_ms) {  /* unreachable single-threaded */
        c->latest -= cost;
        return 0;
    }
    *wait = w > 0 ? w : 0;
    return 1;
}

/* RateLimiterController.canPass (:46-91) on the rule's own latestPassedTime */
static int rl_can_pass(or_ctl* c, int64_t now, int acquire, int64_t* wait) {
    *wait = 0;
    if (acquire <= 0) return 1;
    if (c->rule.count <= 0) return 0;
    int64_t cost = or_math_round(1.0 * (acquire) / c->rule.count * 1000);
    int64_t expected = cost + c->latest;
    if (expected <= now) {
        c->latest = now;
        return 1;
    }
    int64_t w = cost + c->latest - now;
    if (w > c->rule.max_queueing_ms) return 0;
    c->latest += cost;
    w = c->latest - now;
    if (w > c->rule.max_queueing_ms) {
        c->latest -= cost;
        return 0;
    }
    *wait = w > 0 ? w : 0;
    return 1;
}

/* Stand-alone controllers for the reference's own controller tests (mocked nodes). */
or_ctl* or_ctl_new(const sg_local_flow_rule* r, int cold_factor) {
    or_ctl* c = (or_ctl*)malloc(sizeof(or_ctl));
    ctl_init(c, r, cold_factor > 1 ? cold_factor : 3, -1);
    return c;
}
void or_ctl_free(or_ctl* c) { free(c); }
void or_ctl_state(const or_ctl* c, int64_t* out3) {
    out3[0] = c->stored_tokens;
    out3[1] = c->last_filled;
    out3[2] = c->latest;
}
int32_t or_ctl_warning_token(const or_ctl* c) { return c->warning_token; }
int32_t or_ctl_max_token(const or_ctl* c) { return c->max_token; }

/* FlowRuleManager.isOtherOrigin (FlowRuleManager.java:132-148): no rule of the resource names the origin */
static int is_other_origin(const or_node* nd, int origin) {
    if (origin <= 0) return 0;
    for (uint32_t i = 0; i < nd->n_ctl; i++)
        if (nd->ctl[i].rule.limit_app == origin) return 0;
    return 1;
}

/* FlowRuleChecker.selectNodeByRequesterAndStrategy (FlowRuleChecker.java:115-145) with selectReferenceNode
 * (:96-112): 0 the ClusterNode, 1 the origin node, 2 the resource's DefaultNode of the current context (CHAIN),
 * 3 the ClusterNode of ref_resource (RELATE), -1 none (the rule passes). ref_exists: that ClusterNode exists. */
static int select_kind(const or_node* nd, const sg_local_flow_rule* r, int origin, int context, int ref_exists) {
    int matched;   /* 1: limitApp is the origin / "other" (origin node for DIRECT), 0: "default" */
    if (origin > 0 && r->limit_app == origin) matched = 1;   /* limitApp.equals(origin) && filterOrigin(origin) */
    else if (r->limit_app == SG_LIMIT_APP_DEFAULT) matched = 0;
    else if (r->limit_app == SG_LIMIT_APP_OTHER && is_other_origin(nd, origin)) matched = 1;
    else return -1;
    if (r->strategy == SG_STRATEGY_DIRECT) return matched ? 1 : 0;
    if (r->ref_resource < 0) return -1;                         /* StringUtil.isEmpty(refResource) */
    if (r->strategy == SG_STRATEGY_RELATE) return ref_exists ? 3 : -1;   /* ClusterBuilderSlot.getClusterNode */
    if (r->strategy == SG_STRATEGY_CHAIN) return r->ref_resource == context ? 2 : -1;
    return -1;
}

/* For the FlowRuleCheckerTest restatement: the rules of one resource, a request origin / context, and whether the
 * RELATE target's ClusterNode exists. */
int or_select_node(const sg_local_flow_rule* rules, uint32_t n, uint32_t i, int origin, int context, int ref_exists) {
    or_node nd;
    memset(&nd, 0, sizeof(nd));
    or_ctl* c = (or_ctl*)calloc(n ? n : 1, sizeof(or_ctl));
    for (uint32_t j = 0; j < n; j++) c[j].rule = rules[j];
    nd.ctl = c;
    nd.n_ctl = n;
    int r = select_kind(&nd, &rules[i], origin, context, ref_exists);
    free(c);
    return r;
}

static or_node* origin_node(or_local* l, or_node* nd, int origin) {   /* ClusterNode.getOrCreateOriginNode */
    if (origin <= 0 || origin > l->n_origins) return NULL;
    if (origin >= nd->origin_cap) {
        const int32_t cap = l->n_origins + 1;
        nd->origin = (or_node**)realloc(nd->origin, (size_t)cap * sizeof(or_node*));
        for (int32_t o = nd->origin_cap; o < cap; o++) nd->origin[o] = NULL;
        nd->origin_cap = cap;
    }
    if (!nd->origin[origin]) nd->origin[origin] = node_new_plain(l);
    return nd->origin[origin];
}

static or_node* context_node(or_local* l, or_node* nd, int context) {   /* NodeSelectorSlot: DefaultNode per context */
    if (context < 0 || context >= l->n_contexts) return NULL;
    if (context >= nd->ctx_cap) {
        const int32_t cap = l->n_contexts;
        nd->ctxn = (or_node**)realloc(nd->ctxn, (size_t)cap * sizeof(or_node*));
        for (int32_t c = nd->ctx_cap; c < cap; c++) nd->ctxn[c] = NULL;
        nd->ctx_cap = cap;
    }
    if (!nd->ctxn[context]) nd->ctxn[context] = node_new_plain(l);
    return nd->ctxn[context];
}

/* DefaultController.canPass (DefaultController.java:49-76) on the selected node: 1 pass, 0 block, 2 priority wait */
static int default_can_pass(or_local* l, or_node* sn, const or_ctl* c, int64_t t, int count, int prio, int64_t* wait) {
    int32_t cur = c->rule.grade == 0 ? (int32_t)sn->threads : or_d2i(node_pass_qps(sn, t));
    int32_t sum = (int32_t)((uint32_t)cur + (uint32_t)count); /* int + int wraps */
    if (!((double)sum > c->rule.count)) return 1;
    if (prio && c->rule.grade == 1) {
        int64_t w = node_try_occupy_next(l, sn, t, count, c->rule.count);
        if (w < l->occupy_timeout) {
            or_leap_add_waiting(sn->second, t + w, count);        /* addWaitingRequest */
            node_add(sn->minute, t, OR_M_OCCUPIED_PASS, count);   /* addOccupiedPass (StatisticNode.java:333-336) */
            node_add(sn->minute, t, OR_M_PASS, count);
            *wait = w;
            return 2;                                             /* PriorityWaitException */
        }
    }
    return 0;
}

int or_local_attach_cluster(or_local* l, or_cts* cts, int state) {
    if (state == SG_CLUSTER_CLIENT) return SG_E_UNSUPPORTED;
    if (state == SG_CLUSTER_SERVER && !cts) return SG_E_INVAL;
    l->cts = state == SG_CLUSTER_SERVER ? cts : NULL;
    l->cluster_state = state;
    if (l->ps) or_pslot_attach_cluster(l->ps, l->cts, state);  /* one ClusterStateManager per node */
    return 0;
}

/* FlowRuleChecker.passClusterCheck (:147-164) with applyTokenResult (:186-209) on a node whose embedded token server
 * answers (pickClusterService → EmbeddedClusterTokenServerProvider.getServer, :177-184; DefaultEmbeddedTokenServer
 * .requestToken → DefaultTokenService.requestToken, DefaultEmbeddedTokenServer.java:46-51): 1 pass (*wait += the
 * SHOULD_WAIT sleep), 0 BLOCKED, -1 fallbackToLocalOrPass. */
static int cluster_token(or_local* l, const or_ctl* c, int64_t t, int count, int prio, int64_t* wait) {
    sg_req q;
    memset(&q, 0, sizeof(q));
    q.ts_ms = t;
    q.key = (c->rule.cluster_key & SG_KEY_INDEX) | (prio ? SG_KEY_PRIO : 0u);
    q.acquire = count;
    sg_result r;
    or_cts_decide(l->cts, &q, 1, &r);
    switch (r.status) {
    case SG_STATUS_OK: return 1;
    case SG_STATUS_SHOULD_WAIT: *wait += r.wait_ms; return 1;   /* Thread.sleep(waitInMs), then pass */
    case SG_STATUS_NO_RULE_EXISTS:
    case SG_STATUS_BAD_REQUEST:
    case SG_STATUS_FAIL:
    case SG_STATUS_TOO_MANY_REQUEST: return -1;
    default: return 0;                                          /* BLOCKED */
    }
}

/* FlowSlot.checkFlow → FlowRuleChecker.checkFlow (:44-57): the rules in order, the first failure throws. A cluster-mode
 * rule: passClusterCheck (:147-164) — the embedded server's token (SERVER state) or, with no token service
 * (NOT_STARTED) and for the answers applyTokenResult sends there, fallbackToLocalOrPass (:166-175). */
static int check_flow(or_local* l, or_node* nd, int64_t t, int count, int prio, int origin, int context, int64_t* wait) {
    *wait = 0;
    for (uint32_t i = 0; i < nd->n_ctl; i++) {
        or_ctl* c = &nd->ctl[i];
        if (c->rule.cluster_mode != SG_CLUSTER_MODE_OFF && l->cluster_state == SG_CLUSTER_SERVER) {
            const int v = cluster_token(l, c, t, count, prio, wait);
            if (v == 0) return SG_LOCAL_BLOCK_FLOW;
            if (v == 1) continue;
        }
        if (c->rule.cluster_mode == SG_CLUSTER_MODE_NO_FALLBACK) continue;   /* the rule is not activated */
        const int32_t ref = c->rule.ref_resource;
        or_node* rn = (ref >= 0 && (uint32_t)ref < l->n) ? &l->nodes[ref] : NULL;
        int s = select_kind(nd, &c->rule, origin, context, rn && rn->created);
        if (s < 0) continue;
        or_node* sn = s == 0 ? nd : s == 1 ? origin_node(l, nd, origin) : s == 2 ? context_node(l, nd, context) : rn;
        int64_t w = 0;
        switch (c->behavior) {
        case SG_CONTROL_WARM_UP:
            if (!or_warm_can_pass(c, t, node_pass_qps(sn, t), node_previous_pass_qps(sn, t), count))
                return SG_LOCAL_BLOCK_FLOW;
            break;
        case SG_CONTROL_RATE_LIMITER:
            if (!rl_can_pass(c, t, count, &w)) return SG_LOCAL_BLOCK_FLOW;
            *wait += w;   /* each controller sleeps in turn */
            break;
        case SG_CONTROL_WARM_UP_RATE_LIMITER:
            if (!or_warm_rl_can_pass(c, t, node_previous_pass_qps(sn, t), count, &w)) return SG_LOCAL_BLOCK_FLOW;
            *wait += w;
            break;
        default: {
            int r = default_can_pass(l, sn, c, t, count, prio, &w);
            if (r == 0) return SG_LOCAL_BLOCK_FLOW;
            if (r == 2) {
                *wait = w;
                return SG_LOCAL_PASS_WAIT;
            }
        }
        }
    }
    return SG_LOCAL_PASS;
}

/* AbstractCircuitBreaker.tryPass (:73-84); sets *half when this call moved OPEN → HALF_OPEN. */
static int cb_try_pass(or_breaker* cb, int64_t t, int* half) {
    *half = 0;
    if (cb->state == OR_CB_CLOSED) return 1;
    if (cb->state == OR_CB_OPEN) {
        if (t >= cb->next_retry) {
            cb->state = OR_CB_HALF_OPEN;
            *half = 1;
            return 1;
        }
        return 0;
    }
    return 0;
}

static void cb_to_open(or_breaker* cb, int64_t t) { /* transformToOpen / fromHalfOpenToOpen */
    cb->state = OR_CB_OPEN;
    /* recoveryTimeoutMs = rule.getTimeWindow() * 1000 is an int (AbstractCircuitBreaker.java:36,54): wraps */
    cb->next_retry = t + (int64_t)(int32_t)((uint32_t)cb->rule.time_window_sec * 1000u);
}

/* onRequestComplete at exit time t (ResponseTimeCircuitBreaker.java:63-118, ExceptionCircuitBreaker.java:62-113) */
static void cb_on_complete(or_breaker* cb, int64_t t, int64_t rt, int error) {
    int s = or_leap_current_window(cb->stat, t);
    int is_rt = cb->rule.grade == SG_DEGRADE_RT;
    int64_t max_rt = or_math_round(cb->rule.count);
    if (s != -1) {
        if (is_rt ? (rt > max_rt) : error) or_leap_slot_add(cb->stat, s, 0, 1);
        or_leap_slot_add(cb->stat, s, 1, 1);
    }
    if (cb->state == OR_CB_OPEN) return;
    if (cb->state == OR_CB_HALF_OPEN) {
        int bad = is_rt ? (rt > max_rt) : error;
        if (bad) {
            cb_to_open(cb, t);
        } else {
            cb->state = OR_CB_CLOSED; /* fromHalfOpenToClose → resetStat: currentWindow().value().reset() */
            int r = or_leap_current_window(cb->stat, t);
            if (r >= 0 || r == -2) {
                or_bucket* w = slot_ptr(cb->stat, r);
                for (int e = 0; e < OR_MAX_EV; e++) w->c[e] = 0;
            }
        }
        return;
    }
    int64_t bad = 0, total = 0;
    for (int i = 0; i < cb->stat->S; i++) { /* values() at the exit time */
        if (!cb->stat->present[i] || is_deprecated(cb->stat, t, &cb->stat->b[i])) continue;
        bad += cb->stat->b[i].c[0];
        total += cb->stat->b[i].c[1];
    }
    if (total < cb->rule.min_request_amount) return;
    if (is_rt) {
        double ratio = bad * 1.0 / total;
        if (ratio > cb->rule.slow_ratio_threshold) cb_to_open(cb, t);
        if (ratio == cb->rule.slow_ratio_threshold && cb->rule.slow_ratio_threshold == 1.0 && cb->state == OR_CB_CLOSED)
            cb_to_open(cb, t);
    } else {
        double cur = (double)bad;
        if (cb->rule.grade == SG_DEGRADE_EXCEPTION_RATIO) cur = bad * 1.0 / total;
        if (cur > cb->rule.count) cb_to_open(cb, t);
    }
}

/* StatisticSlot.exit → recordCompleteFor (StatisticSlot.java:124-165): addRtAndSuccess, decreaseThreadNum,
 * increaseExceptionQps */
static void record_complete(or_node* nd, int64_t t, int count, int64_t rt, int error) {
    node_add(nd->second, t, OR_M_SUCCESS, count);
    { int s = or_leap_current_window(nd->second, t); if (s != -1) or_leap_slot_add_rt(nd->second, s, rt); }
    node_add(nd->minute, t, OR_M_SUCCESS, count);
    { int s = or_leap_current_window(nd->minute, t); if (s != -1) or_leap_slot_add_rt(nd->minute, s, rt); }
    nd->threads--;
    if (error) {
        node_add(nd->second, t, OR_M_EXCEPTION, count);
        node_add(nd->minute, t, OR_M_EXCEPTION, count);
    }
}

static int pslot_entry(struct or_pslot* s, uint32_t res, int64_t t, int count, const sg_pslot_arg* a, uint32_t na,
                       const uint64_t* values);
static void pslot_exit(struct or_pslot* s, uint32_t res, int64_t t, const sg_pslot_arg* a, uint32_t na,
                       const uint64_t* values, int d);

/* The slot chain for one event (CtSph.entryWithPriority → the ProcessorSlot chain in @Spi order, Constants.java:76-83):
 * StatisticSlot.entry (:55-122) around ParamFlowSlot (order -3000, ParamFlowSlot.java:38-93) → FlowSlot → DegradeSlot;
 * Entry.exit → StatisticSlot.exit (:124-165) with the param exit callback, DegradeSlot.exit. */
static void local_event(or_local* l, const sg_local_event* e, const sg_slot_ext* x, const sg_pslot_arg* args,
                        const uint64_t* values, sg_local_result* out) {
    uint32_t res = e->resource & SG_KEY_INDEX;
    int prio = (e->resource & SG_KEY_PRIO) != 0;
    out->status = SG_LOCAL_PASS;
    out->wait_ms = 0;
    if (res >= l->n) return;
    const int context = x ? (int)x->context : 0;
    const int args_null = !x || x->args_null;
    const sg_pslot_arg* a = x ? args + x->arg_begin : NULL;
    const uint32_t na = x ? x->arg_count : 0;
    or_node* nd = &l->nodes[res];
    or_node* on = origin_node(l, nd, e->origin);   /* context.getCurEntry().getOriginNode() */
    or_node* dn = context_node(l, nd, context);    /* the DefaultNode (NodeSelectorSlot); mirrors into nd */
    or_node* en = l->inbound[res] ? l->entry : NULL; /* EntryType.IN: Constants.ENTRY_NODE (StatisticSlot :71-75) */
    int64_t t = e->ts_ms;
    int count = e->count;
    if (e->kind == SG_LOCAL_ENTRY) {
        nd->created = 1;                           /* ClusterBuilderSlot */
        int64_t wait = 0;
        int status = SG_LOCAL_PASS;
        int32_t prule = -1;
        if (l->ps && !args_null) {                 /* ParamFlowSlot.checkFlow */
            prule = pslot_entry(l->ps, res, t, count, a, na, values);
            if (prule >= 0) status = SG_LOCAL_BLOCK_PARAM;
        }
        if (status == SG_LOCAL_PASS) status = check_flow(l, nd, t, count, prio, e->origin, context, &wait);   /* FlowSlot */
        int half[2] = {0, 0};
        if (status == SG_LOCAL_PASS) { /* DegradeSlot.performChecking */
            for (int j = 0; j < nd->rule.n_breakers && j < 2; j++) {
                if (!cb_try_pass(&nd->cb[j], t, &half[j])) {
                    status = SG_LOCAL_BLOCK_DEGRADE;
                    break;
                }
            }
            if (status == SG_LOCAL_BLOCK_DEGRADE) /* whenTerminate hook: blocked probe → OPEN again */
                for (int j = 0; j < 2; j++)
                    if (half[j] && nd->cb[j].state == OR_CB_HALF_OPEN) nd->cb[j].state = OR_CB_OPEN;
        }
        /* StatisticSlot.entry (:55-122): the DefaultNode (→ ClusterNode) and the origin node */
        or_node* upd[4] = {nd, on, dn, en};
        if (status == SG_LOCAL_PASS) {
            for (int u = 0; u < 4; u++) {
                if (!upd[u]) continue;
                upd[u]->threads++;
                node_add(upd[u]->second, t, OR_M_PASS, count); /* addPassRequest: both windows */
                node_add(upd[u]->minute, t, OR_M_PASS, count);
            }
            out->wait_ms = wait > INT32_MAX ? INT32_MAX : (int32_t)wait;   /* the rate limiters' sleep */
        } else if (status == SG_LOCAL_PASS_WAIT) {
            for (int u = 0; u < 4; u++)
                if (upd[u]) upd[u]->threads++;
            out->wait_ms = (int32_t)wait;
        } else {
            for (int u = 0; u < 4; u++) {
                if (!upd[u]) continue;
                node_add(upd[u]->second, t, OR_M_BLOCK, count); /* increaseBlockQps */
                node_add(upd[u]->minute, t, OR_M_BLOCK, count);
            }
            if (status == SG_LOCAL_BLOCK_PARAM) out->wait_ms = prule;
        }
        /* ParamFlowStatisticEntryCallback.onPass: ParameterMetric.addThreadCount(args) */
        if ((status == SG_LOCAL_PASS || status == SG_LOCAL_PASS_WAIT) && l->ps && !args_null)
            pslot_exit(l->ps, res, t, a, na, values, +1);
        out->status = status;
    } else {
        int error = e->kind == SG_LOCAL_EXIT_ERROR;
        int64_t rt = t - e->create_ts;
        record_complete(nd, t, count, rt, error);
        if (on) record_complete(on, t, count, rt, error);
        if (dn) record_complete(dn, t, count, rt, error);
        if (en) record_complete(en, t, count, rt, error);
        /* ParamFlowStatisticExitCallback.onExit: decreaseThreadCount(args) (the entry passed) */
        if (l->ps && !args_null) pslot_exit(l->ps, res, t, a, na, values, -1);
        /* DegradeSlot.exit → onRequestComplete */
        for (int j = 0; j < nd->rule.n_breakers && j < 2; j++) cb_on_complete(&nd->cb[j], t, rt, error);
    }
}

int or_local_decide_ext(or_local* l, const sg_local_event* ev, const sg_slot_ext* ext, uint64_t n,
                        const sg_pslot_arg* args, const uint64_t* values, sg_local_result* out) {
    for (uint64_t i = 0; i < n; i++) {
        if (ev[i].origin < 0 || ev[i].origin > l->n_origins) return SG_E_INVAL;
        if (ext && (int64_t)ext[i].context >= (int64_t)(l->n_contexts > 0 ? l->n_contexts : 1)) return SG_E_INVAL;
    }
    for (uint64_t i = 0; i < n; i++) local_event(l, &ev[i], ext ? &ext[i] : NULL, args, values, &out[i]);
    if (n) l->batches++;
    return 0;
}

int or_local_decide(or_local* l, const sg_local_event* ev, uint64_t n, sg_local_result* out) {
    return or_local_decide_ext(l, ev, NULL, n, NULL, NULL, out);
}

void or_local_attach_pslot(or_local* l, struct or_pslot* ps) {
    l->ps = ps;
    if (ps) or_pslot_attach_cluster(ps, l->cts, l->cluster_state);
}

int64_t or_local_second_sum(or_local* l, uint32_t res, int64_t t, int ev) {
    return res < l->n ? or_leap_get_sum(l->nodes[res].second, t, ev) : 0;
}
int64_t or_local_minute_sum(or_local* l, uint32_t res, int64_t t, int ev) {
    return res < l->n ? or_leap_get_sum(l->nodes[res].minute, t, ev) : 0;
}
int64_t or_local_thread_num(const or_local* l, uint32_t res) { return res < l->n ? l->nodes[res].threads : 0; }
int64_t or_local_waiting(or_local* l, uint32_t res, int64_t t) {
    return res < l->n ? or_leap_current_waiting(l->nodes[res].second, t) : 0;
}
int or_local_breaker_state(const or_local* l, uint32_t res, int i, int64_t* next_retry) {
    if (res >= l->n || i < 0 || i >= l->nodes[res].rule.n_breakers) return -1;
    *next_retry = l->nodes[res].cb[i].next_retry;
    return l->nodes[res].cb[i].state;
}

static void dump_leap(const or_leap* w, int64_t* out, int with_minrt) {
    for (int i = 0; i < w->S; i++) {
        int64_t* o = out + (size_t)i * (with_minrt ? 8 : 2);
        if (!with_minrt) {
            o[0] = w->present[i] ? w->b[i].start : INT64_MIN;
            o[1] = w->present[i] ? w->b[i].c[OR_M_PASS] : 0;
            continue;
        }
        o[0] = w->present[i] ? w->b[i].start : INT64_MIN;
        for (int e = 0; e < OR_M_NUM; e++) o[1 + e] = w->present[i] ? w->b[i].c[e] : 0;
        o[7] = w->present[i] ? w->b[i].min_rt : 0;
    }
}

int or_local_dump(const or_local* l, uint32_t res, int64_t* second, int64_t* borrow, int64_t* minute) {
    if (res >= l->n) return SG_E_INVAL;
    const or_node* nd = &l->nodes[res];
    dump_leap(nd->second, second, 1);
    dump_leap(nd->second->borrow, borrow, 0);
    dump_leap(nd->minute, minute, 1);
    return 0;
}

static int dump_plain(const or_local* l, const or_node* on, int64_t* second, int64_t* borrow, int64_t* minute,
                      int64_t* threads);

/* The origin node of (res, origin): windows as or_local_dump, *threads = curThreadNum. Returns 1 when the node
 * exists (some event carried the origin), 0 when it was never created (all-empty dumps), < 0 on bad input. */
int or_local_origin_dump(const or_local* l, uint32_t res, int origin, int64_t* second, int64_t* borrow,
                         int64_t* minute, int64_t* threads) {
    if (res >= l->n || origin <= 0 || origin > l->n_origins) return SG_E_INVAL;
    const or_node* nd = &l->nodes[res];
    const or_node* on = origin < nd->origin_cap ? nd->origin[origin] : NULL;
    return dump_plain(l, on, second, borrow, minute, threads);
}

/* The DefaultNode of (res, context) (NodeSelectorSlot): same outputs as or_local_origin_dump. */
int or_local_context_dump(const or_local* l, uint32_t res, int context, int64_t* second, int64_t* borrow,
                          int64_t* minute, int64_t* threads) {
    if (res >= l->n || context < 0 || context >= l->n_contexts) return SG_E_INVAL;
    const or_node* nd = &l->nodes[res];
    return dump_plain(l, context < nd->ctx_cap ? nd->ctxn[context] : NULL, second, borrow, minute, threads);
}

static int dump_plain(const or_local* l, const or_node* on, int64_t* second, int64_t* borrow, int64_t* minute,
                      int64_t* threads) {
    if (!on) {
        for (int i = 0; i < l->S; i++) {
            for (int e = 0; e < 8; e++) second[8 * i + e] = e == 0 ? INT64_MIN : 0;
            borrow[2 * i] = INT64_MIN;
            borrow[2 * i + 1] = 0;
        }
        for (int i = 0; i < 60; i++)
            for (int e = 0; e < 8; e++) minute[8 * i + e] = e == 0 ? INT64_MIN : 0;
        *threads = 0;
        return 0;
    }
    dump_leap(on->second, second, 1);
    dump_leap(on->second->borrow, borrow, 0);
    dump_leap(on->minute, minute, 1);
    *threads = on->threads;
    return 1;
}

/* The input indices of resource res's flow rules in check order; returns their number. */
int or_local_rule_order(const or_local* l, uint32_t res, int32_t* out, uint32_t cap) {
    if (res >= l->n) return SG_E_INVAL;
    const or_node* nd = &l->nodes[res];
    for (uint32_t i = 0; i < nd->n_ctl && i < cap; i++) out[i] = nd->ctl[i].input;
    return (int)nd->n_ctl;
}

/* {storedTokens, lastFilledTime, latestPassedTime} of loaded flow rule i; SG_E_INVAL when it was ignored. */
int or_local_controller(const or_local* l, uint32_t i, int64_t* out3) {
    if (i >= l->n_rules || l->rule_pos[i] < 0) return SG_E_INVAL;
    const or_node* nd = &l->nodes[(uint64_t)l->rule_pos[i] >> 32];
    or_ctl_state(&nd->ctl[l->rule_pos[i] & 0xFFFFFFFF], out3);
    return 0;
}

/* ===================================================================================== */
/* Local-chain trace generator (test infrastructure): a client that exits only the entries */
/* that passed, as SphU.entry callers do (a BlockException means there is no Entry to exit) */
/* ===================================================================================== */

typedef struct or_pending {
    int64_t ts, create_ts, seq;
    uint32_t resource;
    int32_t count, error, origin;
    sg_slot_ext ext;          /* the entry's context and arguments (Entry.exit(count, args) passes them again) */
} or_pending;

struct or_lgen {
    or_local* l;
    or_pending* heap;
    uint64_t n, cap;
    int64_t seq;
};

static int pend_less(const or_pending* a, const or_pending* b) {
    return a->ts < b->ts || (a->ts == b->ts && a->seq < b->seq);
}

static void pend_push(or_lgen* g, or_pending p) {
    if (g->n == g->cap) {
        g->cap = g->cap ? 2 * g->cap : 1024;
        g->heap = (or_pending*)realloc(g->heap, g->cap * sizeof(or_pending));
    }
    uint64_t i = g->n++;
    g->heap[i] = p;
    while (i > 0) {
        uint64_t par = (i - 1) / 2;
        if (!pend_less(&g->heap[i], &g->heap[par])) break;
        or_pending t = g->heap[i];
        g->heap[i] = g->heap[par];
        g->heap[par] = t;
        i = par;
    }
}

static or_pending pend_pop(or_lgen* g) {
    or_pending top = g->heap[0];
    g->heap[0] = g->heap[--g->n];
    uint64_t i = 0;
    for (;;) {
        uint64_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < g->n && pend_less(&g->heap[l], &g->heap[m])) m = l;
        if (r < g->n && pend_less(&g->heap[r], &g->heap[m])) m = r;
        if (m == i) break;
        or_pending t = g->heap[i];
        g->heap[i] = g->heap[m];
        g->heap[m] = t;
        i = m;
    }
    return top;
}

or_lgen* or_lgen_new(or_local* l) {
    or_lgen* g = (or_lgen*)calloc(1, sizeof(or_lgen));
    g->l = l;
    return g;
}

void or_lgen_free(or_lgen* g) {
    if (!g) return;
    free(g->heap);
    free(g);
}

uint64_t or_lgen_pending(const or_lgen* g) { return g->n; }

/* Merge time-ordered entries with the exits of the passed ones (exit at ts + waitInMs + rt; exits due at
 * the same ms as an entry go first), replaying every emitted event through the oracle. Events with
 * ts >= t_end are not emitted (exits stay pending for the next call). Returns the number emitted, or
 * UINT64_MAX when `cap` is too small. ext_in / ext_out (both NULL or both given): each entry's context and
 * arguments, which its exit carries again; args / values: the argument pool the ext records index. */
uint64_t or_lgen_run_ext(or_lgen* g, const sg_local_event* entries, const sg_slot_ext* ext_in, const int32_t* rt,
                         const uint8_t* err, uint64_t n, int64_t t_end, sg_local_event* out, sg_slot_ext* ext_out,
                         sg_local_result* res, uint64_t cap, const sg_pslot_arg* args, const uint64_t* values) {
    uint64_t k = 0, i = 0;
    for (;;) {
        int take_exit;
        if (i < n && g->n) take_exit = g->heap[0].ts <= entries[i].ts_ms;
        else if (g->n) take_exit = 1;
        else if (i < n) take_exit = 0;
        else break;
        if (take_exit && g->heap[0].ts >= t_end) {
            if (i >= n) break;
            take_exit = 0;
        }
        if (k == cap) return UINT64_MAX;
        sg_local_event* e = &out[k];
        sg_slot_ext* x = ext_out ? &ext_out[k] : NULL;
        if (take_exit) {
            or_pending p = pend_pop(g);
            e->ts_ms = p.ts;
            e->create_ts = p.create_ts;
            e->resource = p.resource;
            e->count = p.count;
            e->kind = p.error ? SG_LOCAL_EXIT_ERROR : SG_LOCAL_EXIT;
            e->origin = p.origin;
            if (x) *x = p.ext;
            or_local_decide_ext(g->l, e, x, 1, args, values, &res[k]);
            k++;
            continue;
        }
        *e = entries[i];
        e->kind = SG_LOCAL_ENTRY;
        e->create_ts = 0;
        if (x) *x = ext_in[i];
        or_local_decide_ext(g->l, e, x, 1, args, values, &res[k]);
        if (res[k].status == SG_LOCAL_PASS || res[k].status == SG_LOCAL_PASS_WAIT) {
            or_pending p;
            p.create_ts = e->ts_ms;
            p.ts = e->ts_ms + res[k].wait_ms + (rt ? rt[i] : 0);
            p.seq = g->seq++;
            p.resource = e->resource & SG_KEY_INDEX;
            p.count = e->count;
            p.error = err ? err[i] : 0;
            p.origin = e->origin;
            if (x) p.ext = *x;
            else memset(&p.ext, 0, sizeof(p.ext));
            pend_push(g, p);
        }
        k++;
        i++;
    }
    return k;
}

uint64_t or_lgen_run(or_lgen* g, const sg_local_event* entries, const int32_t* rt, const uint8_t* err, uint64_t n,
                     int64_t t_end, sg_local_event* out, sg_local_result* res, uint64_t cap) {
    return or_lgen_run_ext(g, entries, NULL, rt, err, n, t_end, out, NULL, res, cap, NULL, NULL);
}

/* Breaker i's statistic bucket (LeapArray(1, statIntervalMs)): start (INT64_MIN if never created), slow or
 * error count, total count. */
int or_local_breaker_stat(const or_local* l, uint32_t res, int i, int64_t* start, int64_t* bad, int64_t* total) {
    if (res >= l->n || i < 0 || i >= l->nodes[res].rule.n_breakers) return -1;
    const or_leap* s = l->nodes[res].cb[i].stat;
    *start = s->present[0] ? s->b[0].start : INT64_MIN;
    *bad = s->present[0] ? s->b[0].c[0] : 0;
    *total = s->present[0] ? s->b[0].c[1] : 0;
    return 0;
}


/* ===================================================================================== */
/* ClusterParamMetric (srv/flow/statistic/metric/ClusterParamMetric.java:37-88) over a    */
/* ClusterParameterLeapArray (…/ClusterParameterLeapArray.java:29-51): a LeapArray whose   */
/* buckets are value → LongAdder maps; a reset clears the whole map.                       */
/* ===================================================================================== */

typedef struct or_vmap {       /* open-addressing u64 → i64 map (a bucket's CacheMap, no eviction) */
    uint64_t* k;
    int64_t* v;
    uint8_t* used;
    uint32_t cap, n;
} or_vmap;

static void vmap_clear(or_vmap* m) {
    if (m->used) memset(m->used, 0, m->cap);
    m->n = 0;
}

static int64_t* vmap_find(const or_vmap* m, uint64_t key) {
    if (!m->cap) return NULL;
    uint32_t i = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & (m->cap - 1);
    while (m->used[i]) {
        if (m->k[i] == key) return &m->v[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}

static int64_t* vmap_get_or_add(or_vmap* m, uint64_t key) {
    int64_t* f = vmap_find(m, key);
    if (f) return f;
    if (2 * (m->n + 1) > m->cap) {
        or_vmap g = {0};
        g.cap = m->cap ? 2 * m->cap : 16;
        g.k = (uint64_t*)calloc(g.cap, 8);
        g.v = (int64_t*)calloc(g.cap, 8);
        g.used = (uint8_t*)calloc(g.cap, 1);
        for (uint32_t i = 0; i < m->cap; i++)
            if (m->used[i]) *vmap_get_or_add(&g, m->k[i]) = m->v[i];
        free(m->k);
        free(m->v);
        free(m->used);
        *m = g;
    }
    uint32_t i = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 40) & (m->cap - 1);
    while (m->used[i]) i = (i + 1) & (m->cap - 1);
    m->used[i] = 1;
    m->k[i] = key;
    m->v[i] = 0;
    m->n++;
    return &m->v[i];
}

struct or_cpm {
    int S, wl, interval;
    double isec;
    uint8_t* present;
    int64_t* start;
    or_vmap* maps;
};

static or_cpm* cpm_new(int S, int interval) {
    if (S <= 0 || interval <= 0 || interval % S != 0) return NULL;
    or_cpm* m = (or_cpm*)calloc(1, sizeof(or_cpm));
    m->S = S;
    m->wl = interval / S;
    m->interval = interval;
    m->isec = interval / 1000.0;  /* LeapArray.intervalInSecond */
    m->present = (uint8_t*)calloc(S, 1);
    m->start = (int64_t*)calloc(S, 8);
    m->maps = (or_vmap*)calloc(S, sizeof(or_vmap));
    return m;
}

static void cpm_free(or_cpm* m) {
    if (!m) return;
    for (int i = 0; i < m->S; i++) {
        free(m->maps[i].k);
        free(m->maps[i].v);
        free(m->maps[i].used);
    }
    free(m->maps);
    free(m->start);
    free(m->present);
    free(m);
}

/* LeapArray.currentWindow (LeapArray.java:116-202) with ClusterParameterLeapArray.newEmptyBucket (:43-45,
 * an empty map) and resetWindowTo (:47-51, clear the map). Returns the slot, -2 for a detached bucket. */
static int cpm_current_window(or_cpm* m, int64_t t) {
    int idx = (int)((t / m->wl) % m->S);
    int64_t ws = t - t % m->wl;
    if (!m->present[idx]) {
        m->present[idx] = 1;
        m->start[idx] = ws;
        vmap_clear(&m->maps[idx]);
        return idx;
    }
    if (ws == m->start[idx]) return idx;
    if (ws > m->start[idx]) {
        m->start[idx] = ws;
        vmap_clear(&m->maps[idx]);
        return idx;
    }
    return -2;
}

/* ClusterParamMetric.getSum(value), :48-61: currentWindow(); Σ over values() of bucket.get(value) */
static int64_t cpm_get_sum(or_cpm* m, int64_t t, uint64_t value) {
    cpm_current_window(m, t);
    int64_t sum = 0;
    for (int i = 0; i < m->S; i++) {
        if (!m->present[i] || t - m->start[i] > m->interval) continue;  /* isWindowDeprecated */
        const int64_t* c = vmap_find(&m->maps[i], value);
        if (c) sum += *c;
    }
    return sum;
}

/* ClusterParamMetric.addValue(value, count), :67-78 (a detached bucket's adds are lost) */
static void cpm_add(or_cpm* m, int64_t t, uint64_t value, int count) {
    int s = cpm_current_window(m, t);
    if (s < 0) return;
    *vmap_get_or_add(&m->maps[s], value) += count;
}

/* ClusterParamFlowRuleManager.applyClusterParamRules (…/ClusterParamFlowRuleManager.java:337-360): a flowId
 * that survives keeps its metric (putMetricIfAbsent :354-355), removed ones lose it. */
int or_cts_load_param_rules(or_cts* s, const sg_cparam_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                            uint32_t n_hot) {
    or_cpr* nr = (or_cpr*)calloc(n ? n : 1, sizeof(or_cpr));
    sg_param_hot_item* ph = (sg_param_hot_item*)calloc(n_hot ? n_hot : 1, sizeof(sg_param_hot_item));
    memcpy(ph, hot, n_hot * sizeof(sg_param_hot_item));
    for (uint32_t i = 0; i < n; i++) {
        nr[i].rule = rules[i];
        nr[i].hot = ph + rules[i].hot_begin;
        for (uint32_t j = 0; j < s->n_prules; j++) {
            if (s->prules[j].metric && s->prules[j].rule.flow_id == rules[i].flow_id) {
                nr[i].metric = s->prules[j].metric;
                s->prules[j].metric = NULL;
                break;
            }
        }
        if (!nr[i].metric) nr[i].metric = cpm_new(rules[i].sample_count, rules[i].window_interval_ms);
        if (!nr[i].metric) return SG_E_INVAL;
    }
    for (uint32_t j = 0; j < s->n_prules; j++) cpm_free(s->prules[j].metric);
    free(s->prules);
    free(s->phot);
    s->prules = nr;
    s->n_prules = n;
    s->phot = ph;
    return 0;
}

/* ClusterParamFlowChecker.calcGlobalThreshold / getRawThreshold (:96-116): the value's exclusive item count
 * (ParamFlowRule.retrieveExclusiveItemCount) or rule.count; AVG_LOCAL multiplies by the connected count.
 * (No exceedCount here, unlike ClusterFlowChecker.) */
static double cparam_threshold(const or_cts* s, const or_cpr* r, uint64_t value) {
    double count = r->rule.count;
    for (uint32_t i = 0; i < r->rule.hot_count; i++)
        if (r->hot[i].value == value) {
            count = (double)r->hot[i].threshold;
            break;
        }
    if (r->rule.threshold_type == SG_THRESHOLD_GLOBAL) return count;
    int ns = r->rule.namespace_id;
    int connected = (ns >= 0 && (uint32_t)ns < s->n_ns) ? s->ns[ns].connected_count : 0;
    return count * connected;
}

/* DefaultTokenService.requestParamToken (DefaultTokenService.java:53-64) → ClusterParamFlowChecker.
 * acquireClusterToken (ClusterParamFlowChecker.java:42-87) for one request of m values at time t: all values are
 * checked (first failure blocks, nothing added), then the count is added to every value. *remaining: the last
 * value's nextRemaining (-1 for several values, "remaining is unsupported for multi-values"). */
static int32_t cts_param_token(or_cts* s, uint32_t key, int64_t t, int32_t acquire, const uint64_t* vals, uint32_t m,
                               double* remaining) {
    *remaining = -1;
    key &= SG_KEY_INDEX;
    if (key == SG_KEY_BAD || acquire <= 0 || m == 0) return SG_STATUS_BAD_REQUEST;  /* notValidRequest, params empty */
    if (key >= s->n_prules) return SG_STATUS_NO_RULE_EXISTS;
    or_cpr* r = &s->prules[key];
    int ns = r->rule.namespace_id;  /* allowProceed → GlobalRequestLimiter.tryPass(namespace) */
    if (ns < 0 || (uint32_t)ns >= s->n_ns) return SG_STATUS_TOO_MANY_REQUEST;
    if (s->limiters[ns] && !or_limiter_try_pass(s->limiters[ns], t)) return SG_STATUS_TOO_MANY_REQUEST;
    double rem = -1;
    for (uint32_t v = 0; v < m; v++) {
        double latest = (double)cpm_get_sum(r->metric, t, vals[v]) / r->metric->isec;  /* getAvg */
        double next_remaining = cparam_threshold(s, r, vals[v]) - latest - acquire;
        rem = next_remaining;
        if (next_remaining < 0) return SG_STATUS_BLOCKED;
    }
    for (uint32_t v = 0; v < m; v++) cpm_add(r->metric, t, vals[v], acquire);
    *remaining = m > 1 ? -1 : rem;
    return SG_STATUS_OK;
}

int or_cts_decide_param(or_cts* s, const sg_cparam_req* req, uint64_t n, const uint64_t* values, sg_result* out) {
    for (uint64_t i = 0; i < n; i++) {
        const sg_cparam_req* q = &req[i];
        double remaining;
        const int32_t st = cts_param_token(s, q->key, q->ts_ms, q->acquire, values + q->value_begin, q->value_count,
                                           &remaining);
        out[i] = st == SG_STATUS_OK ? mk(SG_STATUS_OK, or_d2i(remaining), 0) : mk(st, 0, 0);
    }
    return 0;
}

int64_t or_cts_param_sum(or_cts* s, uint32_t key, uint64_t value, int64_t now) {
    if (key >= s->n_prules) return 0;
    return cpm_get_sum(s->prules[key].metric, now, value);
}

/* Standalone ClusterParamMetric for the known-answer tests (ClusterParamMetricTest.java). */
or_cpm* or_cpm_new(int sample_count, int interval_ms) { return cpm_new(sample_count, interval_ms); }
void or_cpm_free(or_cpm* m) { cpm_free(m); }
void or_cpm_add(or_cpm* m, int64_t t, uint64_t value, int count) { cpm_add(m, t, value, count); }
int64_t or_cpm_get_sum(or_cpm* m, int64_t t, uint64_t value) { return cpm_get_sum(m, t, value); }
double or_cpm_get_avg(or_cpm* m, int64_t t, uint64_t value) { return (double)cpm_get_sum(m, t, value) / m->isec; }

/* ==================================================================================== wire codec ==== */
/* Restates the default token server's request decoding and response encoding byte for byte. Paths:
 * srv/ = sentinel-cluster-server-default/.../cluster/server/. Netty's ByteBuf is big-endian:
 * readInt/readLong/writeInt are network order. */

static int64_t or_be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return (int64_t)v;
}

static int32_t or_be32(const uint8_t* p) {
    return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}

static void or_put32(uint8_t* p, int32_t v) {
    p[0] = (uint8_t)((uint32_t)v >> 24);
    p[1] = (uint8_t)((uint32_t)v >> 16);
    p[2] = (uint8_t)((uint32_t)v >> 8);
    p[3] = (uint8_t)v;
}

typedef struct {
    int64_t fid;
    uint32_t idx;
} or_fid;

static int or_fid_cmp(const void* a, const void* b) {
    const or_fid* x = (const or_fid*)a;
    const or_fid* y = (const or_fid*)b;
    return x->fid < y->fid ? -1 : x->fid > y->fid ? 1 : 0;
}

void or_codec_decode_flow(const uint8_t* payload, const uint32_t* offsets, const int64_t* ts_ms, uint64_t n,
                          const int64_t* flow_ids, uint32_t n_rules, sg_req* req_out, int32_t* xid_out,
                          uint8_t* kind_out) {
    /* ClusterFlowRuleManager.getFlowRuleById: flowId → rule (here its index; flowIds are unique) */
    or_fid* map = (or_fid*)malloc(sizeof(or_fid) * (n_rules ? n_rules : 1));
    for (uint32_t i = 0; i < n_rules; ++i) {
        map[i].fid = flow_ids[i];
        map[i].idx = i;
    }
    qsort(map, n_rules, sizeof(or_fid), or_fid_cmp);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* p = payload + offsets[i];
        const uint32_t len = offsets[i + 1] - offsets[i];
        sg_req r;
        r.ts_ms = ts_ms[i];
        r.key = SG_KEY_BAD;
        r.acquire = 0;
        int32_t xid = 0;
        uint8_t kind;
        if (len < 5) {  /* DefaultRequestEntityDecoder.decode (:37): readableBytes() >= 5, else null */
            kind = SG_FRAME_SHORT;
        } else {
            xid = or_be32(p);                 /* :38 source.readInt() */
            const int type = (int8_t)p[4];    /* :39 source.readByte() */
            const uint32_t rem = len - 5;
            if (type != SG_MSG_TYPE_FLOW) {
                kind = SG_FRAME_OTHER;
            } else if (rem < 12) {  /* FlowRequestDataDecoder.decode (:33): readableBytes() >= 12, else null */
                kind = SG_FRAME_NO_DATA;
            } else {
                kind = SG_FRAME_FLOW;
                const int64_t flow_id = or_be64(p + 5);       /* :35 readLong() */
                const int32_t count = or_be32(p + 13);        /* :36 readInt() */
                const int prio = rem >= 13 ? p[17] != 0 : 0;  /* :37-39 readBoolean() when a byte is left */
                r.acquire = count;
                if (flow_id <= 0) {  /* DefaultTokenService.notValidRequest (:87-89) → badRequest() */
                    r.key = SG_KEY_BAD;
                } else {
                    or_fid want = {flow_id, 0};
                    const or_fid* hit = (const or_fid*)bsearch(&want, map, n_rules, sizeof(or_fid), or_fid_cmp);
                    r.key = hit ? hit->idx : SG_KEY_NO_RULE;  /* rule == null → NO_RULE_EXISTS (:44-47) */
                }
                if (prio) r.key |= SG_KEY_PRIO;
            }
        }
        req_out[i] = r;
        xid_out[i] = xid;
        kind_out[i] = kind;
    }
    free(map);
}

void or_codec_encode_flow(const int32_t* xid, const uint8_t* kind, const sg_result* res, uint64_t n,
                          uint8_t* frames_out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t* f = frames_out + (size_t)SG_RESPONSE_FRAME_BYTES * i;
        memset(f, 0, SG_RESPONSE_FRAME_BYTES);
        if (kind[i] != SG_FRAME_FLOW) continue;
        f[0] = 0;  /* LengthFieldPrepender(2) (NettyTransportServer.java:91): payload length 14, big-endian */
        f[1] = 14;
        or_put32(f + 2, xid[i]);                /* DefaultResponseEntityWriter.writeHead: writeInt(id) */
        f[6] = (uint8_t)SG_MSG_TYPE_FLOW;       /* writeByte(type) */
        f[7] = (uint8_t)(int8_t)res[i].status;  /* writeByte(status): the low 8 bits */
        or_put32(f + 8, res[i].remaining);      /* FlowResponseDataWriter.writeTo: writeInt(remainingCount) */
        or_put32(f + 12, res[i].wait_ms);       /* writeInt(waitInMs) */
    }
}

/* ============================================================================== Envoy RLS path ==== */
/* SimpleClusterFlowChecker.acquireClusterToken (sentinel-cluster-server-envoy-rls/.../flow/
 * SimpleClusterFlowChecker.java:33-65) for each request in array order: the same ClusterMetric as the token
 * server, threshold rule.count * exceedCount whatever the threshold type, no namespace limiter, no
 * prioritized occupy. acquire is the service's acquireCount (hitsAddend, 0 → 1,
 * SentinelEnvoyRlsServiceImpl.java:35-44); key >= rules → NO_RULE_EXISTS (checkToken :99-109). */
int or_rls_decide(or_cts* s, const sg_req* req, uint64_t n, sg_result* out) {
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t key = req[i].key & SG_KEY_INDEX;
        const int64_t t = req[i].ts_ms;
        const int acq = req[i].acquire;
        if (key >= s->n_rules) {
            out[i] = mk(SG_STATUS_NO_RULE_EXISTS, 0, 0);
            continue;
        }
        or_cts_rule* r = &s->rules[key];
        const double latest = or_cluster_metric_get_avg(r->metric, t, SG_EV_PASS);  /* :41 */
        const double thr = r->count * s->exceed_count;                              /* :42 */
        const double next_remaining = thr - latest - (double)acq;                   /* :43 */
        if (next_remaining >= 0) {
            or_cluster_metric_add(r->metric, t, SG_EV_PASS, acq);                   /* :46-47 */
            or_cluster_metric_add(r->metric, t, SG_EV_PASS_REQUEST, 1);
            out[i] = mk(SG_STATUS_OK, or_d2i(next_remaining), 0);                   /* :53-55 */
        } else {
            or_cluster_metric_add(r->metric, t, SG_EV_BLOCK, acq);                  /* :58-59 */
            or_cluster_metric_add(r->metric, t, SG_EV_BLOCK_REQUEST, 1);
            out[i] = mk(SG_STATUS_BLOCKED, 0, 0);                                   /* blockedResult :67-71 */
        }
    }
    return 0;
}

/* SentinelEnvoyRlsServiceImpl.shouldRateLimit (sentinel-cluster/sentinel-cluster-server-envoy-rls/src/main/java/com/
 * alibaba/csp/sentinel/cluster/server/envoy/rls/service/v3/SentinelEnvoyRlsServiceImpl.java:34-85), one request after
 * the other: hits_addend < 0 fails the call (onError :36-40), 0 means 1 (:41-44); every descriptor is checkToken →
 * SimpleClusterFlowChecker.acquireClusterToken (or_rls_decide above) on its rule (desc_rule: the rule index
 * EnvoySentinelRuleConverter.generateFlowId resolves to, < 0 or unknown: no rule); NO_RULE_EXISTS passes (:55-58); the
 * call is OVER_LIMIT when any descriptor is not OK (:60-62); a descriptor with a rule reports (int) rule.getCount() and
 * the TokenResult's remaining (:66-73). */
int or_rls_should_rate_limit(or_cts* s, const sg_rls_request* req, uint32_t n, const int32_t* desc_rule,
                             uint64_t n_desc, int32_t* overall, sg_rls_status* status) {
    for (uint64_t d = 0; d < n_desc; d++) memset(&status[d], 0, sizeof(sg_rls_status));
    for (uint32_t j = 0; j < n; j++) {
        const sg_rls_request* q = &req[j];
        if ((uint64_t)q->desc_begin + q->desc_count > n_desc) return SG_E_INVAL;
        if (q->hits_addend < 0) {
            overall[j] = SG_RLS_ERROR;
            continue;
        }
        const int acquire = q->hits_addend == 0 ? 1 : q->hits_addend;
        int blocked = 0;
        for (uint32_t i = 0; i < q->desc_count; i++) {
            const int32_t rule = desc_rule[q->desc_begin + i];
            const int has_rule = rule >= 0 && (uint32_t)rule < s->n_rules;
            sg_req one;
            one.ts_ms = q->ts_ms;
            one.key = has_rule ? (uint32_t)rule : SG_KEY_NO_RULE;
            one.acquire = acquire;
            sg_result r;
            or_rls_decide(s, &one, 1, &r);
            int st = r.status;
            if (st == SG_STATUS_NO_RULE_EXISTS) st = SG_STATUS_OK;
            if (st != SG_STATUS_OK) blocked = 1;
            sg_rls_status* o = &status[q->desc_begin + i];
            o->code = st == SG_STATUS_OK ? SG_RLS_OK : SG_RLS_OVER_LIMIT;
            if (has_rule) {
                o->has_rule = 1;
                o->requests_per_unit = or_d2i(s->rules[rule].count);
                o->limit_remaining = r.remaining;
            }
        }
        overall[j] = blocked ? SG_RLS_OVER_LIMIT : SG_RLS_OK;
    }
    return 0;
}

/* ===================================================================================== */
/* Concurrent cluster tokens: ConcurrentClusterFlowChecker (srv/flow/ConcurrentClusterFlowChecker.java:34-101), */
/* CurrentConcurrencyManager (nowCalls per flowId), TokenCacheNodeManager (the token map) and              */
/* RegularExpireStrategy.clearToken (…/statistic/concurrent/expire/RegularExpireStrategy.java:94-137).    */
/* Token ids are 1 + the number of requests decided before the acquire (sg_conc_req contract).             */
/* ===================================================================================== */

typedef struct or_ctok {         /* TokenCacheNode (TokenCacheNode.java) */
    uint64_t id;
    int64_t flow_id, client_timeout, resource_timeout;
    int32_t acquire;
    uint32_t client;
    int alive;
} or_ctok;

struct or_conc {
    sg_flow_rule* rules;
    int64_t* client_off;          /* ClusterFlowConfig.clientOfflineTime per rule */
    int64_t* res_to;              /* ClusterFlowConfig.resourceTimeout per rule   */
    int32_t* now_calls;           /* CurrentConcurrencyManager.NOW_CALLS_MAP       */
    uint32_t n;
    sg_namespace* ns;
    uint32_t n_ns;
    or_ctok* tok;                 /* in id order (ids increase) */
    uint64_t n_tok, cap_tok, live;
    uint64_t seq;                 /* requests decided so far */
};

or_conc* or_conc_new(void) { return (or_conc*)calloc(1, sizeof(or_conc)); }

void or_conc_free(or_conc* c) {
    if (!c) return;
    free(c->rules);
    free(c->client_off);
    free(c->res_to);
    free(c->now_calls);
    free(c->ns);
    free(c->tok);
    free(c);
}

int or_conc_set_namespaces(or_conc* c, const sg_namespace* ns, uint32_t n) {
    free(c->ns);
    c->ns = (sg_namespace*)malloc((n ? n : 1) * sizeof(sg_namespace));
    memcpy(c->ns, ns, n * sizeof(sg_namespace));
    c->n_ns = n;
    return 0;
}

/* ClusterFlowRuleManager.applyClusterFlowRule: nowCalls put(flowId, 0) when absent (:356-358), removed with the
 * flowId (clearAndResetRulesConditional :287-300) */
int or_conc_load_rules(or_conc* c, const sg_flow_rule* rules, uint32_t n) {
    int32_t* now = (int32_t*)calloc(n ? n : 1, sizeof(int32_t));
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t j = 0; j < c->n; j++)
            if (c->rules[j].flow_id == rules[i].flow_id) now[i] = c->now_calls[j];
    free(c->rules);
    free(c->now_calls);
    free(c->client_off);
    free(c->res_to);
    c->rules = (sg_flow_rule*)malloc((n ? n : 1) * sizeof(sg_flow_rule));
    memcpy(c->rules, rules, n * sizeof(sg_flow_rule));
    c->now_calls = now;
    c->client_off = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    c->res_to = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    for (uint32_t i = 0; i < n; i++) c->client_off[i] = c->res_to[i] = 2000;   /* ClusterFlowConfig defaults */
    c->n = n;
    return 0;
}

int or_conc_set_rule_timeouts(or_conc* c, const int64_t* client_off, const int64_t* res_to, uint32_t n) {
    if (n != c->n) return SG_E_INVAL;
    memcpy(c->client_off, client_off, n * sizeof(int64_t));
    memcpy(c->res_to, res_to, n * sizeof(int64_t));
    return 0;
}

static int conc_rule_of(const or_conc* c, int64_t flow_id) {   /* ClusterFlowRuleManager.getFlowRuleById */
    for (uint32_t i = 0; i < c->n; i++)
        if (c->rules[i].flow_id == flow_id) return (int)i;
    return -1;
}

/* ConcurrentClusterFlowChecker.calcGlobalThreshold (:36-46): no exceedCount on this path */
static double conc_threshold(const or_conc* c, uint32_t k) {
    const sg_flow_rule* r = &c->rules[k];
    if (r->threshold_type == SG_THRESHOLD_GLOBAL) return r->count;
    int connected = (r->namespace_id >= 0 && (uint32_t)r->namespace_id < c->n_ns) ? c->ns[r->namespace_id].connected_count : 0;
    return r->count * connected;
}

static or_ctok* conc_find(or_conc* c, uint64_t id) {          /* TokenCacheNodeManager.getTokenCacheNode */
    uint64_t lo = 0, hi = c->n_tok;
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (c->tok[mid].id < id) lo = mid + 1;
        else hi = mid;
    }
    return (lo < c->n_tok && c->tok[lo].id == id && c->tok[lo].alive) ? &c->tok[lo] : NULL;
}

int or_conc_decide(or_conc* c, const sg_conc_req* req, uint64_t n, sg_conc_result* out) {
    for (uint64_t i = 0; i < n; i++, c->seq++) {
        const sg_conc_req* q = &req[i];
        sg_conc_result* o = &out[i];
        o->reserved = 0;
        o->token_id = 0;
        if (q->kind == SG_CONC_ACQUIRE) {
            /* DefaultTokenService.requestConcurrentToken (:66-77) */
            const uint32_t k = q->key & SG_KEY_INDEX;
            if (q->client == 0 || k == SG_KEY_BAD || q->acquire <= 0) { o->status = SG_STATUS_BAD_REQUEST; continue; }
            if (k >= c->n) { o->status = SG_STATUS_NO_RULE_EXISTS; continue; }
            /* acquireConcurrentToken (:48-79): nowCalls + acquireCount > threshold (int + int, then double) */
            const int32_t sum = (int32_t)((uint32_t)c->now_calls[k] + (uint32_t)q->acquire);
            if ((double)sum > conc_threshold(c, k)) { o->status = SG_STATUS_BLOCKED; continue; }
            c->now_calls[k] = sum;
            if (c->n_tok == c->cap_tok) {
                c->cap_tok = c->cap_tok ? 2 * c->cap_tok : 1024;
                c->tok = (or_ctok*)realloc(c->tok, c->cap_tok * sizeof(or_ctok));
            }
            or_ctok* t = &c->tok[c->n_tok++];
            t->id = c->seq + 1;
            t->flow_id = c->rules[k].flow_id;
            t->client_timeout = c->client_off[k] + q->ts_ms;   /* setClientTimeout: + currentTimeMillis */
            t->resource_timeout = c->res_to[k] + q->ts_ms;
            t->acquire = q->acquire;
            t->client = q->client;
            t->alive = 1;
            c->live++;
            o->status = SG_STATUS_OK;
            o->token_id = t->id;
        } else if (q->kind == SG_CONC_RELEASE) {
            /* releaseConcurrentToken (:81-101) */
            if (q->token_id == 0) { o->status = SG_STATUS_BAD_REQUEST; continue; }
            or_ctok* t = conc_find(c, q->token_id);
            if (!t) { o->status = SG_STATUS_ALREADY_RELEASE; continue; }
            const int r = conc_rule_of(c, t->flow_id);
            if (r < 0) { o->status = SG_STATUS_NO_RULE_EXISTS; continue; }
            t->alive = 0;
            c->live--;
            c->now_calls[r] = (int32_t)((uint32_t)c->now_calls[r] - (uint32_t)t->acquire);
            o->status = SG_STATUS_RELEASE_OK;
        } else {
            o->status = SG_STATUS_BAD_REQUEST;
        }
    }
    return 0;
}

/* RegularExpireStrategy.clearToken over every token: client offline past clientTimeout, or held for more than
 * resourceTimeout past its resource deadline (rule looked up by flowId; tokens of a removed rule only expire by
 * the client condition). Returns the number removed. */
uint64_t or_conc_expire(or_conc* c, int64_t now, const uint8_t* online, uint32_t n_clients) {
    uint64_t removed = 0;
    for (uint64_t i = 0; i < c->n_tok; i++) {
        or_ctok* t = &c->tok[i];
        if (!t->alive) continue;
        const int on = t->client < n_clients && online[t->client];
        const int r = conc_rule_of(c, t->flow_id);
        int drop = !on && t->client_timeout - now < 0;
        if (!drop && r >= 0 && now - t->resource_timeout > c->res_to[r]) drop = 1;
        if (!drop) continue;
        t->alive = 0;
        c->live--;
        removed++;
        if (r >= 0) c->now_calls[r] = (int32_t)((uint32_t)c->now_calls[r] - (uint32_t)t->acquire);
    }
    return removed;
}

int32_t or_conc_now_calls(const or_conc* c, uint32_t k) { return k < c->n ? c->now_calls[k] : 0; }
uint64_t or_conc_live(const or_conc* c) { return c->live; }

/* ===================================================================================== */
/* Metric snapshots: StatisticNode.metrics() rows (core/.../node/StatisticNode.java:116-147 over             */
/* ArrayMetric.details, ArrayMetric.java:156-204) and ClusterParamMetric.getTopValues (…/ClusterParamMetric.java: */
/* 90-133).                                                                                                      */
/* ===================================================================================== */

static int metric_row_less(const sg_metric_node* a, const sg_metric_node* b) {
    return a->timestamp != b->timestamp ? a->timestamp < b->timestamp : a->resource < b->resource;
}

/* MetricTimerListener.run over every resource: rows sorted by (timestamp, resource); returns the number of rows
 * (all of them are written when cap allows; lastFetchTime advances only then). */
/* StatisticNode.metrics() of one node at now (StatisticNode.java:116-147): the minute window's buckets newer than
 * *last_fetch, older than now's second, non-empty; emit: write them (resource id `res`), advance *last_fetch and run
 * currentWindow's side effect. Returns the rows. */
static uint64_t node_rows(or_leap* m, int64_t now, int64_t* last_fetch, uint32_t res, sg_metric_node* out, int emit,
                          int raw) {
    const int64_t cur = now - now % 1000;
    if (emit) or_leap_current_window(m, now);                   /* data.currentWindow() */
    int64_t newest = *last_fetch;
    uint64_t rows = 0;
    for (int j = 0; j < m->S; j++) {                            /* data.list(): not deprecated at now */
        if (!m->present[j] || is_deprecated(m, now, &m->b[j])) continue;
        const or_bucket* b = &m->b[j];
        if (!(b->start > *last_fetch && b->start < cur)) continue;   /* isNodeInTime */
        const int64_t succ = b->c[OR_M_SUCCESS];
        const int64_t rt = succ != 0 ? b->c[OR_M_RT] / succ : b->c[OR_M_RT];
        if (!(b->c[OR_M_PASS] > 0 || b->c[OR_M_BLOCK] > 0 || succ > 0 || b->c[OR_M_EXCEPTION] > 0 || rt > 0 ||
              b->c[OR_M_OCCUPIED_PASS] > 0))
            continue;                                           /* isValidMetricNode */
        if (emit) {
            sg_metric_node* r = &out[rows];
            r->timestamp = b->start;
            r->pass_qps = b->c[OR_M_PASS];
            r->block_qps = b->c[OR_M_BLOCK];
            r->success_qps = succ;
            r->exception_qps = b->c[OR_M_EXCEPTION];
            r->rt = raw ? b->c[OR_M_RT] : rt;   /* raw: the sum, for a node rollup (sg_local_metrics_raw) */
            r->occupied_pass_qps = b->c[OR_M_OCCUPIED_PASS];
            r->resource = res;
            r->concurrency = 0;
            if (b->start > newest) newest = b->start;
        }
        rows++;
    }
    if (emit) *last_fetch = newest;
    return rows;
}

/* MetricTimerListener.run (MetricTimerListener.java:40-55): every resource's ClusterNode, then Constants.ENTRY_NODE
 * (resource id SG_ENTRY_NODE_RESOURCE), rows sorted by (timestamp, resource) as its TreeMap of time → list */
int64_t or_local_metrics_raw(or_local* l, int64_t now, sg_metric_node* out, uint64_t cap, int raw) {
    if (!l->last_fetch) {
        l->last_fetch = (int64_t*)malloc((l->n ? l->n : 1) * sizeof(int64_t));
        for (uint32_t k = 0; k < l->n; k++) l->last_fetch[k] = -1;
    }
    uint64_t rows = 0;
    for (uint32_t k = 0; k < l->n; k++) rows += node_rows(l->nodes[k].minute, now, &l->last_fetch[k], k, NULL, 0, raw);
    if (l->entry) rows += node_rows(l->entry->minute, now, &l->entry_fetch, SG_ENTRY_NODE_RESOURCE, NULL, 0, raw);
    if (rows > cap) return (int64_t)rows;
    rows = 0;
    for (uint32_t k = 0; k < l->n; k++) rows += node_rows(l->nodes[k].minute, now, &l->last_fetch[k], k, out + rows, 1, raw);
    if (l->entry) rows += node_rows(l->entry->minute, now, &l->entry_fetch, SG_ENTRY_NODE_RESOURCE, out + rows, 1, raw);
    for (uint64_t i = 1; i < rows; i++) {                           /* insertion sort by (timestamp, resource) */
        sg_metric_node x = out[i];
        uint64_t j = i;
        while (j > 0 && metric_row_less(&x, &out[j - 1])) {
            out[j] = out[j - 1];
            j--;
        }
        out[j] = x;
    }
    return (int64_t)rows;
}

int64_t or_local_metrics(or_local* l, int64_t now, sg_metric_node* out, uint64_t cap) {
    return or_local_metrics_raw(l, now, out, cap, 0);
}

int or_local_set_entry_types(or_local* l, const uint8_t* inbound, uint32_t n) {
    if (n != l->n) return SG_E_INVAL;
    for (uint32_t k = 0; k < n; k++) l->inbound[k] = inbound[k] ? 1 : 0;
    return 0;
}

typedef struct { uint64_t v; int64_t c; } or_topent;

static int topent_cmp(const void* x, const void* y) {
    const or_topent* a = (const or_topent*)x;
    const or_topent* b = (const or_topent*)y;
    const int32_t ca = (int32_t)a->c, cb = (int32_t)b->c;   /* the comparator compares (int) casts */
    if (ca != cb) return ca > cb ? -1 : 1;
    return a->v < b->v ? -1 : (a->v > b->v ? 1 : 0);          /* ties: value order (HashMap order in Java) */
}

/* ClusterParamMetric.getTopValues(number) at now: values[] / qps[] get up to `number` entries. */
int or_cpm_top(or_cpm* m, int64_t now, int number, uint64_t* values, double* qps) {
    if (number <= 0) return SG_E_INVAL;   /* AssertUtil.isTrue(number > 0) */
    cpm_current_window(m, now);
    uint64_t cap = 0, n = 0;
    for (int i = 0; i < m->S; i++) cap += m->maps[i].n;
    or_topent* e = (or_topent*)malloc((cap ? cap : 1) * sizeof(or_topent));
    for (int i = 0; i < m->S; i++) {                                /* merge the valid buckets' maps */
        if (!m->present[i] || now - m->start[i] > m->interval) continue;
        const or_vmap* mp = &m->maps[i];
        for (uint32_t j = 0; j < mp->cap; j++) {
            if (!mp->used[j]) continue;
            uint64_t x = 0;
            while (x < n && e[x].v != mp->k[j]) x++;
            if (x == n) {
                e[n].v = mp->k[j];
                e[n].c = 0;
                n++;
            }
            e[x].c += mp->v[j];
        }
    }
    qsort(e, n, sizeof(or_topent), topent_cmp);
    int k = 0;
    for (uint64_t i = 0; i < n && k < number; i++) {
        if (e[i].c == 0) break;
        values[k] = e[i].v;
        qps[k] = (double)e[i].c / m->isec;
        k++;
    }
    free(e);
    return k;
}

int or_cts_param_top(or_cts* s, uint32_t key, int64_t now, int number, uint64_t* values, double* qps) {
    if (key >= s->n_prules) return SG_E_INVAL;
    return or_cpm_top(s->prules[key].metric, now, number, values, qps);
}

/* ===================================================================================== */
/* ParamFlowSlot.checkFlow (sentinel-extension/sentinel-parameter-flow-control/.../ParamFlowSlot.java:55-93)  */
/* over ParamFlowChecker.passCheck / passLocalCheck / passSingleValueCheck (ParamFlowChecker.java:48-122)      */
/* and ParameterMetric's thread counts (ParameterMetric.java:125-249), on top of or_pf's token maps.          */
/* ===================================================================================== */

typedef struct or_tc {            /* threadCountMap entry: (resource, paramIdx, value) → count */
    uint64_t value;
    uint32_t res;
    int32_t idx;
    int64_t count;
    uint8_t used;
} or_tc;

struct or_pslot {
    or_pf* pf;                    /* token / time counters per (rule, value) */
    sg_pslot_rule* rules;
    int32_t* cur_idx;             /* the rule's paramIdx (applyRealParamIdx rewrites a negative one once) */
    uint8_t* inited;              /* initParamMetricsFor ran: threadCountMap.get(paramIdx) exists */
    uint32_t n, n_res;
    or_tc* tc;
    uint64_t tc_cap, tc_size;
    int64_t now;                  /* the event's TimeUtil time */
    or_cts* cts;                  /* the embedded token server's DefaultTokenService (cluster_state SERVER) */
    int cluster_state;            /* ClusterStateManager: SG_CLUSTER_NOT_STARTED (default), SERVER */
    uint32_t* res_off;            /* [n_res + 1]: rules of resource r = res_rules[res_off[r] .. res_off[r + 1]) */
    uint32_t* res_rules;          /* rule indices grouped by resource, ascending (getRulesOfResource: load order) */
};

or_pslot* or_pslot_new(void) {
    or_pslot* s = (or_pslot*)calloc(1, sizeof(or_pslot));
    s->pf = or_pf_new();
    s->tc_cap = 1024;
    s->tc = (or_tc*)calloc(s->tc_cap, sizeof(or_tc));
    s->cluster_state = SG_CLUSTER_NOT_STARTED;
    return s;
}

int or_pslot_attach_cluster(or_pslot* s, or_cts* cts, int state) {
    if (state == SG_CLUSTER_SERVER && !cts) return -1;
    s->cts = cts;
    s->cluster_state = state;
    return 0;
}

void or_pslot_free(or_pslot* s) {
    if (!s) return;
    or_pf_free(s->pf);
    free(s->rules);
    free(s->cur_idx);
    free(s->inited);
    free(s->tc);
    free(s->res_off);
    free(s->res_rules);
    free(s);
}

int or_pslot_load_rules(or_pslot* s, const sg_pslot_rule* rules, uint32_t n, const sg_param_hot_item* hot,
                        uint32_t n_hot, uint32_t n_res) {
    sg_param_rule* pr = (sg_param_rule*)calloc(n ? n : 1, sizeof(sg_param_rule));
    for (uint32_t i = 0; i < n; i++) pr[i] = rules[i].rule;
    or_pf_load_rules(s->pf, pr, n, hot, n_hot);
    free(pr);
    free(s->rules);
    free(s->cur_idx);
    free(s->inited);
    s->rules = (sg_pslot_rule*)malloc((n ? n : 1) * sizeof(sg_pslot_rule));
    memcpy(s->rules, rules, n * sizeof(sg_pslot_rule));
    s->cur_idx = (int32_t*)malloc((n ? n : 1) * sizeof(int32_t));
    s->inited = (uint8_t*)calloc(n ? n : 1, 1);
    for (uint32_t i = 0; i < n; i++) s->cur_idx[i] = rules[i].param_idx;
    s->n = n;
    s->n_res = n_res;
    free(s->res_off);
    free(s->res_rules);
    s->res_off = (uint32_t*)calloc((size_t)n_res + 1, sizeof(uint32_t));
    s->res_rules = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; i++)
        if (rules[i].resource < n_res) s->res_off[rules[i].resource + 1]++;
    for (uint32_t r = 0; r < n_res; r++) s->res_off[r + 1] += s->res_off[r];
    {
        uint32_t* fill = (uint32_t*)malloc(((size_t)n_res + 1) * sizeof(uint32_t));
        memcpy(fill, s->res_off, ((size_t)n_res + 1) * sizeof(uint32_t));
        for (uint32_t i = 0; i < n; i++)
            if (rules[i].resource < n_res) s->res_rules[fill[rules[i].resource]++] = i;
        free(fill);
    }
    memset(s->tc, 0, s->tc_cap * sizeof(or_tc));
    s->tc_size = 0;
    return 0;
}

static uint64_t tc_hash(uint32_t res, int32_t idx, uint64_t v) {
    uint64_t z = v + 0x9E3779B97F4A7C15ULL * ((uint64_t)res * 64 + (uint32_t)idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static or_tc* tc_find(const or_pslot* s, uint32_t res, int32_t idx, uint64_t v) {
    uint64_t i = tc_hash(res, idx, v) & (s->tc_cap - 1);
    for (;;) {
        or_tc* e = &s->tc[i];
        if (!e->used || (e->res == res && e->idx == idx && e->value == v)) return e;
        i = (i + 1) & (s->tc_cap - 1);
    }
}

static or_tc* tc_get_or_add(or_pslot* s, uint32_t res, int32_t idx, uint64_t v) {
    if ((s->tc_size + 1) * 2 > s->tc_cap) {
        or_tc* old = s->tc;
        uint64_t oc = s->tc_cap;
        s->tc_cap *= 2;
        s->tc = (or_tc*)calloc(s->tc_cap, sizeof(or_tc));
        for (uint64_t i = 0; i < oc; i++)
            if (old[i].used) *tc_find(s, old[i].res, old[i].idx, old[i].value) = old[i];
        free(old);
    }
    or_tc* e = tc_find(s, res, idx, v);
    if (!e->used) {
        e->used = 1;
        e->res = res;
        e->idx = idx;
        e->value = v;
        e->count = 0;
        s->tc_size++;
    }
    return e;
}

int64_t or_pslot_thread_count(const or_pslot* s, uint32_t res, int32_t idx, uint64_t v) {
    or_tc* e = tc_find(s, res, idx, v);
    return e->used ? e->count : 0;
}

int32_t or_pslot_param_idx(const or_pslot* s, uint32_t rule) { return rule < s->n ? s->cur_idx[rule] : INT32_MIN; }

/* passSingleValueCheck (:106-125) */
static int pslot_single(or_pslot* s, uint32_t ri, uint32_t res, int count, uint64_t v) {
    const sg_pslot_rule* r = &s->rules[ri];
    if (r->grade == 1) {
        if (r->rule.behavior == 2) return pf_throttle(s->pf, ri, v, s->now, count);
        return pf_default(s->pf, ri, v, s->now, count);
    }
    if (r->grade == 0) {
        or_tc* e = tc_find(s, res, s->cur_idx[ri], v);
        int64_t threads = e->used ? e->count : 0;
        for (uint32_t i = 0; i < r->rule.hot_count; i++)   /* exclusionItems: the hot item's threshold */
            if (s->pf->hot[r->rule.hot_begin + i].value == v) return ++threads <= s->pf->hot[r->rule.hot_begin + i].threshold;
        return ++threads <= or_d2l(r->rule.count);
    }
    return 1;
}

/* ParameterMetric.addThreadCount / decreaseThreadCount (:184-239) over the indices whose map exists */
static void pslot_threads(or_pslot* s, uint32_t res, const sg_pslot_arg* args, uint32_t na, const uint64_t* values, int d) {
    for (uint32_t idx = 0; idx < na; idx++) {
        int has_map = 0;
        for (uint32_t q = s->res_off[res]; q < s->res_off[res + 1] && !has_map; q++) {
            const uint32_t r = s->res_rules[q];
            has_map = s->rules[r].cluster_mode != SG_CLUSTER_MODE_INVALID && s->inited[r] && s->cur_idx[r] == (int32_t)idx;
        }
        if (!has_map) continue;
        const sg_pslot_arg* a = &args[idx];
        if (a->kind == SG_ARG_NULL) continue;
        const uint32_t m = a->kind == SG_ARG_COLLECTION ? a->value_count : 1;
        for (uint32_t j = 0; j < m; j++) {
            const uint64_t v = values[a->value_begin + j];
            if (d > 0) {
                tc_get_or_add(s, res, (int32_t)idx, v)->count += 1;
            } else {
                /* putIfAbsent(value, new AtomicInteger()): an absent value is inserted at 0 and not decremented;
                 * a present one is decremented and removed at <= 0 (a removed entry reads 0) */
                or_tc* e = tc_find(s, res, (int32_t)idx, v);
                if (e->used && e->count > 0) e->count -= 1;
                else if (e->used) e->count = 0;
                else tc_get_or_add(s, res, (int32_t)idx, v);
            }
        }
    }
}

/* ParamFlowChecker.passLocalCheck (:78-103): every value of the argument in order, the first failing one blocks */
static int pslot_local(or_pslot* s, uint32_t r, uint32_t res, int count, const sg_pslot_arg* x, const uint64_t* values) {
    const uint32_t m = x->kind == SG_ARG_COLLECTION ? x->value_count : 1;
    for (uint32_t j = 0; j < m; j++)
        if (!pslot_single(s, r, res, count, values[x->value_begin + j])) return 0;
    return 1;
}

/* ParamFlowChecker.passClusterCheck (:278-303): the embedded server's param token for all of the argument's values
 * (toCollection) on SERVER — OK passes, BLOCKED blocks, any other status falls back — else (no token service)
 * fallbackToLocalOrPass (:305-313): the local check with fallbackToLocalWhenFail, a pass without it. */
static int pslot_cluster(or_pslot* s, uint32_t r, uint32_t res, int count, const sg_pslot_arg* x,
                         const uint64_t* values) {
    const sg_pslot_rule* rule = &s->rules[r];
    if (s->cluster_state == SG_CLUSTER_SERVER && s->cts) {
        const uint32_t m = x->kind == SG_ARG_COLLECTION ? x->value_count : 1;
        double rem;
        const int32_t st = cts_param_token(s->cts, rule->cluster_key, s->now, count, values + x->value_begin, m, &rem);
        if (st == SG_STATUS_OK) return 1;
        if (st == SG_STATUS_BLOCKED) return 0;
    }
    if (rule->cluster_mode == SG_CLUSTER_MODE_NO_FALLBACK) return 1;  /* the rule won't be activated: pass */
    return pslot_local(s, r, res, count, x, values);
}

/* ParamFlowSlot.checkFlow (ParamFlowSlot.java:66-93) for one entry with non-null args: the index of the rule that
 * throws ParamFlowException, or -1 */
static int pslot_entry(or_pslot* s, uint32_t res, int64_t t, int count, const sg_pslot_arg* a, uint32_t na,
                       const uint64_t* values) {
    s->now = t;
    if (res >= s->n_res) return -1;
    for (uint32_t q = s->res_off[res]; q < s->res_off[res + 1]; q++) {
        const uint32_t r = s->res_rules[q];
        if (s->rules[r].cluster_mode == SG_CLUSTER_MODE_INVALID) continue;  /* isValidRule → checkCluster: never loaded */
        /* applyRealParamIdx(rule, args.length) */
        if (s->cur_idx[r] < 0) s->cur_idx[r] = (-s->cur_idx[r] <= (int32_t)na) ? (int32_t)na + s->cur_idx[r] : -s->cur_idx[r];
        s->inited[r] = 1;                      /* ParameterMetricStorage.initParamMetricsFor */
        const int32_t idx = s->cur_idx[r];
        if ((int32_t)na <= idx) continue;      /* args.length <= paramIdx */
        const sg_pslot_arg* x = &a[idx];
        if (x->kind == SG_ARG_NULL) continue;
        /* passCheck (:71-75): clusterMode with grade QPS → passClusterCheck, else passLocalCheck */
        const int ok = (s->rules[r].cluster_mode != SG_CLUSTER_MODE_OFF && s->rules[r].grade == 1)
                           ? pslot_cluster(s, r, res, count, x, values)
                           : pslot_local(s, r, res, count, x, values);
        if (!ok) return (int32_t)r;
    }
    return -1;
}

/* ParamFlowStatisticEntryCallback.onPass (d = +1) / ParamFlowStatisticExitCallback.onExit (d = -1) */
static void pslot_exit(or_pslot* s, uint32_t res, int64_t t, const sg_pslot_arg* a, uint32_t na,
                       const uint64_t* values, int d) {
    s->now = t;
    if (res >= s->n_res) return;
    pslot_threads(s, res, a, na, values, d);
}

int or_pslot_decide(or_pslot* s, const sg_pslot_event* ev, uint64_t n, const sg_pslot_arg* args,
                    const uint64_t* values, sg_pslot_result* out) {
    for (uint64_t i = 0; i < n; i++) {
        const sg_pslot_event* e = &ev[i];
        out[i].pass = 1;
        out[i].rule = -1;
        const sg_pslot_arg* a = args + e->arg_begin;
        const uint32_t na = e->arg_count;
        s->now = e->ts_ms;
        if (e->resource >= s->n_res || e->args_null) continue;   /* ParamFlowSlot.checkFlow: args == null */
        if (e->kind != SG_LOCAL_ENTRY) {           /* ParamFlowStatisticExitCallback: passed entries only */
            pslot_exit(s, e->resource, e->ts_ms, a, na, values, -1);
            continue;
        }
        const int r = pslot_entry(s, e->resource, e->ts_ms, e->count, a, na, values);
        out[i].pass = r < 0;
        out[i].rule = r;
        if (r < 0) pslot_exit(s, e->resource, e->ts_ms, a, na, values, +1);   /* onPass */
    }
    return 0;
}

int or_pslot_token_state(const or_pslot* s, uint32_t rule, uint64_t value, int64_t* last_time, int64_t* tokens) {
    return or_pf_read_state(s->pf, rule, value, last_time, tokens);
}
