// token_service.cpp — see token_service.hpp.
#include "token_service.hpp"

#include <algorithm>
#include <cctype>
#include <stdexcept>

namespace sentinel {
namespace cluster {

namespace {

bool isBlank(const std::string& s) {
    return std::all_of(s.begin(), s.end(), [](unsigned char c) { return std::isspace(c); });
}

bool validClusterRuleId(const std::optional<int64_t>& id) { return id.has_value() && *id > 0; }

// FlowRuleUtil.isWindowConfigValid, FlowRuleUtil.java:227-229
bool isWindowConfigValid(int sampleCount, int windowIntervalMs) {
    return sampleCount > 0 && windowIntervalMs > 0 && windowIntervalMs % sampleCount == 0;
}

// FlowRuleUtil.checkClusterField, :206-225
bool checkClusterField(const FlowRule& r) {
    if (!r.clusterMode) return true;
    if (!r.clusterConfig) return false;
    const ClusterFlowConfig& c = *r.clusterConfig;
    if (!validClusterRuleId(c.flowId)) return false;
    if (!isWindowConfigValid(c.sampleCount, c.windowIntervalMs)) return false;
    return c.strategy == ClusterRuleConstant::FLOW_CLUSTER_STRATEGY_NORMAL;
}

// FlowRuleUtil.checkClusterConcurrentField, :184-204
bool checkClusterConcurrentField(const FlowRule& r) {
    if (!r.clusterMode) return true;
    if (!r.clusterConfig) return false;
    const ClusterFlowConfig& c = *r.clusterConfig;
    if (c.clientOfflineTime <= 0 || c.resourceTimeout <= 0) return false;
    if (c.acquireRefuseStrategy < 0 || c.resourceTimeoutStrategy < 0) return false;
    if (!validClusterRuleId(c.flowId)) return false;
    return isWindowConfigValid(c.sampleCount, c.windowIntervalMs);
}

// FlowRuleUtil.checkStrategyField, :231-236
bool checkStrategyField(const FlowRule& r) {
    if (r.strategy == RuleConstant::STRATEGY_RELATE || r.strategy == RuleConstant::STRATEGY_CHAIN)
        return !isBlank(r.refResource);
    return true;
}

// FlowRuleUtil.checkControlBehaviorField, :238-249
bool checkControlBehaviorField(const FlowRule& r) {
    switch (r.controlBehavior) {
    case RuleConstant::CONTROL_BEHAVIOR_WARM_UP: return r.warmUpPeriodSec > 0;
    case RuleConstant::CONTROL_BEHAVIOR_RATE_LIMITER: return r.maxQueueingTimeMs > 0;
    case RuleConstant::CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: return r.warmUpPeriodSec > 0 && r.maxQueueingTimeMs > 0;
    default: return true;
    }
}

int64_t systemMillis() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
        .count();
}

}  // namespace

bool isValidRule(const FlowRule& r) {
    const bool baseValid = !isBlank(r.resource) && r.count >= 0 && r.grade >= 0 && r.strategy >= 0 &&
                           r.controlBehavior >= 0;
    if (!baseValid) return false;
    if (r.grade == RuleConstant::FLOW_GRADE_QPS)
        return checkClusterField(r) && checkStrategyField(r) && checkControlBehaviorField(r);
    if (r.grade == RuleConstant::FLOW_GRADE_THREAD) return checkClusterConcurrentField(r);
    return false;
}

// ParamFlowRuleUtil.isValidRule / checkCluster, ParamFlowRuleUtil.java:46-66
bool isValidParamRule(const ParamFlowRule& r) {
    if (isBlank(r.resource) || !(r.count >= 0) || r.grade < 0 || !r.paramIdx || r.burstCount < 0 ||
        r.controlBehavior < 0 || r.durationInSec <= 0 || r.maxQueueingTimeMs < 0)
        return false;
    if (!r.clusterMode) return true;
    if (!r.clusterConfig) return false;
    const ParamFlowClusterConfig& c = *r.clusterConfig;
    if (!isWindowConfigValid(c.sampleCount, c.windowIntervalMs)) return false;
    return validClusterRuleId(c.flowId);
}

namespace {

// ParamFlowRuleUtil.parseItemValue (:211-240): the classTypes that parse to a primitive wrapper (never equal to
// a String parameter); any other classType, or none, keeps the string.
bool parsesToString(const std::string& classType) {
    static const char* prim[] = {"int", "java.lang.Integer", "boolean", "java.lang.Boolean", "long", "java.lang.Long",
                                 "double", "java.lang.Double", "float", "java.lang.Float", "byte", "java.lang.Byte",
                                 "short", "java.lang.Short", "char"};
    if (isBlank(classType)) return true;
    for (const char* p : prim)
        if (classType == p) return false;
    return true;
}

}  // namespace

GpuTokenService::GpuTokenService(Options opt) : opt_(std::move(opt)) {
    if (!opt_.clock) opt_.clock = systemMillis;
    sg_config cfg{};
    cfg.device = opt_.device;
    cfg.flags = 0;
    cfg.exceed_count = opt_.exceedCount;
    cfg.max_occupy_ratio = opt_.maxOccupyRatio;
    cfg.max_batch = opt_.maxBatch;
    if (!opt_.shardDevices.empty()) {  // node mode: flow tokens over the shards, the rest on the front handle
        std::vector<int32_t> devs(opt_.shardDevices.begin(), opt_.shardDevices.end());
        int rc = sg_node_create(&cfg, devs.data(), (uint32_t)devs.size(), &node_);
        if (rc != SG_OK) throw std::runtime_error("sg_node_create failed: " + std::to_string(rc));
        h_ = sg_node_front(node_);
    } else {
        int rc = sg_create(&cfg, &h_);
        if (rc != SG_OK) throw std::runtime_error("sg_create failed: " + std::to_string(rc));
    }
    const int depth = std::max(1, std::min(3, opt_.pipelineDepth));
    for (int i = 0; i < depth; ++i) {
        sg_req* rq = static_cast<sg_req*>(sg_host_alloc(h_, sizeof(sg_req) * opt_.maxBatch));
        sg_result* rs = static_cast<sg_result*>(sg_host_alloc(h_, sizeof(sg_result) * opt_.maxBatch));
        if (!rq || !rs) {
            sg_host_free(h_, rq);
            sg_host_free(h_, rs);
            for (auto& b : bufs_) {
                sg_host_free(h_, b.first);
                sg_host_free(h_, b.second);
            }
            if (node_) sg_node_destroy(node_);
            else sg_destroy(h_);
            throw std::runtime_error("sg_host_alloc failed");
        }
        bufs_.emplace_back(rq, rs);
        freeBufs_.push_back(i);
    }
    nsIndex("default");  // ServerConstants.DEFAULT_NAMESPACE
    {
        std::lock_guard<std::mutex> lk(mu_);
        pushNamespacesLocked();
    }
    completer_ = std::thread([this] { completerLoop(); });
    flusher_ = std::thread([this] { flusherLoop(); });
}

GpuTokenService::~GpuTokenService() {
    {
        std::unique_lock<std::mutex> lk(mu_);
        stop_ = true;
        if (!pending_.empty()) flushLocked(lk);
    }
    cv_.notify_all();
    if (flusher_.joinable()) flusher_.join();
    waitIdle();
    {
        std::lock_guard<std::mutex> lk(qmu_);
        stopCompleter_ = true;
    }
    qcv_.notify_all();
    if (completer_.joinable()) completer_.join();
    for (auto& b : bufs_) {
        sg_host_free(h_, b.first);
        sg_host_free(h_, b.second);
    }
    if (node_) sg_node_destroy(node_);  // owns the front handle
    else sg_destroy(h_);
}

void GpuTokenService::waitIdle() {
    std::unique_lock<std::mutex> lk(qmu_);
    qcv_.wait(lk, [this] { return inflight_.empty(); });
}

// Answers the micro-batches in submission order: polls the front ticket (without holding the engine lock
// while the GPU works), then fulfils its callers' promises from the pinned result buffer.
void GpuTokenService::completerLoop() {
    for (;;) {
        InFlight f;
        {
            std::unique_lock<std::mutex> lk(qmu_);
            qcv_.wait(lk, [this] { return stopCompleter_ || !inflight_.empty(); });
            if (inflight_.empty()) return;
            f = inflight_.front();
        }
        int rc = f.rc;
        if (rc == SG_OK) {
            for (;;) {
                int r;
                {
                    std::lock_guard<std::mutex> e(engMu_);
                    r = sg_flow_poll(h_, f.ticket);
                    if (r < 0) err_ = sg_last_error(h_);
                }
                if (r != 0) {
                    rc = r < 0 ? r : SG_OK;
                    break;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
        }
        const size_t n = f.waiters.size();
        const sg_result* out = bufs_[f.buf].second;
        if (opt_.onBatch) {
            std::vector<sg_req> rq(bufs_[f.buf].first, bufs_[f.buf].first + n);
            std::vector<sg_result> rs(out, out + n);
            opt_.onBatch(rq, rs, rc);
        }
        for (size_t i = 0; i < n; ++i) {
            if (rc != SG_OK) f.waiters[i]->set_value(TokenResult(TokenResultStatus::FAIL));
            else f.waiters[i]->set_value(TokenResult(out[i].status).setRemaining(out[i].remaining).setWaitInMs(out[i].wait_ms));
        }
        {
            std::lock_guard<std::mutex> lk(qmu_);
            inflight_.pop_front();
            freeBufs_.push_back(f.buf);
        }
        qcv_.notify_all();
    }
}

int GpuTokenService::nsIndex(const std::string& ns) {
    for (size_t i = 0; i < nsNames_.size(); ++i)
        if (nsNames_[i] == ns) return (int)i;
    nsNames_.push_back(ns);
    sg_namespace c{};
    c.limiter_enabled = 0;
    c.connected_count = 0;     // ConnectionManager: no connections until clients connect
    c.max_allowed_qps = 30000; // ServerFlowConfig.DEFAULT_MAX_ALLOWED_QPS
    nsCfg_.push_back(c);
    return (int)nsNames_.size() - 1;
}

void GpuTokenService::pushNamespacesLocked() {
    waitIdle();
    std::lock_guard<std::mutex> e(engMu_);
    if (node_) {
        int rc = sg_node_set_namespaces(node_, nsCfg_.data(), (uint32_t)nsCfg_.size());
        if (rc != SG_OK) err_ = sg_node_last_error(node_);
        return;
    }
    int rc = sg_set_namespaces(h_, nsCfg_.data(), (uint32_t)nsCfg_.size());
    if (rc != SG_OK) err_ = sg_last_error(h_);
}

// All namespaces' rules → one dense rule table, ascending flowId (the engine keeps the windows of
// flowIds that survive, like putMetricIfAbsent).
void GpuTokenService::pushRulesLocked() {
    std::vector<int64_t> ids;
    ids.reserve(rules_.size());
    for (const auto& kv : rules_) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    std::vector<sg_flow_rule> tab(ids.size());
    keyOfFlow_.clear();
    for (size_t i = 0; i < ids.size(); ++i) {
        const RuleEntry& e = rules_.at(ids[i]);
        const ClusterFlowConfig& c = *e.rule.clusterConfig;
        tab[i].flow_id = ids[i];
        tab[i].count = e.rule.count;
        tab[i].threshold_type = c.thresholdType;
        tab[i].sample_count = c.sampleCount;
        tab[i].window_interval_ms = c.windowIntervalMs;
        tab[i].namespace_id = nsIndex(e.ns);
        keyOfFlow_[ids[i]] = (uint32_t)i;
    }
    pushNamespacesLocked();
    std::lock_guard<std::mutex> e(engMu_);
    int rc = node_ ? sg_node_load_flow_rules(node_, tab.data(), (uint32_t)tab.size())
                   : sg_load_flow_rules(h_, tab.data(), (uint32_t)tab.size());
    if (rc != SG_OK) {
        err_ = node_ ? sg_node_last_error(node_) : sg_last_error(h_);
        keyOfFlow_.clear();
    }
}

// ClusterFlowRuleManager.applyClusterFlowRule, ClusterFlowRuleManager.java:325-375
void GpuTokenService::loadRules(const std::string& ns, const std::vector<FlowRule>& list) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);  // a reload is a barrier between batches
    std::map<int64_t, FlowRule> ruleMap;
    for (const FlowRule& r0 : list) {
        if (!r0.clusterMode) continue;
        if (!isValidRule(r0)) continue;   // "Ignoring invalid flow rule"
        FlowRule r = r0;
        if (isBlank(r.limitApp)) r.limitApp = "default";
        const auto& flowId = r.clusterConfig->flowId;
        if (!flowId) continue;
        ruleMap[*flowId] = r;             // the last duplicate wins (ruleMap.put)
    }
    // clearAndResetRulesConditional: drop this namespace's flowIds that are not in the new set
    for (int64_t id : nsFlowIds_[ns])
        if (!ruleMap.count(id)) rules_.erase(id);
    std::vector<int64_t> ids;
    for (auto& kv : ruleMap) {
        rules_[kv.first] = RuleEntry{kv.second, ns};
        ids.push_back(kv.first);
    }
    nsFlowIds_[ns] = ids;
    nsIndex(ns);
    pushRulesLocked();
}

void GpuTokenService::loadServerFlowConfig(const std::string& ns, bool limiterEnabled, double maxAllowedQps) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    const int i = nsIndex(ns);
    nsCfg_[i].limiter_enabled = limiterEnabled ? 1 : 0;
    nsCfg_[i].max_allowed_qps = maxAllowedQps;
    pushNamespacesLocked();
}

void GpuTokenService::setConnectedCount(const std::string& ns, int connected) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    nsCfg_[nsIndex(ns)].connected_count = connected;
    pushNamespacesLocked();
}

std::optional<FlowRule> GpuTokenService::getFlowRuleById(int64_t id) const {
    std::lock_guard<std::mutex> lk(mu_);
    if (id <= 0) return std::nullopt;  // ClusterRuleUtil.validId
    auto it = rules_.find(id);
    if (it == rules_.end()) return std::nullopt;
    return it->second.rule;
}

std::optional<std::string> GpuTokenService::getNamespace(int64_t flowId) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = rules_.find(flowId);
    if (it == rules_.end()) return std::nullopt;
    return it->second.ns;
}

// DefaultTokenService.notValidRequest (id) and the rule lookup (:39-47); acquireCount <= 0 is
// answered BAD_REQUEST by the engine itself.
uint32_t GpuTokenService::keyOf(std::optional<int64_t> ruleId, bool prioritized) const {
    if (!ruleId || *ruleId <= 0) return SG_KEY_BAD;
    auto it = keyOfFlow_.find(*ruleId);
    if (it == keyOfFlow_.end()) return SG_KEY_NO_RULE;
    return it->second | (prioritized ? SG_KEY_PRIO : 0u);
}

std::vector<TokenResult> GpuTokenService::decideLocked(std::vector<sg_req>& reqs) {
    std::vector<TokenResult> res(reqs.size(), TokenResult(TokenResultStatus::FAIL));
    if (reqs.empty()) return res;
    waitIdle();
    std::lock_guard<std::mutex> e(engMu_);
    std::vector<sg_result> out(reqs.size());
    for (size_t off = 0; off < reqs.size(); off += opt_.maxBatch) {
        const size_t n = std::min<size_t>(opt_.maxBatch, reqs.size() - off);
        int rc = node_ ? sg_node_flow_decide_batch_host(node_, reqs.data() + off, n, out.data() + off)
                       : sg_flow_decide_batch_host(h_, reqs.data() + off, n, out.data() + off);
        if (rc != SG_OK) {  // TokenResult(FAIL) → the client falls back to local checking
            err_ = node_ ? sg_node_last_error(node_) : sg_last_error(h_);
            continue;
        }
        for (size_t i = off; i < off + n; ++i)
            res[i] = TokenResult(out[i].status).setRemaining(out[i].remaining).setWaitInMs(out[i].wait_ms);
    }
    return res;
}

std::vector<TokenResult> GpuTokenService::requestTokens(const std::vector<TokenRequest>& reqs) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    std::vector<sg_req> r(reqs.size());
    for (size_t i = 0; i < reqs.size(); ++i) {
        r[i].ts_ms = reqs[i].timeMillis;
        r[i].key = keyOf(reqs[i].ruleId, reqs[i].prioritized);
        r[i].acquire = reqs[i].acquireCount;
        if (reqs[i].timeMillis > lastTs_) lastTs_ = reqs[i].timeMillis;
    }
    return decideLocked(r);
}

TokenResult GpuTokenService::requestToken(std::optional<int64_t> ruleId, int acquireCount, bool prioritized) {
    std::promise<TokenResult> p;
    std::future<TokenResult> f = p.get_future();
    {
        std::unique_lock<std::mutex> lk(mu_);
        sg_req r;
        // TimeUtil.currentTimeMillis at the call; kept non-decreasing in arrival order
        const int64_t now = opt_.clock();
        lastTs_ = std::max(lastTs_, now);
        r.ts_ms = lastTs_;
        r.key = keyOf(ruleId, prioritized);
        r.acquire = acquireCount;
        if (pending_.empty()) oldest_ = std::chrono::steady_clock::now();
        pending_.push_back(Pending{r, &p});
        if (pending_.size() >= opt_.flushSize) flushLocked(lk);
        else if (pending_.size() == 1) cv_.notify_all();
    }
    return f.get();
}

// Submit the pending requests (time-ordered by construction) as micro-batches through the host pipeline;
// called with mu_ held, so submission order = arrival order. Blocks only while every pipeline slot is busy.
void GpuTokenService::flushLocked(std::unique_lock<std::mutex>& lk) {
    std::vector<Pending> batch;
    batch.swap(pending_);
    for (size_t off = 0; off < batch.size(); off += opt_.maxBatch) {
        const size_t n = std::min<size_t>(opt_.maxBatch, batch.size() - off);
        int b;
        {
            std::unique_lock<std::mutex> q(qmu_);
            qcv_.wait(q, [this] { return !freeBufs_.empty(); });
            b = freeBufs_.back();
            freeBufs_.pop_back();
        }
        InFlight f{0, b, SG_OK, {}};
        f.waiters.reserve(n);
        for (size_t i = 0; i < n; ++i) {
            bufs_[b].first[i] = batch[off + i].req;
            f.waiters.push_back(batch[off + i].result);
        }
        {
            std::lock_guard<std::mutex> e(engMu_);
            if (node_) {  // the node routes and decides synchronously (ticket 0: done)
                f.rc = sg_node_flow_decide_batch_host(node_, bufs_[b].first, n, bufs_[b].second);
                if (f.rc != SG_OK) err_ = sg_node_last_error(node_);
            } else {
                f.rc = sg_flow_submit(h_, bufs_[b].first, n, bufs_[b].second, &f.ticket);
                if (f.rc != SG_OK) err_ = sg_last_error(h_);
            }
        }
        {
            std::lock_guard<std::mutex> q(qmu_);
            inflight_.push_back(std::move(f));
        }
        qcv_.notify_all();
    }
    (void)lk;
}

void GpuTokenService::flusherLoop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
        if (pending_.empty()) {
            cv_.wait(lk, [this] { return stop_ || !pending_.empty(); });
            continue;
        }
        const auto deadline = oldest_ + opt_.flushDelay;
        if (std::chrono::steady_clock::now() >= deadline) {
            flushLocked(lk);
        } else {
            cv_.wait_until(lk, deadline);
        }
    }
}

uint64_t GpuTokenService::valueId(const std::string& v) {
    auto it = valueIds_.find(v);
    if (it != valueIds_.end()) return it->second;
    const uint64_t id = (uint64_t)valueIds_.size() + 1;
    valueIds_.emplace(v, id);
    return id;
}

// All namespaces' cluster param rules → one table, ascending flowId; hot items through the value dictionary
// (ParamFlowRuleUtil.parseHotItems :188-209: null object or count < 0 skipped, a later duplicate wins).
void GpuTokenService::pushParamRulesLocked() {
    std::vector<sg_cparam_rule> tab;
    std::vector<sg_param_hot_item> hot;
    keyOfParam_.clear();
    for (const auto& kv : paramRules_) {
        const ParamFlowRule& r = kv.second.rule;
        const ParamFlowClusterConfig& c = *r.clusterConfig;
        sg_cparam_rule t{};
        t.flow_id = kv.first;
        t.count = r.count;
        t.threshold_type = c.thresholdType;
        t.sample_count = c.sampleCount;
        t.window_interval_ms = c.windowIntervalMs;
        t.namespace_id = nsIndex(kv.second.ns);
        std::map<uint64_t, int> items;
        for (const ParamFlowItem& it : r.paramFlowItemList) {
            if (!it.object || !it.count || *it.count < 0) continue;
            if (!parsesToString(it.classType)) continue;  // an Integer / Long … key never equals a String parameter
            items[valueId(*it.object)] = *it.count;
        }
        t.hot_begin = (uint32_t)hot.size();
        t.hot_count = (uint32_t)items.size();
        for (const auto& x : items) {
            sg_param_hot_item h{};
            h.value = x.first;
            h.threshold = x.second;
            hot.push_back(h);
        }
        keyOfParam_[kv.first] = (uint32_t)tab.size();
        tab.push_back(t);
    }
    pushNamespacesLocked();
    std::lock_guard<std::mutex> e(engMu_);
    int rc = sg_cparam_load_rules(h_, tab.data(), (uint32_t)tab.size(), hot.data(), (uint32_t)hot.size(),
                                  opt_.paramCapacityLog2);
    if (rc != SG_OK) {
        err_ = sg_last_error(h_);
        keyOfParam_.clear();
    }
}

// ClusterParamFlowRuleManager.applyClusterParamRules, ClusterParamFlowRuleManager.java:318-365
void GpuTokenService::loadParamRules(const std::string& ns, const std::vector<ParamFlowRule>& list) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    waitIdle();
    std::map<int64_t, ParamFlowRule> ruleMap;
    for (const ParamFlowRule& r0 : list) {
        if (!r0.clusterMode) continue;
        if (!isValidParamRule(r0)) continue;  // "Ignoring invalid param flow rule"
        ParamFlowRule r = r0;
        if (isBlank(r.limitApp)) r.limitApp = "default";
        const auto& flowId = r.clusterConfig->flowId;
        if (!flowId) continue;
        ruleMap[*flowId] = r;
    }
    for (int64_t id : nsParamIds_[ns])
        if (!ruleMap.count(id)) paramRules_.erase(id);
    std::vector<int64_t> ids;
    for (auto& kv : ruleMap) {
        paramRules_[kv.first] = ParamRuleEntry{kv.second, ns};
        ids.push_back(kv.first);
    }
    nsParamIds_[ns] = ids;
    nsIndex(ns);
    pushParamRulesLocked();
}

std::vector<TokenResult> GpuTokenService::decideParamLocked(const std::vector<ParamTokenRequest>& reqs) {
    std::vector<TokenResult> res(reqs.size(), TokenResult(TokenResultStatus::FAIL));
    if (reqs.empty()) return res;
    std::vector<sg_cparam_req> rq(reqs.size());
    std::vector<uint64_t> vals;
    for (size_t i = 0; i < reqs.size(); ++i) {
        const ParamTokenRequest& q = reqs[i];
        sg_cparam_req& r = rq[i];
        r.ts_ms = q.timeMillis;
        r.acquire = q.acquireCount;
        if (!q.ruleId || *q.ruleId <= 0) {
            r.key = SG_KEY_BAD;
        } else {
            auto it = keyOfParam_.find(*q.ruleId);
            r.key = it == keyOfParam_.end() ? SG_KEY_NO_RULE : it->second;
        }
        r.value_begin = (uint32_t)vals.size();
        r.value_count = (uint32_t)q.params.size();
        for (const std::string& v : q.params) vals.push_back(valueId(v));
    }
    std::vector<sg_result> out(reqs.size());
    std::lock_guard<std::mutex> e(engMu_);
    if (sg_cparam_decide_batch_host(h_, rq.data(), rq.size(), vals.data(), vals.size(), out.data()) != SG_OK) {
        err_ = sg_last_error(h_);  // TokenResult(FAIL) → the client falls back to local checking
        return res;
    }
    for (size_t i = 0; i < reqs.size(); ++i)
        res[i] = TokenResult(out[i].status).setRemaining(out[i].remaining).setWaitInMs(out[i].wait_ms);
    return res;
}

// DefaultTokenService.requestParamToken (:53-64) → ClusterParamFlowChecker.acquireClusterToken on the device
// (sg_cparam_*): one request per call, in arrival order with the flow-token micro-batches (they share the
// namespace's GlobalRequestLimiter).
TokenResult GpuTokenService::requestParamToken(std::optional<int64_t> ruleId, int acquireCount,
                                               const std::vector<std::string>& params) {
    if (!ruleId || *ruleId <= 0 || acquireCount <= 0 || params.empty())
        return TokenResult(TokenResultStatus::BAD_REQUEST);  // DefaultTokenService.java:53-56
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    waitIdle();
    ParamTokenRequest q{std::max(lastTs_, opt_.clock()), ruleId, acquireCount, params};
    lastTs_ = q.timeMillis;
    return decideParamLocked({q})[0];
}

std::vector<TokenResult> GpuTokenService::requestParamTokens(const std::vector<ParamTokenRequest>& reqs) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    waitIdle();
    for (const auto& q : reqs) lastTs_ = std::max(lastTs_, q.timeMillis);
    return decideParamLocked(reqs);
}

// DefaultTokenService.requestConcurrentToken (:66-77) → ConcurrentClusterFlowChecker.acquireConcurrentToken on
// the device (sg_conc_*): one request per call, in arrival order with the other concurrency calls.
TokenResult GpuTokenService::requestConcurrentToken(const std::string& clientAddress, std::optional<int64_t> ruleId,
                                                    int acquireCount) {
    if (clientAddress.empty() || !ruleId || *ruleId <= 0 || acquireCount <= 0)
        return TokenResult(TokenResultStatus::BAD_REQUEST);  // DefaultTokenService.java:67-70, 91-93
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    waitIdle();
    auto it = clientIds_.find(clientAddress);
    const uint32_t client = it != clientIds_.end() ? it->second : (clientIds_[clientAddress] = (uint32_t)clientIds_.size() + 1);
    sg_conc_req r{};
    r.ts_ms = std::max(lastTs_, opt_.clock());
    lastTs_ = r.ts_ms;
    r.kind = SG_CONC_ACQUIRE;
    r.key = keyOf(ruleId, false);
    r.acquire = acquireCount;
    r.client = client;
    sg_conc_result o{};
    std::lock_guard<std::mutex> e(engMu_);
    if (sg_conc_decide_batch_host(h_, &r, 1, &o) != SG_OK) {
        err_ = sg_last_error(h_);
        return TokenResult(TokenResultStatus::FAIL);
    }
    TokenResult res(o.status);
    res.setTokenId((int64_t)o.token_id);
    return res;
}

// DefaultTokenService.releaseConcurrentToken (:79-85): null ids are ignored; the checker's status is dropped
// as in the reference (the method is void).
void GpuTokenService::releaseConcurrentToken(std::optional<int64_t> tokenId) {
    if (!tokenId) return;
    std::unique_lock<std::mutex> lk(mu_);
    if (!pending_.empty()) flushLocked(lk);
    waitIdle();
    sg_conc_req r{};
    r.ts_ms = std::max(lastTs_, opt_.clock());
    lastTs_ = r.ts_ms;
    r.kind = SG_CONC_RELEASE;
    r.token_id = (uint64_t)*tokenId;
    sg_conc_result o{};
    std::lock_guard<std::mutex> e(engMu_);
    if (sg_conc_decide_batch_host(h_, &r, 1, &o) != SG_OK) err_ = sg_last_error(h_);
}

}  // namespace cluster
}  // namespace sentinel
