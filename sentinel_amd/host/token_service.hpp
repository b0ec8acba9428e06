// token_service.hpp — C++ host side above the C ABI (include/sentinel_gpu.h), mirroring the Java
// plugin surface this engine replaces, with the same names, argument meaning and error behaviour:
//
//   TokenService / TokenResult / TokenResultStatus  sentinel-core/.../cluster/TokenService.java:26-63,
//                                                   TokenResult.java:26-35, TokenResultStatus.java:22-73
//   FlowRule / ClusterFlowConfig                    sentinel-core/.../slots/block/flow/FlowRule.java,
//                                                   ClusterFlowConfig.java:29-74
//   GpuTokenService::requestToken                   DefaultTokenService.requestToken (srv/flow/DefaultTokenService.java:39-50)
//   GpuTokenService::loadRules                      ClusterFlowRuleManager.loadRules → applyClusterFlowRule
//                                                   (srv/flow/rule/ClusterFlowRuleManager.java:254-260, 325-375)
//   GpuTokenService::requestParamToken              DefaultTokenService.requestParamToken (:53-64) →
//                                                   ClusterParamFlowChecker.acquireClusterToken (:42-87)
//   GpuTokenService::loadParamRules                 ClusterParamFlowRuleManager.loadRules → applyClusterParamRules
//                                                   (srv/flow/rule/ClusterParamFlowRuleManager.java:318-365)
//   GpuTokenService::requestConcurrentToken / releaseConcurrentToken
//                                                   DefaultTokenService (:66-85) → ConcurrentClusterFlowChecker
//   GpuTokenService::loadServerFlowConfig / setConnectedCount
//                                                   ClusterServerConfigManager.loadFlowConfig (:303-346),
//                                                   ConnectionManager.getConnectedCount (:47-51)
//
// requestToken may be called from many threads (the Netty workers of the token server): calls are
// stamped with TimeUtil-equivalent time and an arrival sequence under one lock and micro-batched; a full
// batch goes to the GPU through the asynchronous host pipeline (sg_flow_submit: pinned buffers, up to
// `pipelineDepth` batches in flight, H2D / compute / D2H overlapped) while the next batch keeps filling, and a
// completion thread hands each caller its own result. A failed batch answers FAIL for every request in it,
// so the client's fallbackToLocalOrPass applies (FlowRuleChecker.java:166-209).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/sentinel_gpu.h"

namespace sentinel {
namespace cluster {

struct TokenResultStatus {
    static constexpr int BAD_REQUEST = -4;
    static constexpr int TOO_MANY_REQUEST = -2;
    static constexpr int FAIL = -1;
    static constexpr int OK = 0;
    static constexpr int BLOCKED = 1;
    static constexpr int SHOULD_WAIT = 2;
    static constexpr int NO_RULE_EXISTS = 3;
    static constexpr int NO_REF_RULE_EXISTS = 4;
    static constexpr int NOT_AVAILABLE = 5;
    static constexpr int RELEASE_OK = 6;
    static constexpr int ALREADY_RELEASE = 7;
};

class TokenResult {
public:
    TokenResult() = default;
    explicit TokenResult(int status) : status_(status) {}
    std::optional<int> getStatus() const { return status_; }
    TokenResult& setStatus(int s) { status_ = s; return *this; }
    int getRemaining() const { return remaining_; }
    TokenResult& setRemaining(int r) { remaining_ = r; return *this; }
    int getWaitInMs() const { return waitInMs_; }
    TokenResult& setWaitInMs(int w) { waitInMs_ = w; return *this; }
    int64_t getTokenId() const { return tokenId_; }
    void setTokenId(int64_t id) { tokenId_ = id; }
    bool operator==(const TokenResult& o) const {
        return status_ == o.status_ && remaining_ == o.remaining_ && waitInMs_ == o.waitInMs_;
    }

private:
    std::optional<int> status_;
    int remaining_ = 0;
    int waitInMs_ = 0;
    int64_t tokenId_ = 0;
};

struct RuleConstant {  // sentinel-core/.../slots/block/RuleConstant.java
    static constexpr int FLOW_GRADE_THREAD = 0;
    static constexpr int FLOW_GRADE_QPS = 1;
    static constexpr int STRATEGY_DIRECT = 0;
    static constexpr int STRATEGY_RELATE = 1;
    static constexpr int STRATEGY_CHAIN = 2;
    static constexpr int CONTROL_BEHAVIOR_DEFAULT = 0;
    static constexpr int CONTROL_BEHAVIOR_WARM_UP = 1;
    static constexpr int CONTROL_BEHAVIOR_RATE_LIMITER = 2;
    static constexpr int CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER = 3;
};

struct ClusterRuleConstant {  // ClusterRuleConstant.java:24-30
    static constexpr int FLOW_CLUSTER_STRATEGY_NORMAL = 0;
    static constexpr int FLOW_THRESHOLD_AVG_LOCAL = 0;
    static constexpr int FLOW_THRESHOLD_GLOBAL = 1;
    static constexpr int DEFAULT_CLUSTER_SAMPLE_COUNT = 10;
};

struct ClusterFlowConfig {  // ClusterFlowConfig.java:29-74 (defaults included)
    std::optional<int64_t> flowId;
    int thresholdType = ClusterRuleConstant::FLOW_THRESHOLD_AVG_LOCAL;
    bool fallbackToLocalWhenFail = true;
    int strategy = ClusterRuleConstant::FLOW_CLUSTER_STRATEGY_NORMAL;
    int sampleCount = ClusterRuleConstant::DEFAULT_CLUSTER_SAMPLE_COUNT;
    int windowIntervalMs = 1000;
    int64_t resourceTimeout = 2000;
    int resourceTimeoutStrategy = 0;
    int acquireRefuseStrategy = 0;
    int64_t clientOfflineTime = 2000;
};

struct FlowRule {  // FlowRule.java:52-95
    std::string resource;
    std::string limitApp = "default";
    int grade = RuleConstant::FLOW_GRADE_QPS;
    double count = 0;
    int strategy = RuleConstant::STRATEGY_DIRECT;
    std::string refResource;
    int controlBehavior = RuleConstant::CONTROL_BEHAVIOR_DEFAULT;
    int warmUpPeriodSec = 10;
    int maxQueueingTimeMs = 500;
    bool clusterMode = false;
    std::optional<ClusterFlowConfig> clusterConfig;
};

// FlowRuleUtil.isValidRule (sentinel-core/.../slots/block/flow/FlowRuleUtil.java:167-229)
bool isValidRule(const FlowRule& rule);

struct ParamFlowClusterConfig {  // ParamFlowClusterConfig.java:32-44 (defaults included)
    std::optional<int64_t> flowId;
    int thresholdType = ClusterRuleConstant::FLOW_THRESHOLD_AVG_LOCAL;
    bool fallbackToLocalWhenFail = false;
    int sampleCount = ClusterRuleConstant::DEFAULT_CLUSTER_SAMPLE_COUNT;
    int windowIntervalMs = 1000;
};

struct ParamFlowItem {  // ParamFlowItem.java: object (string form), classType, count
    std::optional<std::string> object;
    std::string classType;
    std::optional<int> count;
};

struct ParamFlowRule {  // ParamFlowRule.java (defaults included)
    std::string resource;
    std::string limitApp = "default";
    int grade = RuleConstant::FLOW_GRADE_QPS;
    std::optional<int> paramIdx;
    double count = 0;
    int controlBehavior = RuleConstant::CONTROL_BEHAVIOR_DEFAULT;
    int maxQueueingTimeMs = 0;
    int burstCount = 0;
    int64_t durationInSec = 1;
    std::vector<ParamFlowItem> paramFlowItemList;
    bool clusterMode = false;
    std::optional<ParamFlowClusterConfig> clusterConfig;
};

// ParamFlowRuleUtil.isValidRule (sentinel-extension/.../param/ParamFlowRuleUtil.java:46-66)
bool isValidParamRule(const ParamFlowRule& rule);

class TokenService {
public:
    virtual ~TokenService() = default;
    virtual TokenResult requestToken(std::optional<int64_t> ruleId, int acquireCount, bool prioritized) = 0;
    virtual TokenResult requestParamToken(std::optional<int64_t> ruleId, int acquireCount,
                                          const std::vector<std::string>& params) = 0;
    virtual TokenResult requestConcurrentToken(const std::string& clientAddress, std::optional<int64_t> ruleId,
                                               int acquireCount) = 0;
    virtual void releaseConcurrentToken(std::optional<int64_t> tokenId) = 0;
};

// One request of the deterministic batch API: requestToken at an explicit TimeUtil time.
struct TokenRequest {
    int64_t timeMillis;
    std::optional<int64_t> ruleId;
    int acquireCount;
    bool prioritized;
};

class GpuTokenService : public TokenService {
public:
    struct Options {
        int device = 0;
        uint64_t maxBatch = 1u << 20;
        double exceedCount = 1.0;      // ServerFlowConfig.DEFAULT_EXCEED_COUNT
        double maxOccupyRatio = 1.0;   // ServerFlowConfig.DEFAULT_MAX_OCCUPY_RATIO
        size_t flushSize = 4096;       // micro-batch: flush at this many pending requests ...
        std::chrono::microseconds flushDelay{200};  // ... or when the oldest has waited this long
        std::function<int64_t()> clock;             // TimeUtil.currentTimeMillis (default: system clock)
        int pipelineDepth = 3;                      // micro-batches in flight on the GPU (1..3)
        // non-empty: one token server over these shard devices (sg_node_*: flowIds hashed over the shards, routing
        // inside the library; a device may repeat); param and concurrent tokens on the node's front handle
        std::vector<int> shardDevices;
        int paramCapacityLog2 = 16;                 // exact (value → window) table per cluster param rule
        // observer of every decided micro-batch (requests as submitted, results, status) — tests and tracing
        std::function<void(const std::vector<sg_req>&, const std::vector<sg_result>&, int)> onBatch;
    };

    explicit GpuTokenService(Options opt);
    ~GpuTokenService() override;
    GpuTokenService(const GpuTokenService&) = delete;
    GpuTokenService& operator=(const GpuTokenService&) = delete;

    // ClusterFlowRuleManager.loadRules(namespace, rules): replaces the namespace's cluster rules.
    void loadRules(const std::string& ns, const std::vector<FlowRule>& rules);
    // ClusterServerConfigManager: per-namespace QPS limiter (GlobalRequestLimiter) and max QPS.
    void loadServerFlowConfig(const std::string& ns, bool limiterEnabled, double maxAllowedQps);
    // ClusterParamFlowRuleManager.loadRules(namespace, rules): replaces the namespace's cluster param rules (a
    // surviving flowId keeps its ClusterParamMetric). Parameters are strings here: a hot item matches when its
    // parsed value is a String (blank or non-primitive classType), as Java's equals would decide.
    void loadParamRules(const std::string& ns, const std::vector<ParamFlowRule>& rules);
    // ConnectionManager.getConnectedCount(namespace), used by FLOW_THRESHOLD_AVG_LOCAL rules.
    void setConnectedCount(const std::string& ns, int connected);

    std::optional<FlowRule> getFlowRuleById(int64_t id) const;  // ClusterFlowRuleManager.getFlowRuleById
    std::optional<std::string> getNamespace(int64_t flowId) const;

    TokenResult requestToken(std::optional<int64_t> ruleId, int acquireCount, bool prioritized) override;
    TokenResult requestParamToken(std::optional<int64_t> ruleId, int acquireCount,
                                  const std::vector<std::string>& params) override;
    TokenResult requestConcurrentToken(const std::string& clientAddress, std::optional<int64_t> ruleId,
                                       int acquireCount) override;
    void releaseConcurrentToken(std::optional<int64_t> tokenId) override;

    // Deterministic replay: decide `reqs` (time-ordered) in one batch.
    std::vector<TokenResult> requestTokens(const std::vector<TokenRequest>& reqs);
    // Deterministic replay of requestParamToken calls at explicit times, one device batch.
    struct ParamTokenRequest {
        int64_t timeMillis;
        std::optional<int64_t> ruleId;
        int acquireCount;
        std::vector<std::string> params;
    };
    std::vector<TokenResult> requestParamTokens(const std::vector<ParamTokenRequest>& reqs);

    const std::string& lastError() const { return err_; }

private:
    struct Pending {
        sg_req req;
        std::promise<TokenResult>* result;
    };
    struct RuleEntry {
        FlowRule rule;
        std::string ns;
    };
    struct InFlight {  // one submitted micro-batch
        uint64_t ticket;
        int buf;
        int rc;        // submit status (non-zero: answered FAIL without a ticket)
        std::vector<std::promise<TokenResult>*> waiters;
    };

    struct ParamRuleEntry {
        ParamFlowRule rule;
        std::string ns;
    };
    uint32_t keyOf(std::optional<int64_t> ruleId, bool prioritized) const;
    uint64_t valueId(const std::string& v);  // exact dictionary: the same string is the same value forever
    void pushParamRulesLocked();
    std::vector<TokenResult> decideParamLocked(const std::vector<ParamTokenRequest>& reqs);
    int nsIndex(const std::string& ns);  // creates the namespace entry if needed
    void pushNamespacesLocked();
    void pushRulesLocked();
    void flushLocked(std::unique_lock<std::mutex>& lk);
    void flusherLoop();
    void completerLoop();
    void waitIdle();  // every submitted micro-batch answered
    std::vector<TokenResult> decideLocked(std::vector<sg_req>& reqs);

    Options opt_;
    sg_handle* h_ = nullptr;               // the engine, or the node's front handle (node mode)
    sg_node* node_ = nullptr;              // node mode: the sharded flow tokens
    std::string err_;

    mutable std::mutex mu_;                // rules, namespaces, pending queue, engine calls
    std::condition_variable cv_;
    std::vector<Pending> pending_;
    std::chrono::steady_clock::time_point oldest_{};
    int64_t lastTs_ = -1;
    bool stop_ = false;
    std::thread flusher_;

    std::mutex engMu_;                     // every sg_* call on h_ (one handle = one submitter)
    std::mutex qmu_;                       // inflight_, freeBufs_, stopCompleter_
    std::condition_variable qcv_;
    std::deque<InFlight> inflight_;
    std::vector<int> freeBufs_;
    std::vector<std::pair<sg_req*, sg_result*>> bufs_;  // pinned staging buffers, one pair per pipeline slot
    bool stopCompleter_ = false;
    std::thread completer_;

    std::vector<std::string> nsNames_;
    std::vector<sg_namespace> nsCfg_;
    std::map<std::string, std::vector<int64_t>> nsFlowIds_;   // NAMESPACE_FLOW_ID_MAP
    std::unordered_map<int64_t, RuleEntry> rules_;            // FLOW_RULES + FLOW_NAMESPACE_MAP
    std::unordered_map<int64_t, uint32_t> keyOfFlow_;         // flowId → dense engine key
    std::unordered_map<std::string, uint32_t> clientIds_;     // client address → sg_conc_req.client (1, 2, …)
    std::map<int64_t, ParamRuleEntry> paramRules_;            // PARAM_RULES (flowId → rule, namespace)
    std::map<std::string, std::vector<int64_t>> nsParamIds_;  // NAMESPACE_FLOW_ID_MAP of the param rules
    std::unordered_map<int64_t, uint32_t> keyOfParam_;        // flowId → dense cparam rule index
    std::unordered_map<std::string, uint64_t> valueIds_;      // parameter string → u64 value
};

}  // namespace cluster
}  // namespace sentinel
