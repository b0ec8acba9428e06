// GPU test of the C++ host mirror (sentinel_amd/host/token_service.cpp) over the REAL library
// (libsentinel_gpu.so): many threads call GpuTokenService::requestToken concurrently, the micro-batcher
// stamps and batches them and decides them through the asynchronous host pipeline (sg_flow_submit). Every
// decided micro-batch is recorded (Options::onBatch); afterwards the recorded stream is replayed through the
// oracle (oracle/sentinel_oracle.c, linked here as test infrastructure) and must match bit-exactly, and the
// results the threads received must be exactly the recorded ones. Prints "OK <requests> <batches>".
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <random>
#include <thread>
#include <tuple>
#include <vector>

#include "../../oracle/sentinel_oracle.h"
#include "../../sentinel_amd/host/token_service.hpp"

using namespace sentinel::cluster;

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__); \
            std::exit(1);                                                 \
        }                                                                 \
    } while (0)

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 16;
    const int per_thread = argc > 2 ? std::atoi(argv[2]) : 20000;
    const int shards = argc > 3 ? std::atoi(argv[3]) : 0;  // > 0: node mode over that many shards of device 0
    const int n_rules = 300;

    std::atomic<int64_t> calls{0};
    std::mutex rec_mu;
    std::vector<sg_req> rec_req;
    std::vector<sg_result> rec_res;
    int batches = 0, failed_batches = 0;

    GpuTokenService::Options opt;
    opt.flushSize = 2048;
    opt.flushDelay = std::chrono::microseconds(150);
    opt.maxBatch = 1 << 16;
    for (int g = 0; g < shards; ++g) opt.shardDevices.push_back(0);
    // TimeUtil: advances 1 ms every 40 calls (read under the batcher's lock, so non-decreasing in arrival order)
    opt.clock = [&] { return (int64_t)1'700'000'000'000 + calls.fetch_add(1) / 40; };
    opt.onBatch = [&](const std::vector<sg_req>& rq, const std::vector<sg_result>& rs, int rc) {
        std::lock_guard<std::mutex> lk(rec_mu);
        ++batches;
        if (rc != SG_OK) {
            ++failed_batches;
            return;
        }
        rec_req.insert(rec_req.end(), rq.begin(), rq.end());
        rec_res.insert(rec_res.end(), rs.begin(), rs.end());
    };
    GpuTokenService svc(opt);

    std::mt19937_64 g(7);
    std::vector<FlowRule> rules;
    std::vector<sg_flow_rule> tab;  // what the mirror pushes: ascending flowId, namespace "default"
    for (int i = 0; i < n_rules; ++i) {
        FlowRule r;
        r.resource = "res" + std::to_string(i);
        r.count = (double)(5 + g() % 60);
        r.clusterMode = true;
        ClusterFlowConfig c;
        c.flowId = 1000 + i;
        c.thresholdType = ClusterRuleConstant::FLOW_THRESHOLD_GLOBAL;
        c.sampleCount = (i % 3 == 0) ? 10 : (i % 3 == 1 ? 2 : 5);
        c.windowIntervalMs = 1000;
        r.clusterConfig = c;
        rules.push_back(r);
        sg_flow_rule t{};
        t.flow_id = 1000 + i;
        t.count = r.count;
        t.threshold_type = c.thresholdType;
        t.sample_count = c.sampleCount;
        t.window_interval_ms = 1000;
        t.namespace_id = 0;
        tab.push_back(t);
    }
    svc.loadRules("default", rules);
    CHECK(svc.lastError().empty());

    // many Netty-worker threads
    std::vector<std::vector<std::tuple<int, int, int>>> got(threads);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        th.emplace_back([&, t] {
            std::mt19937_64 r(100 + t);
            for (int i = 0; i < per_thread; ++i) {
                const int64_t id = (r() % 50 == 0) ? 999999 : 1000 + (int64_t)(r() % n_rules);  // 2 % unknown flowIds
                const int acq = 1 + (int)(r() % 3);
                const bool prio = r() % 20 == 0;
                TokenResult res = svc.requestToken(id, acq, prio);
                got[t].emplace_back(*res.getStatus(), res.getRemaining(), res.getWaitInMs());
            }
        });
    }
    for (auto& x : th) x.join();

    const size_t total = (size_t)threads * per_thread;
    CHECK(failed_batches == 0);
    CHECK(rec_req.size() == total);
    // arrival stamps are non-decreasing across the recorded stream (one batcher, submission order)
    for (size_t i = 1; i < rec_req.size(); ++i) CHECK(rec_req[i].ts_ms >= rec_req[i - 1].ts_ms);

    // the oracle replays the recorded stream: DefaultTokenService + ClusterFlowChecker, sequentially
    or_cts* ora = or_cts_new(1.0, 1.0);
    sg_namespace ns{};
    ns.limiter_enabled = 0;
    ns.connected_count = 0;
    ns.max_allowed_qps = 30000;
    CHECK(or_cts_set_namespaces(ora, &ns, 1) == 0);
    CHECK(or_cts_load_rules(ora, tab.data(), (uint32_t)tab.size()) == 0);
    std::vector<sg_result> want(rec_req.size());
    CHECK(or_cts_decide(ora, rec_req.data(), rec_req.size(), want.data()) == 0);
    for (size_t i = 0; i < want.size(); ++i) {
        if (want[i].status != rec_res[i].status || want[i].remaining != rec_res[i].remaining ||
            want[i].wait_ms != rec_res[i].wait_ms) {
            std::fprintf(stderr, "mismatch at %zu: key %u ts %lld oracle (%d,%d,%d) gpu (%d,%d,%d)\n", i, rec_req[i].key,
                         (long long)rec_req[i].ts_ms, want[i].status, want[i].remaining, want[i].wait_ms,
                         rec_res[i].status, rec_res[i].remaining, rec_res[i].wait_ms);
            return 1;
        }
    }
    or_cts_free(ora);

    // every thread received exactly one of the recorded results for each of its calls
    std::map<std::tuple<int, int, int>, long> a, b;
    for (const auto& v : got)
        for (const auto& x : v) ++a[x];
    for (const auto& r : rec_res) ++b[std::make_tuple(r.status, r.remaining, r.wait_ms)];
    CHECK(a == b);

    // cluster param tokens through the mirror (requestParamTokens: one device batch, explicit times) against the
    // oracle's ClusterParamFlowChecker on the same requests; decisions only depend on value equality, so the
    // test's own string → u64 dictionary stands in for the mirror's
    std::vector<ParamFlowRule> prules;
    std::vector<sg_cparam_rule> ptab;
    std::vector<sg_param_hot_item> phot;
    std::map<std::string, uint64_t> dict;
    auto vid = [&](const std::string& v) {
        auto it = dict.find(v);
        return it != dict.end() ? it->second : (dict[v] = dict.size() + 1);
    };
    for (int i = 0; i < 40; ++i) {
        ParamFlowRule r;
        r.resource = "pres" + std::to_string(i);
        r.paramIdx = 0;
        r.count = (double)(2 + g() % 20);
        r.clusterMode = true;
        ParamFlowClusterConfig c;
        c.flowId = 5000 + i;
        c.thresholdType = ClusterRuleConstant::FLOW_THRESHOLD_GLOBAL;
        c.sampleCount = (i % 2) ? 10 : 5;
        r.clusterConfig = c;
        sg_cparam_rule t{};
        t.flow_id = 5000 + i;
        t.count = r.count;
        t.threshold_type = c.thresholdType;
        t.sample_count = c.sampleCount;
        t.window_interval_ms = 1000;
        t.hot_begin = (uint32_t)phot.size();
        if (i % 4 == 0) {
            r.paramFlowItemList = {{std::string("v1"), "", 40}};
            phot.push_back(sg_param_hot_item{vid("v1"), 40, 0});
        }
        t.hot_count = (uint32_t)phot.size() - t.hot_begin;
        prules.push_back(r);
        ptab.push_back(t);
    }
    svc.loadParamRules("default", prules);
    CHECK(svc.lastError().empty());
    std::vector<GpuTokenService::ParamTokenRequest> preq;
    std::vector<sg_cparam_req> oreq;
    std::vector<uint64_t> ovals;
    std::mt19937_64 pg(11);
    int64_t pt = 1'700'000'100'000;
    for (int i = 0; i < 30000; ++i) {
        pt += (int64_t)(pg() % 3 == 0);
        const int k = (int)(pg() % 42);  // two unknown flowIds
        const int nv = pg() % 10 == 0 ? 2 + (int)(pg() % 2) : 1;
        GpuTokenService::ParamTokenRequest q{pt, (int64_t)(5000 + k), 1 + (int)(pg() % 2), {}};
        sg_cparam_req o{};
        o.ts_ms = pt;
        o.key = k < 40 ? (uint32_t)k : SG_KEY_NO_RULE;
        o.acquire = q.acquireCount;
        o.value_begin = (uint32_t)ovals.size();
        o.value_count = (uint32_t)nv;
        for (int j = 0; j < nv; ++j) {
            const std::string v = "v" + std::to_string(1 + (int)(pg() % 30));
            q.params.push_back(v);
            ovals.push_back(vid(v));
        }
        preq.push_back(q);
        oreq.push_back(o);
    }
    std::vector<TokenResult> pres = svc.requestParamTokens(preq);
    CHECK(svc.lastError().empty());
    or_cts* pora = or_cts_new(1.0, 1.0);
    CHECK(or_cts_set_namespaces(pora, &ns, 1) == 0);
    CHECK(or_cts_load_param_rules(pora, ptab.data(), (uint32_t)ptab.size(), phot.data(), (uint32_t)phot.size()) == 0);
    std::vector<sg_result> pwant(oreq.size());
    CHECK(or_cts_decide_param(pora, oreq.data(), oreq.size(), ovals.data(), pwant.data()) == 0);
    int passes = 0;
    for (size_t i = 0; i < pwant.size(); ++i) {
        if (pwant[i].status != *pres[i].getStatus() || pwant[i].remaining != pres[i].getRemaining()) {
            std::fprintf(stderr, "param mismatch at %zu: oracle (%d,%d) gpu (%d,%d)\n", i, pwant[i].status,
                         pwant[i].remaining, *pres[i].getStatus(), pres[i].getRemaining());
            return 1;
        }
        passes += pwant[i].status == SG_STATUS_OK;
    }
    CHECK(passes > 0 && passes < (int)pwant.size());
    or_cts_free(pora);
    std::printf("OK %zu %d %d\n", total, batches, passes);
    return 0;
}
