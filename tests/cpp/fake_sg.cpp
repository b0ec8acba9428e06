// Recording stand-in for the C ABI, used only by the CPU test of the host mirror: it stores what the
// mirror submits and answers each request with status OK, remaining = key index, wait = acquire, so the
// test can check validation, flowId → key mapping, timestamps and batching without a GPU.
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/sentinel_gpu.h"

struct sg_handle { int dummy; };

namespace fake {
std::mutex mu;
std::vector<sg_flow_rule> rules;
std::vector<sg_namespace> ns;
std::vector<std::vector<sg_req>> batches;
int fail_next = 0;
}  // namespace fake

extern "C" {
int sg_create(const sg_config*, sg_handle** out) { *out = new sg_handle(); return SG_OK; }
void sg_destroy(sg_handle* h) { delete h; }
const char* sg_last_error(const sg_handle*) { return "fake"; }
int sg_set_namespaces(sg_handle*, const sg_namespace* ns, uint32_t n) {
    std::lock_guard<std::mutex> lk(fake::mu);
    fake::ns.assign(ns, ns + n);
    return SG_OK;
}
int sg_load_flow_rules(sg_handle*, const sg_flow_rule* r, uint32_t n) {
    std::lock_guard<std::mutex> lk(fake::mu);
    fake::rules.assign(r, r + n);
    return SG_OK;
}
int sg_flow_decide_batch_host(sg_handle*, const sg_req* req, uint64_t n, sg_result* out) {
    std::lock_guard<std::mutex> lk(fake::mu);
    fake::batches.emplace_back(req, req + n);
    if (fake::fail_next) { --fake::fail_next; return SG_E_DEVICE; }
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t k = req[i].key & SG_KEY_INDEX;
        out[i].status = (k == SG_KEY_BAD) ? SG_STATUS_BAD_REQUEST : (k == SG_KEY_NO_RULE) ? SG_STATUS_NO_RULE_EXISTS : SG_STATUS_OK;
        out[i].remaining = (int32_t)k;
        out[i].wait_ms = req[i].acquire;
    }
    return SG_OK;
}
}
