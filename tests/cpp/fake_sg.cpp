// Recording stand-in for the C ABI, used only by the CPU test of the host mirror: it stores what the
// mirror submits and answers each request with status OK, remaining = key index, wait = acquire, so the
// test can check validation, flowId → key mapping, timestamps and batching without a GPU.
#include <cstdlib>
#include <cstring>
#include <map>
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
std::map<uint64_t, int> tickets;  // submitted batch → its status
std::vector<sg_cparam_rule> cprules;
std::vector<sg_param_hot_item> cphot;
int cp_capacity = 0;
std::vector<sg_cparam_req> cpreqs;
std::vector<uint64_t> cpvalues;
uint64_t next_ticket = 1;
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
void* sg_host_alloc(sg_handle*, uint64_t bytes) { return std::malloc(bytes ? bytes : 1); }
void sg_host_free(sg_handle*, void* p) { std::free(p); }
// the pipeline decides at submit time; the status is handed out by poll / wait
int sg_flow_submit(sg_handle* h, const sg_req* req, uint64_t n, sg_result* out, uint64_t* ticket) {
    const int rc = sg_flow_decide_batch_host(h, req, n, out);
    std::lock_guard<std::mutex> lk(fake::mu);
    *ticket = fake::next_ticket++;
    fake::tickets[*ticket] = rc;
    return SG_OK;
}
int sg_flow_poll(sg_handle*, uint64_t ticket) {
    std::lock_guard<std::mutex> lk(fake::mu);
    auto it = fake::tickets.find(ticket);
    if (it == fake::tickets.end()) return SG_E_INVAL;
    const int rc = it->second;
    fake::tickets.erase(it);
    return rc == SG_OK ? 1 : rc;
}
int sg_flow_wait(sg_handle* h, uint64_t ticket) {
    const int r = sg_flow_poll(h, ticket);
    return r == 1 ? SG_OK : r;
}
int sg_cparam_load_rules(sg_handle*, const sg_cparam_rule* r, uint32_t n, const sg_param_hot_item* hot, uint32_t n_hot,
                         int32_t capacity_log2) {
    std::lock_guard<std::mutex> lk(fake::mu);
    fake::cprules.assign(r, r + n);
    fake::cphot.assign(hot, hot + n_hot);
    fake::cp_capacity = capacity_log2;
    return SG_OK;
}
// records the batch; answers OK with remaining = number of values, wait = key (BAD / NO_RULE as the engine would)
int sg_cparam_decide_batch_host(sg_handle*, const sg_cparam_req* req, uint64_t n, const uint64_t* values,
                                uint64_t n_values, sg_result* out) {
    std::lock_guard<std::mutex> lk(fake::mu);
    fake::cpreqs.assign(req, req + n);
    fake::cpvalues.assign(values, values + n_values);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t k = req[i].key & SG_KEY_INDEX;
        out[i].status = (k == SG_KEY_BAD) ? SG_STATUS_BAD_REQUEST
                        : (k >= fake::cprules.size()) ? SG_STATUS_NO_RULE_EXISTS : SG_STATUS_OK;
        out[i].remaining = (int32_t)req[i].value_count;
        out[i].wait_ms = (int32_t)k;
    }
    return SG_OK;
}
int sg_conc_decide_batch_host(sg_handle*, const sg_conc_req* req, uint64_t n, sg_conc_result* out) {
    std::lock_guard<std::mutex> lk(fake::mu);
    for (uint64_t i = 0; i < n; ++i) {  // acquire: OK with token id 100 + client; release: RELEASE_OK
        out[i].status = req[i].kind == SG_CONC_ACQUIRE ? SG_STATUS_OK : SG_STATUS_RELEASE_OK;
        out[i].reserved = 0;
        out[i].token_id = req[i].kind == SG_CONC_ACQUIRE ? 100 + req[i].client : 0;
    }
    return SG_OK;
}

// node handle: a front handle (param / concurrent tokens) over the same recording flow path
struct sg_node { sg_handle* front; };
int sg_node_create(const sg_config* cfg, const int32_t*, uint32_t, sg_node** out) {
    *out = new sg_node{nullptr};
    return sg_create(cfg, &(*out)->front);
}
void sg_node_destroy(sg_node* nd) {
    sg_destroy(nd->front);
    delete nd;
}
const char* sg_node_last_error(const sg_node*) { return "fake node"; }
sg_handle* sg_node_front(sg_node* nd) { return nd->front; }
int sg_node_set_namespaces(sg_node* nd, const sg_namespace* ns, uint32_t n) { return sg_set_namespaces(nd->front, ns, n); }
int sg_node_load_flow_rules(sg_node* nd, const sg_flow_rule* r, uint32_t n) { return sg_load_flow_rules(nd->front, r, n); }
int sg_node_flow_decide_batch_host(sg_node* nd, const sg_req* req, uint64_t n, sg_result* out) {
    return sg_flow_decide_batch_host(nd->front, req, n, out);
}
}
