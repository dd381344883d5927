#include "prof.h"

#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace qasr {

namespace {
struct Rec {
    std::string name;
    hipEvent_t a, b;
    double flops, bytes;
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t take() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    QASR_HIP(hipEventCreate(&e));
    return e;
}
}  // namespace

bool prof_enabled() { return g_on; }
void prof_set(bool on) { g_on = on; }

void prof_reset() {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& r : g_recs) {
        (void)hipEventSynchronize(r.b);
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
}

ProfScope::ProfScope(hipStream_t s, const char* name, double flops, double bytes) : stream(s) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    Rec r;
    r.name = name;
    r.a = take();
    r.b = take();
    r.flops = flops;
    r.bytes = bytes;
    QASR_HIP(hipEventRecord(r.a, s));
    g_recs.push_back(r);
    slot = (int)g_recs.size() - 1;
}

ProfScope::~ProfScope() {
    if (slot < 0) return;
    std::lock_guard<std::mutex> lk(g_mu);
    (void)hipEventRecord(g_recs[(size_t)slot].b, stream);
}

std::string prof_report() {
    std::lock_guard<std::mutex> lk(g_mu);
    struct Acc {
        long count = 0;
        double ms = 0, flops = 0, bytes = 0;
    };
    std::map<std::string, Acc> acc;
    for (auto& r : g_recs) {
        QASR_HIP(hipEventSynchronize(r.b));
        float ms = 0;
        QASR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        Acc& a = acc[r.name];
        a.count++;
        a.ms += ms;
        a.flops += r.flops;
        a.bytes += r.bytes;
    }
    std::string out = "{";
    bool first = true;
    for (auto& kv : acc) {
        char buf[512];
        snprintf(buf, sizeof buf, "%s\"%s\": {\"count\": %ld, \"ms\": %.6f, \"flops\": %.6e, \"bytes\": %.6e}",
                 first ? "" : ", ", kv.first.c_str(), kv.second.count, kv.second.ms, kv.second.flops, kv.second.bytes);
        out += buf;
        first = false;
    }
    return out + "}";
}

}  // namespace qasr
