// Live per-kernel-class timing for bench.py's roofline line: when enabled, every instrumented launch is
// bracketed by a pair of hipEvents on ITS stream and tagged with its algorithmic FLOPs / bytes.  Disabled
// (the default) it costs one branch per launch.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace qasr {

bool prof_enabled();
void prof_set(bool on);
void prof_reset();
// returns a JSON object {"<name>": {"count", "ms", "flops", "bytes"}, ...} (synchronises the recorded events)
std::string prof_report();

struct ProfScope {
    int slot = -1;
    ProfScope(hipStream_t s, const char* name, double flops, double bytes);
    ~ProfScope();
    hipStream_t stream;
};

}  // namespace qasr
