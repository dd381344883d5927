// extern "C": errors, version, device info.
#include <stdio.h>
#include <string.h>

#include "../../include/qasr.h"
#include "capi_util.h"

namespace qasr {
std::string& last_error_slot() {
    static thread_local std::string s;
    return s;
}
}  // namespace qasr

using namespace qasr;

extern "C" {

QASR_API const char* qasr_last_error(void) { return last_error_slot().c_str(); }

QASR_API const char* qasr_version(void) { return "qasr-mi355x 0.1.0 (gfx950)"; }

QASR_API int qasr_device_info(char* name, size_t name_cap, double* mem_total_gb, int* n_devices) {
    return guard([&] {
        int n = 0;
        QASR_HIP(hipGetDeviceCount(&n));
        if (n_devices) *n_devices = n;
        QASR_CHECK(n > 0, QASR_E_BACKEND, "no HIP device visible");
        int dev = 0;
        QASR_HIP(hipGetDevice(&dev));
        hipDeviceProp_t p;
        QASR_HIP(hipGetDeviceProperties(&p, dev));
        if (name && name_cap) {
            // the marketing name comes from libdrm's amdgpu.ids; without that file it is empty → the ISA name
            char arch[64];
            snprintf(arch, sizeof arch, "AMD Instinct %s", p.gcnArchName);
            strncpy(name, p.name[0] ? p.name : arch, name_cap - 1);
            name[name_cap - 1] = 0;
        }
        if (mem_total_gb) *mem_total_gb = (double)p.totalGlobalMem / (1024.0 * 1024.0 * 1024.0);
    });
}

QASR_API int qasr_set_device(int device) {
    return guard([&] { QASR_HIP(hipSetDevice(device)); });
}

}  // extern "C"

#include "kernels.h"
#include "prof.h"

extern "C" {

QASR_API int qasr_set_deterministic(int32_t on) {
    return guard([&] { qasr::set_deterministic(on != 0); });
}

QASR_API int qasr_get_deterministic(int32_t* on) {
    return guard([&] {
        QASR_CHECK(on, QASR_E_INVALID, "qasr_get_deterministic: null pointer");
        *on = qasr::deterministic() ? 1 : 0;
    });
}

QASR_API int qasr_prof_enable(int on) {
    return guard([&] { qasr::prof_set(on != 0); });
}

QASR_API int qasr_prof_reset(void) {
    return guard([&] { qasr::prof_reset(); });
}

QASR_API int qasr_prof_report(char* buf, size_t cap, size_t* needed) {
    return guard([&] {
        std::string r = qasr::prof_report();
        if (needed) *needed = r.size() + 1;
        QASR_CHECK(!buf || cap > r.size(), QASR_E_CAPACITY, "report buffer too small");
        if (buf) memcpy(buf, r.c_str(), r.size() + 1);
    });
}

}  // extern "C"
