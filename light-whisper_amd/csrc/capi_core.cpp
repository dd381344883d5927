// extern "C": errors, version, device info.
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
            strncpy(name, p.name, name_cap - 1);
            name[name_cap - 1] = 0;
        }
        if (mem_total_gb) *mem_total_gb = (double)p.totalGlobalMem / (1024.0 * 1024.0 * 1024.0);
    });
}

QASR_API int qasr_set_device(int device) {
    return guard([&] { QASR_HIP(hipSetDevice(device)); });
}

}  // extern "C"
