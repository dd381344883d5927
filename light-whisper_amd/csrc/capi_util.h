// Helpers shared by the extern "C" translation units: error capture (no exception crosses the ABI)
// and small host-side tables.
#pragma once
#include <math.h>

#include <exception>
#include <string>

#include "common.h"

namespace qasr {

std::string& last_error_slot();

template <class F>
int guard(F&& f) {
    try {
        f();
        return QASR_OK;
    } catch (const Error& e) {
        last_error_slot() = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        last_error_slot() = "out of host memory";
        return QASR_E_CAPACITY;
    } catch (const std::exception& e) {
        last_error_slot() = e.what();
        return QASR_E_INTERNAL;
    } catch (...) {
        last_error_slot() = "unknown error";
        return QASR_E_INTERNAL;
    }
}

// RoPE (NeoX, rotate-half) cos/sin table [n_ctx][hd/2][2], computed in double like the oracle.
inline void rope_table(int n_ctx, int hd, float theta, float* out) {
    const int half = hd / 2;
    for (int p = 0; p < n_ctx; p++)
        for (int i = 0; i < half; i++) {
            double th = (double)p * pow((double)theta, -2.0 * i / (double)hd);
            out[((size_t)p * half + i) * 2] = (float)cos(th);
            out[((size_t)p * half + i) * 2 + 1] = (float)sin(th);
        }
}

}  // namespace qasr
