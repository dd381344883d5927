// Shared host/device definitions for libqasr (MI355X / gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>

#include <stdexcept>
#include <string>

#include "../../include/qasr_tune.h"

// QASR_FORMAL_HANDOFF=1 (A/B builds): the split-K fix-up and the split decode attention publish their partials with a
// release on the arrival add and read them after an agent-scope acquire fence (the formal C++ memory-model form),
// instead of the measured write-through form (sc1 stores, vmcnt(0), relaxed add, sc1 loads: MI355X_MICROARCH.md,
// inter-workgroup visibility, valid forms table row 1)
#ifndef QASR_FORMAL_HANDOFF
#define QASR_FORMAL_HANDOFF 0
#endif

namespace qasr {

// ------------------------------------------------------------------------------------------------ errors
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define QASR_HIP(expr)                                                                                   \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            throw ::qasr::Error(QASR_E_HIP, std::string("HIP error ") + hipGetErrorString(e_) + \
                                                        " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    } while (0)

#define QASR_CHECK(cond, code, msg)                        \
    do {                                                   \
        if (!(cond)) throw ::qasr::Error((code), (msg));   \
    } while (0)

// ------------------------------------------------------------------------------------------------ Q8_0
constexpr int QK = 32;       // ggml Q8_0 block length
constexpr int QBYTES = 34;   // f16 scale + 32 int8 (GGUF on-disk block)

// Device-resident Q8_0 matrix W[N][K], repacked structure-of-arrays so a wave streams 16-byte vectors:
//   qs : int8 [N][K]      row-major
//   sc : f16  [N][K/32]   per-block scale
struct Q8Mat {
    int8_t* qs = nullptr;
    __half* sc = nullptr;
    int N = 0, K = 0;
    // MXFP8 image of the same rows (precision mode "mxfp8"): e4m3 [N][K] + e8m0 [N][K/32]
    uint8_t* mx = nullptr;
    uint8_t* mxs = nullptr;
    // the same scales regrouped [K/128][N][4] (derived, K % 128 == 0; decoder matrices): a K-128 GEMM stage's
    // column scales are ONE contiguous run of 8 bytes per column, staged by 16-byte DMA (model.cpp
    // ensure_stage_scales, kernels_q8.hip k_gemm_q8d WS4)
    const __half* sc4 = nullptr;
};

// Quantised activations X[M][K]: int8 values + per-32-block f16-rounded scale stored as f32.
struct Q8Act {
    int8_t* q = nullptr;
    float* d = nullptr;
    int M = 0, K = 0;  // capacity metadata only
};

// ------------------------------------------------------------------------------------------------ synth RNG
// Same generator as oracle/qasr_oracle.c (orc_synth_*): splitmix64 over (seed ^ fnv1a(name)) + index.
__host__ __device__ inline uint64_t smix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Row gain of the synthetic vocabulary table (token_embd, the tied lm_head): g = 2^(e/8) with e ≈ 5.77·n, n an
// Irwin-Hall(12) normal from the row's hashes — a log-normal spread of row norms (σ ≈ 0.5 in ln), as real embedding
// tables have, so the synthetic logits have a dominant top entry (a clear top-2 margin on ≥ 90 % of rows instead of
// the ≈ 78 % of i.i.d. rows).  Integer arithmetic and an exact power-of-two table: the same bits on the host
// (oracle/qasr_oracle.c orc_synth_q8) and the device (k_synth_q8).
__host__ __device__ inline float synth_row_gain(uint64_t base, int64_t row) {
    const uint64_t g = smix(base ^ 0x6A09E667F3BCC909ull);
    int64_t sum = 0;
    for (int i = 0; i < 3; i++) {
        const uint64_t h = smix(g + 3 * (uint64_t)row + (uint64_t)i);
        for (int j = 0; j < 4; j++) sum += (int64_t)((h >> (16 * j)) & 0xffff);
    }
    const int64_t num = (sum - 6 * 65536) * 577 / 100;
    const int64_t e = (num + 32768 >= 0) ? (num + 32768) / 65536 : -((-(num + 32768) + 65535) / 65536);
    const float frac[8] = {0x1.000000p+0f, 0x1.172b84p+0f, 0x1.306fe0p+0f, 0x1.4bfdaep+0f,
                           0x1.6a09e6p+0f, 0x1.8ace54p+0f, 0x1.ae89fap+0f, 0x1.d5818ep+0f};
    return ldexpf(frac[e & 7], (int)(e >> 3));
}
inline uint64_t fnv1a(const char* s) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (const unsigned char* p = (const unsigned char*)s; *p; p++) {
        h ^= *p;
        h *= 0x100000001b3ull;
    }
    return h;
}
__host__ __device__ inline float unit_from(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// f32 → f16 after the f32 value has been rounded (blocks hipcc's fused multiply/add → f16 single-rounding
// v_fma_mix* forms, which would differ from the CPU's f32-then-f16 double rounding)
__device__ __forceinline__ __half f2h(float v) {
    asm volatile("" : "+v"(v));
    return __float2half(v);
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace qasr
