// Microbenchmark: issue rate of the i8 MFMA forms on gfx950 (register operands, independent accumulators) and of
// the exact-Q8 rescale loop (MFMA + cvt + fma per output) at 1 and 2 waves per SIMD.  Cycles from s_memtime.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

// MODE 0: 16x16x32_i8  1: 32x32x32_i8  2: 16x16x64_i8  3: 16x16x32_i8 + rescale (4 cvt + 4 fma)
//      4: 32x32x32_i8 + rescale (16 cvt + 16 fma)   5: f32 16x16x1 outer product (4 blocks)
template <int MODE>
__global__ __launch_bounds__(512) void k_rate(int iters, long long* cyc, float* out) {
    const int lane = threadIdx.x & 63;
    long a = 0x0102030405060708ll * (lane + 1), b = 0x0807060504030201ll + lane;
    v4i a4 = {lane, 2, 3, 4}, b4 = {5, lane, 7, 8};
    v4i c4[4] = {};
    v16i c16[2] = {};
    float acc[16] = {};
    v16f o16[2] = {};
    const float sc = 1e-3f * (lane + 1);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int u = 0; u < 4; u++) c4[u] = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c4[u], 0, 0, 0);
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int u = 0; u < 2; u++) c16[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, c16[u], 0, 0, 0);
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int u = 0; u < 4; u++) c4[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a4, b4, c4[u], 0, 0, 0);
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const v4i z = {0, 0, 0, 0};
                const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a + u, b, z, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) acc[4 * u + r] = fmaf((float)c[r], sc, acc[4 * u + r]);
            }
        } else if constexpr (MODE == 4) {
            const v16i z = {};
            const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4 + it, b4, z, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = fmaf((float)c[r], sc, acc[r]);
        } else {
#pragma unroll
            for (int u = 0; u < 2; u++) o16[u] = __builtin_amdgcn_mfma_f32_16x16x1f32(sc + u, sc, o16[u], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int u = 0; u < 4; u++) s += (float)(c4[u][0] + c4[u][3]);
    for (int u = 0; u < 2; u++) s += (float)(c16[u][0] + c16[u][15]) + o16[u][0] + o16[u][15];
    for (int r = 0; r < 16; r++) s += acc[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char* name, int per_iter, int threads) {
    const int iters = 4096, blocks = 256;
    long long* cyc;
    float* out;
    hipMalloc(&cyc, blocks * sizeof(long long));
    hipMalloc(&out, blocks * 512 * sizeof(float));
    k_rate<MODE><<<blocks, threads>>>(iters, cyc, out);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_rate<MODE><<<blocks, threads>>>(iters, cyc, out);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; i++) avg += h[i];
    avg /= blocks;
    const int wps = threads / 256;   // waves per SIMD
    printf("%-28s waves/SIMD %d: %.1f cycles per MFMA-slot per wave (%.1f per SIMD), wall %.3f ms\n", name, wps,
           avg / iters / per_iter, avg / iters / per_iter / wps, ms);
    hipFree(cyc);
    hipFree(out);
}

int main() {
    for (int t : {256, 512}) {
        run<0>("16x16x32_i8", 4, t);
        run<1>("32x32x32_i8", 2, t);
        run<2>("16x16x64_i8", 4, t);
        run<3>("16x16x32_i8+rescale(4+4)", 4, t);
        run<4>("32x32x32_i8+rescale(16+16)", 1, t);
        run<5>("f32 16x16x1 (4 blocks)", 2, t);
    }
    return 0;
}
