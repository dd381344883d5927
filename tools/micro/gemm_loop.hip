// Microbenchmark of the Q8 GEMM inner loop (LDS fragments → MFMA i8 → per-block f32 rescale) with no global
// traffic: isolates the MFMA / VALU / LDS balance of one wave tile.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int GLD = 144;

template <int TI, int TJ, int MODE>
__global__ __launch_bounds__(256) void k_loop(int iters, float* out) {
    constexpr int BM = 32 * TI, BN = 32 * TJ;
    __shared__ __attribute__((aligned(16))) int8_t As[BM * GLD];
    __shared__ __attribute__((aligned(16))) int8_t Bs[BN * GLD];
    __shared__ __attribute__((aligned(16))) float Asc[4 * BM];
    __shared__ __attribute__((aligned(16))) float Bsc[4 * BN];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < BM * GLD; i += 256) As[i] = (int8_t)(i * 7 + blockIdx.x);
    for (int i = tid; i < BN * GLD; i += 256) Bs[i] = (int8_t)(i * 13 + 1);
    for (int i = tid; i < 4 * BM; i += 256) Asc[i] = 1e-3f * (1 + (i & 7));
    for (int i = tid; i < 4 * BN; i += 256) Bsc[i] = 2e-3f * (1 + (i & 3));
    __syncthreads();
    const int wr = wave >> 1, wc = wave & 1;
    const int fr = lane & 15, fk = 8 * (lane >> 4), fq = 4 * (lane >> 4);
    const int arow = wr * 16 * TI, bcol = wc * 16 * TJ;
    float acc[TI][TJ][4] = {};
    v4i iacc[TI][TJ] = {};
    for (int it = 0; it < iters; it++) {
#pragma unroll 1
        for (int kb = 0; kb < 4; kb++) {
            long a[TI], b[TJ];
            float sa[TI][4], sb[TJ];
#pragma unroll
            for (int i = 0; i < TI; i++) {
                a[i] = *(const long*)(As + (arow + i * 16 + fr) * GLD + kb * 32 + fk);
                const float4 v = *(const float4*)(&Asc[kb * BM + arow + i * 16 + fq]);
                sa[i][0] = v.x, sa[i][1] = v.y, sa[i][2] = v.z, sa[i][3] = v.w;
            }
#pragma unroll
            for (int j = 0; j < TJ; j++) b[j] = *(const long*)(Bs + (bcol + j * 16 + fr) * GLD + kb * 32 + fk);
            const float4 v = *(const float4*)(&Bsc[kb * BN + bcol + fr * 4]);
            sb[0] = v.x, sb[1] = v.y, sb[2] = v.z, sb[3] = v.w;
#pragma unroll
            for (int i = 0; i < TI; i++)
#pragma unroll
                for (int j = 0; j < TJ; j++) {
                    if constexpr (MODE == 0) {
                        iacc[i][j] = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i], b[j], iacc[i][j], 0, 0, 0);
                    } else if constexpr (MODE == 1) {
                        const v4i z = {0, 0, 0, 0};
                        v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i], b[j], z, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf((float)c[r], sa[i][r] * sb[j], acc[i][j][r]);
                    } else if constexpr (MODE == 2) {
                        const v4i z = {0, 0, 0, 0};
                        v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i], b[j], z, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf((float)c[r], sa[i][r], acc[i][j][r]);
                    } else {
                        // f16 MFMA on int8-valued f16 operands: block sum arrives as f32
                        typedef _Float16 v8h __attribute__((ext_vector_type(8)));
                        v8h ah, bh;
                        const char* pa = (const char*)&a[i];
                        const char* pb = (const char*)&b[j];
#pragma unroll
                        for (int t = 0; t < 8; t++) ah[t] = (_Float16)pa[t], bh[t] = (_Float16)pb[t];
                        const v4f z = {0.f, 0.f, 0.f, 0.f};
                        v4f c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, z, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf(c[r], sa[i][r] * sb[j], acc[i][j][r]);
                    }
                }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) s += acc[i][j][r] + (float)iacc[i][j][r];
    out[blockIdx.x * 256 + tid] = s;
}

template <int TI, int TJ, int MODE>
void run(const char* name, int wgs) {
    float* out;
    hipMalloc(&out, (size_t)wgs * 256 * 4);
    const int iters = 2000;
    k_loop<TI, TJ, MODE><<<wgs, 256>>>(10, out);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_loop<TI, TJ, MODE><<<wgs, 256>>>(iters, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfma = (double)wgs * 4 * iters * 4 * TI * TJ;   // per wave: 4 kb × TI·TJ
    const double flops = mfma * 16 * 16 * 32 * 2;
    printf("%-28s TI=%d TJ=%d wgs=%5d  %8.3f ms  %7.1f TFLOP/s  %6.2f ns/MFMA/SIMD\n", name, TI, TJ, wgs, ms,
           flops / ms / 1e9, ms * 1e6 / (mfma / 1024.0));
    hipFree(out);
}

int main() {
    for (int wgs : {1024, 2048}) {
        run<4, 4, 0>("mfma only (int acc)", wgs);
        run<4, 4, 1>("rescale cvt+mul+fma", wgs);
        run<4, 4, 2>("rescale cvt+fma", wgs);
        run<4, 4, 3>("f16 mfma + mul+fma", wgs);
        run<2, 2, 0>("mfma only (int acc)", wgs);
        run<2, 2, 1>("rescale cvt+mul+fma", wgs);
        run<2, 2, 2>("rescale cvt+fma", wgs);
        run<2, 4, 1>("rescale cvt+mul+fma", wgs);
        run<4, 8, 1>("rescale cvt+mul+fma", wgs);
    }
    return 0;
}
