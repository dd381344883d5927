// Exact Q8 block-sum rescale, compute ceiling per SIMD: (a) v_mfma_i32_16x16x32_i8 + 4 cvt + 4 fma per block tile
// (the Q8 GEMMs today) against (b) v_mfma_f32_16x16x32_f16 on the same int8 values held as f16 (products exact in f32,
// a 32-block sum < 2^20 exact) + 4 fma — no cvt, at the f16 MFMA rate.  Operands in registers, a 4×4 fragment tile per
// wave, the scale products from one outer-product MFMA per row fragment (as the OP tiles do), W waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o rescale_f16 rescale_f16.hip && ./rescale_f16
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <bool F16>
__global__ __launch_bounds__(512) void k_loop(int iters, const int* seed, float* out) {
    const int lane = threadIdx.x & 63;
    long ai[4], bi[4];
    v8h ah[4], bh[4];
    for (int i = 0; i < 4; i++) {
        ai[i] = (long)seed[lane + 64 * i] * 0x0101010101010101L;
        bi[i] = (long)seed[lane + 64 * i + 256] * 0x0101010101010101L;
        for (int k = 0; k < 8; k++) {
            ah[i][k] = (_Float16)(seed[lane + k] & 127);
            bh[i][k] = (_Float16)(seed[lane + k + 64] & 127);
        }
    }
    float sa = seed[lane] * 1e-3f, sb = seed[lane + 1] * 1e-3f;
    float acc[4][4][4] = {};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const v16f z = {};
            const v16f prod = __builtin_amdgcn_mfma_f32_16x16x1f32(sa, sb, z, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if constexpr (F16) {
                    const v4f c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], v4f{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf(c[r], prod[4 * j + r], acc[i][j][r]);
                } else {
                    const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(ai[i], bi[j], v4i{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf((float)c[r], prod[4 * j + r], acc[i][j][r]);
                }
            }
        }
        sa += 1e-7f;
    }
    float s = 0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            for (int r = 0; r < 4; r++) s += acc[i][j][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int* seed;
    float* out;
    CK(hipMalloc(&seed, 4096 * sizeof(int)));
    CK(hipMalloc(&out, 1 << 24));
    int h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (i * 7919 + 13) % 255 - 127;
    CK(hipMemcpy(seed, h, sizeof h, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 2000, cus = 256;
    for (int waves = 4; waves <= 8; waves += 4)
        for (int f16 = 0; f16 < 2; f16++)
            for (int rep = 0; rep < 2; rep++) {
                auto run = [&] {
                    if (f16) k_loop<true><<<cus, 64 * waves>>>(iters, seed, out);
                    else k_loop<false><<<cus, 64 * waves>>>(iters, seed, out);
                };
                run();
                CK(hipEventRecord(e0));
                run();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                // per SIMD: (waves/4) waves × iters × 16 block MFMAs; at 2.4 GHz
                const double blocks = (double)(waves / 4) * iters * 16;
                printf("%s waves/SIMD %d: %.2f ms, %.1f cycles per block tile per SIMD (2.4 GHz)\n",
                       f16 ? "f16 MFMA + 4 fma     " : "i8 MFMA + 4 cvt + 4 fma", waves / 4, ms,
                       ms * 1e-3 * 2.4e9 / blocks);
            }
    return 0;
}
