// Does the matrix core's f32 outer product (v_mfma_f32_16x16x1_4b_f32 with C = 0, as the Q8 GEMM tiles form d_x·d_w)
// give the same bits as a VALU multiply?  Random f16-valued scales (the Q8 block scales) over the normal range and a
// few subnormal-product cases; prints the mismatch count.  Build: hipcc --offload-arch=gfx950 -O3 -o prod_check
// prod_check.hip
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float v16f __attribute__((ext_vector_type(16)));

// one wave: lane l feeds row / column l & 15 of block l >> 4; every output is compared in-lane with the VALU products
// of the same operands (read back through LDS)
__global__ void k_prod(const float* x, const float* w, int n, unsigned* bad, float* ex) {
    __shared__ float xs[64], wsh[64];
    const int lane = threadIdx.x;
    for (int base = 0; base + 64 <= n; base += 64) {
        const float a = x[base + lane], b = w[base + lane];
        xs[lane] = a;
        wsh[lane] = b;
        __syncthreads();
        const v16f z = {};
        const v16f c = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, z, 0, 0, 0);
        // 4 blocks (operands of block k from lanes 16k..16k+15): C_k[i][j] in lane j + 16·(i/4), register 4k + i%4.
        // Each output must equal the VALU product of one block's operands (all four tried: layout-agnostic).
#pragma unroll
        for (int R = 0; R < 16; R++) {
            const int j = lane & 15, i = 4 * (lane >> 4) + (R & 3);
            bool any = false;
            for (int k = 0; k < 4; k++) {
                const float p = xs[16 * k + i] * wsh[16 * k + j];
                if (__float_as_uint(p) == __float_as_uint(c[R])) any = true;
            }
            if (!any) {
                atomicAdd(bad, 1u);
                if (ex) ex[0] = c[R];
            }
        }
        __syncthreads();
    }
}

int main() {
    const int n = 64 * 65536;
    float* hx = (float*)malloc(n * 4);
    float* hw = (float*)malloc(n * 4);
    srand(1);
    for (int i = 0; i < n; i++) {
        // f16 scales of Q8 blocks: d = amax/127 rounded to f16 (activations ~1e-4..1, weights ~1e-5..1e-1)
        const float ax = powf(10.f, -5.f + 5.f * (float)rand() / RAND_MAX) * (rand() & 1 ? 1.f : -1.f);
        const float aw = powf(10.f, -6.f + 5.f * (float)rand() / RAND_MAX);
        hx[i] = __half2float(__float2half(ax));
        hw[i] = __half2float(__float2half(aw));
    }
    float *dx, *dw, *dex;
    unsigned* dbad;
    hipMalloc(&dx, n * 4);
    hipMalloc(&dw, n * 4);
    hipMalloc(&dbad, 4);
    hipMalloc(&dex, 4);
    hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dw, hw, n * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 4);
    k_prod<<<1, 64>>>(dx, dw, n, dbad, dex);
    unsigned bad = 0;
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("outer-product MFMA vs VALU multiply: %u mismatching products of %d checked\n", bad, n / 64 * 1024);
    return bad != 0;
}
