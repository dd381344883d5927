// Probe of v_mfma_scale_f32_16x16x128_f8f6f4: which B register bytes (lane group g', byte quarter q) fall in the
// K-block whose scale lane `la` of A supplies.  A = 1.0 everywhere; B = 1.0 only in lanes of group g', bytes
// 8q..8q+7; A's scale 2^1 in lane la, 2^0 elsewhere.  C[row la&15][0] = 8·(2 if scaled else 1).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_probe(int la, int gq, int q, float* C) {
    const int l = threadIdx.x;
    v8i a, b;
    for (int j = 0; j < 8; j++) a[j] = 0x38383838, b[j] = ((l >> 4) == gq && (j >> 1) == q) ? 0x38383838 : 0;
    unsigned sa = 0x7f7f7f7fu, sb = 0x7f7f7f7fu;
    if (l == la) sa = 0x7f7f7f80u;
    const v4f z = {0.f, 0.f, 0.f, 0.f};
    const v4f c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, z, 0, 0, 0, (int)sa, 0, (int)sb);
    for (int i = 0; i < 4; i++) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
    float* dC;
    (void)hipMalloc(&dC, 256 * 4);
    float h[256];
    for (int la : {0, 16, 32, 48}) {
        printf("A scale lane %2d:", la);
        for (int g = 0; g < 4; g++)
            for (int q = 0; q < 4; q++) {
                k_probe<<<1, 64>>>(la, g, q, dC);
                (void)hipMemcpy(h, dC, sizeof h, hipMemcpyDeviceToHost);
                printf(" g%dq%d:%g", g, q, h[0]);
            }
        printf("\n");
    }
    return 0;
}
