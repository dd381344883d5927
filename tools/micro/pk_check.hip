// Semantics check for the GEMM rescale: an i8 MFMA seeded with the bits of 1.5·2^23, its result pairs turned into
// floats by one packed add and folded by packed FMAs, against the scalar cvt + fma.  Three ways of forming the
// register pairs (element build, shufflevector, bit-cast halves).  Build: hipcc --offload-arch=gfx950 -O3
// pk_check.hip -o /tmp/pk_check; prints mismatches per variant (all 0 = the packed path is exact).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <int V>
__global__ void k(const long* a, const long* b, const float* s, float* out) {
    const int l = threadIdx.x;
    const v4i magic = {0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000};
    f2v nm = {-12582912.f, -12582912.f};
    asm volatile("" : "+v"(nm));
    f2v acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
    for (int t = 0; t < 4; t++) {
        const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[64 * t + l], b[64 * t + l], magic, 0, 0, 0);
        const v4i z = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[64 * t + l], b[64 * t + l], v4i{0, 0, 0, 0}, 0, 0, 0);
        const float* sp = s + 4 * (64 * t + l);
        f2v lo, hi;
        if constexpr (V == 0) {
            lo = f2v{__builtin_bit_cast(float, c[0]), __builtin_bit_cast(float, c[1])} + nm;
            hi = f2v{__builtin_bit_cast(float, c[2]), __builtin_bit_cast(float, c[3])} + nm;
        } else if constexpr (V == 1) {
            lo = __builtin_bit_cast(f2v, __builtin_shufflevector(c, c, 0, 1)) + nm;
            hi = __builtin_bit_cast(f2v, __builtin_shufflevector(c, c, 2, 3)) + nm;
        } else {
            const long long h0 = __builtin_bit_cast(long long, __builtin_shufflevector(c, c, 0, 1));
            const long long h1 = __builtin_bit_cast(long long, __builtin_shufflevector(c, c, 2, 3));
            lo = __builtin_bit_cast(f2v, h0) + nm;
            hi = __builtin_bit_cast(f2v, h1) + nm;
        }
        acc0 = __builtin_elementwise_fma(lo, f2v{sp[0], sp[1]}, acc0);
        acc1 = __builtin_elementwise_fma(hi, f2v{sp[2], sp[3]}, acc1);
        r0 = fmaf((float)z[0], sp[0], r0);
        r1 = fmaf((float)z[1], sp[1], r1);
        r2 = fmaf((float)z[2], sp[2], r2);
        r3 = fmaf((float)z[3], sp[3], r3);
    }
    out[8 * l + 0] = acc0.x; out[8 * l + 1] = acc0.y; out[8 * l + 2] = acc1.x; out[8 * l + 3] = acc1.y;
    out[8 * l + 4] = r0; out[8 * l + 5] = r1; out[8 * l + 6] = r2; out[8 * l + 7] = r3;
}

int main() {
    const int n = 4 * 64;
    long *a, *b;
    float *s, *o;
    hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&s, n * 16); hipMalloc(&o, 64 * 8 * 4);
    long ha[n], hb[n];
    float hs[4 * n];
    srand(1);
    for (int i = 0; i < n; i++) {
        ha[i] = ((long)rand() << 32) ^ rand();
        hb[i] = ((long)rand() << 32) ^ rand();
    }
    for (int i = 0; i < 4 * n; i++) hs[i] = (rand() % 1000) / 997.f;
    hipMemcpy(a, ha, n * 8, hipMemcpyHostToDevice);
    hipMemcpy(b, hb, n * 8, hipMemcpyHostToDevice);
    hipMemcpy(s, hs, n * 16, hipMemcpyHostToDevice);
    float ho[64 * 8];
    for (int v = 0; v < 3; v++) {
        if (v == 0) k<0><<<1, 64>>>(a, b, s, o);
        if (v == 1) k<1><<<1, 64>>>(a, b, s, o);
        if (v == 2) k<2><<<1, 64>>>(a, b, s, o);
        hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 4; r++) bad += ho[8 * l + r] != ho[8 * l + 4 + r];
        printf("variant %d: %d mismatches of 256 (lane0 %g %g %g %g vs %g %g %g %g)\n", v, bad, ho[0], ho[1], ho[2],
               ho[3], ho[4], ho[5], ho[6], ho[7]);
    }
    return 0;
}
