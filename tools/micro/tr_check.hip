// Checks for the k_attn_tile P·V step: ds_read_b64_tr_b16 on the swizzled 256-B-row V image, and the whole
// stage → transposed read → f16 MFMA sequence with a one-hot P (O[row][dim] must equal V[hot][dim]).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef short v4s __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ int voff(int kr, int ch) { return kr * 256 + 16 * (ch ^ (((kr & 3) << 2 | ((kr >> 2) & 3)) & 15)); }

__global__ void k_tr(int* out) {
    __shared__ __attribute__((aligned(16))) short t[32 * 128];
    const int lane = threadIdx.x;
    for (int i = lane; i < 32 * 128; i += 64) {
        const int row = i / 128, col = i % 128;
        t[(voff(row, col / 8) + 2 * (col % 8)) / 2] = (short)(100 * row + col);
    }
    __syncthreads();
    const int g = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int addr = voff(4 * g + q, p >> 1) + 8 * (p & 1);
    const v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)((__attribute__((address_space(3))) char*)t + addr));
    for (int e = 0; e < 4; e++) out[lane * 4 + e] = r[e];
}

__global__ void k_pv(const __half* V, int hot, float* out) {
    __shared__ __attribute__((aligned(16))) _Float16 vs[32 * 128];
    const int lane = threadIdx.x, fr = lane & 15, kh = lane >> 4;
    int4 vp[8];
    for (int u = 0; u < 8; u++) {
        const int piece = u * 64 + lane, kr = piece / 16, ch = piece % 16;
        vp[u] = *(const int4*)(V + kr * 128 + 8 * ch);
    }
    for (int u = 0; u < 8; u++) {
        const int piece = u * 64 + lane, kr = piece / 16, ch = piece % 16;
        *(int4*)((char*)vs + voff(kr, ch)) = vp[u];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    v8h pf;
    for (int j = 0; j < 8; j++) pf[j] = (_Float16)((16 * (j >> 2) + 4 * kh + (j & 3)) == hot ? 1.f : 0.f);
    const int q = fr >> 2, pp = fr & 3;
    for (int t = 0; t < 8; t++) {
        v4s rr[2];
        for (int h2 = 0; h2 < 2; h2++) {
            const int kr = 16 * h2 + 4 * kh + q, ch = 2 * t + (pp >> 1);
            rr[h2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)((__attribute__((address_space(3))) char*)vs + voff(kr, ch) +
                                                          8 * (pp & 1)));
        }
        typedef _Float16 v4h __attribute__((ext_vector_type(4)));
        const v8h vf = __builtin_shufflevector(__builtin_bit_cast(v4h, rr[0]), __builtin_bit_cast(v4h, rr[1]), 0, 1, 2,
                                               3, 4, 5, 6, 7);
        v4f acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, vf, acc, 0, 0, 0);
        for (int i = 0; i < 4; i++) out[(4 * kh + i) * 128 + 16 * t + fr] = acc[i];
    }
}

int main() {
    int* d;
    (void)hipMalloc(&d, 256 * 4);
    k_tr<<<1, 64>>>(d);
    int h[256];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int lane = 0; lane < 64; lane++)
        for (int e = 0; e < 4; e++)
            if (h[4 * lane + e] != 100 * (4 * (lane >> 4) + e) + (lane & 15)) bad++;
    printf("tr read on the swizzled image: bad=%d (lane 5: %d %d %d %d)\n", bad, h[20], h[21], h[22], h[23]);

    static __half hv[32 * 128];
    for (int k = 0; k < 32; k++)
        for (int dd = 0; dd < 128; dd++) hv[k * 128 + dd] = __float2half((float)k + dd / 256.f);
    __half* dv;
    float* dout;
    (void)hipMalloc(&dv, sizeof(hv));
    (void)hipMalloc(&dout, 16 * 128 * 4);
    (void)hipMemcpy(dv, hv, sizeof(hv), hipMemcpyHostToDevice);
    for (int hot : {0, 1, 2, 3, 5, 17, 30}) {
        k_pv<<<1, 64>>>(dv, hot, dout);
        static float ho[16 * 128];
        (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
        int nb = 0;
        for (int r = 0; r < 16; r++)
            for (int dd = 0; dd < 128; dd++)
                if (ho[r * 128 + dd] != __half2float(hv[hot * 128 + dd])) nb++;
        printf("PV hot=%2d: bad=%d  O[0][0..2]=%g %g %g  O[5][17]=%g\n", hot, nb, ho[0], ho[1], ho[2], ho[5 * 128 + 17]);
    }
    return 0;
}
