// Checks the operand / scale layout of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 × e4m3, e8m0 block scales) with
// exact small-integer data.  Layout (found with mx_probe.hip): lane l holds A[row l&15][k] with
// k = 16(l>>4) + j for operand bytes j = 0..15 and k = 64 + 16(l>>4) + (j-16) for bytes 16..31 (B likewise with
// its column); the scale byte selected by OPSEL in lane l applies to row (col) l&15, K-block l>>4 (k 32b..32b+31)
// — not to the lane's own bytes; C/D the standard 16×16 map.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// e4m3 (OCP) of a small integer |v| <= 15
static unsigned char e4m3(int v) {
    if (v == 0) return 0;
    const int s = v < 0;
    int a = abs(v), e = 0;
    while ((a >> e) > 1) e++;
    const int mant = ((a << 3) >> e) & 7;   // exact for a <= 15
    return (unsigned char)((s << 7) | ((e + 7) << 3) | mant);
}

template <int OPSEL>
__global__ void k_mx(const unsigned char* A, const unsigned char* B, const unsigned* sa, const unsigned* sb,
                     float* C) {
    const int l = threadIdx.x;
    v8i a, b;
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    for (int j = 0; j < 32; j++) {
        const int k = j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16);
        pa[j] = A[(l & 15) * 128 + k];   // A [16][128]
        pb[j] = B[(l & 15) * 128 + k];   // Bᵀ [16 cols][128 k]
    }
    const v4f z = {0.f, 0.f, 0.f, 0.f};
    const v4f c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, z, 0, 0, OPSEL, (int)sa[l], OPSEL, (int)sb[l]);
    for (int i = 0; i < 4; i++) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
    int ai[16 * 128], bi[16 * 128];
    unsigned char ha[16 * 128], hb[16 * 128];
    srand(7);
    for (int i = 0; i < 16 * 128; i++) {
        ai[i] = rand() % 31 - 15;
        bi[i] = rand() % 31 - 15;
        ha[i] = e4m3(ai[i]);
        hb[i] = e4m3(bi[i]);
    }
    int sca[16][4], scb[16][4];   // e8m0 exponents per (row, block) / (col, block)
    for (int r = 0; r < 16; r++)
        for (int k = 0; k < 4; k++) sca[r][k] = 127 + rand() % 7 - 3, scb[r][k] = 127 + rand() % 7 - 3;
    double ref[16][16];
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            double s = 0;
            for (int kb = 0; kb < 4; kb++) {
                double p = 0;
                for (int k = 0; k < 32; k++) p += (double)ai[i * 128 + 32 * kb + k] * bi[j * 128 + 32 * kb + k];
                s += p * ldexp(1.0, sca[i][kb] - 127) * ldexp(1.0, scb[j][kb] - 127);
            }
            ref[i][j] = s;
        }
    unsigned char *dA, *dB;
    unsigned *dsa, *dsb;
    float* dC;
    (void)hipMalloc(&dA, sizeof ha);
    (void)hipMalloc(&dB, sizeof hb);
    (void)hipMalloc(&dsa, 64 * 4);
    (void)hipMalloc(&dsb, 64 * 4);
    (void)hipMalloc(&dC, 256 * 4);
    (void)hipMemcpy(dA, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hb, sizeof hb, hipMemcpyHostToDevice);
    for (int opsel = 0; opsel < 2; opsel++) {
        unsigned hsa[64], hsb[64];
        for (int l = 0; l < 64; l++) {   // scale byte at position OPSEL, garbage elsewhere
            hsa[l] = 0x5a5a5a5au, hsb[l] = 0xa5a5a5a5u;
            const int sh = 8 * opsel;
            hsa[l] = (hsa[l] & ~(0xffu << sh)) | ((unsigned)sca[l & 15][l >> 4] << sh);
            hsb[l] = (hsb[l] & ~(0xffu << sh)) | ((unsigned)scb[l & 15][l >> 4] << sh);
        }
        (void)hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice);
        (void)hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
        if (opsel == 0) k_mx<0><<<1, 64>>>(dA, dB, dsa, dsb, dC);
        else k_mx<1><<<1, 64>>>(dA, dB, dsa, dsb, dC);
        float hc[256];
        (void)hipMemcpy(hc, dC, sizeof hc, hipMemcpyDeviceToHost);
        int bad = 0;
        double maxe = 0;
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                const double e = fabs(hc[i * 16 + j] - ref[i][j]);
                maxe = fmax(maxe, e / (fabs(ref[i][j]) + 1));
                if (e > 1e-3 * (fabs(ref[i][j]) + 1)) bad++;
            }
        printf("opsel %d: mismatches %d / 256, max rel err %.3g  (C[0][0]=%g ref %g, C[3][7]=%g ref %g)\n", opsel, bad,
               maxe, hc[0], ref[0][0], hc[3 * 16 + 7], ref[3][7]);
    }
    return 0;
}
