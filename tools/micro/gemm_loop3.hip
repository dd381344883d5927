// Microbenchmark: Q8 GEMM inner-loop variants, 4 waves (2x2), wave tile 64x64, no global traffic, hashed operands.
//  V1: i8 MFMA, cvt + mul + fma per output and block (round-1 / DMA kernel loop)
//  V3: i8 MFMA, d_x*d_w products from v_mfma_f32_16x16x1_4b_f32 (outer products), cvt + fma
//  V4: f16 MFMA on int-valued f16 operands (exact f32 block sum), outer-product scales, fma only
//  V5: f16 MFMA, mul + fma
// Also checks the 4-block outer-product layout assumption (lane l, reg 4b+r = a[4(l/16)+r] * b[16b + l%16]).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));

__device__ unsigned hsh(unsigned x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }

template <int V>
__global__ __launch_bounds__(256, 2) void k_loop(int iters, float* out) {
    constexpr int TI = 4, TJ = 4, BM = 128, BN = 128;
    constexpr int EB = (V >= 4) ? 2 : 1;
    constexpr int LD = 64 * EB + 16;   // two Q8 blocks per "stage" row
    __shared__ __attribute__((aligned(16))) char As[BM * LD];
    __shared__ __attribute__((aligned(16))) char Bs[BN * LD];
    __shared__ __attribute__((aligned(16))) float Asc[2 * BM];
    __shared__ __attribute__((aligned(16))) float Bsc[2 * BN];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (EB == 1) {
        for (int i = tid; i < BM * LD; i += 256) As[i] = (char)(hsh(i + 77 * blockIdx.x) % 255 - 127);
        for (int i = tid; i < BN * LD; i += 256) Bs[i] = (char)(hsh(i * 3 + 1) % 255 - 127);
    } else {
        for (int i = tid; i < BM * LD / 2; i += 256) ((_Float16*)As)[i] = (_Float16)(int)(hsh(i + 77 * blockIdx.x) % 255 - 127);
        for (int i = tid; i < BN * LD / 2; i += 256) ((_Float16*)Bs)[i] = (_Float16)(int)(hsh(i * 3 + 1) % 255 - 127);
    }
    for (int i = tid; i < 2 * BM; i += 256) Asc[i] = 1e-3f * (1 + (hsh(i) & 7));
    for (int i = tid; i < 2 * BN; i += 256) Bsc[i] = 2e-3f * (1 + (hsh(i + 5) & 3));
    __syncthreads();
    const int wr = wave >> 1, wc = wave & 1;
    const int fr = lane & 15, kh = lane >> 4, fq = 4 * kh;
    const int arow = wr * 64, bcol = wc * 64;
    float acc[TI][TJ][4] = {};
    for (int it = 0; it < iters; it++) {
        asm volatile("" ::: "memory");   // operands are re-read from LDS every iteration (no hoisting)
#pragma unroll
        for (int kb = 0; kb < 2; kb++) {
            float sa[TI][4], sb[TJ], sal[TI], sbl;
#pragma unroll
            for (int i = 0; i < TI; i++) {
                const float4 v = *(const float4*)(&Asc[kb * BM + arow + i * 16 + fq]);
                sa[i][0] = v.x, sa[i][1] = v.y, sa[i][2] = v.z, sa[i][3] = v.w;
                sal[i] = Asc[kb * BM + arow + i * 16 + fr];
            }
#pragma unroll
            for (int j = 0; j < TJ; j++) sb[j] = Bsc[kb * BN + bcol + j * 16 + fr];
            sbl = Bsc[kb * BN + bcol + lane];
            v16f prod[TI];
            if constexpr (V == 3 || V == 4) {
#pragma unroll
                for (int i = 0; i < TI; i++) {
                    v16f z = {};
                    prod[i] = __builtin_amdgcn_mfma_f32_16x16x1f32(sal[i], sbl, z, 0, 0, 0);
                }
            }
#pragma unroll
            for (int i = 0; i < TI; i++) {
#pragma unroll
                for (int j = 0; j < TJ; j++) {
                    v4f c;
                    if constexpr (V <= 3) {
                        const long a = *(const long*)(As + (arow + i * 16 + fr) * LD + kb * 32 + 8 * kh);
                        const long b = *(const long*)(Bs + (bcol + j * 16 + fr) * LD + kb * 32 + 8 * kh);
                        const v4i ci = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, v4i{0, 0, 0, 0}, 0, 0, 0);
                        c = v4f{(float)ci[0], (float)ci[1], (float)ci[2], (float)ci[3]};
                    } else {
                        const v8h a = *(const v8h*)(As + (arow + i * 16 + fr) * LD + kb * 64 + 16 * kh);
                        const v8h b = *(const v8h*)(Bs + (bcol + j * 16 + fr) * LD + kb * 64 + 16 * kh);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        float s;
                        if constexpr (V == 3 || V == 4) s = prod[i][4 * j + r];
                        else s = sa[i][r] * sb[j];
                        acc[i][j][r] = fmaf(c[r], s, acc[i][j][r]);
                    }
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
            for (int r = 0; r < 4; r++) s += acc[i][j][r];
    out[blockIdx.x * 256 + tid] = s;
    // layout check (one block): lane, reg 4b+r must equal a[4(l/16)+r] * b[16b + l%16] for a[i]=i+1, b[j]=100+j
    if (blockIdx.x == 0 && wave == 0 && iters == 1) {
        v16f z = {};
        v16f p = __builtin_amdgcn_mfma_f32_16x16x1f32((float)(fr + 1), (float)(100 + lane), z, 0, 0, 0);
        int bad = 0;
        for (int b = 0; b < 4; b++)
            for (int r = 0; r < 4; r++) {
                const float want = (float)(4 * kh + r + 1) * (float)(100 + 16 * b + fr);
                if (p[4 * b + r] != want) bad++;
            }
        out[1000000 + lane] = (float)bad;
    }
}

template <int V>
void run(const char* name, int wgs, float* out) {
    const int iters = 2000;
    k_loop<V><<<wgs, 256>>>(10, out);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_loop<V><<<wgs, 256>>>(iters, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double mfma = (double)wgs * 4 * iters * 2 * 16;
    printf("%-36s wgs=%5d %8.3f ms %7.1f TFLOP/s\n", name, wgs, ms, mfma * 16 * 16 * 32 * 2 / ms / 1e9);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4 << 22);
    k_loop<3><<<1, 256>>>(1, out);
    float bad[64];
    (void)hipMemcpy(bad, out + 1000000, sizeof(bad), hipMemcpyDeviceToHost);
    float tot = 0;
    for (float b : bad) tot += b;
    printf("outer-product layout mismatches: %g\n", tot);
    for (int wgs : {1024, 2048}) {
        run<1>("V1 i8 cvt+mul+fma", wgs, out);
        run<3>("V3 i8 outer-product, cvt+fma", wgs, out);
        run<4>("V4 f16 outer-product, fma", wgs, out);
        run<5>("V5 f16 mul+fma", wgs, out);
    }
    return 0;
}
