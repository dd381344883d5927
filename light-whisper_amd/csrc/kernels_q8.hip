// Q8_0 kernels for gfx950: weight repack / synthetic weights, activation quantisation, and the two
// W8A8 matmul kernels (wave-per-row GEMV for decode, i8-MFMA GEMM for prefill / batched decode).
//
// Arithmetic contract (ggml Q8_0 conventions behind transcribe_cpp, qwen3_asr_server.py:321):
//   activation block (32): d = amax/127 (f32), q = roundf(x/d) (IEEE division), d kept as f16
//   block dot: exact int32 Σ q_w·q_x, contribution (float)sum · (d_w·d_x), f32 accumulation.
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "exact_rows.h"
#include "kernels.h"
#include "lds_dma.h"
#include "rowops.h"
#include "xlane.h"

#ifndef QASR_DIAG
#define QASR_DIAG 0
#endif
#ifndef QASR_PREOFF_ALL
#define QASR_PREOFF_ALL 1
#endif
// big tiles: unroll the K loop by the ring depth up to this depth (0 = only the pre-offset decode tiles)
#ifndef QASR_UNR_RING
#define QASR_UNR_RING 4
#endif
#ifndef QASR_PIN
#define QASR_PIN 1
#endif

namespace qasr {

// ------------------------------------------------------------------------------------------------ helpers

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ float epi_apply(int epi, float acc, int row, int col, const float* bias, const float* res,
                                           int ldy) {
    if (bias) acc += bias[col];
    if (epi == EPI_RESID) acc += res[(size_t)row * ldy + col];
    else if (epi == EPI_GELU) acc = gelu_erf(acc);
    return acc;
}

// quantise one 32-block held by one thread
__device__ __forceinline__ void quant_block32(const float* v, int8_t* q, float* dout) {
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 32; j++) amax = fmaxf(amax, fabsf(v[j]));
    const float d = amax / 127.f;
    int32_t packed[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            int qv = amax == 0.f ? 0 : (int)roundf(v[4 * j + b] / d);
            w |= (qv & 0xff) << (8 * b);
        }
        packed[j] = w;
    }
    int4* qo = (int4*)q;
    qo[0] = make_int4(packed[0], packed[1], packed[2], packed[3]);
    qo[1] = make_int4(packed[4], packed[5], packed[6], packed[7]);
    *dout = __half2float(f2h(d));
}

// ------------------------------------------------------------------------------------------------ repack / synth
__global__ void k_repack_q8(const uint8_t* __restrict__ blocks, int64_t nblk, int8_t* __restrict__ qs,
                            __half* __restrict__ sc) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    const uint8_t* p = blocks + b * QBYTES;
    uint16_t h = (uint16_t)p[0] | ((uint16_t)p[1] << 8);
    sc[b] = __ushort_as_half(h);
    int32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++)
        w[j] = (int32_t)p[2 + 4 * j] | ((int32_t)p[3 + 4 * j] << 8) | ((int32_t)p[4 + 4 * j] << 16) |
               ((int32_t)p[5 + 4 * j] << 24);
    int4* o = (int4*)(qs + b * QK);
    o[0] = make_int4(w[0], w[1], w[2], w[3]);
    o[1] = make_int4(w[4], w[5], w[6], w[7]);
}

void repack_q8(const uint8_t* blocks, int64_t nblk, int8_t* qs, __half* sc, hipStream_t s) {
    if (nblk <= 0) return;
    k_repack_q8<<<(unsigned)cdiv64(nblk, 256), 256, 0, s>>>(blocks, nblk, qs, sc);
}

__global__ void k_synth_q8(uint64_t base, int64_t nblk, float dbase, int64_t gain_bpr, int8_t* __restrict__ qs,
                           __half* __restrict__ sc) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    uint64_t h = smix(base + (uint64_t)b);
    float d = dbase * (0.5f + unit_from(h));
    if (gain_bpr > 0) d = d * synth_row_gain(base, b / gain_bpr);   // the vocabulary table's row norms
    sc[b] = f2h(d);
    int32_t w[8];
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint64_t r = smix(h + (uint64_t)(g + 1));
#pragma unroll
        for (int half = 0; half < 2; half++) {
            int32_t word = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int v = (int)((r >> (8 * (4 * half + j))) & 0xff) - 128;
                v = v < -127 ? -127 : v;
                word |= (v & 0xff) << (8 * j);
            }
            w[2 * g + half] = word;
        }
    }
    int4* o = (int4*)(qs + b * QK);
    o[0] = make_int4(w[0], w[1], w[2], w[3]);
    o[1] = make_int4(w[4], w[5], w[6], w[7]);
}

void synth_q8(uint64_t base, int64_t nblk, float dbase, int8_t* qs, __half* sc, hipStream_t s, int64_t gain_bpr) {
    if (nblk <= 0) return;
    k_synth_q8<<<(unsigned)cdiv64(nblk, 256), 256, 0, s>>>(base, nblk, dbase, gain_bpr, qs, sc);
}

__global__ void k_synth_f32(uint64_t base, int64_t n, float center, float scale, float* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = fmaf(scale, 2.f * unit_from(smix(base + (uint64_t)i)) - 1.f, center);
}
void synth_f32(uint64_t base, int64_t n, float center, float scale, float* out, hipStream_t s) {
    if (n <= 0) return;
    k_synth_f32<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(base, n, center, scale, out);
}

__global__ void k_synth_f16(uint64_t base, int64_t n, float scale, __half* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = f2h(scale * (2.f * unit_from(smix(base + (uint64_t)i)) - 1.f));
}
void synth_f16(uint64_t base, int64_t n, float scale, __half* out, hipStream_t s) {
    if (n <= 0) return;
    k_synth_f16<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(base, n, scale, out);
}

// ------------------------------------------------------------------------------------------------ quant rows
// one thread per 32-block; 8 × float4 loads
__global__ void k_quant_rows(const float* __restrict__ x, int M, int K, int ldx, int8_t* __restrict__ q,
                             float* __restrict__ d) {
    const int nb = K / QK;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * nb) return;
    const int m = (int)(i / nb), b = (int)(i % nb);
    const float4* src = (const float4*)(x + (size_t)m * ldx + b * QK);
    float v[32];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        float4 t = src[j];
        v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
    }
    quant_block32(v, q + (size_t)m * K + b * QK, d + (size_t)m * nb + b);
}

void quant_rows(const float* x, int M, int K, int ldx, int8_t* q, float* d, hipStream_t s) {
    int64_t n = (int64_t)M * (K / QK);
    if (n <= 0) return;
    k_quant_rows<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(x, M, K, ldx, q, d);
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------------ GEMV
// Weight streaming for M ≤ 8 rows.  One wave per 4 output columns (weight rows): per 2 KB K-segment each lane
// owns two 16-byte chunks (lane, lane+64) of every column, so 8 weight loads per lane are in flight at once and
// the activation chunks it loads are reused for all 4 columns.  The two lanes of a Q8 block (adjacent chunks)
// combine their sdot4 partials with one xor-shuffle, so the block sum is the exact int32 of the contract.
// Every load is unconditional (rows past M are clamped and their results dropped), keeping waits counted.
template <int MR, int GV_COLS>
__global__ __launch_bounds__(256) void k_gemv_q8(const int8_t* __restrict__ W, const __half* __restrict__ Wsc, int N,
                                                 int K, const int8_t* __restrict__ X, const float* __restrict__ Xd,
                                                 int M, const float* __restrict__ bias, const float* res, float* y,
                                                 int ldy, int epi) {
    const int lane = threadIdx.x & 63;
    const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * GV_COLS;
    if (n0 >= N) return;
    const int nb = K / QK;
    const bool even = (lane & 1) == 0;
    float acc[GV_COLS][MR];
#pragma unroll
    for (int c = 0; c < GV_COLS; c++)
#pragma unroll
        for (int m = 0; m < MR; m++) acc[c][m] = 0.f;
    for (int seg = 0; seg < K; seg += 2048) {
        int4 w[GV_COLS][2], x[MR][2];
        float dw[GV_COLS][2], dx[MR][2];
        bool in[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const int k = seg + 16 * (lane + 64 * t);
            in[t] = k < K;
            const int kc = min(k, K - 16), blk = kc >> 5;
#pragma unroll
            for (int c = 0; c < GV_COLS; c++) {
                const int n = min(n0 + c, N - 1);
                const v4i wv = __builtin_nontemporal_load((const v4i*)(W + (size_t)n * K + kc));
                w[c][t] = make_int4(wv.x, wv.y, wv.z, wv.w);
                dw[c][t] = __half2float(Wsc[(size_t)n * nb + blk]);
            }
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const int mm = min(m, M - 1);
                x[m][t] = *(const int4*)(X + (size_t)mm * K + kc);
                dx[m][t] = Xd[(size_t)mm * nb + blk];
            }
        }
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int c = 0; c < GV_COLS; c++) {
#pragma unroll
                for (int m = 0; m < MR; m++) {
                    int p = __builtin_amdgcn_sdot4(w[c][t].x, x[m][t].x, 0, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].y, x[m][t].y, p, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].z, x[m][t].z, p, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].w, x[m][t].w, p, false);
                    p += __builtin_amdgcn_update_dpp(0, p, 0xB1, 0xf, 0xf, false);   // + lane ^ 1
                    if (even && in[t]) acc[c][m] = fmaf((float)p, dw[c][t] * dx[m][t], acc[c][m]);
                }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < GV_COLS; c++) {
#pragma unroll
        for (int m = 0; m < MR; m++) {
            const float v = wave_sum(acc[c][m]);
            const int n = n0 + c;
            if (lane == 0 && m < M && n < N) y[(size_t)m * ldy + n] = epi_apply(epi, v, m, n, bias, res, ldy);
        }
    }
}

static double q8_bytes(int M, const Q8Mat& W, int epi) {
    // weights (int8 + f16 scale per 32) + activations (int8 + f32 scale per 32) + f32 output (+ residual read)
    return (double)W.N * W.K * (1.0 + 2.0 / 32) + (double)M * W.K * (1.0 + 4.0 / 32) +
           (double)M * W.N * 4.0 * (epi == EPI_RESID ? 2 : 1);
}

template <int MR>
static void gemv_launch(int cols, const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias,
                        const float* res, float* y, int ldy, int epi, hipStream_t s) {
    const dim3 g(cdiv(W.N, 4 * cols));
    if (cols == 1) k_gemv_q8<MR, 1><<<g, 256, 0, s>>>(W.qs, W.sc, W.N, W.K, xq, xd, M, bias, res, y, ldy, epi);
    else if (cols == 2) k_gemv_q8<MR, 2><<<g, 256, 0, s>>>(W.qs, W.sc, W.N, W.K, xq, xd, M, bias, res, y, ldy, epi);
    else k_gemv_q8<MR, 4><<<g, 256, 0, s>>>(W.qs, W.sc, W.N, W.K, xq, xd, M, bias, res, y, ldy, epi);
}

void gemv_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res, float* y,
             int ldy, int epi, hipStream_t s, int cols) {
    ProfScope ps(s, "gemv_q8", 2.0 * M * W.N * W.K, q8_bytes(M, W, epi));
    QASR_CHECK(W.K % 32 == 0 && W.K >= 32, QASR_E_INVALID, "gemv_q8: K must be a multiple of 32");
    // measured with cold weights (tools/gemv_tune.py): one column per wave except the vocabulary projection and
    // the single-row QKV, where two per wave keep more loads in flight per lane
    if (cols <= 0) cols = (W.N >= 32768 || (M == 1 && W.K <= 2048 && W.N <= 4096)) ? 2 : 1;
    if (M <= 1) gemv_launch<1>(cols, xq, xd, M, W, bias, res, y, ldy, epi, s);
    else if (M <= 2) gemv_launch<2>(cols, xq, xd, M, W, bias, res, y, ldy, epi, s);
    else if (M <= 4) gemv_launch<4>(cols, xq, xd, M, W, bias, res, y, ldy, epi, s);
    else gemv_launch<8>(std::min(cols, 2), xq, xd, M, W, bias, res, y, ldy, epi, s);
}

// ------------------------------------------------------------------------------------------------ fused decode GEMV
// The 1–4-row decoder's weight-streaming launches with the row operations that feed or follow them folded in (at
// batch 1 a separate norm or SwiGLU launch costs ~2 µs of a ~33 µs layer, tools/graph_cost.py).  About one
// workgroup per CU: a wave owns CPW output columns and issues every 16-byte weight load of them first (T = ⌈K/1024⌉
// chunks per lane per column, lane l reading bytes 16(l + 64t); chunks past K clamped and dropped as in k_gemv_q8),
// so the workgroup's whole weight slice is in flight while it builds its activation rows:
//   GV_RMS:  Q8(RMSNorm(src row)·nw) into LDS by rms_row_q8_wg (rmsnorm_q8's per-row-workgroup arithmetic), once
//            per workgroup (a prologue in every workgroup of a column-group grid costs more than the launch it saves);
//   GV_NONE: the Q8 rows as given (global memory).
// SWI: the workgroup's 64 columns are one h block of the interleaved gate/up matrix, whose SwiGLU + Q8
// (swiglu_q8_block: swiglu_q8's lane arithmetic) is the epilogue, into yq [M][N/2] / yd [M][N/64].
// The dot products, their order and the store / residual epilogue are k_gemv_q8's, so the outputs are bit-identical
// to the separate launches (tests/test_ops_gpu.py::test_gemv_fused_*).
// M > MR (a draft verify pass, up to kExactRows rows): the rows run in groups of MR against the weights held in
// registers, each group with exactly the per-row code of an MR-row launch — so every row's result is the same bits
// as when it runs alone (a 1-row decode step): the exact-row contract of the streaming decode (engine.cpp).
template <int MR, int CPW, int T, int PRO, bool SWI, int NWV>
__global__ __launch_bounds__(64 * NWV) void k_gemv_wide(const int8_t* __restrict__ W, const __half* __restrict__ Wsc,
                                                        int N, int K, int M, const int8_t* __restrict__ X,
                                                        const float* __restrict__ Xd, const float* __restrict__ src,
                                                        int ld_src, const float* __restrict__ nw, float eps,
                                                        const float* res, float* y, int ldy, int epi,
                                                        int8_t* __restrict__ yq, float* __restrict__ yd) {
    static_assert(!SWI || CPW * NWV == 64, "SwiGLU epilogue: one 64-column h block per workgroup");
    extern __shared__ __align__(16) unsigned char gv_smem[];
    __shared__ float part[MR][4];
    __shared__ float gub[SWI ? MR : 1][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n0 = (blockIdx.x * NWV + wv) * CPW;
    const int nb = K / QK;
    // the norm rows' loads go out first (measured: 0.8 µs less than behind the weight stream, whose loads a wave's
    // in-order completion would make them wait for)
    constexpr int RK = PRO == GV_RMS ? T : 1;
    float4 rv[PRO == GV_RMS ? MR : 1][RK], rg[RK];
    if constexpr (PRO == GV_RMS) {
        if (tid < 256) {
#pragma unroll
            for (int m = 0; m < MR; m++)
                if (m < M) rms_row_load<RK>(src + (size_t)m * ld_src, K, nw, rv[m], rg);
        }
    }
    int4 w[CPW][T];
    float dw[CPW][T];
#pragma unroll
    for (int c = 0; c < CPW; c++) {
        const int n = min(n0 + c, N - 1);
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int kc = min(16 * (lane + 64 * t), K - 16);
            const v4i wv4 = __builtin_nontemporal_load((const v4i*)(W + (size_t)n * K + kc));
            w[c][t] = make_int4(wv4.x, wv4.y, wv4.z, wv4.w);
            dw[c][t] = __half2float(Wsc[(size_t)n * nb + (kc >> 5)]);
        }
    }
    const int8_t* xq = X;
    const float* xd = Xd;
    if constexpr (PRO == GV_RMS) {
        // the Q8 rows of all M rows in LDS ([M][K] int8, then [M][K/32] scales)
        int8_t* sq = (int8_t*)gv_smem;
        float* sd = (float*)(gv_smem + (size_t)M * K);
        for (int g0 = 0; g0 < M; g0 += MR) {   // M is uniform: every thread meets the barriers inside
            if (g0 > 0) __syncthreads();   // the previous group's part[] reads are done (MR = 1 reuses part[0])
            if (g0 > 0 && tid < 256) {
#pragma unroll
                for (int m = 0; m < MR; m++)
                    if (g0 + m < M) rms_row_load<RK>(src + (size_t)(g0 + m) * ld_src, K, nw, rv[m], rg);
            }
#pragma unroll
            for (int m = 0; m < MR; m++)
                if (g0 + m < M)
                    rms_row_q8_finish<RK>(rv[m], rg, K, eps, sq + (size_t)(g0 + m) * K, sd + (size_t)(g0 + m) * nb,
                                          part[m], tid < 256);
        }
        __syncthreads();
        xq = sq;
        xd = sd;
    }
    const bool even = (lane & 1) == 0;
    for (int g0 = 0; g0 < M; g0 += MR) {
        float acc[CPW][MR];
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int m = 0; m < MR; m++) acc[c][m] = 0.f;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int k = 16 * (lane + 64 * t);
            const bool in = k < K;
            const int kc = min(k, K - 16), blk = kc >> 5;
            int4 x[MR];
            float dx[MR];
#pragma unroll
            for (int m = 0; m < MR; m++) {
                const int mm = min(g0 + m, M - 1);
                x[m] = *(const int4*)(xq + (size_t)mm * K + kc);
                dx[m] = xd[(size_t)mm * nb + blk];
            }
#pragma unroll
            for (int c = 0; c < CPW; c++) {
#pragma unroll
                for (int m = 0; m < MR; m++) {
                    int p = __builtin_amdgcn_sdot4(w[c][t].x, x[m].x, 0, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].y, x[m].y, p, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].z, x[m].z, p, false);
                    p = __builtin_amdgcn_sdot4(w[c][t].w, x[m].w, p, false);
                    p += __builtin_amdgcn_update_dpp(0, p, 0xB1, 0xf, 0xf, false);   // + lane ^ 1
                    // an explicit fma: the same rounding in every row-group instantiation (see rms_row_q8_finish)
                    if (even && in) acc[c][m] = fmaf((float)p, dw[c][t] * dx[m], acc[c][m]);
                }
            }
        }
        if constexpr (SWI) {
            if (g0 > 0) __syncthreads();   // the previous group's SwiGLU has read gub
#pragma unroll
            for (int c = 0; c < CPW; c++)
#pragma unroll
                for (int m = 0; m < MR; m++) {
                    const float v = wave_sum(acc[c][m]);
                    if (lane == 0 && g0 + m < M) gub[m][wv * CPW + c] = v;
                }
            __syncthreads();
            const int m = 2 * wv + (lane >> 5), j = lane & 31;   // rows 2w, 2w+1 on wave w's lane halves
            if (m < MR && g0 + m < M)   // uniform over each 32-lane group
                swiglu_q8_block(gub[m], j, yq + (size_t)(g0 + m) * (N / 2) + 32 * blockIdx.x + j,
                                yd + (size_t)(g0 + m) * (N / 64) + blockIdx.x);
        } else {
#pragma unroll
            for (int c = 0; c < CPW; c++) {
#pragma unroll
                for (int m = 0; m < MR; m++) {
                    const float v = wave_sum(acc[c][m]);
                    const int n = n0 + c, row = g0 + m;
                    if (lane == 0 && row < M && n < N)
                        y[(size_t)row * ldy + n] = epi_apply(epi, v, row, n, nullptr, res, ldy);
                }
            }
        }
    }
}

struct GvArgs {
    const Q8Mat* W;
    int M;
    const int8_t* xq;
    const float* xd;
    const float* src;
    int ld_src;
    const float* nw;
    float eps;
    const float* res;
    float* y;
    int ldy, epi;
    int8_t* yq;
    float* yd;
};

template <int MR, int CPW, int T, int PRO, bool SWI, int NWV>
static void gv_go(const GvArgs& a, hipStream_t s) {
    const Q8Mat& W = *a.W;
    const dim3 g(cdiv(W.N, NWV * CPW));
    const size_t lds = PRO == GV_RMS ? (size_t)a.M * W.K + (size_t)a.M * (W.K / QK) * sizeof(float) : 0;
    k_gemv_wide<MR, CPW, T, PRO, SWI, NWV><<<g, 64 * NWV, lds, s>>>(W.qs, W.sc, W.N, W.K, a.M, a.xq, a.xd, a.src,
                                                                    a.ld_src, a.nw, a.eps, a.res, a.y, a.ldy, a.epi,
                                                                    a.yq, a.yd);
}

template <int MR, int CPW, int PRO>
static void gv_t(int T, const GvArgs& a, hipStream_t s) {
    switch (T) {
        case 1: gv_go<MR, CPW, 1, PRO, false, 4>(a, s); break;
        case 2: gv_go<MR, CPW, 2, PRO, false, 4>(a, s); break;
        case 3: gv_go<MR, CPW, 3, PRO, false, 4>(a, s); break;
        case 4: gv_go<MR, CPW, 4, PRO, false, 4>(a, s); break;
        default:
            if constexpr (PRO == GV_NONE) gv_go<MR, CPW, 6, PRO, false, 4>(a, s);
            break;
    }
}

template <int MR>
static void gv_mr(int pro, bool swi, int cpw, int T, const GvArgs& a, hipStream_t s) {
    if (swi) {
        switch (T) {
            case 1: gv_go<MR, 8, 1, GV_RMS, true, 8>(a, s); break;
            case 2: gv_go<MR, 8, 2, GV_RMS, true, 8>(a, s); break;
            case 3: gv_go<MR, 8, 3, GV_RMS, true, 8>(a, s); break;
            default: gv_go<MR, 8, 4, GV_RMS, true, 8>(a, s); break;
        }
    } else if (pro == GV_RMS) {
        if (cpw == 4) gv_t<MR, 4, GV_RMS>(T, a, s);
        else if (cpw == 2) gv_t<MR, 2, GV_RMS>(T, a, s);
        else gv_t<MR, 1, GV_RMS>(T, a, s);
    } else {
        if (cpw == 4) gv_t<MR, 4, GV_NONE>(T, a, s);
        else if (cpw == 2) gv_t<MR, 2, GV_NONE>(T, a, s);
        else gv_t<MR, 1, GV_NONE>(T, a, s);
    }
}

int gemv_layer_rows() {
    static const int r = getenv("QASR_GV_ROWS") ? std::max(1, std::min(kGemvWideRows, atoi(getenv("QASR_GV_ROWS"))))
                                                 : kGemvWideRows;
    return r;
}

bool gemv_fused_ok(int pro, int M, int K) {
    if (M < 1 || M > kExactRows || K % QK != 0 || K < QK) return false;
    // GV_RMS keeps the M quantised rows in LDS (K + K/32·4 bytes each) beside the static arrays
    return pro == GV_RMS ? K <= 4096 && (size_t)M * K * 9 / 8 <= 144 * 1024 : K <= 6144;
}

// ------------------------------------------------------------------------------------------------ exact-row GEMM (MFMA)
// The draft verify passes' (and the batch-invariant decode's) linears with EXACTLY the arithmetic of k_gemv_wide's
// 1-row launch, the block dots on the matrix core: exact_rows.h (exact_frag) holds the arithmetic and its derivation.
// A workgroup per 16-column fragment and all RF 16-row fragments (the weight span loaded once for them).
template <int T, int RF>
__global__ __launch_bounds__(256, 2) void k_gemm_q8_exact(const int8_t* __restrict__ X, const float* __restrict__ Xd, int M,
                                                       const int8_t* __restrict__ W, const __half* __restrict__ Wsc,
                                                       int N, int K, const float* res, float* y, int ldy, int epi) {
    __shared__ float hx[4][RF][4][64];   // [wave][row fragment][r][lane]: H_w = O_2w + O_2w+1 of each output
    // rows past 16·RF: grid.y chunks of 16·RF rows, each with the arithmetic of a launch of its own rows (the per-row
    // code depends on nothing but the row)
    {
        const int m0 = (int)blockIdx.y * 16 * RF;
        X += (size_t)m0 * K;
        Xd += (size_t)m0 * (K / QK);
        y += (size_t)m0 * ldy;
        if (res) res += (size_t)m0 * ldy;
        M -= m0;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16;
    float v[4];
    exact_frag<T, RF, XS_PLAIN>(X, Xd, M, W, Wsc, N, K, n0, hx, v);
    if (wv >= RF) return;
    const int f = wv;   // wave f stores row fragment f
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = 16 * f + 4 * (lane >> 4) + r, col = n0 + (lane & 15);
        if (row < M && col < N) y[(size_t)row * ldy + col] = epi_apply(epi, v[r], row, col, nullptr, res, ldy);
    }
}

int exact_mfma_rows() {
    static const int r = getenv("QASR_EXACT_MFMA_ROWS") ? atoi(getenv("QASR_EXACT_MFMA_ROWS")) : 5;
    return r > 0 ? r : kExactRows + 1;   // 0: never (the GEMV rows everywhere)
}

bool gemm_exact_rows_ok(int M, const Q8Mat& W) {
    const int T = W.K / 1024;
    return M >= 1 && W.K % 1024 == 0 && (T == 1 || T == 2 || T == 3 || T == 4 || T == 6) && !W.mx;
}

void gemm_exact_rows(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* res, float* y, int ldy,
                     int epi, hipStream_t s) {
    ProfScope ps(s, "gemm_q8_exact", 2.0 * M * W.N * W.K, q8_bytes(M, W, epi));
    QASR_CHECK(gemm_exact_rows_ok(M, W), QASR_E_INVALID, "gemm_exact_rows: rows ≥ 1, K a multiple of 1024 (T 1-4, 6)");
    QASR_CHECK(epi == EPI_STORE || (epi == EPI_RESID && res), QASR_E_INVALID, "gemm_exact_rows: store or residual");
    // one launch for any row count: 32-row chunks along grid.y (≤ 16 rows: one 16-row chunk)
    const dim3 grid(cdiv(W.N, 16), M <= 16 ? 1 : cdiv(M, 32));
#define EXACT_GO(TT)                                                                                                   \
    do {                                                                                                               \
        if (M <= 16)                                                                                                   \
            k_gemm_q8_exact<TT, 1><<<grid, 256, 0, s>>>(xq, xd, M, W.qs, W.sc, W.N, W.K, res, y, ldy, epi);            \
        else                                                                                                           \
            k_gemm_q8_exact<TT, 2><<<grid, 256, 0, s>>>(xq, xd, M, W.qs, W.sc, W.N, W.K, res, y, ldy, epi);            \
    } while (0)
    switch (W.K / 1024) {
        case 1: EXACT_GO(1); break;
        case 2: EXACT_GO(2); break;
        case 3: EXACT_GO(3); break;
        case 4: EXACT_GO(4); break;
        default: EXACT_GO(6); break;
    }
#undef EXACT_GO
}

void gemv_fused(int pro, const int8_t* xq, const float* xd, const float* src, int ld_src, const float* nw, float eps,
                int M, const Q8Mat& W, const float* res, float* y, int ldy, int epi, int8_t* yq, float* yd,
                hipStream_t s) {
    const bool swi = epi == EPI_SWIGLU;
    ProfScope ps(s, pro == GV_RMS ? (swi ? "gemv_q8_rms_swiglu" : "gemv_q8_rms") : "gemv_q8_wide",
                 2.0 * M * W.N * W.K, q8_bytes(M, W, swi ? EPI_STORE : epi));
    QASR_CHECK(pro == GV_RMS || pro == GV_NONE, QASR_E_INVALID, "gemv_fused: unknown prologue");
    QASR_CHECK(gemv_fused_ok(pro, M, W.K), QASR_E_INVALID, "gemv_fused: rows or K out of range");
    QASR_CHECK(pro != GV_RMS || (nw && ld_src % 4 == 0 && ((uintptr_t)src & 15) == 0), QASR_E_INVALID,
               "gemv_fused: norm rows must be 16-byte aligned float rows with a weight");
    QASR_CHECK(pro != GV_NONE || (xq && xd), QASR_E_INVALID, "gemv_fused: Q8 rows missing");
    QASR_CHECK(epi == EPI_STORE || (epi == EPI_RESID && res) || (swi && pro == GV_RMS && W.N % 64 == 0 && yq && yd),
               QASR_E_INVALID, "gemv_fused: epilogue (SwiGLU needs the norm prologue, N % 64 == 0 and yq / yd)");
    const int T = cdiv(W.K, 1024);
    // columns per wave: about one workgroup of four waves per CU on the decoder shapes (N 1,024–4,096)
    const int cpw = W.N >= 4096 ? 4 : W.N >= 2048 ? 2 : 1;
    const GvArgs a{&W, M, xq, xd, src, ld_src, nw, eps, res, y, ldy, epi, yq, yd};
    // QASR_EXACT_MR (diagnosis): the row-group size of launches with more rows (1, 2, 4 or 8)
    static const int mr = getenv("QASR_EXACT_MR") ? atoi(getenv("QASR_EXACT_MR")) : 8;
    // the SwiGLU launch (8 columns per wave) runs its rows in groups of 4 from K 2,048 up: 8-row groups spill 108 VGPRs
    // there (a row's arithmetic is the same in every group size — test_gemv_exact_rows)
    const bool mr4 = swi && T >= 2;
    if (M <= 1 || mr == 1) gv_mr<1>(pro, swi, cpw, T, a, s);
    else if (M <= 2 || mr == 2) gv_mr<2>(pro, swi, cpw, T, a, s);
    else if (M <= 4 || mr == 4 || mr4) gv_mr<4>(pro, swi, cpw, T, a, s);
    else gv_mr<8>(pro, swi, cpw, T, a, s);
}

// deterministic by default (a transcript is a function of the weights and the audio); QASR_ATOMICS=1 (or
// qasr_set_deterministic(0)) lets decode-shape GEMMs split K with f32 atomics instead (throughput A/B runs)
static std::atomic<int> g_det{[] {
    const char* e = getenv("QASR_ATOMICS");
    return e && atoi(e) != 0 ? 0 : 1;
}()};
// K-128 stages take their scales by 16-byte DMA (WS4) when the matrix carries the regrouped copy (Q8Mat::sc4)
static bool g_ws4 = [] {
    const char* e = getenv("QASR_STAGE_SCALES");
    return !(e && atoi(e) == 0);
}();
void set_stage_scales(bool on) { g_ws4 = on; }
static std::atomic<uint64_t> g_det_gen{0};
void set_deterministic(bool on) {
    if (g_det.exchange(on ? 1 : 0) != (on ? 1 : 0)) g_det_gen++;
}
bool deterministic() { return g_det.load(std::memory_order_relaxed) != 0; }
static thread_local bool g_stable = false;
StableOrderScope::StableOrderScope(bool on) : prev(g_stable) { g_stable = on || prev; }
StableOrderScope::~StableOrderScope() { g_stable = prev; }
bool stable_order() { return g_stable; }
uint64_t deterministic_gen() { return g_det_gen.load(); }


// ------------------------------------------------------------------------------------------------ GEMM (MFMA)
// Tile (32·TI)×(32·TJ), 256 threads = 2×2 waves, each wave (16·TI)×(16·TJ) built from
// v_mfma_i32_16x16x32_i8: one MFMA yields the exact int32 sum of one Q8 block for a 16×16 sub-tile, which is
// rescaled into the f32 accumulator by d_x(row)·d_w(col) (3 VALU ops per output and block — with the MFMA
// this is the whole inner loop).  K step = 128 (four Q8 blocks).  A (activations [M][K]) and B (weights
// [N][K]) are staged through double-buffered LDS with a 144-byte row stride (conflict-free ds_read_b64
// fragments); block scales are stored block-major and lane-permuted so each lane fetches its 4 row scales
// and its TJ column scales with one ds_read_b128 each.  Step s+1 is loaded into registers while step s is
// consumed, one barrier per step.
// Split-K over grid.z fills the chip when M·N has few tiles (decode): partial sums are added with f32 atomics
// (y pre-zeroed for a plain store; the residual already sits in y), the bias is added by split 0.
// Shared GEMM epilogue: the wave's (16·TI)×(16·TJ) f32 accumulators (lane: rows fq..fq+3 of each 16-row
// fragment, column fr of each 16-column fragment) → bias / residual / GELU store, split-K f32 atomics, or the fused
// SwiGLU + Q8 quantisation of interleaved gate/up columns.
template <int TI, int TJ, bool SUMMED = false>
__device__ __forceinline__ void gemm_epilogue(const float (&acc)[TI][TJ][4], int M, int N, int m0, int n0, int arow,
                                              int bcol, int fr, int fq, const float* __restrict__ bias,
                                              const float* res, float* y, int ldy, int epi, int8_t* __restrict__ yq,
                                              float* __restrict__ yd) {
    if constexpr (TJ == 4) {
        if (epi == EPI_SWIGLU) {
            // this wave's 64 columns = gate/up of 32 consecutive h columns = one Q8 block of the SwiGLU output
            const int F = N / 2, hb = (n0 + bcol) / 2;
#pragma unroll
            for (int i = 0; i < TI; i++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = m0 + arow + i * 16 + fq + r;
                    const float g0 = acc[i][0][r], g1 = acc[i][2][r];
                    const float h0 = g0 / (1.f + expf(-g0)) * acc[i][1][r];
                    const float h1 = g1 / (1.f + expf(-g1)) * acc[i][3][r];
                    float am = fmaxf(fabsf(h0), fabsf(h1));
                    am = max16(am);
                    const float dd = am / 127.f;
                    if (row < M && hb < F) {
                        int8_t* qr = yq + (size_t)row * F + hb;
                        qr[fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(h0 / dd));
                        qr[16 + fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(h1 / dd));
                        if (fr == 0) yd[(size_t)row * (F / QK) + hb / QK] = __half2float(f2h(dd));
                    }
                }
            }
            return;
        }
    }
    if constexpr (TJ % 2 == 0) {
        if (epi == EPI_GELU_Q8) {
            // erf-GELU(acc + bias) quantised to Q8 rows: fragments 2b, 2b+1 = one 32-column block of the output
#pragma unroll
            for (int i = 0; i < TI; i++) {
#pragma unroll
                for (int b = 0; b < TJ / 2; b++) {
                    const int c0 = n0 + bcol + 32 * b;
                    const float b0 = bias && c0 + fr < N ? bias[c0 + fr] : 0.f;
                    const float b1 = bias && c0 + 16 + fr < N ? bias[c0 + 16 + fr] : 0.f;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = m0 + arow + i * 16 + fq + r;
                        const float h0 = gelu_erf(acc[i][2 * b][r] + b0), h1 = gelu_erf(acc[i][2 * b + 1][r] + b1);
                        float am = fmaxf(fabsf(h0), fabsf(h1));
                        am = max16(am);
                        const float dd = am / 127.f;
                        if (row < M && c0 < N) {
                            int8_t* qr = yq + (size_t)row * N + c0;
                            qr[fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(h0 / dd));
                            qr[16 + fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(h1 / dd));
                            if (fr == 0) yd[(size_t)row * (N / QK) + c0 / QK] = __half2float(f2h(dd));
                        }
                    }
                }
            }
            return;
        }
    }
    if (epi == EPI_STORE_F16) {
#pragma unroll
        for (int i = 0; i < TI; i++)
#pragma unroll
            for (int j = 0; j < TJ; j++) {
                const int col = n0 + bcol + j * 16 + fr;
                const float bv = bias && col < N ? bias[col] : 0.f;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = m0 + arow + i * 16 + fq + r;
                    if (row < M && col < N) ((__half*)y)[(size_t)row * ldy + col] = f2h(acc[i][j][r] + bv);
                }
            }
        return;
    }
    const bool split = !SUMMED && gridDim.z > 1;   // SUMMED: a split-K fix-up already added the partial tiles
#pragma unroll
    for (int i = 0; i < TI; i++) {
#pragma unroll
        for (int j = 0; j < TJ; j++) {
            const int col = n0 + bcol + j * 16 + fr;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + arow + i * 16 + fq + r;
                if (row >= M || col >= N) continue;
                if (split) {
                    float v = acc[i][j][r];
                    if (bias && blockIdx.z == 0) v += bias[col];
                    atomicAdd(y + (size_t)row * ldy + col, v);
                } else {
                    y[(size_t)row * ldy + col] = epi_apply(epi, acc[i][j][r], row, col, bias, res, ldy);
                }
            }
        }
    }
}

// Split-K fix-up (no output atomics, any epilogue): the S = gridDim.z workgroups of a tile each store their partial
// tile write-through (sc1) into `part`, wait for their stores, and one lane counts the arrival with an agent-scope
// add (MI355X_MICROARCH.md, inter-workgroup visibility: one counter add per storing workgroup, the last adder's
// workgroup reads after a barrier, sc1 loads); the workgroup whose add comes last resets the counter for the next
// launch, adds the S partials in split order — the same sum whatever the arrival order, so the result is
// deterministic — and runs the tile's full epilogue (bias, residual, SwiGLU + Q8, …).  Partial layout per tile:
// [split][wave slot][i·TJ + j][r][lane] floats, 256-B contiguous per store instruction.  Every thread of the
// workgroup calls this (it holds two barriers); `has` = this wave owns accumulators (K group 0, active rows).
// Returns true in the workgroup that must run the epilogue, with acc replaced by the full sums.
// `flag`: one LDS int the caller no longer uses (a static __shared__ here would grow the kernel's LDS past the
// 3-workgroups-per-CU budget of the 3-stage decode tiles).
template <int TI, int TJ>
__device__ __forceinline__ bool splitk_fixup(float (&acc)[TI][TJ][4], bool has, int slot, int nslot, float* part,
                                             unsigned* cnt, int* flag) {
    constexpr int PER = TI * TJ * 4 * 64;   // floats per wave slot
    const int S = gridDim.z, z = blockIdx.z, lane = threadIdx.x & 63;
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    float* tp = part + (size_t)tile * S * nslot * PER + (size_t)slot * PER + lane;
    if (has) {
        float* p = tp + (size_t)z * nslot * PER;
#pragma unroll
        for (int i = 0; i < TI; i++)
#pragma unroll
            for (int j = 0; j < TJ; j++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    __hip_atomic_store(p + ((i * TJ + j) * 4 + r) * 64, acc[i][j][r], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt + tile, 1u, QASR_FORMAL_HANDOFF ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(S - 1);
        if (QASR_FORMAL_HANDOFF && last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (last) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return false;
    if (!has) return true;
    // the S partials in split order; every load of a batch of PB partials in flight at once (partials past S and
    // this workgroup's own are not loaded: its own sums come from registers)
    constexpr int F = TI * TJ * 4, PB = F >= 16 ? 4 : 8;
    float own[F];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) own[(i * TJ + j) * 4 + r] = acc[i][j][r];
    float sum[F];
    for (int u0 = 0; u0 < S; u0 += PB) {
        float v[PB][F];
#pragma unroll
        for (int b = 0; b < PB; b++) {
            const int u = u0 + b;
            if (u < S && u != z) {
                const float* p = tp + (size_t)u * nslot * PER;
#pragma unroll
                for (int e = 0; e < F; e++)
                    v[b][e] = __hip_atomic_load(p + e * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int b = 0; b < PB; b++) {
            const int u = u0 + b;
            if (u >= S) break;
#pragma unroll
            for (int e = 0; e < F; e++) {
                const float x = u == z ? own[e] : v[b][e];
                sum[e] = u == 0 ? x : sum[e] + x;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[i][j][r] = sum[(i * TJ + j) * 4 + r];
    return true;
}

constexpr int GBK = 128;     // K per step
constexpr int GLD = 144;     // LDS row stride (bytes)

template <int TI, int TJ>
__global__ __launch_bounds__(256) void k_gemm_q8(const int8_t* __restrict__ X, const float* __restrict__ Xd, int M,
                                                 const int8_t* __restrict__ W, const __half* __restrict__ Wsc, int N,
                                                 int K, const float* __restrict__ bias, const float* res, float* y,
                                                 int ldy, int epi, int steps_per_split, int8_t* __restrict__ yq,
                                                 float* __restrict__ yd) {
    constexpr int BM = 32 * TI, BN = 32 * TJ;
    constexpr int ACH = BM * 8 / 256, BCH = BN * 8 / 256;     // 16-byte chunks per thread per step
    constexpr int ASC = (BM * 4 + 255) / 256, BSC = (BN * 4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) int8_t As[2][BM * GLD];
    __shared__ __attribute__((aligned(16))) int8_t Bs[2][BN * GLD];
    __shared__ __attribute__((aligned(16))) float Asc[2][4 * BM];   // [kb][row]
    __shared__ __attribute__((aligned(16))) float Bsc[2][4 * BN];   // [kb][wc][fr][j]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int nb = K / QK;
    const int k_begin = blockIdx.z * steps_per_split * GBK;
    const int k_end = min(K, k_begin + steps_per_split * GBK);
    const int nsteps = (k_end - k_begin + GBK - 1) / GBK;

    // global → register staging, two slots: step t's tiles are loaded at step t-2 and written to LDS at the end of
    // step t-1, so each load has two steps of compute to land.  The loads are unconditional (addresses clamped
    // into the matrices, out-of-range data zeroed when written to LDS) and the f16 scales stay raw until then:
    // no branch or conversion touches a load result early, so the compiler's vmcnt waits stay counted instead of
    // draining every load in flight.
    int4 ra[2][ACH], rb[2][BCH];
    float rsa[2][ASC];
    unsigned short rsb[2][BSC];
    unsigned ok_a[2], ok_b[2];
    const int kmax = K - 16;
    auto gload = [&](auto slot_c, int k0) {
        constexpr int sl = decltype(slot_c)::value;
        unsigned oa = 0, ob = 0;
#pragma unroll
        for (int c = 0; c < ACH; c++) {
            const int ch = tid + 256 * c, gm = m0 + (ch >> 3), k = k0 + (ch & 7) * 16;
            oa |= (unsigned)(gm < M && k < k_end) << c;
            ra[sl][c] = *(const int4*)(X + (size_t)min(gm, M - 1) * K + min(k, kmax));
        }
#pragma unroll
        for (int c = 0; c < BCH; c++) {
            const int ch = tid + 256 * c, gn = n0 + (ch >> 3), k = k0 + (ch & 7) * 16;
            ob |= (unsigned)(gn < N && k < k_end) << c;
            rb[sl][c] = *(const int4*)(W + (size_t)min(gn, N - 1) * K + min(k, kmax));
        }
#pragma unroll
        for (int c = 0; c < ASC; c++) {
            const int idx = tid + 256 * c, gm = m0 + (idx >> 2), kb = (k0 >> 5) + (idx & 3);
            oa |= (unsigned)(idx < BM * 4 && gm < M && kb * QK < k_end) << (8 + c);
            rsa[sl][c] = Xd[(size_t)min(gm, M - 1) * nb + min(kb, nb - 1)];
        }
#pragma unroll
        for (int c = 0; c < BSC; c++) {
            const int idx = tid + 256 * c, gn = n0 + (idx >> 2), kb = (k0 >> 5) + (idx & 3);
            ob |= (unsigned)(idx < BN * 4 && gn < N && kb * QK < k_end) << (8 + c);
            rsb[sl][c] = ((const unsigned short*)Wsc)[(size_t)min(gn, N - 1) * nb + min(kb, nb - 1)];
        }
        ok_a[sl] = oa;
        ok_b[sl] = ob;
    };
    auto lstore = [&](auto slot_c, int buf) {
        constexpr int sl = decltype(slot_c)::value;
        auto masked = [](int4 v, unsigned ok) {   // bitwise: a select on the aggregate makes it a memory object
            const int mk = -(int)(ok & 1u);
            return make_int4(v.x & mk, v.y & mk, v.z & mk, v.w & mk);
        };
#pragma unroll
        for (int c = 0; c < ACH; c++) {
            const int ch = tid + 256 * c;
            *(int4*)(As[buf] + (ch >> 3) * GLD + (ch & 7) * 16) = masked(ra[sl][c], ok_a[sl] >> c);
        }
#pragma unroll
        for (int c = 0; c < BCH; c++) {
            const int ch = tid + 256 * c;
            *(int4*)(Bs[buf] + (ch >> 3) * GLD + (ch & 7) * 16) = masked(rb[sl][c], ok_b[sl] >> c);
        }
#pragma unroll
        for (int c = 0; c < ASC; c++) {
            const int idx = tid + 256 * c;
            if (idx < BM * 4) Asc[buf][(idx & 3) * BM + (idx >> 2)] = (ok_a[sl] >> (8 + c)) & 1 ? rsa[sl][c] : 0.f;
        }
#pragma unroll
        for (int c = 0; c < BSC; c++) {
            const int idx = tid + 256 * c;
            if (idx < BN * 4) {
                const int n = idx >> 2, kb = idx & 3;
                const int w = n / (16 * TJ), rem = n % (16 * TJ);
                const float v = __half2float(__ushort_as_half(rsb[sl][c]));
                Bsc[buf][kb * BN + w * 16 * TJ + (rem & 15) * TJ + (rem >> 4)] = (ok_b[sl] >> (8 + c)) & 1 ? v : 0.f;
            }
        }
    };

    float acc[TI][TJ][4];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[i][j][r] = 0.f;

    const int fr = lane & 15, fk = 8 * (lane >> 4), fq = 4 * (lane >> 4);
    const int arow = wr * 16 * TI, bcol = wc * 16 * TJ;
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    if (nsteps > 0) gload(S0{}, k_begin);
    if (nsteps > 1) gload(S1{}, k_begin + GBK);
    if (nsteps > 0) lstore(S0{}, 0);
    __syncthreads();
    // step s computes from LDS buffer s&1 (= register slot s&1, already stored)
    auto step = [&](auto slot_c, int s) {
        constexpr int cur = decltype(slot_c)::value;
        using Other = std::integral_constant<int, cur ^ 1>;
        gload(slot_c, k_begin + (s + 2) * GBK);   // unconditional (clamped) so the vmcnt waits stay counted
        const int8_t* as = As[cur];
        const int8_t* bs = Bs[cur];
#pragma unroll 1
        for (int kb = 0; kb < 4; kb++) {
            long a[TI], b[TJ];
            float sa[TI][4], sb[TJ];
#pragma unroll
            for (int i = 0; i < TI; i++) {
                a[i] = *(const long*)(as + (arow + i * 16 + fr) * GLD + kb * 32 + fk);
                const float4 v = *(const float4*)(&Asc[cur][kb * BM + arow + i * 16 + fq]);
                sa[i][0] = v.x, sa[i][1] = v.y, sa[i][2] = v.z, sa[i][3] = v.w;
            }
#pragma unroll
            for (int j = 0; j < TJ; j++) b[j] = *(const long*)(bs + (bcol + j * 16 + fr) * GLD + kb * 32 + fk);
            if constexpr (TJ == 4) {
                const float4 v = *(const float4*)(&Bsc[cur][kb * BN + bcol + fr * 4]);
                sb[0] = v.x, sb[1] = v.y, sb[2] = v.z, sb[3] = v.w;
            } else if constexpr (TJ == 2) {
                const float2 v = *(const float2*)(&Bsc[cur][kb * BN + bcol + fr * 2]);
                sb[0] = v.x, sb[1] = v.y;
            } else {
#pragma unroll
                for (int j = 0; j < TJ; j++) sb[j] = Bsc[cur][kb * BN + bcol + fr * TJ + j];
            }
#pragma unroll
            for (int i = 0; i < TI; i++) {
#pragma unroll
                for (int j = 0; j < TJ; j++) {
                    v4i c = {0, 0, 0, 0};
                    c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[i], b[j], c, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf((float)c[r], sa[i][r] * sb[j], acc[i][j][r]);
                }
            }
        }
        if (s + 1 < nsteps) lstore(Other{}, cur ^ 1);
        __syncthreads();
    };
    for (int s = 0; s < nsteps; s += 2) {
        step(S0{}, s);
        if (s + 1 < nsteps) step(S1{}, s + 1);
    }
    gemm_epilogue<TI, TJ>(acc, M, N, m0, n0, arow, bcol, fr, fq, bias, res, y, ldy, epi, yq, yd);
}


// ------------------------------------------------------------------------------------------------ GEMM (LDS-DMA)
// The main Q8 W8A8 GEMM (K % 64 == 0).  256 threads = WM×WN waves, wave tile (16·TI)×(16·TJ) of
// v_mfma_i32_16x16x32_i8 (one MFMA = the exact int32 sum of one Q8 block for a 16×16 sub-tile), workgroup tile
// BM×BN = (WM·16·TI)×(WN·16·TJ).  2×2 waves of 64×64 (128×128) serve prefill / encoder shapes; 4×1 waves
// (256×64, 128×64) serve batched decode, where the whole active row set shares every weight panel so the
// weights stream from HBM once per step.
//  * Staging: every operand byte goes global → LDS by `global_load_lds` (LDS-DMA, no VGPR staging, no ds_write):
//    a stage is K = 64 (two Q8 blocks) of A [BM][64 B] and B [BN][64 B], A block scales [2][BM] f32 and B scales
//    [BN] × (2 × f16); an NBUF-stage ring keeps stages s+1 … s+NBUF-1 in flight while stage s is consumed (deep
//    rings for the small decode tiles, whose K loop is latency-bound), with one raw barrier per stage and a
//    counted `vmcnt`.
//  * LDS image: 64-B rows, 16-B chunk c of row r stored at chunk c ^ ((r >> 2) & 3) (the DMA is lane-linear, so the
//    swizzle is applied to each lane's SOURCE address); single ds_read_b64 fragment reads (2 × 32 lanes, 64 banks)
//    are then bank-conflict free.  Fragment addresses are made opaque so the compiler cannot pair two of them
//    into ds_read2st64_b64, whose 16-lane / 32-bank groups would conflict 2-way on this image.
//  * Compute: MFMA q is issued LAG MFMAs before its int32 result is rescaled into the f32 accumulator
//    (cvt, d_x·d_w, fma: 3 VALU per output and block); sched_group_barrier pins the MFMA/VALU interleave.  Waves
//    whose rows all lie past M (padded decode buckets) skip the math but still stage their share.
template <int WM, int WN, int TI, int TJ, int NBUF, int BK = 64, int KG = 1, bool WS4 = false>
__global__ __launch_bounds__(256 * KG, KG == 1 ? 2 : 1) void k_gemm_q8d(const int8_t* __restrict__ X, const float* __restrict__ Xd, int M,
                                                     const int8_t* __restrict__ W, const __half* __restrict__ Wsc,
                                                     const __half* __restrict__ Wsc4,
                                                     int N, int K, const float* __restrict__ bias, const float* res,
                                                     float* y, int ldy, int epi, int steps_per_split,
                                                     int8_t* __restrict__ yq, float* __restrict__ yd,
                                                     float* fix_part, unsigned* fix_cnt) {
    static_assert(WM * WN == 4, "k_gemm_q8d: 4 waves per K group");
    static_assert(BK == 64 || BK == 128, "k_gemm_q8d: a stage is 2 or 4 Q8 blocks");
    // KG K groups of 4 waves share the tile: group g takes blocks [g·KB/KG, (g+1)·KB/KG) of every stage and the
    // groups' accumulators are summed through LDS at the end, in group order (more waves per tile — 8 or 16 — without
    // split-K; deterministic)
    static_assert(KG == 1 || ((KG == 2 || KG == 4) && BK == 128), "k_gemm_q8d: K groups");
    // WS4: the stage's scales by 16-byte DMA — A: one lane per row, its 4 block scales ([M][K/32] f32 rows: 16
    // contiguous bytes), LDS [BM][4]; B: the regrouped copy Wsc4 [K/128][N][4] f16 (Q8Mat::sc4), the tile's 8·BN
    // bytes contiguous, LDS [BN][4].  (Otherwise 4-byte gathers, one cache line per lane: 6 instructions and ~384
    // line touches per 64×64 stage against ~70.)
    static_assert(!WS4 || BK == 128, "k_gemm_q8d: WS4 stages are K = 128");
    constexpr int NW = 4 * KG;
    constexpr int KB = BK / 32, NF = TI * TJ;
    constexpr int BM = WM * 16 * TI, BN = WN * 16 * TJ;
    constexpr int RP = 1024 / BK;                       // rows per 1-KB DMA piece
    static_assert(BM % (4 * RP) == 0 && BN % (4 * RP) == 0 && BN <= 256 && BM <= 256, "k_gemm_q8d: tile sides");
    constexpr int OB = BM * BK, OSA = OB + BN * BK, OSB = OSA + KB * BM * 4, STAGE = OSB + (KB / 2) * BN * 4;
    // A / B pieces per wave per stage; with 16 waves (KG 4) a 64×64 stage has fewer A (B) pieces than waves: then
    // the A and B pieces form one list, PP per wave (UNI)
    constexpr int PA = BM / RP, PB = BN / RP;
    constexpr bool UNI = PA % NW != 0 || PB % NW != 0;
    constexpr int AI = UNI ? 0 : PA / NW, BI = UNI ? 0 : PB / NW, PP = UNI ? (PA + PB) / NW : 0;
    static_assert(UNI ? (PP * NW == PA + PB && PP >= 1) : (AI * RP * NW == BM && BI * RP * NW == BN),
                  "k_gemm_q8d: pieces per wave");
    // A scales: [KB][BM] floats gathered by 4-byte DMA (KB·BM/NW per wave); B scales: [KB/2][BN] dwords (two f16
    // each), BN·KB/(2·NW) per wave.
    constexpr int SAW = KB * BM / NW, ASI = (SAW + 63) / 64;
    constexpr int SBW = BN * KB / (2 * NW), BSI = (SBW + 63) / 64;
    constexpr int AR4 = BM / NW, BL4 = BN / (2 * NW);   // WS4: A-scale rows / B-scale 16-byte lanes per wave
    static_assert(!WS4 || (AR4 * NW == BM && AR4 <= 64 && BL4 * 2 * NW == BN && BL4 >= 1), "k_gemm_q8d: WS4 tile");
    constexpr int SCI = WS4 ? 2 : ASI + BSI;            // scale DMA instructions per wave per stage
    // QASR_DIAG (diagnostic builds only, wrong results): bit 0 skips the scale DMAs, bit 1 the math, bit 2 all DMA
    constexpr int NPW = (QASR_DIAG & 4) ? 0 : AI + BI + PP + ((QASR_DIAG & 1) ? 0 : SCI);   // DMAs per wave per stage
    constexpr int D = NBUF - 1;                         // prefetch distance (stages in flight)
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kg = wave >> 2, lw = wave & 3;
    const int wr = lw / WN, wc = lw % WN;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int nb = K / QK;
    const int k_begin = blockIdx.z * steps_per_split * BK;
    const int k_end = min(K, k_begin + steps_per_split * BK);
    const int nsteps = max(0, (k_end - k_begin) / BK);
    // 16-byte chunk c of row r lives at chunk c ^ swz(r): conflict-free ds_read_b64 fragment reads on BK-byte rows
    auto swz = [](int r) { return BK == 64 ? (r >> 2) & 3 : (r >> 1) & 7; };

    // ---- per-lane DMA sources (k-independent parts)
    const int8_t* a_src[AI ? AI : 1];
    const int8_t* b_src[BI ? BI : 1];
    const int8_t* u_src[PP ? PP : 1];
    uint32_t u_dst[PP ? PP : 1];   // LDS byte offsets of the unified pieces (wave-uniform)
#pragma unroll
    for (int u = 0; u < PP; u++) {
        const int p = wave * PP + u;   // wave-uniform
        const bool isa = p < PA;
        const int row = RP * (isa ? p : p - PA) + lane / (BK / 16), c = (lane % (BK / 16)) ^ swz(row);
        u_src[u] = isa ? X + (size_t)min(m0 + row, M - 1) * K + 16 * c : W + (size_t)min(n0 + row, N - 1) * K + 16 * c;
        u_dst[u] = isa ? 1024 * p : OB + 1024 * (p - PA);
    }
#pragma unroll
    for (int u = 0; u < AI; u++) {
        const int row = RP * (wave * AI + u) + lane / (BK / 16), c = (lane % (BK / 16)) ^ swz(row);
        a_src[u] = X + (size_t)min(m0 + row, M - 1) * K + 16 * c;
    }
#pragma unroll
    for (int u = 0; u < BI; u++) {
        const int row = RP * (wave * BI + u) + lane / (BK / 16), c = (lane % (BK / 16)) ^ swz(row);
        b_src[u] = W + (size_t)min(n0 + row, N - 1) * K + 16 * c;
    }
    const float* sa_src[ASI];
#pragma unroll
    for (int u = 0; u < ASI; u++) {
        const int p = wave * SAW + min(64 * u + lane, SAW - 1);
        sa_src[u] = Xd + (size_t)min(m0 + p % BM, M - 1) * nb + p / BM;
    }
    const uint32_t* sb_src[BSI];
#pragma unroll
    for (int u = 0; u < BSI; u++) {
        const int p = wave * SBW + min(64 * u + lane, SBW - 1);
        sb_src[u] = (const uint32_t*)Wsc + (size_t)min(n0 + p % BN, N - 1) * (nb / 2) + p / BN;
    }
    // WS4 sources: row m0 + wave·AR4 + lane's 16-byte scale group; columns n0 + 2(wave·BL4 + lane) (+1) in Wsc4
    const float* sa4_src = Xd + (size_t)min(m0 + wave * AR4 + min(lane, AR4 - 1), M - 1) * nb;
    const __half* sb4_src = Wsc4 + (size_t)4 * min(n0 + 2 * (wave * BL4 + min(lane, BL4 - 1)), N - 2);

    // LDS byte address of this wave's pieces (wave-uniform → SGPR for M0)
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const uint32_t wa = __builtin_amdgcn_readfirstlane(lds0 + 1024 * (wave * AI));
    const uint32_t wb = __builtin_amdgcn_readfirstlane(lds0 + OB + 1024 * (wave * BI));
    const uint32_t wsa = __builtin_amdgcn_readfirstlane(lds0 + OSA + (WS4 ? wave * AR4 * 16 : wave * SAW * 4));
    const uint32_t wsb = __builtin_amdgcn_readfirstlane(lds0 + OSB + (WS4 ? wave * BL4 * 16 : wave * SBW * 4));
    auto issue = [&](int s, int buf) {
        if constexpr ((QASR_DIAG & 4) != 0) return;
        const int k0 = k_begin + s * BK;
        const uint32_t so = buf * STAGE;
#pragma unroll
        for (int u = 0; u < AI; u++) dma_lds16(a_src[u] + k0, wa + so + 1024 * u);
#pragma unroll
        for (int u = 0; u < BI; u++) dma_lds16(b_src[u] + k0, wb + so + 1024 * u);
#pragma unroll
        for (int u = 0; u < PP; u++)
            dma_lds16(u_src[u] + k0, __builtin_amdgcn_readfirstlane(lds0 + u_dst[u]) + so);
        if constexpr ((QASR_DIAG & 1) != 0) return;
        if constexpr (WS4) {
            if (lane < AR4) dma_lds16(sa4_src + k0 / QK, wsa + so);
            if (lane < BL4) dma_lds16(sb4_src + (size_t)(k0 / 128) * N * 4, wsb + so);
            return;
        }
#pragma unroll
        for (int u = 0; u < ASI; u++) {
            if (64 * u + lane < SAW) dma_lds4(sa_src[u] + k0 / QK, wsa + so + 256 * u);
        }
#pragma unroll
        for (int u = 0; u < BSI; u++)
            if (64 * u + lane < SBW) dma_lds4(sb_src[u] + k0 / 64, wsb + so + 256 * u);
    };

    const int fr = lane & 15, kh = lane >> 4, fq = 4 * kh;
    const int arow = wr * 16 * TI, bcol = wc * 16 * TJ;
    const bool active = (QASR_DIAG & 2) == 0 && m0 + arow < M;   // wave-uniform
    int foff[KB];
#pragma unroll
    for (int kb = 0; kb < KB; kb++) foff[kb] = 16 * ((2 * kb + (kh >> 1)) ^ swz(fr)) + 8 * (kh & 1);

    float acc[TI][TJ][4];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[i][j][r] = 0.f;

    // decode tiles (≤ 64×64): the fragment offsets are computed once, opaque (so no two reads are ever paired into
    // ds_read2st64, whose 16-lane groups would conflict on this image), and the K loop is unrolled by the ring depth,
    // so each stage's LDS base is an immediate of its ds_reads — no per-read address VALU in the K loop (round 3:
    // 180 VALU per 16 MFMAs in the cfg-12 loop, 52 of them moves and adds for addresses)
    // (round 4: every tile — the big tiles' per-read opacity copied each hoisted offset into a temporary, one v_mov per
    // LDS read, 16 per stage of the 128×128 K-64 loop; QASR_PREOFF_ALL=0 restores the per-read form)
    constexpr bool PREOFF = TI * TJ <= 4 || QASR_PREOFF_ALL;
    int offa[PREOFF ? KB : 1][PREOFF ? TI : 1], offb[PREOFF ? KB : 1][PREOFF ? TJ : 1];
    if constexpr (PREOFF) {
#pragma unroll
        for (int kb = 0; kb < KB; kb++) {
#pragma unroll
            for (int i = 0; i < TI; i++) {
                offa[kb][i] = (arow + 16 * i + fr) * BK + foff[kb];
                asm volatile("" : "+v"(offa[kb][i]));
            }
#pragma unroll
            for (int j = 0; j < TJ; j++) {
                offb[kb][j] = OB + (bcol + 16 * j + fr) * BK + foff[kb];
                asm volatile("" : "+v"(offb[kb][j]));
            }
        }
    }

#pragma unroll
    for (int t = 0; t < D; t++)
        if (t < nsteps) issue(t, t);
    // stages per trip of the outer loop (one per ring buffer): each unrolled stage's ring slot is a constant, so its
    // LDS base folds into the ds_read immediates (round 4: also the ≤ 4-deep rings of the big tiles, whose per-stage
    // slot arithmetic cost two VALU per LDS read — 36 of the 128×128 K-64 loop's 311 VALU per stage)
    constexpr int UNR = PREOFF || NBUF <= QASR_UNR_RING ? NBUF : 1;
    for (int s0 = 0; s0 < nsteps; s0 += UNR)
#pragma unroll
    for (int ub = 0; ub < UNR; ub++) {
        const int s = s0 + ub;
        if (UNR > 1 && s >= nsteps) break;
        // this wave's DMAs of stage s have landed and its LDS reads of stage s-1 are done; the barrier then makes
        // that true for every wave, so stage s is readable and buffer (s+D)%NBUF (= stage s-1's) is free
        wait_stages<NPW, D>(min(D - 1, nsteps - 1 - s));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + D < nsteps) issue(s + D, (s + D) % NBUF);
        if (!active) continue;
        const char* st = smem + (UNR > 1 ? ub : s % NBUF) * STAGE;
        // fragments and scales of block kb, read just before its MFMAs (the compiler hoists what registers allow)
        constexpr int KBG = KB / KG;   // blocks of this K group per stage
        // OP (outer-product scales): the 16×16·TJ products d_x(row)·d_w(col) of one i-fragment come from one
        // v_mfma_f32_16x16x1_4b_f32 (lane l supplies d_x of row l&15 and d_w of column l; register 4j+r of lane
        // (fr, kh) = d_x[4kh+r]·d_w[16j+fr]) instead of 4·TJ VALU multiplies — the rescale becomes cvt + fma
        constexpr bool OP = TJ <= 4 && KG == 1 && (BK == 64 || TI == 1);
        float sb[KBG][TJ], sa[KBG][TI][4], sal[KBG][TI], sbl[KBG];
        long a[KBG][TI], b[KBG][TJ];
        // WS4 + OP: lane l's column holds the stage's 4 block scales as 8 contiguous bytes ([BN][4] f16); ONE
        // ds_read_b64 per stage takes all four (64 lanes × 8 B = two conflict-free 32-lane halves), where a 16-bit
        // read per block at an 8-byte lane stride was 2-way bank-conflicted (round 5 PMC: 0.49 conflict cycles per
        // LDS instruction in the decode class, 0.003 before the WS4 layout)
        uint2 sb4w = {0u, 0u};
        const int kb0 = kg * (KB / KG);
        // per-fragment LDS reads of block kb into slot sl: the B scale(s), row fragment i (A bytes + scales), column
        // fragment j (B bytes) — QASR_PIN issues each one right after the previous block's last use of its registers
        auto load_bscale = [&](int sl, int kb) {
            if constexpr (WS4) {   // LDS [BN][4] f16 and [BM][4] f32
                if constexpr (OP) {
                    if (kb == kb0) {   // the stage's first block of this K group: all four scales at once
                        const int cl = min(lane, 16 * TJ - 1);
                        sb4w = *(const uint2*)(st + OSB + 8 * (bcol + cl));
                    }
                    const uint32_t w2 = (kb & 2) ? sb4w.y : sb4w.x;
                    sbl[sl] = __half2float(__ushort_as_half((unsigned short)((kb & 1) ? w2 >> 16 : w2 & 0xffff)));
                } else {
#pragma unroll
                    for (int j = 0; j < TJ; j++)
                        sb[sl][j] = __half2float(*(const __half*)(st + OSB + 8 * (bcol + 16 * j + fr) + 2 * kb));
                }
            } else if constexpr (OP) {
                const int cl = min(lane, 16 * TJ - 1);
                const uint32_t v = *(const uint32_t*)(st + OSB + 4 * ((kb >> 1) * BN + bcol + cl));
                sbl[sl] = __half2float(__ushort_as_half((unsigned short)((kb & 1) ? v >> 16 : v & 0xffff)));
            } else {
#pragma unroll
                for (int j = 0; j < TJ; j++) {
                    const uint32_t v = *(const uint32_t*)(st + OSB + 4 * ((kb >> 1) * BN + bcol + 16 * j + fr));
                    sb[sl][j] = __half2float(__ushort_as_half((unsigned short)((kb & 1) ? v >> 16 : v & 0xffff)));
                }
            }
        };
        auto load_afrag = [&](int sl, int kb, int i) {
            if constexpr (WS4) {
                if constexpr (OP) {
                    sal[sl][i] = *(const float*)(st + OSA + 16 * (arow + 16 * i + fr) + 4 * kb);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        sa[sl][i][r] = *(const float*)(st + OSA + 16 * (arow + 16 * i + fq + r) + 4 * kb);
                }
            } else if constexpr (OP) {
                sal[sl][i] = *(const float*)(st + OSA + 4 * (kb * BM + arow + 16 * i + fr));
            } else {
                const float4 v = *(const float4*)(st + OSA + 4 * (kb * BM + arow + 16 * i + fq));
                sa[sl][i][0] = v.x, sa[sl][i][1] = v.y, sa[sl][i][2] = v.z, sa[sl][i][3] = v.w;
            }
            if constexpr (PREOFF) {
                a[sl][i] = *(const long*)(st + offa[kb][i]);
            } else {
                int off = (arow + 16 * i + fr) * BK + foff[kb];
                asm volatile("" : "+v"(off));
                a[sl][i] = *(const long*)(st + off);
            }
        };
        auto load_bfrag = [&](int sl, int kb, int j) {
            if constexpr (PREOFF) {
                b[sl][j] = *(const long*)(st + offb[kb][j]);
            } else {
                int off = OB + (bcol + 16 * j + fr) * BK + foff[kb];
                asm volatile("" : "+v"(off));
                b[sl][j] = *(const long*)(st + off);
            }
        };
        auto load_block = [&](int sl, int kb) {
            load_bscale(sl, kb);
#pragma unroll
            for (int i = 0; i < TI; i++) load_afrag(sl, kb, i);
#pragma unroll
            for (int j = 0; j < TJ; j++) load_bfrag(sl, kb, j);
        };
        // MFMA q (block q / NF, fragment q % NF) is issued LAG MFMAs before its rescale, so the int32 result has
        // landed by the time the cvt/fma reach it and at most LAG+1 results are live
        // (the 128×128 prefill tile runs LAG 2: one result ring slot fewer keeps it at ≤ 168 VGPRs, 3 waves per SIMD)
        constexpr int LAG = (QASR_PIN != 0 && NF >= 16) ? 2 : 3, NQ = (KB / KG) * NF;
        constexpr int NPR = LAG / TJ + 2;   // outer-product results live at once (ring)
        v4i c[LAG + 1];
        v16f prod[NPR];
        // QASR_PIN (default): the instruction order is pinned per MFMA slot — [OP MFMA] MFMA q, the next block's
        // fragment reads (at a block's first MFMA), then the 4 cvt + 4 fma of MFMA q − LAG — with sched_barrier(0)
        // after each slot.  Left to itself the scheduler consumed every MFMA's result right behind it (an s_nop 7
        // stall per MFMA, no MFMA ∥ VALU overlap inside a wave: profiles/r4_*), whatever the sched_group_barrier mix.
        if constexpr (QASR_PIN != 0) load_block(0, kb0);
#pragma unroll
        for (int q = 0; q < NQ + LAG; q++) {
            if (q < NQ) {
                const int kb = q / NF, f = q % NF;
                if (QASR_PIN == 0 && f == 0) load_block(kb, kb0 + kb);
                if constexpr (OP) {
                    if (f % TJ == 0) {
                        const v16f z = {};
                        prod[(q / TJ) % NPR] = __builtin_amdgcn_mfma_f32_16x16x1f32(sal[kb][f / TJ], sbl[kb], z, 0, 0, 0);
                    }
                }
                c[q % (LAG + 1)] =
                    __builtin_amdgcn_mfma_i32_16x16x32_i8(a[kb][f / TJ], b[kb][f % TJ], v4i{0, 0, 0, 0}, 0, 0, 0);
                if (QASR_PIN != 0 && kb + 1 < KB / KG) {
                    // block kb+1's fragments replace block kb's as soon as their last MFMA has issued: row fragment i
                    // after (i, TJ-1), column fragment j after (TI-1, j), the B scale after the block's last OP MFMA
                    const int i = f / TJ, j = f % TJ;
                    if (j == TJ - 1) load_afrag(kb + 1, kb0 + kb + 1, i);
                    if (i == TI - 1) load_bfrag(kb + 1, kb0 + kb + 1, j);
                    if (i == TI - 1 && j == 0) load_bscale(kb + 1, kb0 + kb + 1);
                }
            }
            if (q >= LAG) {
                const int p = q - LAG, kb = p / NF, f = p % NF, i = f / TJ, j = f % TJ;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if constexpr (OP)
                        acc[i][j][r] = fmaf((float)c[p % (LAG + 1)][r], prod[(p / TJ) % NPR][4 * j + r], acc[i][j][r]);
                    else
                        acc[i][j][r] = fmaf((float)c[p % (LAG + 1)][r], sa[kb][i][r] * sb[kb][j], acc[i][j][r]);
                }
            }
            if constexpr (QASR_PIN != 0) __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (QASR_PIN == 0) {
#pragma unroll
            for (int t = 0; t < NQ; t++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, OP ? 8 : 12, 0);
            }
        }
    }
    if constexpr (KG > 1) {
        // groups 1 … KG-1 hand their partial sums to group 0 through the (now idle) staging LDS; group 0 adds them in
        // group order ((acc0 + acc1) + acc2) + acc3 — the same order in every launch
        static_assert((KG - 1) * 4 * 64 * TI * TJ * 4 * 4 <= NBUF * STAGE, "k_gemm_q8d: reduction buffer");
        __syncthreads();
        float4* red = (float4*)smem + (size_t)lw * 64 * TI * TJ + lane;
        constexpr int GS = 4 * 64 * TI * TJ;   // float4s per group
        if (kg > 0 && active) {
#pragma unroll
            for (int i = 0; i < TI; i++)
#pragma unroll
                for (int j = 0; j < TJ; j++)
                    red[(size_t)(kg - 1) * GS + (i * TJ + j) * 64] =
                        make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
        __syncthreads();
        if (kg > 0 && (TI * TJ > 4 || TJ != 4 || !fix_part)) return;
        if (kg == 0 && active) {
#pragma unroll
            for (int g = 1; g < KG; g++)
#pragma unroll
                for (int i = 0; i < TI; i++)
#pragma unroll
                    for (int j = 0; j < TJ; j++) {
                        const float4 v = red[(size_t)(g - 1) * GS + (i * TJ + j) * 64];
                        acc[i][j][0] += v.x, acc[i][j][1] += v.y, acc[i][j][2] += v.z, acc[i][j][3] += v.w;
                    }
        }
    }
    // split-K fix-up (the 64-column wave tiles of ≤ 64×64 workgroup tiles — the SwiGLU-capable decode tiles; the
    // others keep their register budget): the last workgroup of the tile adds the partials
    if constexpr (TI * TJ <= 4 && TJ == 4) {
        if (fix_part && gridDim.z > 1) {
            if (!splitk_fixup<TI, TJ>(acc, kg == 0 && active, lw, 4, fix_part, fix_cnt, (int*)smem)) return;
            if ((KG > 1 && kg != 0) || !active) return;
            gemm_epilogue<TI, TJ, true>(acc, M, N, m0, n0, arow, bcol, fr, fq, bias, res, y, ldy, epi, yq, yd);
            return;
        }
    }
    if ((KG > 1 && kg != 0) || !active) return;
    gemm_epilogue<TI, TJ>(acc, M, N, m0, n0, arow, bcol, fr, fq, bias, res, y, ldy, epi, yq, yd);
}

// ------------------------------------------------------------------------------------------------ GEMM (decode, K over waves)
// Decode-sized Q8 W8A8 GEMM (a decode step's M ≤ 256 rows; every weight byte is read once per step).  One workgroup
// owns a (16·TI)×(16·TJ) output tile over the WHOLE K and its NW waves split K into equal slices: each wave loads its
// fragments straight from global memory into registers (no LDS staging, no barrier inside the loop — every wave is an
// independent load stream, so a CU keeps NW waves' fragments in flight instead of one pipelined K loop), multiplies
// with v_mfma_i32_16x16x32_i8 (one MFMA = the exact int32 sum of one Q8 block) and rescales into f32 as the other Q8
// GEMMs do ((float)sum · (d_x·d_w), fma).  The NW partial tiles are summed once through LDS, in wave order, and wave
// i < TI runs the shared epilogue for row fragment i.  No split-K atomics, no output memset, one launch.
// Lane (fr, kh) holds row / column fr of a 16-row fragment and bytes [8kh, 8kh + 8) of each block: an 8-byte load per
// fragment and block (4 lanes cover a row's 32-byte block; the G blocks of a load group cover its 128-byte line).
template <int TI, int TJ, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemm_q8_ks(const int8_t* __restrict__ X, const float* __restrict__ Xd,
                                                        int M, const int8_t* __restrict__ W,
                                                        const __half* __restrict__ Wsc, int N, int K,
                                                        const float* __restrict__ bias, const float* res, float* y,
                                                        int ldy, int epi, int8_t* __restrict__ yq,
                                                        float* __restrict__ yd) {
    constexpr int BM = 16 * TI, BN = 16 * TJ, G = 4;   // G blocks per load group
    // dynamic LDS: the tile's activation scales [nb][BM] (block-major, so a lane's 4 rows of one block are one
    // ds_read_b128) during the K loop, then the NW partial tiles [NW][TI·TJ][64] float4 (host sizes the max)
    extern __shared__ float4 smem_ks[];
    float* sas = (float*)smem_ks;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int nb = K / QK, per = nb / NW, b0 = wave * per;   // host: nb % (NW·G) == 0
    const int fr = lane & 15, kh = lane >> 4, fq = 4 * kh;
    for (int idx = threadIdx.x; idx < nb * BM; idx += 64 * NW) {
        const int row = idx / nb, blk = idx % nb;   // consecutive threads read consecutive blocks of a row
        sas[blk * BM + row] = Xd[(size_t)min(m0 + row, M - 1) * nb + blk];
    }
    const int8_t* ap[TI];
    const int8_t* bp[TJ];
    const __half* sbp[TJ];
#pragma unroll
    for (int i = 0; i < TI; i++) ap[i] = X + (size_t)min(m0 + 16 * i + fr, M - 1) * K + 8 * kh;
#pragma unroll
    for (int j = 0; j < TJ; j++) {
        const int c = min(n0 + 16 * j + fr, N - 1);
        bp[j] = W + (size_t)c * K + 8 * kh;
        sbp[j] = Wsc + (size_t)c * nb;
    }
    float acc[TI][TJ][4];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[i][j][r] = 0.f;
    __syncthreads();
    for (int g0 = b0; g0 < b0 + per; g0 += G) {
        long a[G][TI], b[G][TJ];
        uint2 sb[TJ];
#pragma unroll
        for (int g = 0; g < G; g++) {
#pragma unroll
            for (int j = 0; j < TJ; j++) b[g][j] = __builtin_nontemporal_load((const long*)(bp[j] + 32 * (g0 + g)));
#pragma unroll
            for (int i = 0; i < TI; i++) a[g][i] = *(const long*)(ap[i] + 32 * (g0 + g));
        }
#pragma unroll
        for (int j = 0; j < TJ; j++) sb[j] = *(const uint2*)(sbp[j] + g0);
#pragma unroll
        for (int g = 0; g < G; g++) {
            float sw[TJ];
#pragma unroll
            for (int j = 0; j < TJ; j++) {
                const uint32_t h2 = g < 2 ? sb[j].x : sb[j].y;
                sw[j] = __half2float(__ushort_as_half((unsigned short)((g & 1) ? h2 >> 16 : h2 & 0xffff)));
            }
#pragma unroll
            for (int i = 0; i < TI; i++) {
                const float4 sx = *(const float4*)(sas + (g0 + g) * BM + 16 * i + fq);
                const float sxr[4] = {sx.x, sx.y, sx.z, sx.w};
#pragma unroll
                for (int j = 0; j < TJ; j++) {
                    const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a[g][i], b[g][j], v4i{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; r++) acc[i][j][r] = fmaf((float)c[r], sxr[r] * sw[j], acc[i][j][r]);
                }
            }
        }
    }
    __syncthreads();   // the scale image is dead: its LDS takes the partial tiles
    float4* red = smem_ks;   // [NW][TI·TJ][64]
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
            red[(wave * TI * TJ + i * TJ + j) * 64 + lane] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    __syncthreads();
    if (wave >= TI) return;
    float out[1][TJ][4];
#pragma unroll
    for (int j = 0; j < TJ; j++) {
        float4 t = red[(wave * TJ + j) * 64 + lane];
#pragma unroll
        for (int w = 1; w < NW; w++) {
            const float4 v = red[(w * TI * TJ + wave * TJ + j) * 64 + lane];
            t.x += v.x, t.y += v.y, t.z += v.z, t.w += v.w;
        }
        out[0][j][0] = t.x, out[0][j][1] = t.y, out[0][j][2] = t.z, out[0][j][3] = t.w;
    }
    gemm_epilogue<1, TJ>(out, M, N, m0, n0, 16 * wave, 0, fr, fq, bias, res, y, ldy, epi, yq, yd);
}

template <int TI, int TJ>
static void launch_gemm(dim3 grid, hipStream_t s, const int8_t* xq, const float* xd, int M, const Q8Mat& W,
                        const float* bias, const float* res, float* y, int ldy, int epi, int sps, int8_t* yq,
                        float* yd) {
    k_gemm_q8<TI, TJ><<<grid, 256, 0, s>>>(xq, xd, M, W.qs, W.sc, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
}
template <int WM, int WN, int TI, int TJ, int NBUF = 3, int BK = 64, int KG = 1>
static void launch_gemm_dma(dim3 grid, hipStream_t s, const int8_t* xq, const float* xd, int M, const Q8Mat& W,
                            const float* bias, const float* res, float* y, int ldy, int epi, int sps, int8_t* yq,
                            float* yd, float* fix_part, unsigned* fix_cnt) {
    if constexpr (BK == 128) {
        if (W.sc4 && g_ws4 && W.N % 2 == 0) {
            k_gemm_q8d<WM, WN, TI, TJ, NBUF, BK, KG, true><<<grid, 256 * KG, 0, s>>>(
                xq, xd, M, W.qs, W.sc, W.sc4, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd, fix_part, fix_cnt);
            return;
        }
    }
    k_gemm_q8d<WM, WN, TI, TJ, NBUF, BK, KG><<<grid, 256 * KG, 0, s>>>(xq, xd, M, W.qs, W.sc, nullptr, W.N, W.K, bias,
                                                                      res, y, ldy, epi, sps, yq, yd, fix_part, fix_cnt);
}

// GEMM configurations: 0..3 register-staged kernel (any K % 32 == 0), 4..11 LDS-DMA kernel, 2×2 waves, stages of
// 64 (4..7) or 128 (8..11) K (K % bk == 0); 12..13 LDS-DMA, 4×1 waves (64-column wave tiles), K-128 stages.
// ks: waves of the K-over-waves decode kernel (bk unused)
struct GemmCfg { int bm, bn, bk; bool dma; int ks = 0; };
static const GemmCfg kGemmCfgs[] = {
    {128, 128, 128, false}, {64, 128, 128, false}, {64, 64, 128, false}, {32, 64, 128, false},   // 0..3
    {128, 128, 64, true}, {64, 128, 64, true}, {64, 64, 64, true}, {128, 64, 64, true},          // 4..7
    {128, 128, 128, true}, {64, 128, 128, true}, {64, 64, 128, true}, {128, 64, 128, true},      // 8..11
    {64, 64, 128, true}, {128, 64, 128, true},                                                   // 12..13 4×1 waves
    {64, 64, 128, true}, {64, 64, 128, true},                        // 14..15 = 10 / 12 with two K groups (8 waves)
    // decode-sized tiles with deep rings, meant for full-K (no split-K) launches of ≥ 256 workgroups
    {32, 32, 128, true}, {32, 64, 128, true}, {64, 32, 128, true},   // 16..18 rings of 8 / 6 / 6
    {64, 64, 128, true}, {64, 64, 128, true},                        // 19..20 = 14 / 15 (two K groups) with rings of 6
    {64, 64, 128, true}, {64, 64, 128, true}, {32, 128, 128, true},  // 21..23 2×2 / 4×1 waves ring 6, 2×2 (16×64) ring 4
    // 24..30 decode kernel k_gemm_q8_ks<TI, TJ, NW>: full K per workgroup, K split over NW waves
    {32, 16, 0, false, 16}, {32, 32, 0, false, 16}, {64, 16, 0, false, 16}, {64, 32, 0, false, 8},
    {16, 64, 0, false, 16}, {32, 64, 0, false, 8}, {64, 64, 0, false, 8},
    {0, 0, 0, false},   // 31: reserved (the ops' "auto" code)
    // 32..35: reserved (round 4's four-K-group 16-wave tiles: never faster, removed in round 5 — DESIGN §10)
    {0, 0, 0, false}, {0, 0, 0, false}, {0, 0, 0, false}, {0, 0, 0, false},
    // round 4, K-128 stages: 36..37 one K group, ring 6 — 64×32, 32×64 (256 tiles of N 2,048 at 256 rows); 38..39 two
    // K groups — 128×64 4×1, 128×128 2×2.  (40..48, round 4's 32×32×32 kernel k_q8mm: never picked, removed in round 5)
    {64, 32, 128, true}, {32, 64, 128, true}, {128, 64, 128, true}, {128, 128, 128, true},   // 36..39
};
constexpr int kNumGemmCfgs = sizeof(kGemmCfgs) / sizeof(kGemmCfgs[0]);

template <int TI, int TJ, int NW>
static void launch_ks(hipStream_t s, const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias,
                      const float* res, float* y, int ldy, int epi, int8_t* yq, float* yd) {
    const dim3 grid(cdiv(W.N, 16 * TJ), cdiv(M, 16 * TI));
    const size_t lds = std::max<size_t>((size_t)(W.K / QK) * 16 * TI * 4, (size_t)NW * TI * TJ * 64 * 16);
    QASR_CHECK(lds <= 160 * 1024, QASR_E_INVALID, "gemm_q8: decode tile's LDS exceeds 160 KB");
    k_gemm_q8_ks<TI, TJ, NW><<<grid, 64 * NW, lds, s>>>(xq, xd, M, W.qs, W.sc, W.N, W.K, bias, res, y, ldy, epi, yq, yd);
}

static void launch_ks_cfg(int cfg, hipStream_t s, const int8_t* xq, const float* xd, int M, const Q8Mat& W,
                          const float* bias, const float* res, float* y, int ldy, int epi, int8_t* yq, float* yd) {
    switch (cfg) {
        case 24: launch_ks<2, 1, 16>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        case 25: launch_ks<2, 2, 16>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        case 26: launch_ks<4, 1, 16>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        case 27: launch_ks<4, 2, 8>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        case 28: launch_ks<1, 4, 16>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        case 29: launch_ks<2, 4, 8>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
        default: launch_ks<4, 4, 8>(s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd); break;
    }
}

static void launch_cfg(int cfg, dim3 grid, hipStream_t s, const int8_t* xq, const float* xd, int M, const Q8Mat& W,
                       const float* bias, const float* res, float* y, int ldy, int epi, int sps, int8_t* yq,
                       float* yd, float* fp = nullptr, unsigned* fc = nullptr) {
    switch (cfg) {
        case 0: launch_gemm<4, 4>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd); break;
        case 1: launch_gemm<2, 4>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd); break;
        case 2: launch_gemm<2, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd); break;
        case 3: launch_gemm<1, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd); break;
        case 4: launch_gemm_dma<2, 2, 4, 4, 3, 64>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 5: launch_gemm_dma<2, 2, 2, 4, 3, 64>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 6: launch_gemm_dma<2, 2, 2, 2, 3, 64>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 7: launch_gemm_dma<2, 2, 4, 2, 3, 64>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 8: launch_gemm_dma<2, 2, 4, 4, 2, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 9: launch_gemm_dma<2, 2, 2, 4, 3, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 10: launch_gemm_dma<2, 2, 2, 2, 3, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 11: launch_gemm_dma<2, 2, 4, 2, 3, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        // 4×1 waves of 64 columns: the SwiGLU epilogue on 64-column workgroup tiles
        case 12: launch_gemm_dma<4, 1, 1, 4, 3, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 13: launch_gemm_dma<4, 1, 2, 4, 3, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 14: launch_gemm_dma<2, 2, 2, 2, 3, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 15: launch_gemm_dma<4, 1, 1, 4, 3, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 16: launch_gemm_dma<2, 2, 1, 1, 8, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 17: launch_gemm_dma<2, 2, 1, 2, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 18: launch_gemm_dma<2, 2, 2, 1, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 19: launch_gemm_dma<2, 2, 2, 2, 6, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 20: launch_gemm_dma<4, 1, 1, 4, 6, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 21: launch_gemm_dma<2, 2, 2, 2, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 22: launch_gemm_dma<4, 1, 1, 4, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 23: launch_gemm_dma<2, 2, 1, 4, 4, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 36: launch_gemm_dma<2, 2, 2, 1, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 37: launch_gemm_dma<2, 2, 1, 2, 6, 128>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        case 38: launch_gemm_dma<4, 1, 2, 4, 3, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
        default: launch_gemm_dma<2, 2, 4, 4, 2, 128, 2>(grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, fp, fc); break;
    }
}

// ------------------------------------------------------------------------------------------------ MXFP8 (C5)
// The fp8 precision mode (tolerance parity only): operands as OCP MXFP8 — e4m3 elements with one
// e8m0 (power-of-two) scale per 32-element block — multiplied by v_mfma_scale_f32_16x16x128_f8f6f4, which applies
// the block scales inside the matrix core: no per-block VALU rescale, K = 128 per instruction at twice the bf16
// rate.  Operand layout of that instruction (pinned by tools/micro/mx_check.hip / mx_probe.hip): lane l holds
// row (or column) l&15, bytes 0-15 = k 16(l>>4)+j, bytes 16-31 = k 64+16(l>>4)+j; its scale byte is that of
// K-block l>>4 (k 32b..32b+31), not of its own bytes.

// e8m0 exponent E of a block: the smallest E with amax·2^-E ≤ 448 (the e4m3 maximum), clamped to [-127, 127]
__device__ __forceinline__ int mx_block_exp(float amax) {
    if (!(amax > 0.f)) return -127;
    int e;
    const float m = frexpf(amax, &e);   // amax = m·2^e, m ∈ [0.5, 1); 448 = 0.875·2^9
    return max(-127, min(127, m <= 0.875f ? e - 9 : e - 8));
}

// e4m3 (OCP, no inf, 0x7f = NaN never produced) of |v| ≤ 448, round to nearest even; subnormals below 2^-6
__device__ __forceinline__ uint32_t e4m3_rne(float v) {
    const uint32_t sg = v < 0.f ? 0x80u : 0u;
    const float a = fabsf(v);
    if (a < 0.015625f) return sg | (uint32_t)__builtin_rintf(a * 512.f);   // 0..8 (8 = 2^-6, the same bits)
    int x;
    frexpf(a, &x);
    int e = x - 1;                                                      // a ∈ [2^e, 2^(e+1))
    int m = (int)__builtin_rintf(ldexpf(a, 3 - e));                     // 8..16
    if (m == 16) e++, m = 8;
    return sg | (uint32_t)((e + 7) << 3) | (uint32_t)(m - 8);
}

// Q8 blocks (int8 q + scale d) → MXFP8 (e4m3 q·d·2^-E, e8m0 E+127): one thread per 32-block
template <typename SC>
__global__ __launch_bounds__(256) void k_q8_to_mx(const int8_t* __restrict__ q, const SC* __restrict__ d, int64_t nblk,
                                                  uint8_t* __restrict__ q8, uint8_t* __restrict__ s8) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    const int4 w0 = *(const int4*)(q + b * 32), w1 = *(const int4*)(q + b * 32 + 16);
    const int8_t* v = (const int8_t*)&w0;
    const int8_t* u = (const int8_t*)&w1;
    const float dd = (float)d[b];
    int mq = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) mq = max(mq, max(abs((int)v[j]), abs((int)u[j])));
    const int E = mx_block_exp(fabsf(dd) * (float)mq);
    const float sc = mq == 0 ? 0.f : ldexpf(dd, -E);   // exact power-of-two rescale of d (empty block: 0)
    uint32_t o[8];
#pragma unroll
    for (int w = 0; w < 8; w++) {
        uint32_t r = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int j = 4 * w + t;
            const float x = (float)(j < 16 ? v[j] : u[j - 16]) * sc;   // q·d·2^-E: 18 significant bits, exact
            r |= e4m3_rne(x) << (8 * t);
        }
        o[w] = r;
    }
    *(int4*)(q8 + b * 32) = make_int4((int)o[0], (int)o[1], (int)o[2], (int)o[3]);
    *(int4*)(q8 + b * 32 + 16) = make_int4((int)o[4], (int)o[5], (int)o[6], (int)o[7]);
    s8[b] = (uint8_t)(E + 127);
}

void q8_to_mx(const int8_t* q, const float* d, int64_t nblk, uint8_t* q8, uint8_t* s8, hipStream_t s) {
    if (nblk > 0) k_q8_to_mx<float><<<(unsigned)cdiv64(nblk, 256), 256, 0, s>>>(q, d, nblk, q8, s8);
}
void q8w_to_mx(const int8_t* q, const __half* d, int64_t nblk, uint8_t* q8, uint8_t* s8, hipStream_t s) {
    if (nblk > 0) k_q8_to_mx<__half><<<(unsigned)cdiv64(nblk, 256), 256, 0, s>>>(q, d, nblk, q8, s8);
}

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// MXFP8 GEMM y = epi(X·Wᵀ): 2×2 waves of (16·TI)×(16·TJ), K stages of 128 (one MFMA deep) staged global → LDS by
// DMA in an NBUF ring (the k_gemm_q8d pipeline: counted vmcnt, one barrier per stage, 128-B rows with chunk
// c ^ ((r >> 1) & 7)); the stage's block scales are one dword per row (4 e8m0 bytes), lane l picks byte l>>4.
template <int TI, int TJ, int NBUF>
__global__ __launch_bounds__(256, NBUF <= 2 ? 2 : 1) void k_gemm_mx(const uint8_t* __restrict__ X,
                                                             const uint8_t* __restrict__ Xs, int M,
                                                             const uint8_t* __restrict__ W,
                                                             const uint8_t* __restrict__ Ws, int N, int K,
                                                             const float* __restrict__ bias, const float* res,
                                                             float* y, int ldy, int epi, int steps_per_split,
                                                             int8_t* __restrict__ yq, float* __restrict__ yd) {
    constexpr int BK = 128, NW = 4, RP = 8;
    constexpr int BM = 32 * TI, BN = 32 * TJ;
    constexpr int OB = BM * BK, OSA = OB + BN * BK, OSB = OSA + BM * 4, STAGE = OSB + BN * 4;
    constexpr int AI = BM / RP / NW, BI = BN / RP / NW;
    static_assert(AI * RP * NW == BM && BI * RP * NW == BN, "k_gemm_mx: pieces per wave");
    constexpr int SAW = BM / NW, SBW = BN / NW;   // scale dwords per wave per stage (≤ 64)
    constexpr int NPW = AI + BI + 2;
    constexpr int D = NBUF - 1;
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int kq = K / BK;   // scale dwords per row
    const int k_begin = blockIdx.z * steps_per_split * BK;
    const int k_end = min(K, k_begin + steps_per_split * BK);
    const int nsteps = max(0, (k_end - k_begin) / BK);
    auto swz = [](int r) { return (r >> 1) & 7; };

    const uint8_t* a_src[AI];
    const uint8_t* b_src[BI];
#pragma unroll
    for (int u = 0; u < AI; u++) {
        const int row = RP * (wave * AI + u) + lane / 8, c = (lane % 8) ^ swz(row);
        a_src[u] = X + (size_t)min(m0 + row, M - 1) * K + 16 * c;
    }
#pragma unroll
    for (int u = 0; u < BI; u++) {
        const int row = RP * (wave * BI + u) + lane / 8, c = (lane % 8) ^ swz(row);
        b_src[u] = W + (size_t)min(n0 + row, N - 1) * K + 16 * c;
    }
    const uint32_t* sa_src = (const uint32_t*)Xs + (size_t)min(m0 + wave * SAW + min(lane, SAW - 1), M - 1) * kq;
    const uint32_t* sb_src = (const uint32_t*)Ws + (size_t)min(n0 + wave * SBW + min(lane, SBW - 1), N - 1) * kq;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const uint32_t wa = __builtin_amdgcn_readfirstlane(lds0 + 1024 * (wave * AI));
    const uint32_t wb = __builtin_amdgcn_readfirstlane(lds0 + OB + 1024 * (wave * BI));
    const uint32_t wsa = __builtin_amdgcn_readfirstlane(lds0 + OSA + wave * SAW * 4);
    const uint32_t wsb = __builtin_amdgcn_readfirstlane(lds0 + OSB + wave * SBW * 4);
    auto issue = [&](int s, int buf) {
        if constexpr ((QASR_DIAG & 4) != 0) return;
        const int k0 = k_begin + s * BK;
        const uint32_t so = buf * STAGE;
#pragma unroll
        for (int u = 0; u < AI; u++) dma_lds16(a_src[u] + k0, wa + so + 1024 * u);
#pragma unroll
        for (int u = 0; u < BI; u++) dma_lds16(b_src[u] + k0, wb + so + 1024 * u);
        if (lane < SAW) dma_lds4(sa_src + k0 / BK, wsa + so);
        if (lane < SBW) dma_lds4(sb_src + k0 / BK, wsb + so);
    };

    const int fr = lane & 15, kh = lane >> 4, fq = 4 * kh;
    const int arow = wr * 16 * TI, bcol = wc * 16 * TJ;
    const bool active = m0 + arow < M;
    const int flo = 16 * (kh ^ swz(fr)), fhi = 16 * ((4 + kh) ^ swz(fr));
    v4f acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int t = 0; t < D; t++)
        if (t < nsteps) issue(t, t);
    for (int s = 0; s < nsteps; s++) {
        wait_stages<NPW, D>(min(D - 1, nsteps - 1 - s));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + D < nsteps) issue(s + D, (s + D) % NBUF);
        if (!active) continue;
        const char* st = smem + (s % NBUF) * STAGE;
        v8i a[TI], b[TJ];
        int sa[TI], sb[TJ];
#pragma unroll
        for (int i = 0; i < TI; i++) {
            const char* r = st + (arow + 16 * i + fr) * BK;
            const int4 lo = *(const int4*)(r + flo), hi = *(const int4*)(r + fhi);
            a[i] = (v8i){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            sa[i] = (int)((*(const uint32_t*)(st + OSA + 4 * (arow + 16 * i + fr)) >> (8 * kh)) & 0xffu);
        }
#pragma unroll
        for (int j = 0; j < TJ; j++) {
            const char* r = st + OB + (bcol + 16 * j + fr) * BK;
            const int4 lo = *(const int4*)(r + flo), hi = *(const int4*)(r + fhi);
            b[j] = (v8i){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            sb[j] = (int)((*(const uint32_t*)(st + OSB + 4 * (bcol + 16 * j + fr)) >> (8 * kh)) & 0xffu);
        }
#pragma unroll
        for (int i = 0; i < TI; i++)
#pragma unroll
            for (int j = 0; j < TJ; j++)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, sa[i], 0,
                                                                           sb[j]);
    }
    if (!active) return;
    float out[TI][TJ][4];
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) out[i][j][r] = acc[i][j][r];
    gemm_epilogue<TI, TJ>(out, M, N, m0, n0, arow, bcol, fr, fq, bias, res, y, ldy, epi, yq, yd);
}

// workspace for the activations' MXFP8 image (set by the session before its GEMMs; sized for its largest M·K)
static thread_local uint8_t* g_mx_ws = nullptr;
static thread_local size_t g_mx_ws_bytes = 0;
void set_mx_workspace(void* p, size_t bytes) {
    g_mx_ws = (uint8_t*)p;
    g_mx_ws_bytes = bytes;
}
size_t mx_workspace_bytes(int64_t M, int64_t K) { return (size_t)(M * K + M * (K / QK) + 256); }

void gemm_mx(const uint8_t* x8, const uint8_t* xs, int M, const Q8Mat& W, const float* bias, const float* res,
             float* y, int ldy, int epi, hipStream_t s, int8_t* yq, float* yd, bool y_zeroed, int force_cfg) {
    ProfScope ps(s, "gemm_mx", 2.0 * M * W.N * W.K, (double)W.N * W.K * (1 + 1.0 / 32) + (double)M * W.K * (1 + 1.0 / 32));
    QASR_CHECK(W.mx && W.K % 128 == 0, QASR_E_INVALID, "gemm_mx: needs the MXFP8 weights and K % 128 == 0");
    // measured (tools/gemm_mx_tune.py): 128×128 tiles for prefill-sized M and the batched vocabulary projection
    // (128×64 where K ≤ 1024 or N, K ≤ 2048: more tiles, shorter K loops), 64×128 for the vocabulary projection of
    // fewer rows, 64×64 (+ split-K) for the other decode GEMMs;
    // SwiGLU needs 64-column wave tiles
    int cfg = force_cfg;
    if (cfg < 0)
        cfg = M > 256 ? ((W.K <= 1024 || (W.N <= 2048 && W.K <= 2048)) ? 4 : 0) : W.N >= 32768 ? (M > 128 ? 0 : 2) : 1;
    // the SwiGLU epilogue needs 64-column wave tiles (TJ = 4): cfg 0 / 2 / 3; 64×64 → 64×128, 128×64 → 128×128
    if (epi == EPI_SWIGLU && (cfg == 1 || cfg == 4)) cfg = cfg == 1 ? 2 : 0;
    QASR_CHECK(epi != EPI_SWIGLU || cfg == 0 || cfg == 2 || cfg == 3, QASR_E_INVALID,
               "gemm_mx: SwiGLU epilogue needs a 64-column wave tile");
    const int bm = cfg == 0 || cfg == 3 || cfg == 4 ? 128 : 64, bn = cfg == 0 || cfg == 2 || cfg == 3 ? 128 : 64;
    const int steps = W.K / 128, tiles = cdiv(W.N, bn) * cdiv(M, bm);
    const bool can_split = (epi == EPI_STORE || epi == EPI_RESID) && ldy == W.N && (epi != EPI_RESID || res == y);
    int splits = 1;
    if (tiles < 256 && can_split) splits = std::max(1, std::min(std::min(cdiv(512, tiles), steps / 2), 8));
    if (deterministic()) splits = 1;
    const int sps = cdiv(steps, splits);
    splits = cdiv(steps, sps);
    if (splits > 1 && epi == EPI_STORE && !y_zeroed) QASR_HIP(hipMemsetAsync(y, 0, (size_t)M * ldy * sizeof(float), s));
    if (epi == EPI_SWIGLU) QASR_CHECK(W.N % 64 == 0 && yq && yd, QASR_E_INVALID, "gemm_mx: SwiGLU epilogue shape");
    if (epi == EPI_GELU_Q8) QASR_CHECK(W.N % 32 == 0 && yq && yd, QASR_E_INVALID, "gemm_mx: GELU+Q8 epilogue shape");
    const dim3 grid(cdiv(W.N, bn), cdiv(M, bm), splits);
    if (cfg == 0)
        k_gemm_mx<4, 4, 2><<<grid, 256, 0, s>>>(x8, xs, M, W.mx, W.mxs, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
    else if (cfg == 1)
        k_gemm_mx<2, 2, 3><<<grid, 256, 0, s>>>(x8, xs, M, W.mx, W.mxs, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
    else if (cfg == 2)
        k_gemm_mx<2, 4, 3><<<grid, 256, 0, s>>>(x8, xs, M, W.mx, W.mxs, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
    else if (cfg == 3)
        k_gemm_mx<4, 4, 3><<<grid, 256, 0, s>>>(x8, xs, M, W.mx, W.mxs, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
    else
        k_gemm_mx<4, 2, 2><<<grid, 256, 0, s>>>(x8, xs, M, W.mx, W.mxs, W.N, W.K, bias, res, y, ldy, epi, sps, yq, yd);
}

// Q8 activations in, MXFP8 GEMM: the activations' MXFP8 image goes to the session workspace first
static void gemm_mx_q8in(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias,
                         const float* res, float* y, int ldy, int epi, hipStream_t s, int8_t* yq, float* yd,
                         bool y_zeroed) {
    const size_t need = mx_workspace_bytes(M, W.K);
    QASR_CHECK(g_mx_ws && g_mx_ws_bytes >= need, QASR_E_INVALID, "gemm_mx: MXFP8 activation workspace too small");
    uint8_t* x8 = g_mx_ws;
    uint8_t* xs = g_mx_ws + (size_t)M * W.K;
    q8_to_mx(xq, xd, (int64_t)M * (W.K / QK), x8, xs, s);
    gemm_mx(x8, xs, M, W, bias, res, y, ldy, epi, s, yq, yd, y_zeroed, -1);
}

// Split-K fix-up workspace (thread-local registration, like the MXFP8 workspace): partial tiles + one arrival
// counter per tile, zero between launches.  Unregistered (or QASR_NO_FIXUP=1): split-K adds with f32 atomics.
static thread_local float* g_fix_part = nullptr;
static thread_local size_t g_fix_floats = 0;
static thread_local unsigned* g_fix_cnt = nullptr;
static thread_local int g_fix_ncnt = 0;
static thread_local bool g_fix_all = false;
void set_gemm_fixup(float* part, size_t floats, unsigned* cnt, int ncnt, bool all_epilogues) {
    static const bool off = getenv("QASR_NO_FIXUP") && atoi(getenv("QASR_NO_FIXUP")) != 0;
    const bool on = !off && part && cnt;
    g_fix_part = on ? part : nullptr;
    g_fix_floats = on ? floats : 0;
    g_fix_cnt = on ? cnt : nullptr;
    g_fix_ncnt = on ? ncnt : 0;
    g_fix_all = on && all_epilogues;
}

// Decode-step table (M = the step's row bucket ≤ 256, K % 128 == 0): configuration and split-K count per row range,
// from tools/dec_gemm_sweep.py with cold weights on MI355X (profiles/r2_dec_gemm_sweep.log) — every configuration ×
// split count timed per shape; the winners per class of the decoder's shapes: QKV (plain store, K ≤ 2048), the
// attention output projection (residual, K ≤ 2048) and the down projection (residual, K > 2048).
struct DecPick { int m_max, cfg, splits; };
static const DecPick kDecQkv[] = {{16, 17, 6}, {32, 16, 4}, {64, 18, 4}, {128, 14, 2}, {256, 14, 1}};
static const DecPick kDecO[] = {{64, 16, 4}, {128, 18, 4}, {192, 15, 3}, {256, 14, 2}};
static const DecPick kDecDown[] = {{32, 16, 8}, {64, 15, 8}, {96, 10, 8}, {128, 14, 4}, {192, 10, 8}, {256, 15, 4}};
// gate/up with the SwiGLU epilogue: split-K through the fix-up workspace pays off only at ≤ 32 rows
static const DecPick kDecGu[] = {{16, 15, 2}, {32, 23, 2}};

// Deterministic mode (the default): split-K only through the fix-up of the wave-64 tiles (12, 15, 20, 22, 23), else
// unsplit (one-K-group, two-K-group or K-over-waves tiles); the winners of tools/dec_gemm_sweep.py run in that mode
// (profiles/r3a_dec_sweep_det.log, cold weights, every configuration × split).  Used when the fix-up workspace is
// registered (the session's decode steps), else the heuristic below.
// round 4 (pinned slot schedule + 16-byte stage scales): profiles/r4b_sweep*, r4c_sweep* (cold weights)
static const DecPick kDetQkv[] = {{192, 12, 4}, {256, 12, 3}};
static const DecPick kDetO[] = {{16, 24, 0}, {64, 12, 4}, {128, 16, 1}, {192, 12, 4}, {256, 12, 3}};
static const DecPick kDetDown[] = {{192, 12, 8}, {256, 12, 4}};
static const DecPick kDetGu[] = {{64, 12, 4}, {128, 12, 2}, {256, 12, 1}};

static bool dec_table_pick(int M, const Q8Mat& W, int epi, int& cfg, int& splits) {
    if (M > 256 || W.K % 128 != 0 || W.N >= 32768) return false;
    const DecPick* t = nullptr;
    int n = 0;
    const bool det = deterministic() && g_fix_part;
#define QASR_TAB(a, b) (det ? (t = a, n = sizeof(a) / sizeof(DecPick)) : (t = b, n = sizeof(b) / sizeof(DecPick)))
    if (epi == EPI_STORE && W.K <= 2048) QASR_TAB(kDetQkv, kDecQkv);
    else if (epi == EPI_RESID && W.K <= 2048) QASR_TAB(kDetO, kDecO);
    else if (epi == EPI_RESID) QASR_TAB(kDetDown, kDecDown);
    else if (epi == EPI_SWIGLU && g_fix_part) QASR_TAB(kDetGu, kDecGu);
#undef QASR_TAB
    if (!t) return false;
    for (int i = 0; i < n; i++)
        if (M <= t[i].m_max) {
            cfg = t[i].cfg, splits = t[i].splits;
            return true;
        }
    return false;
}

// The configurations whose outputs are each one fma chain over the K blocks in order (one K group, no split): the
// register-staged tiles 0–3 and the LDS-DMA tiles 4–13, 16–18, 21–23.  Stable order picks among them (K % 128 == 0):
// 128×128 for prefill-sized M, else the largest of 64×64 / 32×64 / 32×32 that fills the chip (≥ 256 tiles) — the
// smallest otherwise; the SwiGLU epilogue needs 64-column wave tiles (12), GELU+Q8 64-column workgroup tiles.
static int stable_pick(int M, int N, int epi) {
    if (M > 256) return N >= 32768 ? 8 : 4;   // (the SwiGLU epilogue too: cfg 4's wave tiles are 64 columns wide)
    if (epi == EPI_SWIGLU) return 12;
    const int cand[3] = {10, 17, 16};
    const int n = epi == EPI_GELU_Q8 ? 2 : 3;
    for (int i = 0; i < n; i++) {
        const GemmCfg& g = kGemmCfgs[cand[i]];
        if ((long)cdiv(N, g.bn) * cdiv(M, g.bm) >= 256) return cand[i];
    }
    return cand[n - 1];
}

// force_cfg: -1 auto, else an index into kGemmCfgs (a DMA config on K % 64 != 0 falls back to auto);
// force_splits: split-K (0 = heuristic).
void gemm_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res, float* y,
             int ldy, int epi, hipStream_t s, int force_cfg, int force_splits, int8_t* yq, float* yd, bool y_zeroed) {
    if (W.mx && force_cfg < 0 && W.K % 128 == 0) {   // the model runs in MXFP8 precision mode
        gemm_mx_q8in(xq, xd, M, W, bias, res, y, ldy, epi, s, yq, yd, y_zeroed);
        return;
    }
    // two classes for the bench's roofline: prefill / encoder shapes (M > 256 rows, MFMA-bound) and decode-step
    // shapes (≤ 256 rows, bound by the weight stream and the per-block rescale)
    ProfScope ps(s, M > 256 ? "gemm_q8_prefill" : "gemm_q8_decode", 2.0 * M * W.N * W.K, q8_bytes(M, W, epi));
    auto usable = [&](int c) {
        const GemmCfg& g = kGemmCfgs[c];
        if (g.bm == 0) return false;   // reserved slot
        if (g.ks) return W.K % (QK * 4 * g.ks) == 0 && (epi != EPI_GELU_Q8 || g.bn % 32 == 0);
        return !g.dma || W.K % g.bk == 0;
    };
    int pick;
    if (g_stable && W.K % 128 == 0 && force_cfg < 0) {
        // row-count-independent order (StableOrderScope): a one-K-group configuration without split — every output is
        // its blocks' fma chain in K order, acc = fma((float)Σq·q, d_x·d_w, acc), the same bits for any tile shape and
        // any M (tests/test_ops_gpu.py::test_gemm_chain_configs_bit_identical); the tile by the row count
        pick = stable_pick(M, W.N, epi);
        force_splits = 1;
    } else if (W.K % 64 == 0) {
        // measured on the engine's shapes (tools/gemm_tune.py, profiles/): 128×128 tiles with K-64 stages on prefill
        // / encoder shapes; 64×64 tiles with K-128 stages (+ split-K) on batched decode; the vocabulary projection
        // by row count; decode SwiGLU epilogue on 4×1 waves of 64 columns; two K groups (8 waves per tile) where
        // the tile count is low
        const bool k128 = W.K % 128 == 0;
        // (the vocabulary projection: 128×128 tiles from 97 rows — 163.6 against 202.5 µs for cfg 9 at 128 rows,
        // cold weights, profiles/r6e_lmhead_sweep.log)
        if (W.N >= 32768) pick = !k128 ? 5 : M > 96 ? 8 : M > 32 ? 9 : 10;
        else if (M > 256) pick = 4;
        else if (epi == EPI_SWIGLU) pick = !k128 ? 5 : M > 128 ? 12 : 15;
        else pick = !k128 ? 6 : W.N <= 4096 ? 14 : 10;
        if (force_cfg < 0 && force_splits <= 0) {
            int c, sp;
            if (dec_table_pick(M, W, epi, c, sp) && usable(c)) pick = c, force_splits = sp;   // (K-over-waves tiles
                                                                                                // need K % 2,048)
        }
    } else {
        const int first = M <= 32 ? 3 : M <= 64 ? 1 : 0, last = M <= 32 ? 3 : 2;
        pick = last;
        for (int c = first; c <= last; c++)
            if ((long)cdiv(W.N, kGemmCfgs[c].bn) * cdiv(M, kGemmCfgs[c].bm) >= 256) {
                pick = c;
                break;
            }
    }
    if (force_cfg >= 0 && force_cfg < kNumGemmCfgs && usable(force_cfg)) pick = force_cfg;
    const GemmCfg& cf = kGemmCfgs[pick];
    if (cf.ks) {   // decode kernel: one launch over the whole K, no split-K, no memset
        QASR_CHECK(epi != EPI_SWIGLU || (cf.bn == 64 && W.N % 64 == 0 && yq && yd), QASR_E_INVALID,
                   "gemm_q8: SwiGLU epilogue needs a 64-column wave tile");
        QASR_CHECK(epi != EPI_GELU_Q8 || (W.N % 32 == 0 && yq && yd), QASR_E_INVALID, "gemm_q8: GELU+Q8 epilogue shape");
        launch_ks_cfg(pick, s, xq, xd, M, W, bias, res, y, ldy, epi, yq, yd);
        return;
    }
    const int steps = cf.dma ? W.K / cf.bk : cdiv(W.K, GBK);
    const int tiles = cdiv(W.N, cf.bn) * cdiv(M, cf.bm);
    // split-K through the fix-up workspace (any epilogue, deterministic): a forced / table split count of a DMA tile
    auto fixup_ok = [&](int sp) {
        const bool wave64 = pick == 12 || pick == 15 || pick == 20 || pick == 22 || pick == 23;   // TJ = 4 tiles
        return cf.dma && wave64 && sp > 1 && g_fix_part && tiles <= g_fix_ncnt &&
               (size_t)tiles * sp * cf.bm * cf.bn <= g_fix_floats;
    };
    // The fix-up's serial tail (store → count → reload) costs more than f32 atomics on the plain-store / residual
    // decode shapes (profiles/r2_dec_gemm_sweep_fixup.log), so those keep the atomics (deterministic mode: no split);
    // the SwiGLU epilogue (no atomic form) splits only through the fix-up, deterministic either way.
    // deterministic mode: every split epilogue goes through the fix-up (the tiles that have it; the others run unsplit)
    const bool fix_epi = epi == EPI_SWIGLU || g_fix_all || deterministic();
    if (force_splits > 1 && fix_epi && fixup_ok(std::min(force_splits, steps))) {
        const int sps = cdiv(steps, std::min(force_splits, steps));
        dim3 grid(cdiv(W.N, cf.bn), cdiv(M, cf.bm), cdiv(steps, sps));
        if (epi == EPI_SWIGLU)
            QASR_CHECK(W.N % 64 == 0 && yq && yd && (cf.bn == 128 || pick == 12 || pick == 13 || pick == 15 ||
                                                     pick == 20 || pick == 22 || pick == 38),
                       QASR_E_INVALID, "gemm_q8: SwiGLU epilogue needs a 64-column wave tile");
        launch_cfg(pick, grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd, g_fix_part, g_fix_cnt);
        return;
    }
    if (epi == EPI_SWIGLU) {
        QASR_CHECK(W.N % 64 == 0 && yq && yd, QASR_E_INVALID, "gemm_q8: SwiGLU epilogue needs N % 64 == 0");
        QASR_CHECK(cf.bn == 128 || pick == 12 || pick == 13 || pick == 15 || pick == 20 || pick == 22 || pick == 38,
                   QASR_E_INVALID,
                   "gemm_q8: SwiGLU epilogue needs a 64-column wave tile");
        dim3 grid(cdiv(W.N, cf.bn), cdiv(M, cf.bm), 1);
        launch_cfg(pick, grid, s, xq, xd, M, W, bias, res, y, ldy, epi, steps, yq, yd);
        return;
    }
    const bool can_split = (epi == EPI_STORE || epi == EPI_RESID) && ldy == W.N && (epi != EPI_RESID || res == y);
    if (epi == EPI_GELU_Q8)
        QASR_CHECK(W.N % 32 == 0 && yq && yd && cf.bn >= 64, QASR_E_INVALID, "gemm_q8: GELU+Q8 epilogue shape");
    int splits = 1;
    if (tiles < 256 && can_split) splits = std::max(1, std::min(std::min(cdiv(512, tiles), steps / 2), 8));
    if (force_splits > 0) splits = can_split ? std::min(force_splits, steps) : 1;
    if (deterministic()) splits = 1;
    const int sps = cdiv(steps, splits);
    splits = cdiv(steps, sps);
    if (splits > 1 && epi == EPI_STORE && !y_zeroed)
        QASR_HIP(hipMemsetAsync(y, 0, (size_t)M * ldy * sizeof(float), s));
    dim3 grid(cdiv(W.N, cf.bn), cdiv(M, cf.bm), splits);
    launch_cfg(pick, grid, s, xq, xd, M, W, bias, res, y, ldy, epi, sps, yq, yd);
}

int64_t gate_up_interleaved_row(int64_t r, int64_t F) {
    return r < F ? 32 * (r / 16) + r % 16 : 32 * ((r - F) / 16) + 16 + (r - F) % 16;
}

__global__ void k_gather_rows_q8(const int8_t* __restrict__ qs, const __half* __restrict__ sc, int64_t F, int K,
                                 int8_t* __restrict__ qo, __half* __restrict__ so) {
    const int64_t r = blockIdx.x;   // logical row
    int64_t p = r < F ? 32 * (r / 16) + r % 16 : 32 * ((r - F) / 16) + 16 + (r - F) % 16;
    for (int k = threadIdx.x; k < K; k += blockDim.x) qo[p * K + k] = qs[r * K + k];
    for (int b = threadIdx.x; b < K / QK; b += blockDim.x) so[p * (K / QK) + b] = sc[r * (K / QK) + b];
}

void interleave_gate_up(Q8Mat& W, hipStream_t s) {
    QASR_CHECK(W.N % 32 == 0, QASR_E_INVALID, "interleave_gate_up: N % 32 != 0");
    int8_t* q2 = nullptr;
    __half* s2 = nullptr;
    QASR_HIP(hipMalloc(&q2, (size_t)W.N * W.K));
    QASR_HIP(hipMalloc(&s2, (size_t)W.N * (W.K / QK) * sizeof(__half)));
    k_gather_rows_q8<<<W.N, 256, 0, s>>>(W.qs, W.sc, W.N / 2, W.K, q2, s2);
    QASR_HIP(hipMemcpyAsync(W.qs, q2, (size_t)W.N * W.K, hipMemcpyDeviceToDevice, s));
    QASR_HIP(hipMemcpyAsync(W.sc, s2, (size_t)W.N * (W.K / QK) * sizeof(__half), hipMemcpyDeviceToDevice, s));
    QASR_HIP(hipStreamSynchronize(s));
    QASR_HIP(hipFree(q2));
    QASR_HIP(hipFree(s2));
}

// out[(b/4)·N·4 + 4n + b%4] = sc[n·nb + b]: a K-128 stage's 4 block scales of column n are 8 contiguous bytes and
// the stage's columns n0… one contiguous run (the 16-byte DMA of k_gemm_q8d<…, WS4>)
__global__ void k_stage_scales(const __half* __restrict__ sc, int N, int nb, __half* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // output index
    if (i >= (int64_t)N * nb) return;
    const int64_t g = i / ((int64_t)N * 4), r = i % ((int64_t)N * 4);
    const int64_t n = r / 4, b = 4 * g + r % 4;
    out[i] = sc[n * nb + b];
}

void q8_stage_scales(const __half* sc, int N, int K, __half* out, hipStream_t s) {
    QASR_CHECK(K % 128 == 0 && N > 0, QASR_E_INVALID, "q8_stage_scales: K % 128 != 0");
    const int64_t n = (int64_t)N * (K / QK);
    k_stage_scales<<<(unsigned)cdiv(n, 256), 256, 0, s>>>(sc, N, K / QK, out);
}

void linear_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res,
               float* y, int ldy, int epi, hipStream_t s, bool y_zeroed) {
    if (M <= 0) return;
    if (M <= kGemvRows && !(g_stable && W.K % 128 == 0)) gemv_q8(xq, xd, M, W, bias, res, y, ldy, epi, s);
    else gemm_q8(xq, xd, M, W, bias, res, y, ldy, epi, s, -1, 0, nullptr, nullptr, y_zeroed);
}

// ------------------------------------------------------------------------------------------------ embeddings
__global__ void k_embed_rows(const int* __restrict__ ids, int n, const int8_t* __restrict__ qs,
                             const __half* __restrict__ sc, int K, const float* __restrict__ alt,
                             float* __restrict__ out) {
    const int nb = K / QK;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * nb) return;
    const int r = (int)(i / nb), b = (int)(i % nb);
    const int id = ids[r];
    float4* dst = (float4*)(out + (size_t)r * K + b * QK);
    if (id < 0) {
        const float4* src = (const float4*)(alt + (size_t)(-(id + 1)) * K + b * QK);
#pragma unroll
        for (int j = 0; j < 8; j++) dst[j] = src[j];
        return;
    }
    dequant_block_q8(qs, sc, K, id, b, (float*)dst);
}

void embed_rows(const int* ids, int n, const Q8Mat& W, const float* alt, float* out, hipStream_t s) {
    int64_t total = (int64_t)n * (W.K / QK);
    if (total <= 0) return;
    k_embed_rows<<<(unsigned)cdiv64(total, 256), 256, 0, s>>>(ids, n, W.qs, W.sc, W.K, alt, out);
}

}  // namespace qasr
