// Row-level device routines shared by the stand-alone norm / activation kernels (kernels_nn.hip) and the prologues
// of the fused decode GEMVs (kernels_q8.hip): one definition of the arithmetic, so a row quantised inside a GEMV
// prologue is bit-identical to the one the separate launch writes (the decode-fusion parity contract).
#pragma once
#include "common.h"
#include "wt.h"
#include "xlane.h"

namespace qasr {

// one 32-value block b of Q8 row `id` (qs [..][K] int8, sc [..][K/32] f16) dequantised into dst[0..32): the
// embedding lookup's arithmetic (k_embed_rows, and the decode step's fused plan + embed)
__device__ __forceinline__ void dequant_block_q8(const int8_t* __restrict__ qs, const __half* __restrict__ sc, int K,
                                                 int id, int b, float* __restrict__ dstf) {
    const int nb = K / QK;
    float4* dst = (float4*)dstf;
    const float d = __half2float(sc[(size_t)id * nb + b]);
    const int4* q4 = (const int4*)(qs + (size_t)id * K + b * QK);
#pragma unroll
    for (int h = 0; h < 2; h++) {
        int4 v = q4[h];
        int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            dst[h * 4 + j] = make_float4(d * (float)(int8_t)(w[j] & 0xff), d * (float)(int8_t)((w[j] >> 8) & 0xff),
                                         d * (float)(int8_t)((w[j] >> 16) & 0xff), d * (float)(int8_t)((w[j] >> 24) & 0xff));
        }
    }
}

// one float4 chunk c of a row → 4 int8 of its Q8 block (8 consecutive lanes = one 32-block: amax by three DPP
// steps); the block's first lane writes the scale.  q / d may point to global memory or LDS.
// WT: stored write-through (sc1, wt.h: qrow / drow wave-uniform), for a hand-off inside one launch
template <bool WT = false>
__device__ __forceinline__ void quant4_store(float4 v, int c, int lane, int8_t* qrow, float* drow) {
    const float am = max8(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    const float dd = am / 127.f;
    int32_t w = 0;
    if (am != 0.f) {
        w = ((int)roundf(v.x / dd) & 0xff) | (((int)roundf(v.y / dd) & 0xff) << 8) |
            (((int)roundf(v.z / dd) & 0xff) << 16) | (((int)roundf(v.w / dd) & 0xff) << 24);
    }
    if constexpr (WT) {
        wt_st32(qrow, (uint32_t)c * 4u, w);
        if ((lane & 7) == 0) wt_stf(drow, (uint32_t)(c >> 3) * 4u, __half2float(f2h(dd)));
    } else {
        ((int32_t*)qrow)[c] = w;
        if ((lane & 7) == 0) drow[c >> 3] = __half2float(f2h(dd));
    }
}

// RMSNorm(x)·w of one row of H (H % 32 == 0, H ≤ 1024·KC) → Q8 (q [H], d [H/32]) by a whole 256-thread workgroup:
// thread t holds float4 chunks t, t+256, …; the sum of squares is reduced by wave shuffles, then across the four
// waves through part[4] (LDS).  Split in two so a caller can issue the row's loads before other memory traffic:
// rms_row_load (registers) then rms_row_q8_finish, which ends with every thread past one workgroup barrier (part may
// be reused only after another barrier).  Threads 256+ of a larger workgroup pass active = false (barrier only).
// WT: the row is read write-through (sc1: it was written by another workgroup of the same launch; xr wave-uniform)
// (tid < 0: threadIdx.x)
template <int KC, bool WT = false>
__device__ __forceinline__ void rms_row_load(const float* __restrict__ xr, int H, const float* __restrict__ w,
                                             float4 (&v)[KC], float4 (&gw)[KC], int tid_ = -1) {
    const int tid = tid_ < 0 ? (int)threadIdx.x : tid_, nc = H / 4;
    const float4* x4 = (const float4*)xr;
    const float4* g4 = (const float4*)w;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = tid + 256 * k;
        if constexpr (WT) v[k] = c < nc ? wt_ldf4(xr, (uint32_t)c * 16u) : make_float4(0.f, 0.f, 0.f, 0.f);
        else v[k] = c < nc ? x4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        gw[k] = c < nc ? g4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <int KC, bool WT = false>
__device__ __forceinline__ void rms_row_q8_finish(const float4 (&v)[KC], const float4 (&gw)[KC], int H, float eps,
                                                  int8_t* q, float* d, float* part, bool active = true,
                                                  int tid_ = -1) {
    const int tid = tid_ < 0 ? (int)threadIdx.x : tid_, lane = tid & 63, nc = H / 4;
    if (!active) {   // waves past the first four of a larger workgroup: only the barrier
        __syncthreads();
        return;
    }
    // separately rounded operations: a caller that runs several rows (k_gemv_wide's row groups) may have them packed
    // or fused differently by the compiler, and a one-ulp change of the sum can flip a Q8 rounding of the row.  (HIP's
    // __fmul_rn / __fadd_rn are the plain operators: the build's -ffp-contract=off is what keeps them unfused.)
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < KC; k++)
        ss = __fadd_rn(ss, __fadd_rn(__fadd_rn(__fmul_rn(v[k].x, v[k].x), __fmul_rn(v[k].y, v[k].y)),
                                     __fadd_rn(__fmul_rn(v[k].z, v[k].z), __fmul_rn(v[k].w, v[k].w))));
    ss = wave_sum(ss);
    if (lane == 0) part[tid >> 6] = ss;
    __syncthreads();
    ss = __fadd_rn(__fadd_rn(part[0], part[1]), __fadd_rn(part[2], part[3]));
    const float inv = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(__fdiv_rn(ss, (float)H), eps)));
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = tid + 256 * k;
        if (256 * k + (tid & ~7) < nc) {   // 8-thread blocks are all in or all out (nc % 8 == 0)
            const float4 g = gw[k];
            const float4 y = make_float4(__fmul_rn(__fmul_rn(v[k].x, inv), g.x), __fmul_rn(__fmul_rn(v[k].y, inv), g.y),
                                         __fmul_rn(__fmul_rn(v[k].z, inv), g.z), __fmul_rn(__fmul_rn(v[k].w, inv), g.w));
            quant4_store<WT>(y, c, lane, q, d);
        }
    }
}

template <int KC>
__device__ __forceinline__ void rms_row_q8_wg(const float* __restrict__ xr, int H, const float* __restrict__ w,
                                              float eps, int8_t* q, float* d, float* part) {
    float4 v[KC], gw[KC];
    rms_row_load<KC>(xr, H, w, v, gw);
    rms_row_q8_finish<KC>(v, gw, H, eps, q, d, part);
}

// SwiGLU of element j (0..31) of one h block from the block's 64 gate/up values in the interleaved layout
// ([g 16 | u 16 | g 16 | u 16]) → its Q8 value; one lane per element, a 32-lane group = one Q8 block (every lane of
// the group active).  Writes *q and, from the block's first lane, *d.
// the value form: element j's Q8 value, dq = the block's scale (f16-rounded)
__device__ __forceinline__ int swiglu_q8_value(const float* blk64, int j, float& dq) {
    const int c = j < 16 ? j : j + 16;
    const float g = blk64[c], u = blk64[c + 16];
    const float v = g / (1.f + expf(-g)) * u;
    float amax = fabsf(v);
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float dd = amax / 127.f;
    dq = __half2float(f2h(dd));
    return amax == 0.f ? 0 : (int)roundf(v / dd);
}
__device__ __forceinline__ void swiglu_q8_block(const float* blk64, int j, int8_t* q, float* d) {
    float dq;
    *q = (int8_t)swiglu_q8_value(blk64, j, dq);
    if (j == 0) *d = dq;
}

// SwiGLU of element f of a gate/up row (interleaved by 16, or [gate F | up F]) → q[f] / d[f/32]; as above
__device__ __forceinline__ void swiglu_lane_q8(const float* __restrict__ row, int F, int f, bool interleaved,
                                               int8_t* q, float* d) {
    const int b = f >> 5, j = f & 31;
    if (interleaved) {
        swiglu_q8_block(row + 64 * b, j, q + f, d + b);
        return;
    }
    const float g = row[f], u = row[F + f];
    const float v = g / (1.f + expf(-g)) * u;
    float amax = fabsf(v);
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float dd = amax / 127.f;
    q[f] = (int8_t)(amax == 0.f ? 0 : (int)roundf(v / dd));
    if (j == 0) d[b] = __half2float(f2h(dd));
}

}  // namespace qasr
