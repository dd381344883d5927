// Norm / activation / RoPE / reduction kernels for gfx950 (wave64).  Each fuses the Q8_0 activation
// quantisation that feeds the next W8A8 matmul, so an activation row is written once as int8+scale.
#include <algorithm>

#include "kernels.h"
#include "qk_rope.h"
#include "rowops.h"
#include "xlane.h"

namespace qasr {

__device__ __forceinline__ float wsum(float v) { return wave_sum(v); }

__device__ __forceinline__ void quant32(const float* v, int8_t* q, float* dout) {
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

__device__ __forceinline__ void load32(const float* p, float* v) {
    const float4* s = (const float4*)p;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        float4 t = s[j];
        v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
    }
}

// Row kernels: one wave per row, the row held in registers as float4 chunks (lane + 64·k), one HBM pass.  A Q8
// block is 8 consecutive lanes' chunks: its amax is three DPP steps, each lane packs its 4 int8 into one
// dword (coalesced stores), the block's first lane writes the scale.  Rows up to RW_MAX·256 elements.
constexpr int RW_MAX = 16;

template <int KC>
__global__ __launch_bounds__(256) void k_rmsnorm_q8(const float* __restrict__ x, int M, int H, int ldx,
                                                    const float* __restrict__ w, float eps, int8_t* __restrict__ q,
                                                    float* __restrict__ d) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int nc = H / 4;
    const float4* xr = (const float4*)(x + (size_t)row * ldx);
    const float4* g4 = (const float4*)w;
    // every load of the row and of the weights is issued before the first use (one memory round trip)
    float4 v[KC], gw[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = lane + 64 * k;
        v[k] = c < nc ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        gw[k] = c < nc ? g4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < KC; k++) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    ss = wsum(ss);
    const float inv = 1.0f / sqrtf(ss / (float)H + eps);
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = lane + 64 * k;
        if (64 * k < nc && c < nc) {   // 8-lane blocks are all in or all out (nc % 8 == 0)
            const float4 g = gw[k];
            const float4 y = make_float4(v[k].x * inv * g.x, v[k].y * inv * g.y, v[k].z * inv * g.z, v[k].w * inv * g.w);
            quant4_store(y, c, lane, q + (size_t)row * H, d + (size_t)row * (H / 32));
        }
    }
}

// One 256-thread workgroup per row (decode-sized launches have few rows: a wave per row leaves the chip idle and
// serialises 8 chunks of divisions and shuffles per lane).  Thread t holds float4 chunks t, t+256, …; the sum of
// squares is reduced by wave shuffles then across the four waves through LDS.
template <int KC>
__global__ __launch_bounds__(256) void k_rmsnorm_q8_wg(const float* __restrict__ x, int H, int ldx,
                                                       const float* __restrict__ w, float eps, int8_t* __restrict__ q,
                                                       float* __restrict__ d, float4* __restrict__ zero,
                                                       int64_t nzero4) {
    __shared__ float part[4];
    const int tid = threadIdx.x, row = blockIdx.x;
    // optional: clear the next split-K GEMM's output (saves a memset launch per layer)
    for (int64_t i = (int64_t)row * 256 + tid; i < nzero4; i += (int64_t)gridDim.x * 256)
        zero[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    rms_row_q8_wg<KC>(x + (size_t)row * ldx, H, w, eps, q + (size_t)row * H, d + (size_t)row * (H / 32), part);
}

void rmsnorm_q8(const float* x, int M, int H, int ldx, const float* w, float eps, int8_t* q, float* d, hipStream_t s,
                float* zero, int64_t nzero) {
    if (M <= 0) return;
    QASR_CHECK(H % 32 == 0 && H <= RW_MAX * 256 && ldx % 4 == 0, QASR_E_INVALID, "rmsnorm_q8: unsupported width");
    QASR_CHECK(nzero % 4 == 0 && ((uintptr_t)zero & 15) == 0, QASR_E_INVALID, "rmsnorm_q8: zero range alignment");
    const int kc = cdiv(H, 1024);   // float4 chunks per thread with a workgroup per row
    // a workgroup per row for every row count (round 4): the wave-per-row kernel below sums the squares in another
    // order, so a prefill of > 2,048 rows (a batch) rounded a row differently from the same row in a smaller one —
    // the batch-invariant contract needs one reduction order per row width
    if (kc <= 4) {
        float4* z = zero ? (float4*)zero : nullptr;
        const int64_t nz = zero ? nzero / 4 : 0;
        if (kc <= 1) k_rmsnorm_q8_wg<1><<<M, 256, 0, s>>>(x, H, ldx, w, eps, q, d, z, nz);
        else if (kc <= 2) k_rmsnorm_q8_wg<2><<<M, 256, 0, s>>>(x, H, ldx, w, eps, q, d, z, nz);
        else k_rmsnorm_q8_wg<4><<<M, 256, 0, s>>>(x, H, ldx, w, eps, q, d, z, nz);
        return;
    }
    if (zero && nzero) QASR_HIP(hipMemsetAsync(zero, 0, (size_t)nzero * sizeof(float), s));
    const int kcw = cdiv(H, 256);
    if (kcw <= 4)
        k_rmsnorm_q8<4><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, ldx, w, eps, q, d);
    else if (kcw <= 8)
        k_rmsnorm_q8<8><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, ldx, w, eps, q, d);
    else
        k_rmsnorm_q8<RW_MAX><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, ldx, w, eps, q, d);
}

// ------------------------------------------------------------------------------------------------ LayerNorm
template <int KC>
__global__ __launch_bounds__(256) void k_layernorm_q8(const float* __restrict__ x, int M, int H,
                                                      const float* __restrict__ w, const float* __restrict__ bb,
                                                      float eps, int8_t* __restrict__ q, float* __restrict__ d,
                                                      float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int nc = H / 4;
    const float4* xr = (const float4*)(x + (size_t)row * H);
    float4 v[KC];
    float s1 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = lane + 64 * k;
        v[k] = c < nc ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        s1 += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    const float mean = wsum(s1) / (float)H;
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        if (lane + 64 * k < nc) {
            const float a = v[k].x - mean, b = v[k].y - mean, c = v[k].z - mean, e = v[k].w - mean;
            s2 += a * a + b * b + c * c + e * e;
        }
    }
    const float inv = 1.0f / sqrtf(wsum(s2) / (float)H + eps);
    const float4* g4 = (const float4*)w;
    const float4* b4 = (const float4*)bb;
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int c = lane + 64 * k;
        if (64 * k >= nc) break;
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < nc) {
            const float4 g = g4[c], e = b4[c];
            o = make_float4((v[k].x - mean) * inv * g.x + e.x, (v[k].y - mean) * inv * g.y + e.y,
                            (v[k].z - mean) * inv * g.z + e.z, (v[k].w - mean) * inv * g.w + e.w);
            if (y) ((float4*)(y + (size_t)row * H))[c] = o;
        }
        if (q) {
            if (c < nc) quant4_store(o, c, lane, q + (size_t)row * H, d + (size_t)row * (H / 32));
            else max8(0.f);
        }
    }
}

void layernorm_q8(const float* x, int M, int H, const float* w, const float* b, float eps, int8_t* q, float* d,
                  float* y_opt, hipStream_t s) {
    if (M <= 0) return;
    QASR_CHECK(H % 32 == 0 && H <= RW_MAX * 256, QASR_E_INVALID, "layernorm_q8: unsupported width");
    const int kc = cdiv(H, 256);
    if (kc <= 4)
        k_layernorm_q8<4><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, w, b, eps, q, d, y_opt);
    else if (kc <= 8)
        k_layernorm_q8<8><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, w, b, eps, q, d, y_opt);
    else
        k_layernorm_q8<RW_MAX><<<cdiv(M, 4), 256, 0, s>>>(x, M, H, w, b, eps, q, d, y_opt);
}

// ------------------------------------------------------------------------------------------------ SwiGLU / GELU
__global__ void k_swiglu_q8(const float* __restrict__ gu, int M, int F, int8_t* __restrict__ q, float* __restrict__ d,
                            int interleaved) {
    const int nb = F / 32;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * nb) return;
    const int m = (int)(i / nb), b = (int)(i % nb);
    float g[32], u[32];
    const float* row = gu + (size_t)m * 2 * F;
    if (interleaved) {   // h columns 32b..32b+31 = [g 16 | u 16 | g 16 | u 16] at 64b
        float t[64];
        load32(row + 64 * b, t);
        load32(row + 64 * b + 32, t + 32);
#pragma unroll
        for (int j = 0; j < 16; j++) {
            g[j] = t[j], u[j] = t[16 + j], g[16 + j] = t[32 + j], u[16 + j] = t[48 + j];
        }
    } else {
        load32(row + b * 32, g);
        load32(row + F + b * 32, u);
    }
#pragma unroll
    for (int j = 0; j < 32; j++) g[j] = g[j] / (1.f + expf(-g[j])) * u[j];
    quant32(g, q + (size_t)m * F + b * 32, d + (size_t)m * nb + b);
}

// one lane per element (a Q8 block = 32 lanes, amax by xor-shuffles): the decode's few-row case, where one
// thread per block leaves the chip idle behind a 32-deep serial chain.  Same arithmetic as k_swiglu_q8 / quant32.
__global__ __launch_bounds__(256) void k_swiglu_q8_lane(const float* __restrict__ gu, int M, int F,
                                                        int8_t* __restrict__ q, float* __restrict__ d, int interleaved) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * F) return;     // F % 32 == 0: a 32-lane group never straddles the bound
    const int m = (int)(i / F), f = (int)(i % F);
    swiglu_lane_q8(gu + (size_t)m * 2 * F, F, f, interleaved != 0, q + (size_t)m * F, d + (size_t)m * (F / 32));
}

void swiglu_q8(const float* gu, int M, int F, int8_t* q, float* d, hipStream_t s, bool interleaved) {
    int64_t n = (int64_t)M * (F / 32);
    if (n <= 0) return;
    if (M <= 64)   // (the verify passes' ≤ 32 rows included: one lane per element, no 32-deep serial chain)
        k_swiglu_q8_lane<<<(unsigned)cdiv64(n * 32, 256), 256, 0, s>>>(gu, M, F, q, d, interleaved ? 1 : 0);
    else
        k_swiglu_q8<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(gu, M, F, q, d, interleaved ? 1 : 0);
}

__global__ void k_gelu_q8(const float* __restrict__ x, int M, int K, int8_t* __restrict__ q, float* __restrict__ d) {
    const int nb = K / 32;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * nb) return;
    const int m = (int)(i / nb), b = (int)(i % nb);
    float v[32];
    load32(x + (size_t)m * K + b * 32, v);
#pragma unroll
    for (int j = 0; j < 32; j++) v[j] = 0.5f * v[j] * (1.f + erff(v[j] * 0.70710678118654752f));
    quant32(v, q + (size_t)m * K + b * 32, d + (size_t)m * nb + b);
}

void gelu_q8(const float* x, int M, int K, int8_t* q, float* d, hipStream_t s) {
    int64_t n = (int64_t)M * (K / 32);
    if (n <= 0) return;
    k_gelu_q8<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(x, M, K, q, d);
}

// ------------------------------------------------------------------------------------------------ q/k norm + RoPE
// one wave per (row, head slot); slots [0,nh) = q heads, [nh,nh+nkv) = k heads, [nh+nkv, nh+2nkv) = v heads.
// hd = 128 (2 dims per lane) or 64 (1 dim per lane); the RoPE partner of lane l is lane l^32.
template <int HD>
__global__ __launch_bounds__(256) void k_qk_norm_rope(const float* __restrict__ qkv, int rows, int nh, int nkv,
                                                      const int* __restrict__ pos, const int* __restrict__ slot,
                                                      const float* __restrict__ qnw, const float* __restrict__ knw,
                                                      const float* __restrict__ rope_cs, float eps,
                                                      __half* __restrict__ qout, __half* __restrict__ kc,
                                                      __half* __restrict__ vc) {
    constexpr int DPL = HD / 64;
    const int lane = threadIdx.x & 63;
    const int nslot = nh + 2 * nkv;
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= rows * nslot) return;
    const int r = g / nslot, h = g % nslot;
    const int ld = nslot * HD;
    const float* src = qkv + (size_t)r * ld + h * HD;
    // issue the independent loads first: row data, position, slot, norm weights, then the RoPE pair
    const int p = pos[r], sl = slot[r];
    float v[DPL], nwv[DPL];
    const float* nw = h < nh ? qnw : knw;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
        v[j] = src[lane * DPL + j];
        nwv[j] = nw[lane * DPL + j];
    }
    const int half = HD / 2;
    float cs[DPL], sn[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) {
        const int dim = lane * DPL + j;
        const int e = dim < half ? dim : dim - half;
        const float2 t = *(const float2*)(rope_cs + ((size_t)p * half + e) * 2);
        cs[j] = t.x;
        sn[j] = t.y;
    }
    const int kvd = nkv * HD;
    if (h >= nh + nkv) {  // v head: copy to cache
        __half* dst = vc + (size_t)sl * kvd + (h - nh - nkv) * HD;
#pragma unroll
        for (int j = 0; j < DPL; j++) dst[lane * DPL + j] = f2h(v[j]);
        return;
    }
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < DPL; j++) ss += v[j] * v[j];
    ss = wsum(ss);
    const float inv = 1.0f / sqrtf(ss / (float)HD + eps);
#pragma unroll
    for (int j = 0; j < DPL; j++) v[j] = v[j] * inv * nwv[j];
    float o[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) {
        const float partner = __shfl_xor(v[j], 32);
        const int dim = lane * DPL + j;
        o[j] = dim < half ? v[j] * cs[j] - partner * sn[j] : v[j] * cs[j] + partner * sn[j];
    }
    if (h < nh) {
        __half* dst = qout + (size_t)r * nh * HD + h * HD;
#pragma unroll
        for (int j = 0; j < DPL; j++) dst[lane * DPL + j] = f2h(o[j]);
    } else {
        __half* dst = kc + (size_t)sl * kvd + (h - nh) * HD;
#pragma unroll
        for (int j = 0; j < DPL; j++) dst[lane * DPL + j] = f2h(o[j]);
    }
}

// Row-per-workgroup form (hd = 128): the row's position, slot and RoPE factors are loaded once per wave and
// reused for every head the wave takes (heads w, w+4, …); all head loads are issued before the first use, 8-byte
// loads and 4-byte f16 stores per lane.
template <int NHW>
__global__ __launch_bounds__(256) void k_qk_norm_rope_row(const float* __restrict__ qkv, int nh, int nkv,
                                                          const int* __restrict__ pos, const int* __restrict__ slot,
                                                          const float* __restrict__ qnw, const float* __restrict__ knw,
                                                          const float* __restrict__ rope_cs, float eps,
                                                          __half* __restrict__ qout, __half* __restrict__ kc,
                                                          __half* __restrict__ vc) {
    constexpr int HD = 128, half = 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = blockIdx.x;
    const int nslot = nh + 2 * nkv, ld = nslot * HD, kvd = nkv * HD;
    const float* src = qkv + (size_t)r * ld;
    float2 v[NHW];
#pragma unroll
    for (int t = 0; t < NHW; t++) {
        const int h = w + 4 * t;
        v[t] = h < nslot ? *(const float2*)(src + h * HD + 2 * lane) : make_float2(0.f, 0.f);
    }
    const float2 qw = *(const float2*)(qnw + 2 * lane), kw = *(const float2*)(knw + 2 * lane);
    const int p = pos[r], sl = slot[r];
    // dims 2·lane, 2·lane+1: RoPE pair index e = dim mod 64, partner lane = lane ^ 32
    const int e0 = (2 * lane) & (half - 1);
    const float4 cs = *(const float4*)(rope_cs + ((size_t)p * half + e0) * 2);   // (cos, sin) of e0, e0+1
    const bool lo = 2 * lane < half;
#pragma unroll
    for (int t = 0; t < NHW; t++) {
        const int h = w + 4 * t;
        if (h >= nslot) break;
        if (h >= nh + nkv) {   // v head: copy into its cache slot
            *(__half2*)(vc + (size_t)sl * kvd + (h - nh - nkv) * HD + 2 * lane) = __floats2half2_rn(v[t].x, v[t].y);
            continue;
        }
        __half* dst = h < nh ? qout + (size_t)r * nh * HD + h * HD : kc + (size_t)sl * kvd + (h - nh) * HD;
        *(__half2*)(dst + 2 * lane) = norm_rope_hd128(v[t], h < nh ? qw : kw, cs, lo, eps);
    }
}

void qk_norm_rope(const float* qkv, int rows, int nh, int nkv, int hd, const int* pos, const int* slot,
                  const float* qnw, const float* knw, const float* rope_cs, float eps, __half* qout, __half* kc,
                  __half* vc, hipStream_t s) {
    if (rows <= 0) return;
    const int nslot = nh + 2 * nkv;
    if (hd == 128 && nslot <= 32) {
        k_qk_norm_rope_row<8><<<rows, 256, 0, s>>>(qkv, nh, nkv, pos, slot, qnw, knw, rope_cs, eps, qout, kc, vc);
        return;
    }
    const int waves = rows * nslot;
    if (hd == 128)
        k_qk_norm_rope<128><<<cdiv(waves, 4), 256, 0, s>>>(qkv, rows, nh, nkv, pos, slot, qnw, knw, rope_cs, eps, qout, kc, vc);
    else if (hd == 64)
        k_qk_norm_rope<64><<<cdiv(waves, 4), 256, 0, s>>>(qkv, rows, nh, nkv, pos, slot, qnw, knw, rope_cs, eps, qout, kc, vc);
    else
        throw Error(QASR_E_INVALID, "qk_norm_rope: head_dim must be 64 or 128");
}

// ------------------------------------------------------------------------------------------------ misc
__global__ void k_to_f16(const float* __restrict__ x, int rows, int cols, int ldx, __half* __restrict__ y, int ldy) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)rows * cols) return;
    const int r = (int)(i / cols), c = (int)(i % cols);
    y[(size_t)r * ldy + c] = f2h(x[(size_t)r * ldx + c]);
}

void to_f16(const float* x, int rows, int cols, int ldx, __half* y, int ldy, hipStream_t s) {
    int64_t n = (int64_t)rows * cols;
    if (n <= 0) return;
    k_to_f16<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(x, rows, cols, ldx, y, ldy);
}

// first index of the maximum (ties → lowest index, like the oracle's strict '>' scan)
__global__ __launch_bounds__(256) void k_argmax(const float* __restrict__ x, int V, int* __restrict__ out) {
    const float* r = x + (size_t)blockIdx.x * V;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < V; i += 256) {
        float v = r[i];
        if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float ov = __shfl_xor(best, o);
        int oi = __shfl_xor(bi, o);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    __shared__ float sv[4];
    __shared__ int si[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sv[w] = best; si[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 1; j < 4; j++)
            if (sv[j] > best || (sv[j] == best && si[j] < bi)) { best = sv[j]; bi = si[j]; }
        out[blockIdx.x] = bi;
    }
}

// two-stage argmax: ARG_P workgroups per row each reduce a slice to one 64-bit key (order-preserving float bits
// high, inverted index low, so the maximum key is the largest value at the lowest index), then one wave per row
constexpr int ARG_P = kArgParts;

__device__ __forceinline__ unsigned long long argkey(float v, int i) {
    unsigned u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
    const unsigned lo = __shfl_xor((unsigned)v, o), hi = __shfl_xor((unsigned)(v >> 32), o);
    return ((unsigned long long)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void k_argmax_part(const float* __restrict__ x, int V, int L,
                                                     unsigned long long* __restrict__ part) {
    const float* r = x + (size_t)blockIdx.y * V;
    const int lo = blockIdx.x * L, hi = min(V, lo + L);
    unsigned long long best = 0;
    if ((V & 3) == 0) {
        for (int i = lo + 4 * threadIdx.x; i < hi; i += 4 * 256) {
            const float4 v = *(const float4*)(r + i);
            best = max(best, argkey(v.x, i));
            best = max(best, argkey(v.y, i + 1));
            best = max(best, argkey(v.z, i + 2));
            best = max(best, argkey(v.w, i + 3));
        }
    } else {
        for (int i = lo + threadIdx.x; i < hi; i += 256) best = max(best, argkey(r[i], i));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = max(best, shfl_xor_u64(best, o));
    __shared__ unsigned long long sk[4];
    if ((threadIdx.x & 63) == 0) sk[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0)
        part[(size_t)blockIdx.y * ARG_P + blockIdx.x] = max(max(sk[0], sk[1]), max(sk[2], sk[3]));
}

__global__ __launch_bounds__(64) void k_argmax_final(const unsigned long long* __restrict__ part, int* __restrict__ out) {
    unsigned long long k = threadIdx.x < ARG_P ? part[(size_t)blockIdx.x * ARG_P + threadIdx.x] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k = max(k, shfl_xor_u64(k, o));
    if (threadIdx.x == 0) out[blockIdx.x] = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
}

size_t argmax_scratch_bytes(int M) { return (size_t)std::max(M, 1) * ARG_P * sizeof(unsigned long long); }

void argmax_rows_partial(const float* x, int M, int V, void* scratch, hipStream_t s) {
    if (M <= 0) return;
    const int L = ((cdiv(V, ARG_P) + 3) / 4) * 4;
    k_argmax_part<<<dim3(ARG_P, M), 256, 0, s>>>(x, V, L, (unsigned long long*)scratch);
}

void argmax_rows(const float* x, int M, int V, int* out, hipStream_t s, void* scratch) {
    if (M <= 0) return;
    if (!scratch) {
        k_argmax<<<M, 256, 0, s>>>(x, V, out);
        return;
    }
    const int L = ((cdiv(V, ARG_P) + 3) / 4) * 4;
    k_argmax_part<<<dim3(ARG_P, M), 256, 0, s>>>(x, V, L, (unsigned long long*)scratch);
    k_argmax_final<<<M, 64, 0, s>>>((const unsigned long long*)scratch, out);
}

// audio encoder: gather the valid post-CNN positions of every chunk and add the sinusoid embedding
__global__ void k_posemb_gather(const float* __restrict__ proj, int T, int d, const float* __restrict__ pe,
                                const int* __restrict__ valid_idx, int n_out, float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_out * d) return;
    const int r = (int)(i / d), c = (int)(i % d);
    const int src = valid_idx[r];
    out[i] = proj[(size_t)src * d + c] + pe[(size_t)(src % T) * d + c];
}

void add_posemb_gather(const float* proj, int n_chunks, int T, int d, const float* pe, const int* valid_idx,
                       int n_out, float* out, hipStream_t s) {
    (void)n_chunks;
    int64_t n = (int64_t)n_out * d;
    if (n <= 0) return;
    k_posemb_gather<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(proj, T, d, pe, valid_idx, n_out, out);
}

}  // namespace qasr
