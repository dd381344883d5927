// Variable-length attention over f16 K/V (decoder KV cache slots or encoder window buffers), gfx950.
//
// One wave per (query row, KV head), the G = n_heads/n_kv_heads query heads of the group sharing every K/V load.  Keys are processed in LDS-resident chunks of 256 with an online softmax
// (running max / sum, f32).  QKᵀ: 8 lanes per key (16-dim slices, 3 xor-shuffles), 32 keys per unrolled
// iteration so eight 16-byte K loads per lane are in flight together.  PV: each lane owns hd/64 dims and
// walks the keys 8 at a time with eight independent 4-byte V loads in flight (each V row is one coalesced
// 256-byte segment).  Row r attends slots [kv_start[r], kv_start[r]+kv_len[r]) — causal prefill, single-token
// decode and the encoder's bidirectional 104-token windows (modeling_qwen3_asr.py:276-315) are all expressed
// by the per-row ranges.  The output is written as f32 and/or directly as Q8 blocks for the O-projection.
#include <type_traits>

#include "kernels.h"

namespace qasr {

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wsum_a(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int QD>
__device__ __forceinline__ float qk_dot(const float* qv, const __half* kr) {
    float part = 0.f;
    if constexpr (QD == 16) {
        const int4 a = *(const int4*)kr, b = *(const int4*)(kr + 8);
        const __half2* ha = (const __half2*)&a;
        const __half2* hb = (const __half2*)&b;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const float2 fa = __half22float2(ha[t]), fb = __half22float2(hb[t]);
            part += qv[2 * t] * fa.x + qv[2 * t + 1] * fa.y;
            part += qv[8 + 2 * t] * fb.x + qv[8 + 2 * t + 1] * fb.y;
        }
    } else {
        const int4 a = *(const int4*)kr;
        const __half2* ha = (const __half2*)&a;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const float2 fa = __half22float2(ha[t]);
            part += qv[2 * t] * fa.x + qv[2 * t + 1] * fa.y;
        }
    }
    return part;
}

template <int HD, int G, int NW>
__global__ __launch_bounds__(256) void k_attention(const __half* __restrict__ Q, int ldq, const __half* __restrict__ K,
                                                   const __half* __restrict__ V, int ldkv,
                                                   const int* __restrict__ kv_start, const int* __restrict__ kv_len,
                                                   int rows, int nh, int nkv, float scale, float* __restrict__ o,
                                                   int8_t* __restrict__ oq, float* __restrict__ od) {
    constexpr int CH = 256;
    constexpr int QD = HD / 8;    // dims per lane in QKᵀ
    constexpr int PD = HD / 64;   // dims per lane in PV / output
    constexpr int KU = 4;         // 8-key groups per QKᵀ iteration
    constexpr int VU = 8;         // keys per PV iteration
    __shared__ float sp[4][G][CH];
    __shared__ float cm_s[4][G], cl_s[4][G];
    __shared__ float ca_s[4][G][HD];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // NW = 4: one workgroup per (row, KV head), its 4 waves take contiguous quarters of the key range and merge
    // their partial softmax states through LDS (long decoder KV ranges).  NW = 1: one wave per (row, KV head)
    // (the encoder's 104-key windows).  The G query heads of a KV group share every K/V load.
    const int gw = NW == 4 ? blockIdx.x : blockIdx.x * 4 + w;
    if (NW == 1 && gw >= rows * nkv) return;
    const int part = NW == 4 ? w : 0;
    const int r = gw / nkv, kvh = gw % nkv;
    const int Lr = kv_len[r], qn = (Lr + NW - 1) / NW;
    const int s0 = kv_start[r] + part * qn, L = max(0, min(qn, Lr - part * qn));
    const int sub = lane & 7, kk = lane >> 3;

    float qv[G][QD];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const __half* qp = Q + (size_t)r * ldq + (kvh * G + g) * HD + sub * QD;
#pragma unroll
        for (int j = 0; j < QD; j++) qv[g][j] = __half2float(qp[j]);
    }
    float acc[G][PD];
    float m[G], lsum[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
        m[g] = -INFINITY;
        lsum[g] = 0.f;
#pragma unroll
        for (int j = 0; j < PD; j++) acc[g][j] = 0.f;
    }
    const __half* kbase = K + (size_t)kvh * HD + sub * QD;
    const __half* vbase = V + (size_t)kvh * HD + lane * PD;

    for (int c0 = 0; c0 < L; c0 += CH) {
        const int n = min(CH, L - c0);
        const __half* kc = kbase + (size_t)(s0 + c0) * ldkv;
        const __half* vb = vbase + (size_t)(s0 + c0) * ldkv;
        for (int j0 = 0; j0 < n; j0 += 8 * KU) {
            float part[KU][G];
#pragma unroll
            for (int u = 0; u < KU; u++) {
                const int j = j0 + u * 8 + kk;
                if (j < n) {
                    const __half* kr = kc + (size_t)j * ldkv;
#pragma unroll
                    for (int g = 0; g < G; g++) part[u][g] = qk_dot<QD>(qv[g], kr);
                } else {
#pragma unroll
                    for (int g = 0; g < G; g++) part[u][g] = 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < KU; u++) {
                const int j = j0 + u * 8 + kk;
#pragma unroll
                for (int g = 0; g < G; g++) {
                    float p = part[u][g];
                    p += __shfl_xor(p, 1);
                    p += __shfl_xor(p, 2);
                    p += __shfl_xor(p, 4);
                    if (sub == 0 && j < n) sp[w][g][j] = p * scale;
                }
            }
        }
        wave_sync_lds();
#pragma unroll
        for (int g = 0; g < G; g++) {
            float* spw = sp[w][g];
            float cm = -INFINITY;
            for (int i = lane; i < n; i += 64) cm = fmaxf(cm, spw[i]);
            cm = wmax(cm);
            const float mnew = fmaxf(m[g], cm);
            const float alpha = expf(m[g] - mnew);
#pragma unroll
            for (int j = 0; j < PD; j++) acc[g][j] *= alpha;
            float ps = 0.f;
            for (int i = lane; i < n; i += 64) {
                const float p = expf(spw[i] - mnew);
                spw[i] = p;
                ps += p;
            }
            lsum[g] = lsum[g] * alpha + wsum_a(ps);
            m[g] = mnew;
        }
        wave_sync_lds();
        int j = 0;
        for (; j + VU <= n; j += VU) {
            if constexpr (PD == 2) {
                __half2 vv[VU];
#pragma unroll
                for (int u = 0; u < VU; u++) vv[u] = *(const __half2*)(vb + (size_t)(j + u) * ldkv);
#pragma unroll
                for (int u = 0; u < VU; u++) {
                    const float2 f = __half22float2(vv[u]);
#pragma unroll
                    for (int g = 0; g < G; g++) {
                        const float p = sp[w][g][j + u];
                        acc[g][0] += p * f.x;
                        acc[g][1] += p * f.y;
                    }
                }
            } else {
                __half vv[VU];
#pragma unroll
                for (int u = 0; u < VU; u++) vv[u] = vb[(size_t)(j + u) * ldkv];
#pragma unroll
                for (int u = 0; u < VU; u++) {
                    const float f = __half2float(vv[u]);
#pragma unroll
                    for (int g = 0; g < G; g++) acc[g][0] += sp[w][g][j + u] * f;
                }
            }
        }
        for (; j < n; j++) {
            if constexpr (PD == 2) {
                const float2 f = __half22float2(*(const __half2*)(vb + (size_t)j * ldkv));
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const float p = sp[w][g][j];
                    acc[g][0] += p * f.x;
                    acc[g][1] += p * f.y;
                }
            } else {
                const float f = __half2float(vb[(size_t)j * ldkv]);
#pragma unroll
                for (int g = 0; g < G; g++) acc[g][0] += sp[w][g][j] * f;
            }
        }
        wave_sync_lds();
    }
    // merge the NW partial states (m, l, acc) of this row's key ranges
    if constexpr (NW == 1) {
#pragma unroll
        for (int g = 0; g < G; g++) {
            if (lane == 0) {
                cm_s[w][g] = m[g];
                cl_s[w][g] = lsum[g];
            }
#pragma unroll
            for (int j = 0; j < PD; j++) ca_s[w][g][lane * PD + j] = acc[g][j];
        }
        wave_sync_lds();
    } else {
#pragma unroll
        for (int g = 0; g < G; g++) {
            if (lane == 0) {
                cm_s[w][g] = m[g];
                cl_s[w][g] = lsum[g];
            }
#pragma unroll
            for (int j = 0; j < PD; j++) ca_s[w][g][lane * PD + j] = acc[g][j];
        }
        __syncthreads();
        if (w != 0) return;
    }
    const int wb = NW == 1 ? w : 0;   // first partial state of this item
    const int D = nh * HD;
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int h = kvh * G + g;
        float mt = -INFINITY;
#pragma unroll
        for (int u = 0; u < NW; u++) mt = fmaxf(mt, cm_s[wb + u][g]);
        float lt = 0.f, sc[NW];
#pragma unroll
        for (int u = 0; u < NW; u++) {
            sc[u] = cm_s[wb + u][g] == -INFINITY ? 0.f : expf(cm_s[wb + u][g] - mt);
            lt += cl_s[wb + u][g] * sc[u];
        }
        const float inv = Lr > 0 ? 1.f / lt : 0.f;
        float out[PD];
#pragma unroll
        for (int j = 0; j < PD; j++) {
            float a = 0.f;
#pragma unroll
            for (int u = 0; u < NW; u++) a += ca_s[wb + u][g][lane * PD + j] * sc[u];
            out[j] = a * inv;
        }
        if (o) {
#pragma unroll
            for (int j = 0; j < PD; j++) o[(size_t)r * D + h * HD + lane * PD + j] = out[j];
        }
        if (oq) {
            // a 32-dim block spans 32/PD lanes
            float amax = 0.f;
#pragma unroll
            for (int j = 0; j < PD; j++) amax = fmaxf(amax, fabsf(out[j]));
#pragma unroll
            for (int off = 1; off < 32 / PD; off <<= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
            const float d = amax / 127.f;
#pragma unroll
            for (int j = 0; j < PD; j++) {
                const int qv2 = amax == 0.f ? 0 : (int)roundf(out[j] / d);
                oq[(size_t)r * D + h * HD + lane * PD + j] = (int8_t)qv2;
            }
            if ((lane & (32 / PD - 1)) == 0)
                od[(size_t)r * (D / 32) + (h * HD + lane * PD) / 32] = __half2float(f2h(d));
        }
    }
}

template <int HD>
static void launch_attention(int G, int rows, hipStream_t s, const __half* Q, int ldq, const __half* K,
                             const __half* V, int ldkv, const int* kv_start, const int* kv_len, int nh, int nkv,
                             float scale, float* o, int8_t* oq, float* od) {
    const unsigned b4 = (unsigned)(rows * nkv), b1 = (unsigned)cdiv(rows * nkv, 4);
    switch (G) {
        case 1: k_attention<HD, 1, 1><<<b1, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o, oq, od); break;
        case 2: k_attention<HD, 2, 4><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o, oq, od); break;
        case 4: k_attention<HD, 4, 4><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o, oq, od); break;
        default: throw Error(QASR_E_INVALID, "attention: query heads per KV head must be 1, 2 or 4");
    }
}

void attention(const __half* Q, int ldq, const __half* K, const __half* V, int ldkv, const int* kv_start,
               const int* kv_len, int rows, int nh, int nkv, int hd, float scale, float* o, int8_t* oq, float* od,
               hipStream_t s, int64_t total_keys) {
    if (rows <= 0) return;
    // QKᵀ + PV: 4·hd flops per (query head, key); f16 K/V bytes read per (query head, key)
    ProfScope ps(s, "attention", 4.0 * hd * nh * (double)total_keys, 4.0 * hd * nh * (double)total_keys);
    QASR_CHECK(nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "attention: bad head counts");
    const int G = nh / nkv;
    if (hd == 128)
        launch_attention<128>(G, rows, s, Q, ldq, K, V, ldkv, kv_start, kv_len, nh, nkv, scale, o, oq, od);
    else if (hd == 64)
        launch_attention<64>(G, rows, s, Q, ldq, K, V, ldkv, kv_start, kv_len, nh, nkv, scale, o, oq, od);
    else
        throw Error(QASR_E_INVALID, "attention: head_dim must be 64 or 128");
}

}  // namespace qasr
