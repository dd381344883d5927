// The exact-row linear's fragment body: one 16-column fragment of W·Xᵀ for up to 16·RF rows with EXACTLY the
// arithmetic of k_gemv_wide's 1-row launch (the exact-row contract, engine.cpp), shared by the k_gemm_q8_exact
// launches (kernels_q8.hip) and the per-phase xr launches (kernels_xr.hip) — one definition, so both give the
// same bits.
//
// The GEMV's result for output (m, n), K = 1024·T, is: lane ℓ = 2l (l = 0…31) accumulates the blocks b = l + 32t in t
// order, leaf_l = fma((float)Σ_b q·q, d_w[n][b]·d_x[m][b], leaf_l) from 0, the odd lanes hold 0, and wave_sum's DPP
// tree adds them as ((H0 + H1) + (H2 + H3)), H_h = O_2h + O_2h+1, O_g = ((l'_4g + l'_4g+1) + (l'_4g+2 + l'_4g+3)), l'
// = leaf + 0 (the xor-1 step's add of an odd lane's 0: -0 → +0).  Here the four waves of a 256-thread workgroup own
// leaves 8w … 8w+7 (blocks 8w + 2j + {0,1} + 32t: spans 4w + j + 16t); the exact int32 block sums come from
// v_mfma_i32_16x16x64_i8 on 64-byte spans (the weight span masked to lane groups 0–1 / 2–3 gives blocks 2s / 2s+1),
// each lane keeps the 8 leaves of its 4 outputs per row fragment in registers, and the same fma chains and the same
// tree run in-lane and across the waves through LDS — the same bits, whatever the row count.  Rows past M are computed
// on clamped inputs and must not be stored by the caller.
#pragma once
#include "kernels.h"

#ifndef QASR_XR_FENCE
#define QASR_XR_FENCE 2
#endif
#include "wt.h"

namespace qasr {

typedef int xr_v4i __attribute__((ext_vector_type(4)));

enum ExactSrc : int {
    XS_PLAIN = 0,   // X / Xd in global memory, plain loads
    XS_WT = 1,      // X / Xd handed over inside one launch: sc1 buffer loads (wt.h; X / Xd wave-uniform bases)
};

// Lane (fr = lane & 15, g = lane >> 4) of wave w < RF ends with out[r] = the output of row 16w + 4g + r, column
// n0 + fr (waves ≥ RF: undefined).  hx: the workgroup's LDS exchange, [4 waves][RF][4][64] floats.  Every thread of
// the workgroup must call it (one barrier inside); hx may be reused after the caller's next barrier.
template <int T, int RF, int SRC>
__device__ __forceinline__ void exact_frag(const int8_t* __restrict__ X, const float* __restrict__ Xd, int M,
                                           const int8_t* __restrict__ W, const __half* __restrict__ Wsc, int N, int K,
                                           int n0, float (*hx)[RF][4][64], float (&out)[4]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int fr = lane & 15, g = lane >> 4;
    const int nb = K / QK;
    const int8_t* wp = W + (size_t)min(n0 + fr, N - 1) * K + 16 * g;
    const uint32_t* sp = (const uint32_t*)(Wsc + (size_t)min(n0 + fr, N - 1) * nb);
    uint32_t aoff[RF];        // byte offset of row fr of fragment f, lane group g
    uint32_t doff[RF][4];     // byte offset of the block scales of row 4g + r of fragment f
#pragma unroll
    for (int f = 0; f < RF; f++) {
        aoff[f] = (uint32_t)(min(16 * f + fr, M - 1) * K + 16 * g);
#pragma unroll
        for (int r = 0; r < 4; r++) doff[f][r] = (uint32_t)(min(16 * f + 4 * g + r, M - 1) * nb) * 4u;
    }
    constexpr int NS = 4 * T;                            // spans of this wave
    constexpr int G8 = RF == 1 && NS % 8 == 0 ? 8 : 4;   // spans loaded per group
    float leaf[RF][8][4];
#pragma unroll
    for (int f = 0; f < RF; f++)
#pragma unroll
        for (int l = 0; l < 8; l++)
#pragma unroll
            for (int r = 0; r < 4; r++) leaf[f][l][r] = 0.f;   // (the chains start at t = 0 from 0.f either way)
    const bool lo = g < 2;
    const xr_v4i zero = {0, 0, 0, 0};
#pragma unroll
    for (int q0 = 0; q0 < NS; q0 += G8) {
        xr_v4i wq[G8], aq[G8][RF];
        uint32_t ws[G8];
        float2 dx[G8][RF][4];
#pragma unroll
        for (int u = 0; u < G8; u++) {
            const int i = q0 + u, s = 4 * wv + (i & 3) + 16 * (i >> 2);
            wq[u] = __builtin_nontemporal_load((const xr_v4i*)(wp + 64 * (size_t)s));
            ws[u] = sp[s];
#pragma unroll
            for (int f = 0; f < RF; f++) {
                if constexpr (SRC == XS_WT) {
                    aq[u][f] = wt_ld16(X, aoff[f] + 64u * (uint32_t)s);
#pragma unroll
                    for (int r = 0; r < 4; r++) dx[u][f][r] = wt_ldf2(Xd, doff[f][r] + 8u * (uint32_t)s);
                } else {
                    aq[u][f] = *(const xr_v4i*)(X + aoff[f] + 64 * (size_t)s);
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        dx[u][f][r] = *(const float2*)((const char*)Xd + doff[f][r] + 8 * (size_t)s);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < G8; u++) {
            const int i = q0 + u, j = i & 3, t = i >> 2;   // blocks 8w + 2j + h + 32t → leaves 2j + h (of this wave)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const xr_v4i bm = (lo == (h == 0)) ? wq[u] : zero;
                const float dw = __half2float(__ushort_as_half((unsigned short)(h ? ws[u] >> 16 : ws[u] & 0xffff)));
                const int l = 2 * j + h;
#pragma unroll
                for (int f = 0; f < RF; f++) {
                    const xr_v4i c = __builtin_amdgcn_mfma_i32_16x16x64_i8(aq[u][f], bm, zero, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float dxr = h ? dx[u][f][r].y : dx[u][f][r].x;
                        leaf[f][l][r] = fmaf((float)c[r], dw * dxr, t == 0 ? 0.f : leaf[f][l][r]);
                    }
                }
            }
        }
    }
    // this wave's leaves l' = leaf + 0 (the GEMV's xor-1 add of an odd lane's 0), O_2w, O_2w+1, H_w
#pragma unroll
    for (int f = 0; f < RF; f++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float o[2];
#pragma unroll
            for (int gq = 0; gq < 2; gq++) {
                const float a0 = leaf[f][4 * gq][r] + 0.f, a1 = leaf[f][4 * gq + 1][r] + 0.f;
                const float a2 = leaf[f][4 * gq + 2][r] + 0.f, a3 = leaf[f][4 * gq + 3][r] + 0.f;
                o[gq] = (a0 + a1) + (a2 + a3);
            }
            hx[wv][f][r][lane] = o[0] + o[1];
        }
    __syncthreads();
    if (wv < RF) {
        const int f = wv;   // wave f finishes row fragment f
#pragma unroll
        for (int r = 0; r < 4; r++)
            out[r] = (hx[0][f][r][lane] + hx[1][f][r][lane]) + (hx[2][f][r][lane] + hx[3][f][r][lane]);
    }
}

// ---- the xr launches' form: weights held in registers (loaded at the workgroup's start), activations from an
// LDS tile (staged once per phase).  Same lanes, spans, chains and tree as exact_frag: the same bits.

// row stride (floats) of the LDS tile's block scales (exact_frag_lds below)
__host__ __device__ constexpr int xr_sd_stride(int K) { return K / 32 + 4; }

// one wave's weight spans of a 16-column fragment: spans 4w + j + 16t, i = 4t + j (NS = 4T).  XS = 2 (the leaf split
// of the per-phase launches): the fragment's 32 leaves are shared by TWO workgroups, half h taking leaves 16h … 16h+15
// (wave w: leaves 16h + 4w … +3 = O_{4h+w}; spans 8h + 2w + j + 16t, i = 2t + j, NS = 2T); each half's workgroup
// tree gives H_{2h} + H_{2h+1}, and the two halves are added in half order — ((H0 + H1) + (H2 + H3)), the same bits.
template <int T, int XS = 1>
struct XWeights {
    xr_v4i wq[4 * T / XS];
    uint32_t ws[4 * T / XS];
};
template <int XS>
__device__ __forceinline__ int xr_span(int i, int wv, int half) {
    return XS == 1 ? 4 * wv + (i & 3) + 16 * (i >> 2) : 8 * half + 2 * wv + (i & 1) + 16 * (i >> 1);
}

// tid: the thread index
// spans [I0, I1) only (a caller that loads a matrix in two parts, e.g. half ahead of a grid wait)
template <int T, int I0 = 0, int I1 = 4 * T, int XS = 1>
__device__ __forceinline__ void exact_load_w(XWeights<T, XS>& w, const int8_t* __restrict__ W,
                                             const __half* __restrict__ Wsc, int N, int K, int n0, int tid,
                                             int half = 0) {
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, g = lane >> 4;
    const int nb = K / QK;
    const int8_t* wp = W + (size_t)min(n0 + fr, N - 1) * K + 16 * g;
    const uint32_t* sp = (const uint32_t*)(Wsc + (size_t)min(n0 + fr, N - 1) * nb);
#pragma unroll
    for (int i = I0; i < I1; i++) {
        const int s = xr_span<XS>(i, wv, half);
        w.wq[i] = __builtin_nontemporal_load((const xr_v4i*)(wp + 64 * (size_t)s));
        w.ws[i] = sp[s];
    }
}

// sX: the tile's int8 rows (row stride ldx bytes, 16-B aligned, ldx ≡ 16 mod 256 so the 16 rows of a fragment read
// conflict-free), sXd: its f32 block scales (row stride xr_sd_stride(K) = K/32 + 4 floats: the four lane groups of a
// span's scale read fetch rows 4g + r, which at the unpadded stride (a multiple of 32 floats) sat in one bank — a
// 4-way conflict on every read, round 6 PMC 2.3–2.8 conflict cycles per LDS instruction in the xr launches; with 4
// floats of padding the rows start 16 banks apart and 16-B aligned); rows [0, M) valid (later rows clamped to M − 1)
// XS = 2: this workgroup's half of the leaves (XWeights above); out = H_{2h} + H_{2h+1} of half h
template <int T, int RF, int XS = 1>
__device__ __forceinline__ void exact_frag_lds(const XWeights<T, XS>& w, const int8_t* sX, int ldx, const float* sXd,
                                               int M, float (*hx)[RF][4][64], float (&out)[4], int tid,
                                               int half = 0) {
    constexpr int LW = 8 / XS;   // leaves per wave
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, g = lane >> 4;
    constexpr int nb = xr_sd_stride(1024 * T);   // K / 32 + 4
    const int8_t* ap[RF];
    const float* dp[RF][4];
#pragma unroll
    for (int f = 0; f < RF; f++) {
        ap[f] = sX + min(16 * f + fr, M - 1) * ldx + 16 * g;
#pragma unroll
        for (int r = 0; r < 4; r++) dp[f][r] = sXd + min(16 * f + 4 * g + r, M - 1) * nb;
    }
    float leaf[RF][LW][4];
#pragma unroll
    for (int f = 0; f < RF; f++)
#pragma unroll
        for (int l = 0; l < LW; l++)
#pragma unroll
            for (int r = 0; r < 4; r++) leaf[f][l][r] = 0.f;   // fma(c, p, +0) = the chains' first step
    const bool lo = g < 2;
    const xr_v4i zero = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4 * T / XS; i++) {
        // a scheduling fence every QASR_XR_FENCE spans (default 2): unfenced, the scheduler hoisted every span's LDS
        // reads (and the weights of the next fragment) and spilled at 512 registers
        if (i % QASR_XR_FENCE == 0) __builtin_amdgcn_sched_barrier(0);
        const int j = i & (4 / XS - 1), s = xr_span<XS>(i, wv, half);
        xr_v4i aq[RF];
        float2 dx[RF][4];
#pragma unroll
        for (int f = 0; f < RF; f++) {
            aq[f] = *(const xr_v4i*)(ap[f] + 64 * s);
#pragma unroll
            for (int r = 0; r < 4; r++) dx[f][r] = *(const float2*)(dp[f][r] + 2 * s);
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const xr_v4i bm = (lo == (h == 0)) ? w.wq[i] : zero;
            const float dw = __half2float(__ushort_as_half((unsigned short)(h ? w.ws[i] >> 16 : w.ws[i] & 0xffff)));
            const int l = 2 * j + h;
#pragma unroll
            for (int f = 0; f < RF; f++) {
                const xr_v4i c = __builtin_amdgcn_mfma_i32_16x16x64_i8(aq[f], bm, zero, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float dxr = h ? dx[f][r].y : dx[f][r].x;
                    leaf[f][l][r] = fmaf((float)c[r], dw * dxr, leaf[f][l][r]);
                }
            }
        }
    }
#pragma unroll
    for (int f = 0; f < RF; f++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            float o[2];
#pragma unroll
            for (int gq = 0; gq < LW / 4; gq++) {
                const float a0 = leaf[f][4 * gq][r] + 0.f, a1 = leaf[f][4 * gq + 1][r] + 0.f;
                const float a2 = leaf[f][4 * gq + 2][r] + 0.f, a3 = leaf[f][4 * gq + 3][r] + 0.f;
                o[gq] = (a0 + a1) + (a2 + a3);
            }
            hx[wv][f][r][lane] = XS == 1 ? o[0] + o[1] : o[0];   // H_w, or (XS = 2) O_{4h+w}
        }
    __syncthreads();
    if (wv < RF) {
        const int f = wv;
#pragma unroll
        for (int r = 0; r < 4; r++)
            out[r] = (hx[0][f][r][lane] + hx[1][f][r][lane]) + (hx[2][f][r][lane] + hx[3][f][r][lane]);
    }
}

}  // namespace qasr
