// The per-row attention body (decode rows, encoder windows, the fused decode q/k prologue and the split key range),
// of the k_attention launches (kernels_attn.hip; round 5's persistent decode kernel ran it too, hence the header).
// `bid` is the work item (the launch's blockIdx.x).  Every
// early `return` is either uniform over the workgroup (before any barrier) or leaves wave 0 alone past the last
// barrier, so a caller that runs items back to back needs only a workgroup barrier between them.  `tid` is the thread
// index.
#pragma once
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "qk_rope.h"
#include "wt.h"
#include "xlane.h"

namespace qasr {

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));

// one lane's QD dims of q·k: v_dot2_f32_f16 on the f16 q and K (products exact in f32, f32 accumulation)
template <int QD>
__device__ __forceinline__ float qk_dot(const h2v* qh, const __half* kr) {
    float part = 0.f;
    const int4 a = *(const int4*)kr;
    const h2v* ha = (const h2v*)&a;
#pragma unroll
    for (int t = 0; t < 4; t++) part = __builtin_amdgcn_fdot2(qh[t], ha[t], part, false);
    if constexpr (QD == 16) {
        const int4 b = *(const int4*)(kr + 8);
        const h2v* hb = (const h2v*)&b;
#pragma unroll
        for (int t = 0; t < 4; t++) part = __builtin_amdgcn_fdot2(qh[4 + t], hb[t], part, false);
    }
    return part;
}

// acc + p·(low / high f16 half of h), one v_fma_mix_f32 (the f16 operand is widened inside the FMA: no converts,
// so the V registers stay packed)
__device__ __forceinline__ float fma_mix_lo(float p, uint32_t h, float acc) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(p), "v"(h), "v"(acc));
    return d;
}
__device__ __forceinline__ float fma_mix_hi(float p, uint32_t h, float acc) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(p), "v"(h), "v"(acc));
    return d;
}

// q·k of one lane's 16 dims held in two registers (the decode path's chunk-wide loads)
__device__ __forceinline__ float qk_dot16(const h2v* qh, int4 a, int4 b) {
    float part = 0.f;
    const h2v* ha = (const h2v*)&a;
    const h2v* hb = (const h2v*)&b;
#pragma unroll
    for (int t = 0; t < 4; t++) part = __builtin_amdgcn_fdot2(qh[t], ha[t], part, false);
#pragma unroll
    for (int t = 0; t < 4; t++) part = __builtin_amdgcn_fdot2(qh[4 + t], hb[t], part, false);
    return part;
}

template <int HD, int G, int NW, bool FUSED = false, int CK = 64>
__device__ __forceinline__ void attention_rows(unsigned bid, int tid, const __half* __restrict__ Q, int ldq, const __half* K,
                                                   const __half* V, int ldkv,
                                                   const int* __restrict__ kv_start, const int* __restrict__ kv_len,
                                                   int rows, int nh, int nkv, float scale, float* __restrict__ o,
                                                   int8_t* __restrict__ oq, float* __restrict__ od, QkFuse fz = {}) {
    constexpr int CH = 256;
    constexpr int QD = HD / 8;    // dims per lane in QKᵀ
    constexpr int PD = HD / 64;   // dims per lane in PV / output
    constexpr int KU = 4;         // 8-key groups per QKᵀ iteration
    constexpr int VU = 8;         // keys per PV iteration
    __shared__ float sp[4][G][CH];
    __shared__ float cm_s[4][G], cl_s[4][G];
    __shared__ __align__(16) float ca_s[4][G][HD];
    __shared__ __align__(16) __half2 kn[FUSED ? HD / 2 : 1];   // FUSED: the new K row (f16), see the K preload
    // tid: threadIdx.x
    const int lane = tid & 63, w = tid >> 6;
    // NW = 4: one workgroup per (row, KV head), its 4 waves take contiguous quarters of the key range and merge
    // their partial softmax states through LDS (long decoder KV ranges).  NW = 1: one wave per (row, KV head)
    // (the encoder's 104-key windows).  The G query heads of a KV group share every K/V load.
    // FUSED with fz.part: kAttnSplitMax workgroups per (row, KV head); a range longer than fz.split_min keys is
    // cut into S ≤ kAttnSplitMax contiguous pieces (≥ fz.split_keys each), the rest exit at once.  Each piece's
    // merged (m, l, Σp·v) goes to fz.part; the last piece to arrive (fz.cnt) combines them in piece order.
    const bool spl = FUSED && fz.part != nullptr;   // uniform
    // split grid piece-major: every (row, KV head)'s piece 0 is dispatched first, the pieces a short range does not
    // need (they exit at once) after them, so they never queue ahead of real work
    const int nitems = rows * nkv;
    const int gw = spl ? (int)(bid % nitems) : NW == 4 ? bid : bid * 4 + w;
    const int piece = spl ? (int)(bid / nitems) : 0;
    if (NW == 1 && gw >= rows * nkv) return;
    const int part = NW == 4 ? w : 0;
    const int r = gw / nkv, kvh = gw % nkv;
    const int Lr = kv_len[r];
    int S = 1, per = Lr;
    if (spl && Lr > fz.split_min) {
        S = min(kAttnSplitMax, (Lr + fz.split_keys - 1) / fz.split_keys);
        per = (Lr + S - 1) / S;
    }
    if (piece >= S) return;   // whole workgroup, before any barrier
    const int kb0 = kv_start[r] + piece * per, Ls = min(per, Lr - piece * per);
    const int qn = (Ls + NW - 1) / NW;
    const int s0 = kb0 + part * qn, L = max(0, min(qn, Ls - part * qn));
    const int sub = lane & 7, kk = lane >> 3;
    constexpr bool DEC = HD == 128 && NW == 4;
    // FUSED decode: the first chunk's K loads go out before the q/k prologue (they do not wait for its barrier).
    // Only the new row (slot sl_new, written by the prologue) would be stale: its lanes take it from LDS (kn).
    constexpr int KP = DEC ? CK / 8 : 1;
    int4 ka[KP], kb[KP];   // the decode chunk loop's K registers (chunk 0 preloaded when FUSED)
    int sl_new = -1;
    // (G = 2 only: with 4 query heads the preload costs a wave per SIMD; the 64-key kernel preloads only ranges
    // of ≤ 32 keys per wave, which it runs as one 32-key chunk)
    constexpr bool PRE = FUSED && DEC && G == 2;
    const bool pre = PRE && (CK == 32 || L <= 32);   // uniform
    if (pre) {
        const int C0 = 32;
        const int n0 = min(C0, L);
        const __half* kc = K + (size_t)kvh * HD + sub * QD + (size_t)s0 * ldkv;
#pragma unroll
        for (int u = 0; u < KP; u++) {
            if (8 * u < C0 && n0 > 0) {
                const int j = min(8 * u + kk, n0 - 1);
                ka[u] = *(const int4*)(kc + (size_t)j * ldkv);
                kb[u] = *(const int4*)(kc + (size_t)j * ldkv + 8);
            }
        }
    }

    h2v qv[G][QD / 2];   // the f16 q dims of this lane (q is f16-rounded on every path)
    if constexpr (FUSED) {
        // decode rows (NW = 4, hd = 128): the q/k RMS-norm + RoPE of this row's G query heads and its KV head, and
        // the new K/V cache row, computed here instead of by k_qk_norm_rope_row (same arithmetic, same f16
        // rounding: bit-identical).  q stays in LDS; K/V go to the cache and the barrier makes the new row
        // visible to the waves that read it below (workgroup-scope ordering of global memory).
        static_assert(HD == 128 && NW == 4, "fused q/k prologue: hd 128 decode kernel");
        // q rows in LDS with 4 floats of padding per 16 (element e at e + 4·(e/16)): the 8 lanes groups' ds_read_b128 of
        // dims 16·sub … 16·sub + 15 then fall in distinct banks (unpadded, sub and sub + 4 collided)
        __shared__ __align__(16) float qs[G][HD + HD / 4];
        const int nslot = nh + 2 * nkv, kvd = nkv * HD;
        const float* src = fz.qkv + (size_t)r * nslot * HD;
        const int p = fz.pos[r], sl = fz.slot[r];
        // the new K/V row is written (and read back through the barrier) by the piece whose range holds its slot;
        // a slot outside the row's key range (never from the engine) is written by piece 0, as the unsplit kernel does
        const bool own = S == 1 || (sl >= kb0 && sl < kb0 + Ls) ||
                         (piece == 0 && (sl < kv_start[r] || sl >= kv_start[r] + Lr));
        sl_new = own ? sl : -1;
        const int e0 = (2 * lane) & (HD / 2 - 1);
        const float4 cs = *(const float4*)(fz.rope_cs + ((size_t)p * (HD / 2) + e0) * 2);
        const bool lo = 2 * lane < HD / 2;
        for (int t = w; t < G + 2; t += 4) {
            if (t >= G && !own) continue;
            const int h = t < G ? kvh * G + t : t == G ? nh + kvh : nh + nkv + kvh;
            const float2 v = *(const float2*)(src + h * HD + 2 * lane);
            if (t == G + 1) {
                *(__half2*)(fz.vc + (size_t)sl * kvd + kvh * HD + 2 * lane) = __floats2half2_rn(v.x, v.y);
                continue;
            }
            const float2 g = *(const float2*)((t < G ? fz.qnw : fz.knw) + 2 * lane);
            const __half2 hv = norm_rope_hd128(v, g, cs, lo, fz.eps);
            if (t < G) {
                const float2 back = __half22float2(hv);
                *(float2*)&qs[t][2 * lane + 4 * (lane >> 3)] = make_float2(back.x, back.y);
            } else {
                *(__half2*)(fz.kc + (size_t)sl * kvd + kvh * HD + 2 * lane) = hv;
                kn[lane] = hv;
            }
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < QD / 2; j++)
                qv[g][j] = (h2v){(_Float16)qs[g][sub * (QD + 4) + 2 * j], (_Float16)qs[g][sub * (QD + 4) + 2 * j + 1]};
    } else {
#pragma unroll
        for (int g = 0; g < G; g++) {
            const __half* qp = Q + (size_t)r * ldq + (kvh * G + g) * HD + sub * QD;
#pragma unroll
            for (int j = 0; j < QD / 2; j++) qv[g][j] = *(const h2v*)(qp + 2 * j);
        }
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
    // decoder rows (hd 128, 4 waves): 64-key chunks whose K and V loads are all issued together (one memory round
    // trip per chunk instead of one per 8 keys); PV with 16 lanes per key (16-B V loads, dims 8·(lane&15)..+8,
    // key group lane>>4), the 4 key groups summed once at the end
    const int vg = lane >> 4, vd = 8 * (lane & 15);
    float av[G][8];
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
        for (int j = 0; j < 8; j++) av[g][j] = 0.f;
    if constexpr (DEC) {
        // C keys per chunk and wave: K as C/8 row groups of 8 lanes × 32 B, V as C/4 groups of 16 lanes × 16 B.
        // CK = 64 kernels run a wave with ≤ 32 keys in 32-key chunks (half the clamped re-reads; the registers are
        // sized by the 64-key path anyway); CK = 32 kernels (many rows: occupancy 4, not 3) only in 32-key chunks.
        static_assert(CK == 32 || CK == 64, "k_attention: decode chunk of 32 or 64 keys");
        const __half* vbase16 = V + (size_t)kvh * HD + vd;
        auto run = [&](auto ckc) {
        constexpr int C = decltype(ckc)::value;
        constexpr int KU8 = C / 8, VU4 = C / 4;
        for (int c0 = 0; c0 < L; c0 += C) {
            const int n = min(C, L - c0);
            const __half* kc = kbase + (size_t)(s0 + c0) * ldkv;
            const __half* vc = vbase16 + (size_t)(s0 + c0) * ldkv;
            static_assert(KU8 <= KP, "k_attention: chunk wider than the K registers");
            int4 vr[VU4];
            if (!pre || c0 > 0) {
#pragma unroll
                for (int u = 0; u < KU8; u++) {
                    const int j = min(8 * u + kk, n - 1);   // rows past n re-read row n-1 (their scores are dropped)
                    ka[u] = *(const int4*)(kc + (size_t)j * ldkv);
                    kb[u] = *(const int4*)(kc + (size_t)j * ldkv + 8);
                }
            }
            if constexpr (FUSED) {
                if (sl_new >= s0 + c0 && sl_new < s0 + c0 + n) {   // this chunk holds the new row
#pragma unroll
                    for (int u = 0; u < KU8; u++) {
                        if (s0 + c0 + min(8 * u + kk, n - 1) == sl_new) {
                            ka[u] = *(const int4*)(kn + sub * (QD / 2));
                            kb[u] = *(const int4*)(kn + sub * (QD / 2) + 4);
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < KU8; u++) {
                const int j = 8 * u + kk;
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const float p = sum8(qk_dot16(qv[g], ka[u], kb[u]));
                    if (sub == 0 && j < n) sp[w][g][j] = p * scale;
                }
            }
            wave_sync_lds();
            // the V loads fly while the softmax runs (issued after the scores so K and V are never live together:
            // issuing them with K costs the 32-key kernel its 4th wave per SIMD, 31.9 → 33.8 µs at 256 rows,
            // profiles/r2s2_attn_v_early_ab.jsonl)
#pragma unroll
            for (int u = 0; u < VU4; u++) {
                const int j = min(4 * u + vg, n - 1);   // rows past n: weight p = 0
                vr[u] = *(const int4*)(vc + (size_t)j * ldkv);
            }
#pragma unroll
            for (int g = 0; g < G; g++) {
                const float x = lane < n ? sp[w][g][lane] : -INFINITY;
                const float mnew = fmaxf(m[g], wave_max(x));
                const float alpha = expf(m[g] - mnew);
                const float p = lane < n ? expf(x - mnew) : 0.f;
                lsum[g] = fmaf(lsum[g], alpha, wave_sum(p));
                m[g] = mnew;
                sp[w][g][lane] = p;
#pragma unroll
                for (int j = 0; j < 8; j++) av[g][j] *= alpha;
            }
            wave_sync_lds();
#pragma unroll
            for (int u = 0; u < VU4; u++) {
                const uint32_t* hv = (const uint32_t*)&vr[u];
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const float p = sp[w][g][4 * u + vg];
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        av[g][2 * t] = fma_mix_lo(p, hv[t], av[g][2 * t]);
                        av[g][2 * t + 1] = fma_mix_hi(p, hv[t], av[g][2 * t + 1]);
                    }
                }
            }
            wave_sync_lds();
        }
        };
        if (CK == 32 || L <= 32) run(std::integral_constant<int, 32>{});
        else run(std::integral_constant<int, CK>{});
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                av[g][j] += __shfl_xor(av[g][j], 16);   // once per workgroup: ds_bpermute is fine here
                av[g][j] += __shfl_xor(av[g][j], 32);
            }
    }

    for (int c0 = 0; c0 < (DEC ? 0 : L); c0 += CH) {
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
                    p = sum8(p);
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
            cm = wave_max(cm);
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
            lsum[g] = lsum[g] * alpha + wave_sum(ps);
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
    // merge the NW partial states (m, l, acc) of this row's key ranges.  Every multiply-add of the decode softmax
    // and merges is an explicit fmaf: left to contraction, each instantiation's SLP packing decides mul+add (two
    // roundings, v_pk_*) or fma (one), and the fused and unfused kernels then differ in the last bit
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
            if constexpr (DEC) {
                if (vg == 0) {
#pragma unroll
                    for (int j = 0; j < 8; j += 4)   // two ds_write_b128 per lane (8 scalar writes were 2-way conflicted)
                        *(float4*)&ca_s[w][g][vd + j] = make_float4(av[g][j], av[g][j + 1], av[g][j + 2], av[g][j + 3]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < PD; j++) ca_s[w][g][lane * PD + j] = acc[g][j];
            }
        }
        __syncthreads();
        if (w != 0) return;
    }
    const int wb = NW == 1 ? w : 0;   // first partial state of this item
    const int D = nh * HD;
    float* pbase = spl ? fz.part + (size_t)gw * kAttnSplitMax * G * (2 + HD) : nullptr;
    if (S > 1) {
        // this piece's merged state → fz.part; the last piece to arrive goes on to combine all S of them
#pragma unroll
        for (int g = 0; g < G; g++) {
            float mt = -INFINITY;
#pragma unroll
            for (int u = 0; u < NW; u++) mt = fmaxf(mt, cm_s[wb + u][g]);
            float lt = 0.f, sc[NW];
#pragma unroll
            for (int u = 0; u < NW; u++) {
                sc[u] = cm_s[wb + u][g] == -INFINITY ? 0.f : expf(cm_s[wb + u][g] - mt);
                lt = fmaf(cl_s[wb + u][g], sc[u], lt);
            }
            float* pp = pbase + (size_t)(piece * G + g) * (2 + HD);
#pragma unroll
            for (int j = 0; j < PD; j++) {
                float a = 0.f;
#pragma unroll
                for (int u = 0; u < NW; u++) a = fmaf(ca_s[wb + u][g][lane * PD + j], sc[u], a);
                __hip_atomic_store(pp + 2 + lane * PD + j, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) {
                __hip_atomic_store(pp, mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pp + 1, lt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // hand-off without cache-wide fences (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1): the
        // state is stored write-through (sc1) by this one wave, which waits for its stores, then counts the arrival
        // with an agent-scope add; the piece whose add comes last reads every state with sc1 loads
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int prev = 0;
        if (lane == 0)
            prev = __hip_atomic_fetch_add(fz.cnt + gw, 1, QASR_FORMAL_HANDOFF ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        prev = __builtin_amdgcn_readfirstlane(prev);
        if (prev != S - 1) return;
        if constexpr (QASR_FORMAL_HANDOFF) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 0) __hip_atomic_store(fz.cnt + gw, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int h = kvh * G + g;
        float out[PD];
        if (S > 1) {
            // combine the S pieces in piece order (deterministic whatever the arrival order)
            // every load in flight at once: lane u reads piece u's (m, l); each lane reads its dims of all pieces
            // (unconditionally, pieces past S clamped and weighted 0); fixed order, so deterministic
            auto ld = [](const float* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
            const float* pl = pbase + (size_t)(min(lane, S - 1) * G + g) * (2 + HD);
            const float mu = ld(pl), lu = ld(pl + 1);
            float av2[kAttnSplitMax][PD];
#pragma unroll
            for (int u = 0; u < kAttnSplitMax; u++)
#pragma unroll
                for (int j = 0; j < PD; j++)
                    av2[u][j] = ld(pbase + (size_t)(min(u, S - 1) * G + g) * (2 + HD) + 2 + lane * PD + j);
            const float mt = wave_max(lane < S ? mu : -INFINITY);
            const float su = lane < S ? expf(mu - mt) : 0.f;
            const float lt = wave_sum(lu * su);
            float a[PD];
#pragma unroll
            for (int j = 0; j < PD; j++) a[j] = 0.f;
#pragma unroll
            for (int u = 0; u < kAttnSplitMax; u++) {
                const float sc = lane_f(su, u);   // 0 for pieces past S
#pragma unroll
                for (int j = 0; j < PD; j++) a[j] = fmaf(av2[u][j], sc, a[j]);
            }
#pragma unroll
            for (int j = 0; j < PD; j++) out[j] = a[j] / lt;
        } else {
            float mt = -INFINITY;
#pragma unroll
            for (int u = 0; u < NW; u++) mt = fmaxf(mt, cm_s[wb + u][g]);
            float lt = 0.f, sc[NW];
#pragma unroll
            for (int u = 0; u < NW; u++) {
                sc[u] = cm_s[wb + u][g] == -INFINITY ? 0.f : expf(cm_s[wb + u][g] - mt);
                lt = fmaf(cl_s[wb + u][g], sc[u], lt);
            }
            const float inv = Lr > 0 ? 1.f / lt : 0.f;
#pragma unroll
            for (int j = 0; j < PD; j++) {
                float a = 0.f;
#pragma unroll
                for (int u = 0; u < NW; u++) a = fmaf(ca_s[wb + u][g][lane * PD + j], sc[u], a);
                out[j] = a * inv;
            }
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
            if constexpr (PD == 2) {
                amax = max16(amax);
            } else {
#pragma unroll
                for (int off = 1; off < 32 / PD; off <<= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
            }
            const float d = amax / 127.f;
            int qb[PD];
#pragma unroll
            for (int j = 0; j < PD; j++) qb[j] = amax == 0.f ? 0 : (int)roundf(out[j] / d);
            const float dq = __half2float(f2h(d));
#pragma unroll
            for (int j = 0; j < PD; j++) oq[(size_t)r * D + h * HD + lane * PD + j] = (int8_t)qb[j];
            if ((lane & (32 / PD - 1)) == 0) od[(size_t)r * (D / 32) + (h * HD + lane * PD) / 32] = dq;
        }
    }
}

}  // namespace qasr
