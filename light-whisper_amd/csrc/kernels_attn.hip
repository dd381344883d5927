// Variable-length attention over f16 K/V (decoder KV cache slots or encoder window buffers), gfx950.
//
// One wave per (query row, KV head), the G = n_heads/n_kv_heads query heads of the group sharing every K/V load.  Keys are processed in LDS-resident chunks of 256 with an online softmax
// (running max / sum, f32).  QKᵀ: 8 lanes per key (16-dim slices, 3 xor-shuffles), 32 keys per unrolled
// iteration so eight 16-byte K loads per lane are in flight together.  PV: each lane owns hd/64 dims and
// walks the keys 8 at a time with eight independent 4-byte V loads in flight (each V row is one coalesced
// 256-byte segment).  Row r attends slots [kv_start[r], kv_start[r]+kv_len[r]) — causal prefill, single-token
// decode and the encoder's bidirectional 104-token windows (modeling_qwen3_asr.py:276-315) are all expressed
// by the per-row ranges.  The output is written as f32 and/or directly as Q8 blocks for the O-projection.
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "qk_rope.h"
#include "xlane.h"

// decode rows from which the fused decode attention takes the 32-key-chunk kernel (4 waves per SIMD) instead of the
// 64-key one (3 per SIMD, one chunk for per-wave ranges of 33–64 keys)
#ifndef QASR_ATTN_CK32_ROWS
#define QASR_ATTN_CK32_ROWS 192
#endif

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
__global__ __launch_bounds__(256) void k_attention(const __half* __restrict__ Q, int ldq, const __half* K,
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
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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
    const int gw = spl ? (int)(blockIdx.x % nitems) : NW == 4 ? blockIdx.x : blockIdx.x * 4 + w;
    const int piece = spl ? (int)(blockIdx.x / nitems) : 0;
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


// ------------------------------------------------------------------------------------------------ tiled (MFMA)
// Prefill / encoder attention: rows come in runs that share their key range (an utterance's causal prompt rows,
// an encoder window), so 16 consecutive rows form one tile and every K/V chunk loaded is used by all 16.
// One wave per (16-row tile, KV head) with the G query heads of the group in the same wave:
//   Sᵀ = K·Qᵀ on v_mfma_f32_16x16x32_f16 (keys on the MFMA rows, so each lane owns one query row's scores for
//   its keys — row max / sum are a few in-lane ops plus two xor-shuffles), online softmax in f32, P rounded to
//   f16 and O += P·V on the same MFMA with V read column-wise by ds_read_b64_tr_b16 from a per-wave LDS chunk.
// Each row's own range [kv_start, kv_start+kv_len) is applied as a mask inside the union range of the tile.
// Precision: scores and the softmax in f32, P in f16 (relative 2^-11) — the test states the tolerance.
template <int HD, int G, bool SINGLE>
__global__ __launch_bounds__(256) void k_attn_tile(const __half* __restrict__ Q, int ldq, const __half* __restrict__ K,
                                                   const __half* __restrict__ V, int ldkv,
                                                   const int* __restrict__ kv_start, const int* __restrict__ kv_len,
                                                   int rows, int nkv, float scale, float* __restrict__ o,
                                                   int8_t* __restrict__ oq, float* __restrict__ od) {
    typedef _Float16 v8h __attribute__((ext_vector_type(8)));
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef _Float16 v4h __attribute__((ext_vector_type(4)));
    typedef float v4f __attribute__((ext_vector_type(4)));
    constexpr int KC = 32;          // keys per chunk
    constexpr int DC = HD / 32;     // 32-dim slices of the QKᵀ reduction
    constexpr int DT = HD / 16;     // 16-dim output tiles of PV
    constexpr int CPR = HD / 8;     // 16-byte chunks per V row
    __shared__ __attribute__((aligned(16))) _Float16 vs_all[4][KC * HD];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // SINGLE (decode): one query row per wave, replicated on the 16 MFMA rows (the MFMA work is idle capacity
    // beside the K/V stream; only output row 0 is stored)
    const int ntiles = SINGLE ? rows : (rows + 15) >> 4;
    const int item = blockIdx.x * 4 + w;
    if (item >= ntiles * nkv) return;   // whole wave
    const int tile = item / nkv, kvh = item % nkv;
    const int fr = lane & 15, kh = lane >> 4;
    const int r0 = SINGLE ? tile : tile * 16;
    _Float16* vs = vs_all[w];
    // V image: 16-byte chunk ch of key row kr at kr·HD·2 + 16·(ch ^ swz(kr)), swz(kr) = ((kr >> 1) & 3) << 1 |
    // (kr & 1) << 3 (mod the row's chunks): each ds_read_b64_tr_b16 32-lane group (8 key rows × 2 chunks) and each
    // ds_write_b128 8-lane group hits distinct banks for hd 64 and 128 (MI355X_MICROARCH.md §LDS; the r2 swizzle was
    // 4-way / 2-way on the reads: 0.82 conflict cycles per LDS instruction)
    auto voff = [&](int kr, int ch) -> int {
        return kr * HD * 2 + 16 * (ch ^ (((((kr >> 1) & 3) << 1) | ((kr & 1) << 3)) & (CPR - 1)));
    };

    // this lane's query row (fr) and its key range
    const int myrow = SINGLE ? r0 : min(r0 + fr, rows - 1);
    const bool row_ok = SINGLE || r0 + fr < rows;
    const int st = kv_start[myrow], en = row_ok ? st + kv_len[myrow] : st;
    int lo = 0, hi = 0;
    // Q fragments (B operand of K·Qᵀ): lane (row fr, kh) holds Q[row][32c + 8kh .. +8]
    v8h qf[G][DC];
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
        for (int c = 0; c < DC; c++)
            qf[g][c] = *(const v8h*)(Q + (size_t)myrow * ldq + (kvh * G + g) * HD + 32 * c + 8 * kh);
    v4f acc[G][DT];
    float m[G], l[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
        m[g] = -INFINITY;
        l[g] = 0.f;
#pragma unroll
        for (int t = 0; t < DT; t++) acc[g][t] = v4f{0.f, 0.f, 0.f, 0.f};
    }
    const __half* kbase = K + (size_t)kvh * HD;
    const __half* vbase = V + (size_t)kvh * HD;
    // K/V of chunk k0 + KC are loaded while chunk k0 is computed (one chunk in flight ahead)
    constexpr int VP = KC * CPR / 64;   // 16-byte V pieces per lane
    int4 vp[VP];
    v8h kn[2][DC];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int u = 0; u < VP; u++) {
            const int piece = u * 64 + lane, kr = piece / CPR, ch = piece % CPR;
            vp[u] = *(const int4*)(vbase + (size_t)min(c0 + kr, hi - 1) * ldkv + 8 * ch);
        }
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int c = 0; c < DC; c++)
                kn[t][c] = *(const v8h*)(kbase + (size_t)min(c0 + 16 * t + fr, hi - 1) * ldkv + 32 * c + 8 * kh);
    };
    // One pass per distinct range start among the tile's rows (encoder windows / packed utterances meeting inside a
    // 16-row tile): the rows that share a start take every key in chunks aligned at THAT start, the others see the
    // pass fully masked (state unchanged bit for bit: alpha 1, p 0).  A row's result is then independent of where its
    // range sits relative to the tile — the streaming encoder cache recomputes a window as rows 0… of a shorter run.
    // Tiles whose rows share one start (nearly all) run exactly one pass, as before.
    bool pend = row_ok && en > st;
    for (;;) {
    int s0 = pend ? st : INT_MAX;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) s0 = min(s0, __shfl_xor(s0, off));
    if (s0 == INT_MAX) break;
    const bool in = pend && st == s0;
    int e0 = in ? en : INT_MIN;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) e0 = max(e0, __shfl_xor(e0, off));
    lo = s0;
    hi = e0;
    pend = pend && !in;
    load_chunk(lo);
    for (int k0 = lo; k0 < hi; k0 += KC) {
        // ---- this chunk: V into the wave's LDS image, K fragments to registers; then prefetch the next chunk
#pragma unroll
        for (int u = 0; u < VP; u++) {
            const int piece = u * 64 + lane, kr = piece / CPR, ch = piece % CPR;
            *(int4*)((char*)vs + voff(kr, ch)) = vp[u];
        }
        v8h kf[2][DC];
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int c = 0; c < DC; c++) kf[t][c] = kn[t][c];
        if (k0 + KC < hi) load_chunk(k0 + KC);
        // ---- Sᵀ tiles: lane (row fr, kh) gets keys 16t + 4kh + i
        float p[G][2][4];
#pragma unroll
        for (int g = 0; g < G; g++) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
                v4f sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int c = 0; c < DC; c++) sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[t][c], qf[g][c], sacc, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int key = k0 + 16 * t + 4 * kh + i;
                    p[g][t][i] = (in && key >= st && key < en) ? sacc[i] * scale : -INFINITY;
                }
            }
        }
        // ---- online softmax per row (lane-local over its 8 keys, then across the 4 kh groups)
        float alpha[G];
        _Float16 ph[G][8];
#pragma unroll
        for (int g = 0; g < G; g++) {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int i = 0; i < 4; i++) mx = fmaxf(mx, p[g][t][i]);
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            const float mn = fmaxf(m[g], mx);
            alpha[g] = mn == -INFINITY ? 1.f : expf(m[g] - mn);
            float ps = 0.f;
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float e = mn == -INFINITY ? 0.f : expf(p[g][t][i] - mn);
                    ps += e;
                    ph[g][4 * t + i] = (_Float16)e;
                }
            ps += __shfl_xor(ps, 16);
            ps += __shfl_xor(ps, 32);
            l[g] = l[g] * alpha[g] + ps;
            m[g] = mn;
        }
        // rescale O: acc rows are 4kh+i (row on the register), alpha lives on lane (row fr)
#pragma unroll
        for (int g = 0; g < G; g++) {
            float ar[4];
#pragma unroll
            for (int i = 0; i < 4; i++) ar[i] = __shfl(alpha[g], 4 * kh + i);
#pragma unroll
            for (int t = 0; t < DT; t++)
#pragma unroll
                for (int i = 0; i < 4; i++) acc[g][t][i] *= ar[i];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- O += P·V: P slots j ↔ keys 16(j>>2) + 4kh + (j&3); V fragment = two transposed 4×16 reads
        const int q = fr >> 2, pp = fr & 3;
#pragma unroll
        for (int t = 0; t < DT; t++) {
            v4s rr[2];
#pragma unroll
            for (int h2 = 0; h2 < 2; h2++) {
                const int kr = 16 * h2 + 4 * kh + q, ch = 2 * t + (pp >> 1);
                rr[h2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) v4s*)((__attribute__((address_space(3))) char*)vs +
                                                              voff(kr, ch) + 8 * (pp & 1)));
            }
            // whole-vector bit casts: assembling vf element by element from the shorts miscompiles (ROCm 7.2,
            // tools/micro/tr_check.hip)
            const v8h vf = __builtin_shufflevector(__builtin_bit_cast(v4h, rr[0]), __builtin_bit_cast(v4h, rr[1]), 0, 1,
                                                   2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int g = 0; g < G; g++) {
                v8h pf;
#pragma unroll
                for (int j = 0; j < 8; j++) pf[j] = ph[g][j];
                acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, vf, acc[g][t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    }
    // ---- normalise and store: acc[g][t][i] = O[row 4kh+i][dim 16t + fr] of head kvh·G + g
    const int D = nkv * G * HD;
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int h = kvh * G + g;
        float inv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float li = __shfl(l[g], 4 * kh + i);
            inv[i] = li > 0.f ? 1.f / li : 0.f;
        }
#pragma unroll
        for (int t = 0; t < DT; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) acc[g][t][i] *= inv[i];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = SINGLE ? (4 * kh + i == 0 ? r0 : rows) : r0 + 4 * kh + i;   // rows = "not stored"
            if (o && row < rows) {
#pragma unroll
                for (int t = 0; t < DT; t++) o[(size_t)row * D + h * HD + 16 * t + fr] = acc[g][t][i];
            }
            if (oq) {
                // a Q8 block = 32 dims = tiles 2b, 2b+1 across the 16 lanes of this kh group
#pragma unroll
                for (int b = 0; b < DT / 2; b++) {
                    float am = fmaxf(fabsf(acc[g][2 * b][i]), fabsf(acc[g][2 * b + 1][i]));
#pragma unroll
                    for (int off = 1; off < 16; off <<= 1) am = fmaxf(am, __shfl_xor(am, off));
                    const float dd = am / 127.f;
                    if (row < rows) {
                        int8_t* qr = oq + (size_t)row * D + h * HD + 32 * b;
                        qr[fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(acc[g][2 * b][i] / dd));
                        qr[16 + fr] = (int8_t)(am == 0.f ? 0 : (int)roundf(acc[g][2 * b + 1][i] / dd));
                        if (fr == 0) od[(size_t)row * (D / 32) + (h * HD) / 32 + b] = __half2float(f2h(dd));
                    }
                }
            }
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
        // the fused decode kernel's chunk policy (attention_decode_fused), so the two paths stay bit-identical
        case 2:
            if (HD == 128 && rows >= QASR_ATTN_CK32_ROWS)
                k_attention<HD, 2, 4, false, 32><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                                     scale, o, oq, od);
            else
                k_attention<HD, 2, 4><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o,
                                                         oq, od);
            break;
        case 4:
            if (HD == 128 && rows >= QASR_ATTN_CK32_ROWS)
                k_attention<HD, 4, 4, false, 32><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                                     scale, o, oq, od);
            else
                k_attention<HD, 4, 4><<<b4, 256, 0, s>>>(Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o,
                                                         oq, od);
            break;
        default: throw Error(QASR_E_INVALID, "attention: query heads per KV head must be 1, 2 or 4");
    }
}

void attention_decode_fused(const QkFuse& fz, int ldkv, const int* kv_start, const int* kv_len, int rows, int nh,
                            int nkv, int hd, float scale, int8_t* oq, float* od, hipStream_t s, int64_t total_keys) {
    if (rows <= 0) return;
    // QKᵀ + PV: 4·hd flops per (query head, key); bytes: the f16 K and V rows once per (KV head, key) — the G query
    // heads of a group share every load
    ProfScope ps(s, "attention_decode", 4.0 * hd * nh * (double)total_keys, 4.0 * hd * nkv * (double)total_keys);
    QASR_CHECK(hd == 128 && nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "attention_decode_fused: hd 128 only");
    const int G = nh / nkv;
    QASR_CHECK(!fz.part || (rows <= fz.part_rows && fz.cnt), QASR_E_INVALID,
               "attention_decode_fused: more split rows than the scratch holds");
    const unsigned b4 = (unsigned)(rows * nkv * (fz.part ? kAttnSplitMax : 1));
    // many rows (≥ 192: ≥ 1,536 workgroups) → the 32-key-chunk kernel, 103 VGPRs and 4 waves per SIMD instead of 3
    // (tools/attn_batch.py, profiles/r2_attn_batch_chunk.jsonl: 256 rows 35.9 → 31.2 µs); fewer rows → the 64-key
    // kernel, which still runs its ≤ 32-key waves in 32-key chunks (1 key 6.35 → 5.37 µs)
    const bool ck32 = rows >= QASR_ATTN_CK32_ROWS && !fz.fixed_chunk;
    // (a 5-waves-per-SIMD build of the 32-key kernel, 95 VGPRs, streamed the same: 31.1 against 31.5 µs at 256
    // rows, profiles/r2s2_attn_occupancy_ab.jsonl — the kernel is not occupancy-bound)
    if (G == 2 && ck32)
        k_attention<128, 2, 4, true, 32><<<b4, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh,
                                                            nkv, scale, nullptr, oq, od, fz);
    else if (G == 2)
        k_attention<128, 2, 4, true><<<b4, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                        scale, nullptr, oq, od, fz);
    else if (G == 4 && ck32)
        k_attention<128, 4, 4, true, 32><<<b4, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh,
                                                            nkv, scale, nullptr, oq, od, fz);
    else if (G == 4)
        k_attention<128, 4, 4, true><<<b4, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                        scale, nullptr, oq, od, fz);
    else
        throw Error(QASR_E_INVALID, "attention_decode_fused: query heads per KV head must be 2 or 4");
}

void attention(const __half* Q, int ldq, const __half* K, const __half* V, int ldkv, const int* kv_start,
               const int* kv_len, int rows, int nh, int nkv, int hd, float scale, float* o, int8_t* oq, float* od,
               hipStream_t s, int64_t total_keys, bool dense) {
    if (rows <= 0) return;
    // QKᵀ + PV: 4·hd flops per (query head, key); bytes: K and V once per (KV head, key) for per-row decode rows, once
    // per (16-row tile, KV head, key) for the dense tile kernel (prefill / encoder: MFMA-priced in bench.py)
    ProfScope ps(s, dense ? "attention_tile" : "attention_decode", 4.0 * hd * nh * (double)total_keys,
                 4.0 * hd * nkv * (double)total_keys / (dense ? 16.0 : 1.0));
    QASR_CHECK(nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "attention: bad head counts");
    const int G = nh / nkv;
    // QASR_ATTN_SINGLE=1 (A/B only): decode rows as single-row MFMA tiles instead of the f32 per-row kernel, which
    // streams the decode KV at 4-5 TB/s (tools/attn_tune.py; the single-row tiles reach 2.4-2.8)
    static const bool single_tiles = [] {
        const char* e = getenv("QASR_ATTN_SINGLE");
        return e && *e == '1';
    }();
    if ((G == 1 || G == 2) && (hd == 64 || hd == 128) && ldq % 8 == 0 && ldkv % 8 == 0 && (dense || single_tiles)) {
        const unsigned grid = (unsigned)cdiv((dense ? cdiv(rows, 16) : rows) * nkv, 4);
#define QASR_TILE(HD_, G_)                                                                                         \
    (dense ? k_attn_tile<HD_, G_, false> : k_attn_tile<HD_, G_, true>)<<<grid, 256, 0, s>>>(                       \
        Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nkv, scale, o, oq, od)
        if (hd == 128 && G == 2) QASR_TILE(128, 2);
        else if (hd == 128) QASR_TILE(128, 1);
        else if (G == 2) QASR_TILE(64, 2);
        else QASR_TILE(64, 1);
#undef QASR_TILE
        return;
    }
    if (hd == 128)
        launch_attention<128>(G, rows, s, Q, ldq, K, V, ldkv, kv_start, kv_len, nh, nkv, scale, o, oq, od);
    else if (hd == 64)
        launch_attention<64>(G, rows, s, Q, ldq, K, V, ldkv, kv_start, kv_len, nh, nkv, scale, o, oq, od);
    else
        throw Error(QASR_E_INVALID, "attention: head_dim must be 64 or 128");
}

}  // namespace qasr
