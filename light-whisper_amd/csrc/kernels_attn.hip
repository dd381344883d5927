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

#include "attn_rows.h"
#include "kernels.h"
#include "qk_rope.h"
#include "xlane.h"

// decode rows from which the fused decode attention takes the 32-key-chunk kernel (4 waves per SIMD) instead of the
// 64-key one (3 per SIMD, one chunk for per-wave ranges of 33–64 keys)
#ifndef QASR_ATTN_CK32_ROWS
#define QASR_ATTN_CK32_ROWS 192
#endif

namespace qasr {

// one workgroup per item (see attention_rows)
template <int HD, int G, int NW, bool FUSED = false, int CK = 64>
__global__ __launch_bounds__(256) void k_attention(const __half* __restrict__ Q, int ldq, const __half* K,
                                                   const __half* V, int ldkv,
                                                   const int* __restrict__ kv_start, const int* __restrict__ kv_len,
                                                   int rows, int nh, int nkv, float scale, float* __restrict__ o,
                                                   int8_t* __restrict__ oq, float* __restrict__ od, QkFuse fz = {}) {
    attention_rows<HD, G, NW, FUSED, CK>(blockIdx.x, threadIdx.x, Q, ldq, K, V, ldkv, kv_start, kv_len, rows, nh, nkv, scale, o, oq,
                                         od, fz);
}


// ------------------------------------------------------------------------------------------------ one wave per item
// Decode rows of many-row steps (round 5): ONE wave per (row, KV head) over its whole key range, 4
// items per workgroup, no LDS merge and no workgroup barrier — the 4-wave kernel's chain (prologue → barrier → K → V
// → merge barrier) per item is replaced by a per-wave chunk loop in which chunk c+1's K loads are issued as soon as
// chunk c's scores are out of the K registers, so K(c+1) and V(c) are in flight together (one memory round trip per
// 32-key chunk).  Same per-key arithmetic as the decode chunk loop of attention_rows (v_dot2 q·k, f32 online softmax,
// v_fma_mix PV over 4 key groups of 16 lanes), one key range instead of four merged quarters: NOT bit-identical to
// the 4-wave kernel, so it runs only where the engine's contract is tolerance-level (the table path's batched decode
// rows; exact rows, verify passes and batch invariance keep attention_rows).  FUSED: the q/k RMSNorm + RoPE and the
// new K/V row in the wave's prologue (qk_rope.h arithmetic); the new row's K and V are patched in from LDS.
template <int G, bool FUSED>
__global__ __launch_bounds__(256) void k_attn_wave(const __half* __restrict__ Q, int ldq, __half* K, __half* V,
                                                   int ldkv, const int* __restrict__ kv_start,
                                                   const int* __restrict__ kv_len, int rows, int nh, int nkv,
                                                   float scale, int8_t* __restrict__ oq, float* __restrict__ od,
                                                   QkFuse fz) {
    constexpr int HD = 128, QD = 16, C = 32;
    __shared__ float sp_all[4][G][C];
    __shared__ __align__(16) float qs_all[FUSED ? 4 : 1][G][HD + HD / 4];
    __shared__ __align__(16) __half2 kn_all[FUSED ? 4 : 1][HD / 2];
    __shared__ __align__(16) __half2 vn_all[FUSED ? 4 : 1][HD / 2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int gw = blockIdx.x * 4 + w;
    if (gw >= rows * nkv) return;   // whole wave (no workgroup barrier below)
    const int r = gw / nkv, kvh = gw % nkv;
    const int L = kv_len[r], s0 = kv_start[r];
    const int sub = lane & 7, kk = lane >> 3, vg = lane >> 4, vd = 8 * (lane & 15);
    float (*sp)[C] = sp_all[w];
    const __half* kbase = K + (size_t)kvh * HD + sub * QD;
    const __half* vbase = V + (size_t)kvh * HD + vd;
    int4 ka[4], kb[4];
    auto load_k = [&](int c0) {
        const int n = min(C, L - c0);
        const __half* kc = kbase + (size_t)(s0 + c0) * ldkv;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int j = min(8 * u + kk, n - 1);   // rows past n re-read row n-1 (their scores are dropped)
            ka[u] = *(const int4*)(kc + (size_t)j * ldkv);
            kb[u] = *(const int4*)(kc + (size_t)j * ldkv + 8);
        }
    };
    if (L > 0) load_k(0);   // chunk 0's K goes out before the prologue (the new row is patched from LDS below)
    h2v qv[G][QD / 2];
    int sl_new = -1;
    if constexpr (FUSED) {
        float* qs = &qs_all[w][0][0];
        const int nslot = nh + 2 * nkv, kvd = nkv * HD;
        const float* src = fz.qkv + (size_t)r * nslot * HD;
        const int p = fz.pos[r], sl = fz.slot[r];
        sl_new = sl;
        const int e0 = (2 * lane) & (HD / 2 - 1);
        const float4 cs = *(const float4*)(fz.rope_cs + ((size_t)p * (HD / 2) + e0) * 2);
        const bool lo = 2 * lane < HD / 2;
        float2 v[G + 2];
#pragma unroll
        for (int t = 0; t < G + 2; t++) {
            const int h = t < G ? kvh * G + t : t == G ? nh + kvh : nh + nkv + kvh;
            v[t] = *(const float2*)(src + h * HD + 2 * lane);
        }
        const float2 gq = *(const float2*)(fz.qnw + 2 * lane), gk = *(const float2*)(fz.knw + 2 * lane);
#pragma unroll
        for (int t = 0; t < G + 1; t++) {
            const __half2 hv = norm_rope_hd128(v[t], t < G ? gq : gk, cs, lo, fz.eps);
            if (t < G) {
                const float2 back = __half22float2(hv);
                *(float2*)&qs[t * (HD + HD / 4) + 2 * lane + 4 * (lane >> 3)] = make_float2(back.x, back.y);
            } else {
                *(__half2*)(fz.kc + (size_t)sl * kvd + kvh * HD + 2 * lane) = hv;
                kn_all[w][lane] = hv;
            }
        }
        const __half2 vh = __floats2half2_rn(v[G + 1].x, v[G + 1].y);
        *(__half2*)(fz.vc + (size_t)sl * kvd + kvh * HD + 2 * lane) = vh;
        vn_all[w][lane] = vh;
        wave_sync_lds();
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < QD / 2; j++)
                qv[g][j] = (h2v){(_Float16)qs[g * (HD + HD / 4) + sub * (QD + 4) + 2 * j],
                                 (_Float16)qs[g * (HD + HD / 4) + sub * (QD + 4) + 2 * j + 1]};
    } else {
#pragma unroll
        for (int g = 0; g < G; g++) {
            const __half* qp = Q + (size_t)r * ldq + (kvh * G + g) * HD + sub * QD;
#pragma unroll
            for (int j = 0; j < QD / 2; j++) qv[g][j] = *(const h2v*)(qp + 2 * j);
        }
    }
    float m[G], lsum[G], av[G][8];
#pragma unroll
    for (int g = 0; g < G; g++) {
        m[g] = -INFINITY;
        lsum[g] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) av[g][j] = 0.f;
    }
    for (int c0 = 0; c0 < L; c0 += C) {
        const int n = min(C, L - c0);
        if constexpr (FUSED) {
            if (sl_new >= s0 + c0 && sl_new < s0 + c0 + n) {   // this chunk holds the new row: K from LDS
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (s0 + c0 + min(8 * u + kk, n - 1) == sl_new) {
                        ka[u] = *(const int4*)(&kn_all[w][0] + sub * (QD / 2));
                        kb[u] = *(const int4*)(&kn_all[w][0] + sub * (QD / 2) + 4);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int j = 8 * u + kk;
#pragma unroll
            for (int g = 0; g < G; g++) {
                const float p = sum8(qk_dot16(qv[g], ka[u], kb[u]));
                if (sub == 0 && j < n) sp[g][j] = p * scale;
            }
        }
        // the K registers are free: the next chunk's K loads go out now, beside this chunk's V loads
        if (c0 + C < L) load_k(c0 + C);
        int4 vr[8];
        const __half* vc = vbase + (size_t)(s0 + c0) * ldkv;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int j = min(4 * u + vg, n - 1);   // rows past n: weight p = 0
            vr[u] = *(const int4*)(vc + (size_t)j * ldkv);
        }
        wave_sync_lds();
#pragma unroll
        for (int g = 0; g < G; g++) {
            const float x = lane < n ? sp[g][lane] : -INFINITY;
            const float mnew = fmaxf(m[g], wave_max(x));
            const float alpha = expf(m[g] - mnew);
            const float p = lane < n ? expf(x - mnew) : 0.f;
            lsum[g] = fmaf(lsum[g], alpha, wave_sum(p));
            m[g] = mnew;
            if (lane < C) sp[g][lane] = p;
#pragma unroll
            for (int j = 0; j < 8; j++) av[g][j] *= alpha;
        }
        wave_sync_lds();
        if constexpr (FUSED) {
            if (sl_new >= s0 + c0 && sl_new < s0 + c0 + n) {   // the new row's V from LDS
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (s0 + c0 + min(4 * u + vg, n - 1) == sl_new) vr[u] = *(const int4*)(&vn_all[w][0] + vd / 2);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t* hv = (const uint32_t*)&vr[u];
#pragma unroll
            for (int g = 0; g < G; g++) {
                const float p = sp[g][4 * u + vg];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    av[g][2 * t] = fma_mix_lo(p, hv[t], av[g][2 * t]);
                    av[g][2 * t + 1] = fma_mix_hi(p, hv[t], av[g][2 * t + 1]);
                }
            }
        }
        wave_sync_lds();
    }
    const int D = nh * HD;
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int h = kvh * G + g;
        const float inv = L > 0 ? 1.f / lsum[g] : 0.f;
        float out[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float a = av[g][j];
            a += __shfl_xor(a, 16);
            a += __shfl_xor(a, 32);
            out[j] = a * inv;
        }
        // lane (lane & 15) holds dims vd … vd+7: a Q8 block = 32 dims = 4 lanes
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(out[j]));
        amax = fmaxf(amax, __shfl_xor(amax, 1));
        amax = fmaxf(amax, __shfl_xor(amax, 2));
        const float d = amax / 127.f;
        if (lane < 16) {
            uint32_t lo4 = 0, hi4 = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t b = (uint32_t)(uint8_t)(int8_t)(amax == 0.f ? 0 : (int)roundf(out[j] / d));
                if (j < 4) lo4 |= b << (8 * j);
                else hi4 |= b << (8 * (j - 4));
            }
            *(uint2*)(oq + (size_t)r * D + h * HD + vd) = make_uint2(lo4, hi4);
            if ((lane & 3) == 0) od[(size_t)r * (D / 32) + (h * HD + vd) / 32] = __half2float(f2h(d));
        }
    }
}

// the one-wave kernel from this many decode rows (engine's table path; QASR_ATTN_WAVE_ROWS / set_attn_wave_rows,
// 0 = never)
static int g_attn_wave_rows = [] {
    const char* e = getenv("QASR_ATTN_WAVE_ROWS");
    return e ? atoi(e) : 0;
}();
static int attn_wave_rows() { return g_attn_wave_rows; }
void set_attn_wave_rows(int rows) { g_attn_wave_rows = rows < 0 ? 0 : rows; }

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
    // the fused decode kernel's one-wave policy (attention_decode_fused), so the two paths stay bit-identical
    if (HD == 128 && !o && oq && (G == 2 || G == 4) && attn_wave_rows() > 0 && rows >= attn_wave_rows()) {
        if (G == 2)
            k_attn_wave<2, false><<<b1, 256, 0, s>>>(Q, ldq, (__half*)K, (__half*)V, ldkv, kv_start, kv_len, rows, nh,
                                                     nkv, scale, oq, od, QkFuse{});
        else
            k_attn_wave<4, false><<<b1, 256, 0, s>>>(Q, ldq, (__half*)K, (__half*)V, ldkv, kv_start, kv_len, rows, nh,
                                                     nkv, scale, oq, od, QkFuse{});
        return;
    }
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
    if (!fz.part && !fz.fixed_chunk && attn_wave_rows() > 0 && rows >= attn_wave_rows() && (G == 2 || G == 4)) {
        const unsigned b1 = (unsigned)cdiv(rows * nkv, 4);
        if (G == 2)
            k_attn_wave<2, true><<<b1, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                    scale, oq, od, fz);
        else
            k_attn_wave<4, true><<<b1, 256, 0, s>>>(nullptr, 0, fz.kc, fz.vc, ldkv, kv_start, kv_len, rows, nh, nkv,
                                                    scale, oq, od, fz);
        return;
    }
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
