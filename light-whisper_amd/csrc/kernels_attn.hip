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
