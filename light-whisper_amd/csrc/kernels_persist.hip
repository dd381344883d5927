// Persistent decode: the whole decoder stack of a ≤ 32-row decode step (one token for each of up to 32 utterances)
// as ONE launch of about one 256-thread workgroup per CU, gfx950.
//
// Why: at ≤ 32 rows a decode step is a chain of ~8 launches per layer whose kernel times add up to the wall time
// (4,520 RMSNorm launches per 32-segment bench step, ~200 launches per decode iteration, the N = 8 share
// latency-bound).  Here a layer is a sequence of phases inside the launch:
//   N1  RMSNorm + Q8 of each row (one item per row)          → xq / xd
//   QKV exact-row linear (16-column items)                    → qkv f32
//   ATT q/k-norm + RoPE + KV write + attention + Q8 output (items (row, KV head, key-range piece)) → xq / xd
//   O   exact-row linear + residual (16-column items)         → x
//   N2  RMSNorm + Q8                                          → xq / xd
//   GU  exact-row gate/up (64-column items = one h block) + SwiGLU + Q8 → hq / hd
//   D   exact-row down-projection + residual                  → x
// separated by grid-wide waits: every workgroup counts its arrival on one of 8 per-XCD counters (agent-scope add)
// after its stores, and proceeds when the counters sum to the phase's total.  Hand-offs follow MI355X_MICROARCH.md
// (inter-workgroup visibility, table row 1): every handed-off byte stored write-through (sc1, wt.h), the storing waves'
// vmcnt(0), a workgroup barrier, ONE lane's add; the consumer polls with sc1 loads and reads with sc1 loads.
//
// Numerics: every row runs the arithmetic of the 1-row decode step — the same device bodies as the stand-alone
// launches (rms_row_q8_* of rmsnorm_q8 / the GEMV prologue, exact_frag of gemm_exact_rows = k_gemv_wide's 1-row bits,
// attention_rows of the fused split decode attention, swiglu_q8_value of the SwiGLU epilogue), so a row's logits are
// the bits of its own single-utterance step whatever else shares the launch (tests/test_model_real_gpu.py::
// test_real_persistent_decode_*).
//
// Liveness: the waits need every workgroup resident.  The grid is sized by the occupancy query (one per CU), only one
// persistent launch runs at a time per process (engine.cpp), and every wait is bounded: after timeout_ticks (100 MHz)
// the waiting workgroup sets sync[kPersistAbortWord] and every workgroup leaves at its next wait, so the grid always
// drains; the host turns a set abort word into an error.
#include "attn_rows.h"
#include "exact_rows.h"
#include "kernels.h"
#include "rowops.h"
#include "wt.h"
#include "xlane.h"

namespace qasr {

namespace {
constexpr int kSyncStride = 32;                   // words between the per-XCD arrival counters (one 128-B line each)
constexpr int kExitWord = kPersistAbortWord + kSyncStride;
static_assert(kPersistAbortWord == 8 * kSyncStride, "abort word after the 8 counters");
// s_getreg_b32 HW_REG_XCC_ID (id 20, bits 0..15): which XCD this CU sits on (speed only: any counter is correct)
constexpr int kHwRegXccId = 20 | (15 << 11);
}  // namespace

size_t persist_sync_words() { return kExitWord + kSyncStride; }

// End of a phase, part 1: this workgroup's write-through stores are complete; count its arrival.  (The caller may then
// issue the next phase's weight loads — they do not depend on any activation — before grid_wait.)
__device__ __forceinline__ int grid_arrive(const PersistArgs& a, unsigned& target, int tid) {
    __builtin_amdgcn_sched_barrier(0);   // phases are not interleaved by the scheduler (register pressure)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores have completed
    __syncthreads();
    const int wi = (int)(target / gridDim.x);          // this wait's index in the launch
    target += gridDim.x;
    if (tid == 0) {
        if (a.stamps && wi < kPersistMaxWaits)
            a.stamps[((size_t)blockIdx.x * kPersistMaxWaits + wi) * 2] = __builtin_amdgcn_s_memrealtime();
        const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(kHwRegXccId) & 7u;
        __hip_atomic_fetch_add(a.sync + kSyncStride * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return wi;
}

// part 2: wave 0 polls until every workgroup has arrived (or the launch aborted); the workgroup leaves together.
// Returns false (uniformly) on abort.
__device__ __forceinline__ bool grid_wait(const PersistArgs& a, unsigned target, int wi, int* s_ok, int tid) {
    if (tid < 64) {
        const int lane = tid;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        for (;;) {
            unsigned v = 0;
            if (lane < 8) v = __hip_atomic_load(a.sync + kSyncStride * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (lane == 8) v = __hip_atomic_load(a.sync + kPersistAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned sum = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) sum += (unsigned)__builtin_amdgcn_readlane((int)v, i);
            if (sum >= target) break;
            if (__builtin_amdgcn_readlane((int)v, 8) != 0) {
                ok = 0;
                break;
            }
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
                if (lane == 0) __hip_atomic_store(a.sync + kPersistAbortWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) {
            *s_ok = ok;
            if (a.stamps && wi < kPersistMaxWaits)
                a.stamps[((size_t)blockIdx.x * kPersistMaxWaits + wi) * 2 + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    return *s_ok != 0;
}

// rows [r0, r0 + n) of Q8 rows X [*][K] / Xd [*][K/32] written earlier in this launch → the LDS tile (row stride ldx
// bytes; scales with row stride K/32), sc1 loads, 16 chunks of 16 bytes per thread in flight
__device__ __forceinline__ void stage_tile(const int8_t* X, const float* Xd, int K, int r0, int n, int8_t* sX, int ldx,
                                           float* sXd, int tid) {
    const int cpr = K / 16, total = n * cpr;
    const uint32_t base = (uint32_t)r0 * (uint32_t)K;
    for (int c0 = 0; c0 < total; c0 += 256 * 16) {
        xr_v4i v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int c = c0 + 256 * u + tid;
            if (c < total) v[u] = wt_ld16(X, base + 16u * (uint32_t)c);
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const int c = c0 + 256 * u + tid;
            if (c < total) {
                const int row = c / cpr, col = c - row * cpr;
                *(xr_v4i*)(sX + row * ldx + 16 * col) = v[u];
            }
        }
    }
    const int nbr = K / QK, t4 = n * nbr / 4;   // float4 chunks of the scales (nbr % 4 == 0)
    const uint32_t dbase = (uint32_t)r0 * (uint32_t)nbr * 4u;
    for (int c0 = 0; c0 < t4; c0 += 256 * 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = c0 + 256 * u + tid;
            if (c < t4) v[u] = wt_ldf4(Xd, dbase + 16u * (uint32_t)c);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = c0 + 256 * u + tid;
            if (c < t4) *(float4*)(sXd + 4 * c) = v[u];
        }
    }
}

// RMSNorm(x rows [0, R))·w → Q8 into the LDS tile (rmsnorm_q8's arithmetic: rms_row_q8_finish into LDS), eight rows'
// loads in flight at a time; part: [8][4] floats
template <int KC>
__device__ __forceinline__ void norm_tile(const float* x, int H, float eps, int R, const float* w, int8_t* sX, int ldx,
                                          float* sXd, float (*part)[4], int tid) {
    for (int r0 = 0; r0 < R; r0 += 8) {
        float4 v[8][KC], gw[KC];
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (r0 + u < R) rms_row_load<KC, true>(x + (size_t)(r0 + u) * H, H, w, v[u], gw, tid);
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (r0 + u < R)
                rms_row_q8_finish<KC, false>(v[u], gw, H, eps, sX + (r0 + u) * ldx, sXd + (r0 + u) * (H / QK), part[u],
                                             true, tid);
        __syncthreads();   // part reuse
    }
}

// N1 / N2 (rows > kFoldRows): row r's RMSNorm(x)·w → Q8 rows in global memory, write-through
template <int KC>
__device__ __forceinline__ void norm_row(const PersistArgs& a, int r, const float* w, float* part, int tid) {
    float4 v[KC], gw[KC];
    rms_row_load<KC, true>(a.x + (size_t)r * a.H, a.H, w, v, gw, tid);
    rms_row_q8_finish<KC, true>(v, gw, a.H, a.eps, a.xq + (size_t)r * a.H, a.xd + (size_t)r * (a.H / QK), part, true,
                                tid);
}


// the epilogue of an exact-row linear item: rows [row0, row0 + 16·RF) ∩ [row0, rows_end), write-through, + residual
// (rv, read before the compute) when RESID
template <int RF, bool RESID>
__device__ __forceinline__ void item_store(const float (&v)[4], const float (&rv)[4], int row0, int rows_end, int n0,
                                           int N, float* y, int ldy, int tid) {
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wv < RF) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int row = row0 + 16 * wv + 4 * (lane >> 4) + r, col = n0 + (lane & 15);
            if (row < rows_end && col < N) wt_stf(y, (uint32_t)(row * ldy + col) * 4u, RESID ? v[r] + rv[r] : v[r]);
        }
    }
}
template <int RF>
__device__ __forceinline__ void resid_load(float (&rv)[4], int row0, int rows_end, int n0, int N, const float* y,
                                           int ldy, int tid) {
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = row0 + 16 * wv + 4 * (lane >> 4) + r, col = n0 + (lane & 15);
        rv[r] = wv < RF && row < rows_end && col < N ? wt_ldf(y, (uint32_t)(row * ldy + col) * 4u) : 0.f;
    }
}

template <int TH, int TQ, int TF, int RF, int G>
__global__ __launch_bounds__(256, 1) void k_dec_persist(PersistArgs a) {
    // the activation tile: QKV / GU all 16·RF rows × H, O / D 16 rows × QD / F (rows past 16 split over items)
    constexpr int H = 1024 * TH, QD = 1024 * TQ, F = 1024 * TF;
    constexpr int LX_H = H + 16, LX_Q = QD + 16, LX_F = F + 16;
    constexpr int TILE_A = 16 * RF * LX_H + 16 * RF * (H / QK) * 4;
    constexpr int TILE_O = 16 * LX_Q + 16 * (QD / QK) * 4;
    constexpr int TILE_D = 16 * LX_F + 16 * (F / QK) * 4;
    constexpr int TILE = TILE_A > TILE_O ? (TILE_A > TILE_D ? TILE_A : TILE_D) : (TILE_O > TILE_D ? TILE_O : TILE_D);
    __shared__ __align__(16) int8_t tile[TILE];
    __shared__ float hx[4][RF][4][64];
    __shared__ float part[8][4];
    __shared__ float gub[16 * RF][64];                  // a GU item's 64 gate/up outputs per row
    __shared__ __align__(16) int8_t hqb[16 * RF][32];   // its SwiGLU Q8 values
    __shared__ float hdb[16 * RF];
    __shared__ int s_ok;
    __shared__ int pre[33];                             // attention items before row r (pieces × KV heads)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int R = a.R, nkv = a.nkv;
    const int KD = nkv * 128, NQKV = QD + 2 * KD;
    const int gsz = gridDim.x, b = blockIdx.x;
    // norms inside the QKV / GU phases (every workgroup normalises all rows from x into its own tile: no norm phase,
    // no grid wait) up to fold_rows rows, else as phases of their own
    const bool fold = R <= a.fold_rows;
    // O / D items: 16-column fragments × row halves (rows > 16: 2 halves, so all workgroups have an item)
    const int halves = R > 16 ? 2 : 1;
    const int nQ = NQKV / 16, nO = (H / 16) * halves, nG = F / 32, nD = (H / 16) * halves;
    unsigned target = 0;
    int wi = 0;

    // the attention's work list (fixed for the launch: every layer attends the same key ranges): row r has S_r
    // pieces of its key range (attention_rows' split rule), items (r, piece, KV head) numbered row-major
    if (tid < 64) {
        int S = 0;
        if (lane < R) {
            const int L = a.kvl[lane];
            S = 1;
            if (a.apart && L > a.split_min) S = min(kAttnSplitMax, (L + a.split_keys - 1) / a.split_keys);
        }
        int inc = S * nkv;   // inclusive scan over the 32 rows (lanes ≥ R hold 0)
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            const int t = __shfl_up(inc, o);
            if (lane >= o) inc += t;
        }
        if (lane < 32) pre[lane + 1] = inc;
        if (lane == 0) pre[0] = 0;
    }
    __syncthreads();
    const int n_att = pre[R];

    // this workgroup's first item of each phase is loaded into registers a phase ahead, before the grid wait (the
    // weights depend on no activation).  wq crosses the layer loop's back edge, so its load is unconditional (a
    // clamped item where the workgroup has none): a conditional load would keep the previous value live all round.
    XWeights<TH> wq;
    exact_load_w<TH>(wq, a.layers[0].qkv_q, a.layers[0].qkv_s, NQKV, H, 16 * min(b, nQ - 1), tid);

    for (int l = 0; l < a.n_layers; l++) {
        // the thread index as a value the compiler cannot hoist out of this loop: every per-lane address below is
        // recomputed per layer instead of being kept live across the whole loop (it spilled at 512 registers)
        int tl = tid;
        asm volatile("" : "+v"(tl) : "s"(l));
        const PersistLayer Ly = a.layers[l];
        __half* kc = a.kc + (size_t)l * a.layer_kv;
        __half* vc = a.vc + (size_t)l * a.layer_kv;
        int8_t* sX = tile;
        XWeights<TQ> wo;     // (declared per layer: their values never cross the back edge)
        XWeights<TH> wg[4];
        XWeights<TF> wd;
        // ---- N1 (many rows) or its fold into QKV
        if (!fold) {
            for (int r = b; r < R; r += gsz) {
                norm_row<TH>(a, r, Ly.attn_norm, part[0], tl);
                __syncthreads();
            }
            wi = grid_arrive(a, target, tl);
            if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        }
        // ---- QKV
        if (b < nQ) {
            float* sXd = (float*)(tile + 16 * RF * LX_H);
            if (fold) norm_tile<TH>(a.x, H, a.eps, R, Ly.attn_norm, sX, LX_H, sXd, part, tl);
            else stage_tile(a.xq, a.xd, H, 0, R, sX, LX_H, sXd, tl);
            __syncthreads();
            // (the first item on the prefetched weights, further ones — fewer CUs than items — on their own: one
            // weight variable per path, no merge of two 40–160-register values)
            auto q_item = [&](int it, const XWeights<TH>& w) {
                float v[4], rv[4];
                exact_frag_lds<TH, RF>(w, sX, LX_H, sXd, R, hx, v, tl);
                item_store<RF, false>(v, rv, 0, R, 16 * it, NQKV, a.qkv, NQKV, tl);
                __syncthreads();
            };
            q_item(b, wq);
            for (int it = b + gsz; it < nQ; it += gsz) {
                XWeights<TH> w2;
                exact_load_w<TH>(w2, Ly.qkv_q, Ly.qkv_s, NQKV, H, 16 * it, tl);
                q_item(it, w2);
            }
        }
        wi = grid_arrive(a, target, tl);
        if (b < nO) exact_load_w<TQ>(wo, Ly.o_q, Ly.o_s, H, QD, 16 * (b % (H / 16)), tl);
        if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        // ---- ATT
        {
            QkFuse fz{a.qkv, a.pos, a.slot, Ly.q_norm, Ly.k_norm, a.rope_cs, a.eps, kc, vc};
            fz.part = a.apart;
            fz.cnt = a.acnt;
            fz.part_rows = a.part_rows;
            fz.fixed_chunk = true;
            fz.split_min = a.split_min;
            fz.split_keys = a.split_keys;
            for (int it = b; it < n_att; it += gsz) {
                int r = 0;
                while (pre[r + 1] <= it) r++;   // uniform
                const int k = it - pre[r], piece = k / nkv, kvh = k - piece * nkv;
                const unsigned bid = a.apart ? (unsigned)(piece * (R * nkv) + r * nkv + kvh) : (unsigned)(r * nkv + kvh);
                attention_rows<128, G, 4, true, 64, true>(bid, tl, nullptr, 0, kc, vc, KD, a.kvs, a.kvl, R, a.nh, nkv,
                                                          a.scale, nullptr, a.xq, a.xd, fz);
                __syncthreads();   // waves 1-3 may have left the body early; LDS reuse
            }
        }
        wi = grid_arrive(a, target, tl);
        if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        // ---- O + residual: item = (16-column fragment, row half)
        {
            auto o_item = [&](int it, const XWeights<TQ>& w) {
                const int fi = it % (H / 16), r0 = 16 * (it / (H / 16)), rn = min(16, R - r0);
                float* sXd = (float*)(tile + 16 * LX_Q);
                float rv[4], v[4];
                resid_load<1>(rv, r0, R, 16 * fi, H, a.x, H, tl);
                stage_tile(a.xq, a.xd, QD, r0, rn, sX, LX_Q, sXd, tl);
                __syncthreads();
                exact_frag_lds<TQ, 1>(w, sX, LX_Q, sXd, rn, (float(*)[1][4][64])hx, v, tl);
                item_store<1, true>(v, rv, r0, R, 16 * fi, H, a.x, H, tl);
                __syncthreads();
            };
            if (b < nO) o_item(b, wo);
            for (int it = b + gsz; it < nO; it += gsz) {
                XWeights<TQ> w2;
                exact_load_w<TQ>(w2, Ly.o_q, Ly.o_s, H, QD, 16 * (it % (H / 16)), tl);
                o_item(it, w2);
            }
        }
        wi = grid_arrive(a, target, tl);
        if (b < nG)   // (fragments 0-1 ahead; 2-3 at the phase start — all four ahead spilled)
#pragma unroll
            for (int c = 0; c < 2; c++) exact_load_w<TH>(wg[c], Ly.gu_q, Ly.gu_s, 2 * F, H, 64 * b + 16 * c, tl);
        if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        // ---- N2 (many rows)
        if (!fold) {
            for (int r = b; r < R; r += gsz) {
                norm_row<TH>(a, r, Ly.ffn_norm, part[0], tl);
                __syncthreads();
            }
            wi = grid_arrive(a, target, tl);
            if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        }
        // ---- GU + SwiGLU + Q8: item = one 32-wide h block = 64 interleaved gate/up columns (4 fragments)
        if (b < nG) {
#pragma unroll
            for (int c = 2; c < 4; c++) exact_load_w<TH>(wg[c], Ly.gu_q, Ly.gu_s, 2 * F, H, 64 * b + 16 * c, tl);
            float* sXd = (float*)(tile + 16 * RF * LX_H);
            if (fold) norm_tile<TH>(a.x, H, a.eps, R, Ly.ffn_norm, sX, LX_H, sXd, part, tl);
            else stage_tile(a.xq, a.xd, H, 0, R, sX, LX_H, sXd, tl);
            __syncthreads();
            auto g_item = [&](int it, const XWeights<TH>(&w)[4]) {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    float v[4];
                    exact_frag_lds<TH, RF>(w[c], sX, LX_H, sXd, R, hx, v, tl);
                    if ((tl >> 6) < RF) {
#pragma unroll
                        for (int r = 0; r < 4; r++)
                            gub[16 * (tl >> 6) + 4 * ((tl & 63) >> 4) + r][16 * c + (tl & 15)] = v[r];
                    }
                    __syncthreads();
                }
                // SwiGLU of row m on the 32-lane group m % 8 (swiglu_q8_block's arithmetic)
                const int grp = tl >> 5, j = tl & 31;
                for (int m = grp; m < 16 * RF; m += 8) {   // every lane of the group active (max over 32 lanes)
                    float dq;
                    const int q = swiglu_q8_value(gub[m], j, dq);
                    hqb[m][j] = (int8_t)q;
                    if (j == 0) hdb[m] = dq;
                }
                __syncthreads();
                if (tl < R * 8) {
                    const int m = tl >> 3, w4 = tl & 7;
                    wt_st32(a.hq, (uint32_t)(m * F + 32 * it + 4 * w4), ((const int32_t*)hqb[m])[w4]);
                }
                if (tl < R) wt_stf(a.hd, (uint32_t)(tl * (F / QK) + it) * 4u, hdb[tl]);
                __syncthreads();
            };
            g_item(b, wg);
            for (int it = b + gsz; it < nG; it += gsz) {
                XWeights<TH> w2[4];
#pragma unroll
                for (int c = 0; c < 4; c++) exact_load_w<TH>(w2[c], Ly.gu_q, Ly.gu_s, 2 * F, H, 64 * it + 16 * c, tl);
                g_item(it, w2);
            }
        }
        wi = grid_arrive(a, target, tl);
        // (the first half of the spans ahead, the rest at the phase start: all of them ahead spilled at 1.7B)
        if (b < nD) exact_load_w<TF, 0, 2 * TF>(wd, Ly.dn_q, Ly.dn_s, H, F, 16 * (b % (H / 16)), tl);
        if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        // ---- D + residual: item = (16-column fragment, row half)
        {
            auto d_item = [&](int it, const XWeights<TF>& w) {
                const int fi = it % (H / 16), r0 = 16 * (it / (H / 16)), rn = min(16, R - r0);
                float* sXd = (float*)(tile + 16 * LX_F);
                float rv[4], v[4];
                resid_load<1>(rv, r0, R, 16 * fi, H, a.x, H, tl);
                stage_tile(a.hq, a.hd, F, r0, rn, sX, LX_F, sXd, tl);
                __syncthreads();
                exact_frag_lds<TF, 1>(w, sX, LX_F, sXd, rn, (float(*)[1][4][64])hx, v, tl);
                item_store<1, true>(v, rv, r0, R, 16 * fi, H, a.x, H, tl);
                __syncthreads();
            };
            if (b < nD) {
                exact_load_w<TF, 2 * TF, 4 * TF>(wd, Ly.dn_q, Ly.dn_s, H, F, 16 * (b % (H / 16)), tl);
                d_item(b, wd);
            }
            for (int it = b + gsz; it < nD; it += gsz) {
                XWeights<TF> w2;
                exact_load_w<TF>(w2, Ly.dn_q, Ly.dn_s, H, F, 16 * (it % (H / 16)), tl);
                d_item(it, w2);
            }
        }
        if (l + 1 < a.n_layers) {
            wi = grid_arrive(a, target, tl);
            exact_load_w<TH>(wq, a.layers[l + 1].qkv_q, a.layers[l + 1].qkv_s, NQKV, H, 16 * min(b, nQ - 1), tl);
            if (!grid_wait(a, target, wi, &s_ok, tl)) return;
        }
    }
    // every workgroup is past its last wait once it counts here: the last one resets the counters for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.sync + kExitWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)gsz - 1) {
#pragma unroll
            for (int i = 0; i < 8; i++) __hip_atomic_store(a.sync + kSyncStride * i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sync + kExitWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------------------ per-phase launches
// The persistent kernel's item bodies as plain launches (a kernel boundary instead of a grid wait): the ≤ 32-row decode
// linears with exact-row arithmetic (bit-identical to the 1-row GEMV step and to gemm_exact_rows), every weight span
// of a workgroup's fragment(s) loaded at its start, the activation rows staged once into LDS (or, FOLD, normalised
// there from x: rmsnorm_q8's arithmetic — no separate norm launch).  One workgroup per CU (512 registers).
//   k_xr_linear: a 16-column fragment × the rows of blockIdx.y's slice (16·RF rows), + residual (RESID)
//   k_xr_gu:     one h block = 64 interleaved gate/up columns (4 fragments) + SwiGLU + Q8
// The residual launches' fused RMSNorm (XrNorm::w != nullptr; the output rows are whole rows of H = N): once every
// workgroup has stored its columns (write-through, counted on cnt[0]), the last R workgroups to arrive wait
// for the count to reach the grid and normalise the rows into q / d — rmsnorm_q8's arithmetic on the finished rows,
// so the next launch needs no norm launch of its own.  The grid (≤ 256 workgroups, one per CU) is resident as a
// whole, so the wait ends; it is bounded anyway (cnt[2] = 1 flags a timeout, the engine checks it).  cnt[1] counts
// the finished norm workgroups; the last one leaves cnt[0..1] zero for the next launch.
template <int KC>
__device__ __forceinline__ void xr_norm_tail(const XrNorm& nm, const float* x, int H, int R, float* part, int tid) {
    __shared__ int s_prev;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores of x have completed
    __syncthreads();
    const unsigned G = gridDim.x * gridDim.y;
    if (tid == 0) s_prev = (int)__hip_atomic_fetch_add(nm.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int NL = R, k = s_prev - (int)(G - (unsigned)NL);   // one row per norm workgroup (8 rows each: slower than a launch)
    if (k < 0) return;   // uniform: not one of the norm workgroups
    if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(nm.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // 0.2 s: never, with the grid resident
                __hip_atomic_store(nm.cnt + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    for (int r = k; r < R; r += NL) {
        float4 v[KC], gw[KC];
        rms_row_load<KC, true>(x + (size_t)r * H, H, nm.w, v, gw, tid);
        rms_row_q8_finish<KC, false>(v, gw, H, nm.eps, nm.q + (size_t)r * H, nm.d + (size_t)r * (H / QK), part, true,
                                     tid);
        __syncthreads();
    }
    if (tid == 0) {
        const unsigned d = __hip_atomic_fetch_add(nm.cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == (unsigned)NL - 1) {   // every norm workgroup is past its wait
            __hip_atomic_store(nm.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(nm.cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int T, int RF, bool FOLD, bool RESID, int XS = 1>
__global__ __launch_bounds__(256, 1) void k_xr_linear(const int8_t* X, const float* Xd, const float* src,
                                                      const float* nw, float eps, int R, const int8_t* Wq,
                                                      const __half* Ws, int N, float* y, int ldy, XrNorm nm,
                                                      XrSplit xs) {
    constexpr int K = 1024 * T, LX = K + 16;
    __shared__ __align__(16) int8_t tile[16 * RF * LX + 16 * RF * (K / QK) * 4];
    __shared__ float hx[4][RF][4][64];
    __shared__ float part[8][4];
    __shared__ unsigned s_prev;
    const int tid = threadIdx.x;
    // XS = 2: blockIdx.x = 2·fragment + half (the halves of a fragment are neighbours, dispatched together)
    const int half = XS == 2 ? (int)(blockIdx.x & 1) : 0, frag = XS == 2 ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const int n0 = 16 * frag, r0 = 16 * RF * blockIdx.y, rn = min(16 * RF, R - r0);
    XWeights<T, XS> w;
    exact_load_w<T, 0, 4 * T / XS, XS>(w, Wq, Ws, N, K, n0, tid, half);
    float rv[4] = {0.f, 0.f, 0.f, 0.f}, v[4];
    if (RESID) resid_load<RF>(rv, r0, R, n0, N, y, ldy, tid);
    float* sXd = (float*)(tile + 16 * RF * LX);
    if constexpr (FOLD) norm_tile<T>(src + (size_t)r0 * K, K, eps, rn, nw, tile, LX, sXd, part, tid);
    else stage_tile(X, Xd, K, r0, rn, tile, LX, sXd, tid);
    __syncthreads();
    exact_frag_lds<T, RF, XS>(w, tile, LX, sXd, rn, hx, v, tid, half);
    if constexpr (XS == 2) {
        // hand-off (MI355X_MICROARCH.md inter-workgroup visibility, table row 1): this half's tree stored write-through,
        // the storing waves' vmcnt(0), a barrier, one agent-scope add; the second to arrive reads the first's with sc1
        // loads and adds the two in half order
        const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int item = frag * (int)gridDim.y + (int)blockIdx.y;
        float* pp = xs.part + (size_t)item * 2 * (RF * 256);
        if (wv < RF) {
#pragma unroll
            for (int r = 0; r < 4; r++) wt_stf(pp, (uint32_t)(((half * RF + wv) * 4 + r) * 64 + lane) * 4u, v[r]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) s_prev = __hip_atomic_fetch_add(xs.cnt + item, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (s_prev == 0) return;   // uniform: the first half to arrive is done
        if (tid == 0) __hip_atomic_store(xs.cnt + item, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
        if (wv < RF) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float o = wt_ldf(pp, (uint32_t)((((1 - half) * RF + wv) * 4 + r) * 64 + lane) * 4u);
                v[r] = half == 0 ? v[r] + o : o + v[r];
            }
        }
    }
    item_store<RF, RESID>(v, rv, r0, R, n0, N, y, ldy, tid);
    if constexpr (RESID) {
        if (nm.w) {   // uniform
            if (N == 1024) xr_norm_tail<1>(nm, y, N, R, part[0], tid);
            else xr_norm_tail<2>(nm, y, N, R, part[0], tid);
        }
    }
}

template <int T, int RF, bool FOLD>
__global__ __launch_bounds__(256, 1) void k_xr_gu(const int8_t* X, const float* Xd, const float* src, const float* nw,
                                                  float eps, int R, const int8_t* Wq, const __half* Ws, int F,
                                                  int8_t* hq, float* hd) {
    constexpr int K = 1024 * T, LX = K + 16;
    __shared__ __align__(16) int8_t tile[16 * RF * LX + 16 * RF * (K / QK) * 4];
    __shared__ float hx[4][RF][4][64];
    __shared__ float part[8][4];
    __shared__ float gub[16 * RF][64];
    __shared__ __align__(16) int8_t hqb[16 * RF][32];
    __shared__ float hdb[16 * RF];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int it = blockIdx.x;
    XWeights<T> w[4];
#pragma unroll
    for (int c = 0; c < 4; c++) exact_load_w<T>(w[c], Wq, Ws, 2 * F, K, 64 * it + 16 * c, tid);
    float* sXd = (float*)(tile + 16 * RF * LX);
    if constexpr (FOLD) norm_tile<T>(src, K, eps, R, nw, tile, LX, sXd, part, tid);
    else stage_tile(X, Xd, K, 0, R, tile, LX, sXd, tid);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++) {
        float v[4];
        exact_frag_lds<T, RF>(w[c], tile, LX, sXd, R, hx, v, tid);
        if (wv < RF) {
#pragma unroll
            for (int r = 0; r < 4; r++) gub[16 * wv + 4 * (lane >> 4) + r][16 * c + (lane & 15)] = v[r];
        }
        __syncthreads();
    }
    const int grp = tid >> 5, j = tid & 31;   // row m on the 32-lane group m % 8 (swiglu_q8_block's arithmetic)
    for (int m = grp; m < 16 * RF; m += 8) {
        float dq;
        const int q = swiglu_q8_value(gub[m], j, dq);
        hqb[m][j] = (int8_t)q;
        if (j == 0) hdb[m] = dq;
    }
    __syncthreads();
    if (tid < R * 8) {
        const int m = tid >> 3, w4 = tid & 7;
        ((int32_t*)(hq + (size_t)m * F + 32 * it))[w4] = ((const int32_t*)hqb[m])[w4];
    }
    if (tid < R) hd[(size_t)tid * (F / QK) + it] = hdb[tid];
}

bool xr_ok(int R, int K) { return R >= 1 && R <= 32 && (K == 1024 || K == 2048 || K == 3072 || K == 6144); }

size_t xr_split_bytes() { return (size_t)kXrSplitItems * (2 * 2 * 256 * sizeof(float) + sizeof(unsigned)); }

// QASR_XR_SPLIT=0 turns the leaf split off (A/B)
static bool xr_split_on() {
    static const bool on = !(getenv("QASR_XR_SPLIT") && atoi(getenv("QASR_XR_SPLIT")) == 0);
    return on;
}

void xr_linear(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps, int R, const Q8Mat& W,
               float* y, int ldy, bool resid, hipStream_t s, const XrNorm* norm, const XrSplit* split) {
    const bool fold = src != nullptr;
    ProfScope ps(s, fold ? "xr_linear_rms" : "xr_linear", 2.0 * R * W.N * W.K,
                 (double)W.N * W.K * (1.0 + 2.0 / 32) + (double)R * W.K * (fold ? 4.0 : 1.125) +
                     (double)R * W.N * 4.0 * (resid ? 2 : 1));
    QASR_CHECK(xr_ok(R, W.K) && W.N % 16 == 0 && (!fold || (R <= 8 && nw)), QASR_E_INVALID,
               "xr_linear: rows 1-32 (fold: ≤ 8), K 1,024 / 2,048 / 3,072 / 6,144");
    QASR_CHECK(!norm || (resid && ldy == W.N && (W.N == 1024 || W.N == 2048) && norm->w && norm->q && norm->d &&
                         norm->cnt),
               QASR_E_INVALID, "xr_linear: the fused norm needs whole residual rows of 1,024 / 2,048");
    const XrNorm nm = norm ? *norm : XrNorm{};
    // rows > 16: two 16-row slices (one row fragment each) where a 32-row tile would not fit LDS (K 6,144), else one
    // 32-row slice
    const bool two = R > 16 && W.K > 3072;
    const int rf = R > 16 && !two ? 2 : 1;
    // the leaf split (two workgroups per fragment) where one per fragment leaves CUs idle and the doubled grid is
    // still resident at once (LDS: the activation tile bounds the workgroups per CU), on the long-K projection only:
    // down (K 6,144) 11.5 / 12.8 → 9.5 / 10.8 µs at 8 / 16 rows, but QKV and O (K 2,048) 5.5 / 5.5 → 7.5 / 7.0 µs at
    // 8 rows — there the hand-off's round trip costs more than the halved weight stream saves (profiles/
    // r5_xr_cost_split.log)
    const int slices = two ? 2 : 1, items = W.N / 16 * slices;
    const size_t lds = (size_t)16 * rf * (W.K + 16) + (size_t)16 * rf * (W.K / QK) * 4 + 8192;
    const int per_cu = (int)std::min<size_t>(2, 160 * 1024 / lds);
    const bool xs2 = split && split->part && split->cnt && !norm && !fold && W.K > 3072 && items <= split->items &&
                     items < 256 * per_cu && 2 * items <= 256 * per_cu && xr_split_on();
    const XrSplit xsp = xs2 ? *split : XrSplit{};
    const dim3 g(W.N / 16 * (xs2 ? 2 : 1), slices);
#define XR_GO(TT, RFF, FF, RR)                                                                                        \
    do {                                                                                                              \
        if (xs2 && !FF)                                                                                               \
            k_xr_linear<TT, RFF, FF, RR, 2><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, W.N, y, ldy, nm,   \
                                                              xsp);                                                   \
        else                                                                                                          \
            k_xr_linear<TT, RFF, FF, RR><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, W.N, y, ldy, nm, xsp); \
    } while (0)
#define XR_RF(TT, FF, RR)                      \
    do {                                       \
        if (rf == 2) XR_GO(TT, 2, FF, RR);     \
        else XR_GO(TT, 1, FF, RR);             \
    } while (0)
#define XR_T(FF, RR)                                        \
    do {                                                    \
        switch (W.K) {                                      \
            case 1024: XR_RF(1, FF, RR); break;             \
            case 2048: XR_RF(2, FF, RR); break;             \
            case 3072: XR_RF(3, FF, RR); break;             \
            default: XR_GO(6, 1, FF, RR); break;            \
        }                                                   \
    } while (0)
    if (fold) {
        QASR_CHECK(W.K <= 2048 && !resid, QASR_E_INVALID, "xr_linear: the norm fold is for the QKV input (K ≤ 2,048)");
        if (W.K == 1024) XR_GO(1, 1, true, false);
        else XR_GO(2, 1, true, false);
    } else if (resid) {
        XR_T(false, true);
    } else {
        XR_T(false, false);
    }
#undef XR_T
#undef XR_RF
#undef XR_GO
    QASR_HIP(hipGetLastError());
}

void xr_gu_swiglu(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps, int R,
                  const Q8Mat& W, int8_t* hq, float* hd, hipStream_t s) {
    const bool fold = src != nullptr;
    ProfScope ps(s, fold ? "xr_gu_rms" : "xr_gu", 2.0 * R * W.N * W.K,
                 (double)W.N * W.K * (1.0 + 2.0 / 32) + (double)R * W.K * (fold ? 4.0 : 1.125) + R * W.N * 0.5625);
    QASR_CHECK(xr_ok(R, W.K) && W.K <= 2048 && W.N % 64 == 0 && (!fold || (R <= 8 && nw)), QASR_E_INVALID,
               "xr_gu_swiglu: rows 1-32 (fold: ≤ 8), K 1,024 / 2,048, interleaved gate/up");
    const int F = W.N / 2;
    const dim3 g(F / 32);
    if (W.K == 1024) {
        if (fold) k_xr_gu<1, 1, true><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
        else if (R <= 16) k_xr_gu<1, 1, false><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
        else k_xr_gu<1, 2, false><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
    } else {
        if (fold) k_xr_gu<2, 1, true><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
        else if (R <= 16) k_xr_gu<2, 1, false><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
        else k_xr_gu<2, 2, false><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd);
    }
    QASR_HIP(hipGetLastError());
}

namespace {
typedef void (*PersistKernel)(PersistArgs);
template <int TH, int TQ, int TF>
PersistKernel pick_rf(int R) {
    return R <= 16 ? k_dec_persist<TH, TQ, TF, 1, 2> : k_dec_persist<TH, TQ, TF, 2, 2>;
}
PersistKernel pick(int H, int F, int nh, int R) {
    const int TH = H / 1024, TQ = nh * 128 / 1024, TF = F / 1024;
    if (R < 1 || R > 32 || TQ != 2) return nullptr;
    if (TH == 1 && TF == 3) return pick_rf<1, 2, 3>(R);   // qwen3-asr-0.6b
    if (TH == 2 && TF == 6) return pick_rf<2, 2, 6>(R);   // qwen3-asr-1.7b
    return nullptr;
}
}  // namespace

bool persist_supported(int H, int F, int nh, int nkv, int hd) {
    return hd == 128 && nkv > 0 && nh == 2 * nkv && H % 1024 == 0 && F % 1024 == 0 && pick(H, F, nh, 1) != nullptr;
}

int persist_grid(int H, int F, int nh, int nkv, int R) {
    PersistKernel k = pick(H, F, nh, R);
    if (!k || nh != 2 * nkv) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k), 256, 0) != hipSuccess)
        return 0;
    return per_cu >= 1 ? cus : 0;   // one workgroup per CU: every grid wait needs all of them resident
}

void decoder_persistent(const PersistArgs& a, hipStream_t s) {
    const double QD = a.nh * 128.0, KD = a.nkv * 128.0;
    const double wbytes = (double)a.n_layers * ((QD + 2 * KD) * a.H + a.H * QD + 2.0 * a.F * a.H + a.H * (double)a.F) *
                          (1.0 + 2.0 / 32);
    ProfScope ps(s, "dec_persist", 2.0 * a.R * wbytes / (1.0 + 2.0 / 32), wbytes);
    PersistKernel k = pick(a.H, a.F, a.nh, a.R);
    QASR_CHECK(k && a.nh == 2 * a.nkv && a.grid > 0, QASR_E_INVALID, "decoder_persistent: unsupported shape");
    QASR_CHECK(a.R <= 32 && (!a.apart || (a.acnt && a.R <= a.part_rows)), QASR_E_INVALID,
               "decoder_persistent: rows or split-attention scratch");
    hipLaunchKernelGGL(k, dim3(a.grid), dim3(256), 0, s, a);
    QASR_HIP(hipGetLastError());
}

}  // namespace qasr
