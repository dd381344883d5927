// The ≤ 32-row decode linears as exact-row launches (k_xr_linear, k_xr_gu), gfx950: every row with the arithmetic of
// the 1-row decode step (exact_frag = k_gemv_wide's 1-row bits, shared with gemm_exact_rows through exact_rows.h), the
// workgroup's weight spans loaded at its start, the rows' Q8 activations staged once into LDS.
//
// (Round 5 also built the whole ≤ 32-row decoder stack as ONE persistent launch over these bodies; bit-identical but
// 0.56× the launch chain — DESIGN §10 keeps its measurements — so round 6 removed it from libqasr.)
#include <algorithm>

#include "exact_rows.h"
#include "kernels.h"
#include "rowops.h"
#include "wt.h"
#include "xlane.h"

namespace qasr {

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
    const int nbr = K / QK, t4 = n * nbr / 4, c4 = nbr / 4;   // float4 chunks of the scales (nbr % 4 == 0)
    const int sds = xr_sd_stride(K);                             // the tile's padded scale row stride
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
            if (c < t4) {
                const int row = c / c4, col = c - row * c4;
                *(float4*)(sXd + row * sds + 4 * col) = v[u];
            }
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
                rms_row_q8_finish<KC, false>(v[u], gw, H, eps, sX + (r0 + u) * ldx, sXd + (r0 + u) * xr_sd_stride(H), part[u],
                                             true, tid);
        __syncthreads();   // part reuse
    }
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

// ------------------------------------------------------------------------------------------------ per-phase launches
// The ≤ 32-row decode linears with exact-row arithmetic (bit-identical to the 1-row GEMV step and to gemm_exact_rows), every weight span
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
    __shared__ __align__(16) int8_t tile[16 * RF * LX + 16 * RF * xr_sd_stride(K) * 4];
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
        float* pp = xs.part + (size_t)item * kXrSplitPart;
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
    __shared__ __align__(16) int8_t tile[16 * RF * LX + 16 * RF * xr_sd_stride(K) * 4];
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

// The vocabulary projection of a 5–16-row decode step (N 151,936 at both sizes) with the exact-row arithmetic: a
// workgroup stages the rows' Q8 activations into LDS ONCE and then walks fragments f, f + G, f + 2G, … (G = the grid,
// every workgroup resident), the next fragment's weight spans loaded into the other register set while this one's
// exact_frag runs — one launch streams the 155 MB matrix with every CU busy, where one launch of a workgroup per
// 16-column fragment re-staged the activation tile 9,496 times (k_gemm_q8_exact 97–111 µs at 5–16 rows) and the table
// GEMM took 79–86 µs; this: 72–74 µs, the 1-row GEMV's bits per row (profiles/r6n_lmhead_cost.log).  17–32 rows stay on
// the table / exact kernels: the exact fragment is latency-bound per workgroup, so two 16-row slices per fragment
// took 136–151 µs against the table's 83–93 (a three-deep weight ring changed nothing: it is not the weight stream).
__device__ __forceinline__ void vocab_store(const float (&v)[4], int R, int n0, int N, float* y, int ldy, int tid) {
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (wv == 0) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int row = 4 * (lane >> 4) + r, col = n0 + (lane & 15);
            if (row < R && col < N) y[(size_t)row * ldy + col] = v[r];
        }
    }
}

template <int T>
__global__ __launch_bounds__(256) void k_xr_vocab(const int8_t* X, const float* Xd, int R, const int8_t* Wq,
                                                  const __half* Ws, int N, float* y, int ldy) {
    constexpr int K = 1024 * T, LX = K + 16;
    __shared__ __align__(16) int8_t tile[16 * LX + 16 * xr_sd_stride(K) * 4];
    __shared__ float hx[4][1][4][64];
    const int tid = threadIdx.x, nfrag = N / 16, G = (int)gridDim.x;
    float* sXd = (float*)(tile + 16 * LX);
    XWeights<T> w0, w1;   // alternated by unrolling (a runtime-indexed pair would go to scratch)
    int f = blockIdx.x;
    if (f < nfrag) exact_load_w<T>(w0, Wq, Ws, N, K, 16 * f, tid);
    stage_tile(X, Xd, K, 0, R, tile, LX, sXd, tid);
    __syncthreads();
    float v[4];
    while (f < nfrag) {
        int fn = f + G;
        if (fn < nfrag) exact_load_w<T>(w1, Wq, Ws, N, K, 16 * fn, tid);
        exact_frag_lds<T, 1>(w0, tile, LX, sXd, R, hx, v, tid);
        vocab_store(v, R, 16 * f, N, y, ldy, tid);
        __syncthreads();   // hx is reused by the next fragment's exchange
        f = fn;
        if (f >= nfrag) break;
        fn = f + G;
        if (fn < nfrag) exact_load_w<T>(w0, Wq, Ws, N, K, 16 * fn, tid);
        exact_frag_lds<T, 1>(w1, tile, LX, sXd, R, hx, v, tid);
        vocab_store(v, R, 16 * f, N, y, ldy, tid);
        __syncthreads();
        f = fn;
    }
}

bool xr_vocab_ok(int R, int K, int N) { return R >= 1 && R <= 16 && (K == 1024 || K == 2048) && N % 16 == 0; }

void xr_vocab(const int8_t* xq, const float* xd, int R, const Q8Mat& W, float* y, int ldy, hipStream_t s) {
    ProfScope ps(s, "xr_vocab", 2.0 * R * W.N * W.K, (double)W.N * W.K * (1.0 + 2.0 / 32) + (double)R * W.K * 1.125 +
                                                          (double)R * W.N * 4.0);
    QASR_CHECK(xr_vocab_ok(R, W.K, W.N) && ldy >= W.N, QASR_E_INVALID,
               "xr_vocab: rows 1-16, K 1,024 / 2,048, N % 16 == 0");
    typedef void (*VocabKernel)(const int8_t*, const float*, int, const int8_t*, const __half*, int, float*, int);
    const VocabKernel k = W.K == 1024 ? k_xr_vocab<1> : k_xr_vocab<2>;
    // the grid: every workgroup resident at once (the occupancy query per instantiation: a persistent walk with more
    // workgroups than slots would run its second half after the first)
    static int cus = 0, occ[2] = {0, 0};
    const int ki = W.K == 1024 ? 0 : 1;
    if (!cus) {
        int dev = 0;
        QASR_HIP(hipGetDevice(&dev));
        QASR_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (!occ[ki]) {
        int per_cu = 0;
        QASR_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k), 256, 0));
        occ[ki] = std::max(1, std::min(per_cu, 2));
    }
    const int g = std::min(W.N / 16, occ[ki] * cus);
    hipLaunchKernelGGL(k, dim3(g), dim3(256), 0, s, xq, xd, R, W.qs, W.sc, W.N, y, ldy);
    QASR_HIP(hipGetLastError());
}

bool xr_ok(int R, int K) { return R >= 1 && R <= 32 && (K == 1024 || K == 2048 || K == 3072 || K == 6144); }

size_t xr_split_bytes() { return (size_t)kXrSplitItems * (kXrSplitPart * sizeof(float) + sizeof(unsigned)); }

XrSplit xr_split_view(void* mem) {
    XrSplit v;
    v.part = (float*)mem;
    v.cnt = (unsigned*)((char*)mem + (size_t)kXrSplitItems * kXrSplitPart * sizeof(float));
    v.items = kXrSplitItems;
    return v;
}

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
    const size_t lds = (size_t)16 * rf * (W.K + 16) + (size_t)16 * rf * xr_sd_stride(W.K) * 4 + 8192;
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
    // (round 6: a leaf split like k_xr_linear's — two workgroups per h block, half the leaves each, the second adding
    // the first's values — measured slower at every row count: 17.1 / 29.2 / 30.7 against 15.7 / 19.0 / 19.3 µs at
    // 16 / 24 / 32 rows, profiles/r6h_xr_cost.log: both halves stage the whole activation tile)
#define XR_GU(TT, RFF, FF) k_xr_gu<TT, RFF, FF><<<g, 256, 0, s>>>(xq, xd, src, nw, eps, R, W.qs, W.sc, F, hq, hd)
    if (W.K == 1024) {
        if (fold) XR_GU(1, 1, true);
        else if (R <= 16) XR_GU(1, 1, false);
        else XR_GU(1, 2, false);
    } else {
        if (fold) XR_GU(2, 1, true);
        else if (R <= 16) XR_GU(2, 1, false);
        else XR_GU(2, 2, false);
    }
#undef XR_GU
    QASR_HIP(hipGetLastError());
}


}  // namespace qasr
