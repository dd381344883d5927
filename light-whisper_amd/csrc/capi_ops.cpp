// extern "C" kernel-level entry points (qasr_op_*) — see include/qasr.h.
#include <math.h>
#include <string.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/qasr.h"
#include "capi_util.h"
#include "kernels.h"

using namespace qasr;

namespace {
inline hipStream_t S(void* s) { return (hipStream_t)s; }
inline void launched() { QASR_HIP(hipGetLastError()); }
}  // namespace

extern "C" {

QASR_API int qasr_op_quant_rows(const float* x, int32_t M, int32_t K, int32_t ldx, int8_t* q, float* d, void* stream) {
    return guard([&] {
        QASR_CHECK(K % QK == 0 && M >= 0 && ldx >= K, QASR_E_INVALID, "quant_rows: K must be a multiple of 32");
        quant_rows(x, M, K, ldx, q, d, S(stream));
        launched();
    });
}

// Tests and tuning tools: the regrouped stage scales (Q8Mat::sc4, [K/128][N][4]) of a raw weight matrix given to the
// qasr_op_* GEMM entry points, registered by its scale pointer AND shape (a model's matrices carry theirs, model.cpp):
// a later matrix of another shape at a recycled address never picks up a stale registration
struct S4Reg {
    const void* wsc;
    int32_t N, K;
    const __half* sc4;
};
static std::mutex g_s4_mu;
static std::vector<S4Reg> g_s4;
static const __half* stage_scales_of(const void* wsc, int32_t N, int32_t K) {
    std::lock_guard<std::mutex> lk(g_s4_mu);
    for (auto& e : g_s4)
        if (e.wsc == wsc && e.N == N && e.K == K) return e.sc4;
    return nullptr;
}

QASR_API int qasr_op_stage_scales(const void* wsc, int32_t N, int32_t K, void* out, void* stream) {
    return guard([&] {
        q8_stage_scales((const __half*)wsc, N, K, (__half*)out, S(stream));
        launched();
    });
}

QASR_API int qasr_op_register_stage_scales(const void* wsc, int32_t N, int32_t K, const void* sc4) {
    return guard([&] {
        QASR_CHECK(wsc && N > 0 && K > 0 && K % 128 == 0, QASR_E_INVALID, "stage scales: scale pointer, N, K % 128");
        std::lock_guard<std::mutex> lk(g_s4_mu);
        for (size_t i = 0; i < g_s4.size(); i++)
            if (g_s4[i].wsc == wsc) {   // one registration per address (whatever shape it had)
                g_s4.erase(g_s4.begin() + (long)i);
                break;
            }
        if (sc4) g_s4.push_back(S4Reg{wsc, N, K, (const __half*)sc4});
    });
}

QASR_API int qasr_op_repack_q8(const uint8_t* blocks, int64_t nblk, int8_t* qs, void* sc, void* stream) {
    return guard([&] {
        repack_q8(blocks, nblk, qs, (__half*)sc, S(stream));
        launched();
    });
}

QASR_API int qasr_op_linear_q8(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                               int32_t N, int32_t K, const float* bias, const float* res, float* y, int32_t ldy,
                               int32_t epi, int32_t path, void* stream) {
    return guard([&] {
        QASR_CHECK(K % QK == 0 && N > 0 && M >= 0 && ldy >= N, QASR_E_INVALID, "linear_q8: bad shape");
        QASR_CHECK(epi >= 0 && epi <= 2, QASR_E_INVALID, "linear_q8: bad epilogue");
        QASR_CHECK(epi != EPI_RESID || res, QASR_E_INVALID, "linear_q8: residual epilogue needs res");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        if (path == 1 || (path >= 3 && path <= 5)) {   // GEMV: auto, or 1 / 2 / 4 columns per wave
            QASR_CHECK(M <= 8, QASR_E_INVALID, "linear_q8: GEMV path supports M <= 8");
            gemv_q8(xq, xd, M, W, bias, res, y, ldy, epi, S(stream), path == 1 ? 0 : 1 << (path - 3));
        } else if (path == 2) {
            gemm_q8(xq, xd, M, W, bias, res, y, ldy, epi, S(stream));
        } else if (path >= 4096) {   // any configuration index: 4096 + cfg + 256·splits
            const int cfg = (path - 4096) % 256, splits = (path - 4096) / 256;
            gemm_q8(xq, xd, M, W, bias, res, y, ldy, epi, S(stream), cfg, splits);
        } else if (path >= 16) {
            const int cfg = (path - 16) % 32, splits = (path - 16) / 32;
            gemm_q8(xq, xd, M, W, bias, res, y, ldy, epi, S(stream), cfg == 31 ? -1 : cfg, splits);
        } else {
            linear_q8(xq, xd, M, W, bias, res, y, ldy, epi, S(stream));
        }
        launched();
    });
}

QASR_API int qasr_op_q8_to_mx(const int8_t* q, const void* d, int32_t d_is_f16, int64_t nblk, uint8_t* q8,
                             uint8_t* s8, void* stream) {
    return guard([&] {
        QASR_CHECK(nblk >= 0, QASR_E_INVALID, "q8_to_mx: bad size");
        if (d_is_f16) q8w_to_mx(q, (const __half*)d, nblk, q8, s8, S(stream));
        else q8_to_mx(q, (const float*)d, nblk, q8, s8, S(stream));
        launched();
    });
}

QASR_API int qasr_op_gemm_mx(const uint8_t* x8, const uint8_t* xs, int32_t M, const uint8_t* w8, const uint8_t* ws,
                             int32_t N, int32_t K, const float* bias, const float* res, float* y, int32_t ldy,
                             int32_t epi, int8_t* yq, float* yd, int32_t cfg, void* stream) {
    return guard([&] {
        QASR_CHECK(K % 128 == 0 && N > 0 && M > 0 && ldy >= (epi == EPI_SWIGLU ? 0 : N) && epi >= 0 && epi <= 4,
                   QASR_E_INVALID, "gemm_mx: bad shape / epilogue");
        Q8Mat W;
        W.N = N;
        W.K = K;
        W.mx = (uint8_t*)w8;
        W.mxs = (uint8_t*)ws;
        gemm_mx(x8, xs, M, W, bias, res, y, ldy, epi, S(stream), yq, yd, false, cfg);
        launched();
    });
}

QASR_API int qasr_op_linear_q8_ex(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                  int32_t N, int32_t K, const float* bias, void* y, int32_t ldy, int32_t epi,
                                  int8_t* yq, float* yd, int32_t cfg, void* stream) {
    return guard([&] {
        QASR_CHECK(K % QK == 0 && N > 0 && M > 8 && ldy >= N && (epi == 4 || epi == 5), QASR_E_INVALID,
                   "linear_q8_ex: bad shape / epilogue");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        gemm_q8(xq, xd, M, W, bias, nullptr, (float*)y, ldy, epi, S(stream), cfg, 0, yq, yd);
        launched();
    });
}


QASR_API int qasr_op_rmsnorm_q8(const float* x, int32_t M, int32_t H, const float* w, float eps, int8_t* q, float* d,
                                void* stream) {
    return guard([&] {
        QASR_CHECK(H % QK == 0, QASR_E_INVALID, "rmsnorm_q8: H must be a multiple of 32");
        rmsnorm_q8(x, M, H, H, w, eps, q, d, S(stream));
        launched();
    });
}

QASR_API int qasr_op_layernorm_q8(const float* x, int32_t M, int32_t H, const float* w, const float* b, float eps,
                                  int8_t* q, float* d, float* y, void* stream) {
    return guard([&] {
        QASR_CHECK(H % QK == 0, QASR_E_INVALID, "layernorm_q8: H must be a multiple of 32");
        layernorm_q8(x, M, H, w, b, eps, q, d, y, S(stream));
        launched();
    });
}

QASR_API int qasr_op_swiglu_q8(const float* gu, int32_t M, int32_t F, int8_t* q, float* d, void* stream) {
    return guard([&] {
        QASR_CHECK(F % QK == 0, QASR_E_INVALID, "swiglu_q8: F must be a multiple of 32");
        swiglu_q8(gu, M, F, q, d, S(stream));
        launched();
    });
}

QASR_API int qasr_op_interleave_gate_up(int8_t* qs, void* sc, int32_t N, int32_t K, void* stream) {
    return guard([&] {
        QASR_CHECK(N % 32 == 0 && K % QK == 0, QASR_E_INVALID, "interleave_gate_up: bad shape");
        Q8Mat W;
        W.qs = qs;
        W.sc = (__half*)sc;
        W.N = N;
        W.K = K;
        interleave_gate_up(W, S(stream));
        launched();
    });
}

QASR_API int qasr_op_gemm_swiglu_q8(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                    int32_t N, int32_t K, int8_t* hq, float* hd, void* stream) {
    return guard([&] {
        QASR_CHECK(N % 64 == 0 && K % QK == 0 && M >= 0, QASR_E_INVALID, "gemm_swiglu_q8: bad shape");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        gemm_q8(xq, xd, M, W, nullptr, nullptr, nullptr, N, EPI_SWIGLU, S(stream), -1, 0, hq, hd);
        launched();
    });
}

QASR_API int qasr_op_gemm_swiglu_q8_cfg(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs,
                                        const void* wsc, int32_t N, int32_t K, int8_t* hq, float* hd, int32_t cfg,
                                        void* stream) {
    return guard([&] {
        QASR_CHECK(N % 64 == 0 && K % QK == 0 && M >= 0, QASR_E_INVALID, "gemm_swiglu_q8: bad shape");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        // cfg + 32·splits (cfg < 31), or 4096 + cfg + 256·splits (any configuration index)
        const int c = cfg < 0 ? -1 : cfg >= 4096 ? (cfg - 4096) % 256 : cfg % 32;
        const int sp = cfg < 0 ? 0 : cfg >= 4096 ? (cfg - 4096) / 256 : cfg / 32;
        gemm_q8(xq, xd, M, W, nullptr, nullptr, nullptr, N, EPI_SWIGLU, S(stream), c, sp, hq, hd);
        launched();
    });
}

QASR_API int qasr_op_gemm_exact_rows(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                     int32_t N, int32_t K, const float* res, float* y, int32_t ldy, int32_t epi,
                                     void* stream) {
    return guard([&] {
        QASR_CHECK(N > 0 && ldy >= N && (epi == EPI_STORE || (epi == EPI_RESID && res)), QASR_E_INVALID,
                   "gemm_exact_rows: bad shape / epilogue");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        gemm_exact_rows(xq, xd, M, W, res, y, ldy, epi, S(stream));
        launched();
    });
}

// the xr launches' leaf-split scratch: one process-wide buffer for the op entry points (tests / tools, one stream; every
// launch leaves its counters zero)
static const XrSplit& op_xr_split() {
    static const XrSplit xs = [] {
        void* mem = nullptr;
        QASR_HIP(hipMalloc(&mem, xr_split_bytes()));
        QASR_HIP(hipMemset(mem, 0, xr_split_bytes()));
        return xr_split_view(mem);
    }();
    return xs;
}

QASR_API int qasr_op_xr_linear(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps,
                               int32_t M, const int8_t* wqs, const void* wsc, int32_t N, int32_t K, float* y,
                               int32_t ldy, int32_t resid, void* stream) {
    return guard([&] {
        QASR_CHECK(N > 0 && ldy >= N && (src || (xq && xd)), QASR_E_INVALID, "xr_linear: bad arguments");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.N = N;
        W.K = K;
        xr_linear(xq, xd, src, nw, eps, M, W, y, ldy, resid != 0, S(stream), nullptr, &op_xr_split());
        launched();
    });
}

QASR_API int qasr_op_xr_vocab(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                             int32_t N, int32_t K, float* y, int32_t ldy, void* stream) {
    return guard([&] {
        QASR_CHECK(xq && xd && y && N > 0 && ldy >= N, QASR_E_INVALID, "xr_vocab: bad arguments");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.N = N;
        W.K = K;
        xr_vocab(xq, xd, M, W, y, ldy, S(stream));
        launched();
    });
}

QASR_API int qasr_op_xr_gu_swiglu(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps,
                                  int32_t M, const int8_t* wqs, const void* wsc, int32_t N, int32_t K, int8_t* hq,
                                  float* hd, void* stream) {
    return guard([&] {
        QASR_CHECK(N > 0 && (src || (xq && xd)) && hq && hd, QASR_E_INVALID, "xr_gu_swiglu: bad arguments");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.N = N;
        W.K = K;
        xr_gu_swiglu(xq, xd, src, nw, eps, M, W, hq, hd, S(stream));
        launched();
    });
}

QASR_API int qasr_op_set_gemm_fixup(void* part, int64_t part_bytes, void* cnt, int32_t ncnt) {
    return guard([&] {
        QASR_CHECK(part_bytes >= 0 && ncnt >= 0, QASR_E_INVALID, "set_gemm_fixup: bad size");
        set_gemm_fixup((float*)part, (size_t)part_bytes / sizeof(float), (unsigned*)cnt, ncnt, true);
    });
}

QASR_API int qasr_op_swiglu_q8_interleaved(const float* gu, int32_t M, int32_t F, int8_t* q, float* d, void* stream) {
    return guard([&] {
        QASR_CHECK(F % QK == 0, QASR_E_INVALID, "swiglu_q8: F must be a multiple of 32");
        swiglu_q8(gu, M, F, q, d, S(stream), true);
        launched();
    });
}

QASR_API int qasr_op_gemv_fused(int32_t pro, const float* src, int32_t ld_src, const float* nw, float eps, int32_t M,
                                const int8_t* xq, const float* xd, const int8_t* wqs, const void* wsc, int32_t N,
                                int32_t K, const float* res, float* y, int32_t ldy, int32_t epi, int8_t* hq,
                                float* hd, void* stream) {
    return guard([&] {
        QASR_CHECK(N > 0 && (epi == EPI_SWIGLU || (y && ldy >= N)), QASR_E_INVALID, "gemv_fused: bad shape");
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.sc4 = stage_scales_of(wsc, N, K);
        W.N = N;
        W.K = K;
        gemv_fused(pro, xq, xd, src, ld_src, nw, eps, M, W, res, y, ldy, epi, hq, hd, S(stream));
        launched();
    });
}

QASR_API int qasr_op_qk_norm_rope(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                  const int32_t* pos, const int32_t* slot, const float* qnw, const float* knw,
                                  const float* rope_cs, float eps, void* qout, void* kc, void* vc, void* stream) {
    return guard([&] {
        QASR_CHECK(nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "qk_norm_rope: bad head counts");
        qk_norm_rope(qkv, rows, nh, nkv, hd, pos, slot, qnw, knw, rope_cs, eps, (__half*)qout, (__half*)kc,
                     (__half*)vc, S(stream));
        launched();
    });
}

QASR_API int qasr_op_attention_decode_fused(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                            const int32_t* pos, const int32_t* slot, const float* qnw,
                                            const float* knw, const float* rope_cs, float eps, void* kc, void* vc,
                                            const int32_t* kv_start, const int32_t* kv_len, float scale, int8_t* oq,
                                            float* od, void* stream) {
    return guard([&] {
        QASR_CHECK(hd == 128 && nkv > 0 && nh % nkv == 0 && oq && od, QASR_E_INVALID,
                   "attention_decode_fused: hd 128, Q8 output");
        const QkFuse fz{qkv, pos, slot, qnw, knw, rope_cs, eps, (__half*)kc, (__half*)vc};
        attention_decode_fused(fz, nkv * hd, kv_start, kv_len, rows, nh, nkv, hd, scale, oq, od, S(stream));
        launched();
    });
}

QASR_API int qasr_op_attention_decode_split(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                            const int32_t* pos, const int32_t* slot, const float* qnw,
                                            const float* knw, const float* rope_cs, float eps, void* kc, void* vc,
                                            const int32_t* kv_start, const int32_t* kv_len, float scale, int8_t* oq,
                                            float* od, float* part, int32_t* cnt, void* stream) {
    return guard([&] {
        QASR_CHECK(hd == 128 && nkv > 0 && nh % nkv == 0 && oq && od && part && cnt && rows <= kExactRows,
                   QASR_E_INVALID, "attention_decode_split: hd 128, Q8 output, ≤ 32 rows, scratch");
        QkFuse fz{qkv, pos, slot, qnw, knw, rope_cs, eps, (__half*)kc, (__half*)vc};
        fz.part = part;
        fz.cnt = cnt;
        attention_decode_fused(fz, nkv * hd, kv_start, kv_len, rows, nh, nkv, hd, scale, oq, od, S(stream));
        launched();
    });
}

QASR_API int qasr_op_attention(const void* q, int32_t ldq, const void* k, const void* v, int32_t ldkv,
                               const int32_t* kv_start, const int32_t* kv_len, int32_t rows, int32_t nh, int32_t nkv,
                               int32_t hd, float scale, float* o, int8_t* oq, float* od, void* stream) {
    return guard([&] {
        QASR_CHECK(nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "attention: bad head counts");
        attention((const __half*)q, ldq, (const __half*)k, (const __half*)v, ldkv, kv_start, kv_len, rows, nh, nkv,
                  hd, scale, o, oq, od, S(stream));
        launched();
    });
}

QASR_API int qasr_op_attention_dense(const void* q, int32_t ldq, const void* k, const void* v, int32_t ldkv,
                                     const int32_t* kv_start, const int32_t* kv_len, int32_t rows, int32_t nh,
                                     int32_t nkv, int32_t hd, float scale, float* o, int8_t* oq, float* od,
                                     int32_t dense, void* stream) {
    return guard([&] {
        QASR_CHECK(nkv > 0 && nh % nkv == 0, QASR_E_INVALID, "attention: bad head counts");
        attention((const __half*)q, ldq, (const __half*)k, (const __half*)v, ldkv, kv_start, kv_len, rows, nh, nkv,
                  hd, scale, o, oq, od, S(stream), 0, dense != 0);
        launched();
    });
}

QASR_API int qasr_op_argmax(const float* x, int32_t M, int32_t V, int32_t* out, void* stream) {
    return guard([&] {
        argmax_rows(x, M, V, out, S(stream));
        launched();
    });
}

QASR_API int qasr_op_embed_rows(const int32_t* ids, int32_t n, const int8_t* wqs, const void* wsc, int32_t K,
                                const float* alt, float* out, void* stream) {
    return guard([&] {
        Q8Mat W;
        W.qs = (int8_t*)wqs;
        W.sc = (__half*)wsc;
        W.K = K;
        embed_rows(ids, n, W, alt, out, S(stream));
        launched();
    });
}

QASR_API int qasr_op_synth_q8(uint64_t seed, const char* name, int64_t N, int64_t K, float sigma, int8_t* qs, void* sc,
                              void* stream) {
    return guard([&] {
        QASR_CHECK(K % QK == 0, QASR_E_INVALID, "synth_q8: K must be a multiple of 32");
        synth_q8(smix(seed ^ fnv1a(name)), N * (K / QK), sigma / 73.6f, qs, (__half*)sc, S(stream),
                 strcmp(name, "token_embd.weight") == 0 ? K / QK : 0);
        launched();
    });
}

QASR_API int qasr_op_rope_table(int32_t n_ctx, int32_t head_dim, float theta, float* host_out) {
    return guard([&] { rope_table(n_ctx, head_dim, theta, host_out); });
}

QASR_API int qasr_stream_sync(void* stream) {
    return guard([&] { QASR_HIP(hipStreamSynchronize(S(stream))); });
}

}  // extern "C"
