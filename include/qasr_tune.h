/*
 * qasr_tune.h — engine-internal tuning, A/B and test hooks of libqasr (NOT part of the drop-in boundary in qasr.h:
 * no reference interface corresponds to them).  The GEMM tuning tools (tools/gemm_tune.py, tools/dec_gemm_sweep.py)
 * and the kernel parity tests force configurations through them; a host binding the reference's interface never
 * needs them.  Pointer arguments are DEVICE pointers, `stream` a hipStream_t (NULL = default stream).
 */
#ifndef QASR_TUNE_H
#define QASR_TUNE_H

#include "qasr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* qasr_op_gemm_swiglu_q8 with the GEMM configuration forced (kernels_q8.hip kGemmCfgs index + 32 × split-K count, or
   4096 + cfg + 256 × split-K count for configurations ≥ 32; -1 = heuristic).  Split-K needs a fix-up workspace
   (qasr_op_set_gemm_fixup). */
QASR_API int qasr_op_gemm_swiglu_q8_cfg(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs,
                                        const void* wsc, int32_t N, int32_t K, int8_t* hq, float* hd, int32_t cfg,
                                        void* stream);
/* Register (this thread) the split-K fix-up workspace the op-level Q8 GEMMs use: part_bytes of device memory for
   partial tiles and ncnt device uint32 arrival counters, ZEROED by the caller (the kernels leave them zero).  With
   it, every split-K GEMM stores partial tiles and the tile's last workgroup adds them in split order and runs the
   full epilogue (deterministic, any epilogue); without it (part = NULL) split-K adds with f32 atomics.  Sessions
   register their own for the decode steps (used there for the SwiGLU epilogue).  Not in
   the reference (an engine-internal tuning / test hook). */
QASR_API int qasr_op_set_gemm_fixup(void* part, int64_t part_bytes, void* cnt, int32_t ncnt);
/* Regrouped stage scales of a Q8 matrix (sc [N][K/32] f16 → out [K/128][N][4] f16, K % 128 == 0): a K-128 GEMM
   stage's column scales as one contiguous run (the decode GEMMs' 16-byte scale DMA; a model's decoder matrices
   carry theirs).  qasr_op_register_stage_scales(wsc, N, K, out) makes the qasr_op_* GEMM entry points use `out` for
   the N × K matrix whose scale pointer is `wsc` (out NULL unregisters; a call with another N or K at that address
   finds no registration) — tests and tuning tools. */
QASR_API int qasr_op_stage_scales(const void* wsc, int32_t N, int32_t K, void* out, void* stream);
QASR_API int qasr_op_register_stage_scales(const void* wsc, int32_t N, int32_t K, const void* sc4);
/* The ≤ 32-row decode's exact-row launches (kernels_xr.hip, xr_*): the same outputs bit for bit as
   qasr_op_gemm_exact_rows (and, with src, as qasr_op_rmsnorm_q8 + it), one workgroup per 16-column fragment with its
   weights loaded up front and the rows staged once in LDS.  qasr_op_xr_linear: y = X·Wᵀ (+ y when resid); src != NULL
   (M ≤ 8, K ≤ 2,048): X = Q8(RMSNorm(src)·nw) computed inside.  qasr_op_xr_gu_swiglu: W = interleaved gate/up [2F][K],
   hq / hd = Q8(silu(g)·u) (qasr_op_swiglu_q8_interleaved's arithmetic).  M 1-32, K ∈ {1,024, 2,048, 3,072, 6,144}. */
QASR_API int qasr_op_xr_linear(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps,
                               int32_t M, const int8_t* wqs, const void* wsc, int32_t N, int32_t K, float* y,
                               int32_t ldy, int32_t resid, void* stream);
/* the vocabulary projection of 1–16 rows with the exact-row arithmetic (each row the 1-row GEMV's bits): a grid sized
   by the occupancy query staging the rows once per workgroup and walking the 16-column fragments (kernels_xr.hip
   k_xr_vocab) */
QASR_API int qasr_op_xr_vocab(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                             int32_t N, int32_t K, float* y, int32_t ldy, void* stream);
QASR_API int qasr_op_xr_gu_swiglu(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps,
                                  int32_t M, const int8_t* wqs, const void* wsc, int32_t N, int32_t K, int8_t* hq,
                                  float* hd, void* stream);
#ifdef __cplusplus
}
#endif

#endif /* QASR_TUNE_H */
