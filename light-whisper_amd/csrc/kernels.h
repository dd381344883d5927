// Launch wrappers for the hand-written gfx950 kernels (definitions in kernels_*.hip).
// Every wrapper takes device pointers and a stream; none allocates or synchronises (graph-capturable).
#pragma once
#include "common.h"
#include "prof.h"

namespace qasr {

enum Epi : int {
    EPI_STORE = 0,  // y = acc (+ bias)
    EPI_RESID = 1,  // y = res + acc (+ bias)      (y may alias res)
    EPI_GELU = 2,   // y = gelu_erf(acc + bias)
    EPI_SWIGLU = 3, // W rows gate/up interleaved by 16 (interleave_gate_up): h = silu(g)·u → Q8 rows (yq, yd)
    EPI_GELU_Q8 = 4,   // h = gelu_erf(acc + bias) → Q8 rows (yq [M][N], yd [M][N/32]); y unused
    EPI_STORE_F16 = 5, // y (as __half, row stride ldy) = f16(acc + bias)
};

// ---- Q8_0 weights / activations (kernels_q8.hip)
void repack_q8(const uint8_t* blocks, int64_t nblk, int8_t* qs, __half* sc, hipStream_t s);
// gain_bpr > 0: blocks per row of a table whose rows get synth_row_gain (token_embd.weight, see common.h)
void synth_q8(uint64_t base, int64_t nblk, float dbase, int8_t* qs, __half* sc, hipStream_t s, int64_t gain_bpr = 0);
void synth_f32(uint64_t base, int64_t n, float center, float scale, float* out, hipStream_t s);
void synth_f16(uint64_t base, int64_t n, float scale, __half* out, hipStream_t s);
// quantise rows of x (row stride ldx floats) into q [M][K] / d [M][K/32]
void quant_rows(const float* x, int M, int K, int ldx, int8_t* q, float* d, hipStream_t s);
// y[M][N] (row stride ldy) = epi(X·Wᵀ); dispatches GEMV (M ≤ 8) or the MFMA GEMM
// y_zeroed: y is already all-zero (a split-K GEMM then skips its memset)
void linear_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res,
               float* y, int ldy, int epi, hipStream_t s, bool y_zeroed = false);
// rows up to which linear_q8 streams weights with the GEMV kernel; more rows take the MFMA GEMM and its fused
// epilogues (tools/gemv_tune.py: at 8 rows the GEMM is faster on every decoder shape, at 4 the GEMV mostly is)
constexpr int kGemvRows = 4;
// rows up to which the decoder layer runs on the fused weight-streaming GEMVs (gemv_fused: norm prologue, SwiGLU
// epilogue, 5 launches per layer) instead of the MFMA GEMMs (QASR_GV_ROWS overrides, for A/B timing).  Round 5: 4 —
// the 5–8-row GEMV group (v_dot4 rows, 8 rows against the weight registers) cost 19–26 µs per QKV / down / gate-up
// launch in the 32-segment share; the MFMA paths take 5–15 µs (32-segment share 1,107 → 1,188 audio-s/s,
// profiles/r5_seg32_*.log)
constexpr int kGemvWideRows = 4;
// rows up to which gemv_fused runs (groups of 8 against the weights held in registers, each row with the per-row
// arithmetic of a 1-row launch): the draft verify passes of the streaming decode, whose rows must be the same bits
// as one-token greedy steps (engine.cpp, exact rows)
constexpr int kExactRows = 32;
int gemv_layer_rows();
void gemv_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res, float* y,
             int ldy, int epi, hipStream_t s, int cols = 0);
// the 1–8-row decoder GEMVs, about one workgroup per CU, with the row operations around them fused (bit-identical to
// the separate rmsnorm_q8 / gemv_q8 / swiglu_q8 launches): pro GV_RMS: activations = Q8(RMSNorm(src rows, stride
// ld_src floats)·nw), K ≤ 4096; GV_NONE: the Q8 rows xq / xd, K ≤ 6144.  epi EPI_STORE / EPI_RESID into y, or
// EPI_SWIGLU (GV_RMS only; W = interleaved gate/up, N % 64 == 0): h = Q8(silu(g)·u) into yq [M][N/2] / yd [M][N/64].
enum GvPro : int { GV_NONE = 0, GV_RMS = 1 };
// The draft verify passes' linears on the matrix core with EXACTLY k_gemv_wide's 1-row arithmetic (the same block fma
// chains and wave-sum tree, run in-lane): any row count (32-row chunks in one launch), K a multiple of 1,024 (K/1024 ∈ {1,2,3,4,6}), epi store
// or residual — bit-identical to gemv_fused(GV_NONE) on the same Q8 rows, and to the fused norm / SwiGLU launches when
// preceded by rmsnorm_q8 / followed by swiglu_q8(interleaved)
bool gemm_exact_rows_ok(int M, const Q8Mat& W);
// verify-pass rows from which the engine takes gemm_exact_rows (default 5; QASR_EXACT_MFMA_ROWS, 0 = never)
int exact_mfma_rows();
void gemm_exact_rows(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* res, float* y, int ldy,
                     int epi, hipStream_t s);
bool gemv_fused_ok(int pro, int M, int K);
void gemv_fused(int pro, const int8_t* xq, const float* xd, const float* src, int ld_src, const float* nw, float eps,
                int M, const Q8Mat& W, const float* res, float* y, int ldy, int epi, int8_t* yq, float* yd,
                hipStream_t s);
// deterministic mode (process-wide): GEMMs never split K with float atomics (split-K sums landing by atomics, whose
// order varies run to run); deterministic_gen() changes on every switch so captured step graphs are re-captured
void set_deterministic(bool on);
bool deterministic();
uint64_t deterministic_gen();
// Row-count-independent summation order for the Q8 GEMMs in its scope (thread-local): one tile configuration with one
// K group and no split for every M (and no GEMV rows), so a row's outputs are the same bits whatever other rows the
// call carries — the streaming encoder cache reuses rows of an earlier, shorter run bit for bit.
struct StableOrderScope {
    explicit StableOrderScope(bool on);
    ~StableOrderScope();
    bool prev;
};
bool stable_order();
// force_cfg: index into kernels_q8.hip kGemmCfgs (-1 = heuristic); force_splits: split-K (0 = heuristic)
void gemm_q8(const int8_t* xq, const float* xd, int M, const Q8Mat& W, const float* bias, const float* res, float* y,
             int ldy, int epi, hipStream_t s, int force_cfg = -1, int force_splits = 0, int8_t* yq = nullptr,
             float* yd = nullptr, bool y_zeroed = false);
// MXFP8 precision mode (C5): Q8 blocks → e4m3 elements + e8m0 block exponents (activations f32 d, weights f16 d);
// the block-scaled fp8 GEMM (same epilogues as gemm_q8, K % 128 == 0); gemm_q8 routes to it when W.mx is set,
// converting the Q8 activations into the workspace registered by set_mx_workspace
void q8_to_mx(const int8_t* q, const float* d, int64_t nblk, uint8_t* q8, uint8_t* s8, hipStream_t s);
void q8w_to_mx(const int8_t* q, const __half* d, int64_t nblk, uint8_t* q8, uint8_t* s8, hipStream_t s);
void gemm_mx(const uint8_t* x8, const uint8_t* xs, int M, const Q8Mat& W, const float* bias, const float* res,
             float* y, int ldy, int epi, hipStream_t s, int8_t* yq = nullptr, float* yd = nullptr,
             bool y_zeroed = false, int force_cfg = -1);
void set_mx_workspace(void* p, size_t bytes);
// split-K fix-up workspace for gemm_q8 (thread-local): `floats` partial-tile floats and `ncnt` arrival counters that
// are zero between launches (the kernels keep them so); nullptr = split-K adds with f32 atomics.  The fix-up serves
// the SwiGLU epilogue (deterministic), or every split epilogue with all_epilogues (op-level tests / tuning).
void set_gemm_fixup(float* part, size_t floats, unsigned* cnt, int ncnt, bool all_epilogues = false);
// rows up to which gemm_q8's automatic choice takes the weight-streaming kernel (≤ 64; 0 = never); all_shapes: on
// every shape it supports, not only the wide decoder matrices where it is faster (tests)
constexpr int kFixSplits = 8, kFixCounters = 8192;
struct FixupScope {   // registers a fix-up workspace for the calls in its scope, unregisters on exit (throws included)
    FixupScope(float* part, size_t floats, unsigned* cnt, int ncnt) { set_gemm_fixup(part, floats, cnt, ncnt); }
    ~FixupScope() { set_gemm_fixup(nullptr, 0, nullptr, 0); }
    FixupScope(const FixupScope&) = delete;
    FixupScope& operator=(const FixupScope&) = delete;
};
size_t mx_workspace_bytes(int64_t M, int64_t K);
// rows of a [2F][K] gate|up matrix → interleaved by 16 (32j+t: t<16 gate 16j+t, else up 16j+t-16)
int64_t gate_up_interleaved_row(int64_t r, int64_t F);
void interleave_gate_up(Q8Mat& W, hipStream_t s);
// sc [N][K/32] → out [K/128][N][4] (Q8Mat::sc4), K % 128 == 0
void q8_stage_scales(const __half* sc, int N, int K, __half* out, hipStream_t s);
// rows of a Q8 table (token embeddings), dequantised; ids < 0 take row -(id+1) of `alt` [*][K] f32 instead
void embed_rows(const int* ids, int n, const Q8Mat& W, const float* alt, float* out, hipStream_t s);

// ---- norms / elementwise (kernels_nn.hip)
// zero/nzero (optional): a float range cleared by the same launch (the next split-K GEMM's output)
void rmsnorm_q8(const float* x, int M, int H, int ldx, const float* w, float eps, int8_t* q, float* d, hipStream_t s,
                float* zero = nullptr, int64_t nzero = 0);
void layernorm_q8(const float* x, int M, int H, const float* w, const float* b, float eps, int8_t* q, float* d,
                  float* y_opt, hipStream_t s);
// gu rows [gate F | up F], or interleaved by 16 (interleave_gate_up layout)
void swiglu_q8(const float* gu, int M, int F, int8_t* q, float* d, hipStream_t s, bool interleaved = false);
void gelu_q8(const float* x, int M, int K, int8_t* q, float* d, hipStream_t s);
// Qwen3 q/k RMSNorm + NeoX RoPE; Q → qout f16 [rows][nh*hd], K/V → cache slots (f16)
void qk_norm_rope(const float* qkv, int rows, int nh, int nkv, int hd, const int* pos, const int* slot,
                  const float* qnw, const float* knw, const float* rope_cs, float eps, __half* qout, __half* kc,
                  __half* vc, hipStream_t s);
// f32 [rows][ld_in] column range → f16 [rows][cols]
void to_f16(const float* x, int rows, int cols, int ldx, __half* y, int ldy, hipStream_t s);
// argmax per row (lowest index on ties); scratch (argmax_scratch_bytes(M)) selects the two-stage kernel
void argmax_rows(const float* x, int M, int V, int* out, hipStream_t s, void* scratch = nullptr);
size_t argmax_scratch_bytes(int M);
// the first half of argmax_rows (scratch required): kArgParts slice maxima per row as order-preserving 64-bit keys
// (value bits, then the complement of the index, so ties keep the lowest index); argmax_accept finishes it
constexpr int kArgParts = 32;
void argmax_rows_partial(const float* x, int M, int V, void* scratch, hipStream_t s);
void add_posemb_gather(const float* proj, int n_chunks, int T, int d, const float* pe, const int* valid_idx,
                       int n_out, float* out, hipStream_t s);

// ---- attention (kernels_attn.hip)
// one query row r: Q[r] (f16) against keys/values slots [kv_start[r], kv_start[r]+kv_len[r]) of K/V (f16);
// output quantised (q/d, row stride nh*hd) and/or f32 (o).  dense: runs of 16 consecutive rows share most of their
// key range (prefill prompt rows, encoder windows) → the MFMA tile kernel; otherwise the per-row kernel (decode).
// decode attention with the q/k RMS-norm + RoPE and the KV-cache write of the new row fused in (hd 128, G 2 / 4):
// reads the f32 QKV rows directly; same results as qk_norm_rope followed by attention
struct QkFuse {
    const float* qkv;
    const int* pos;
    const int* slot;
    const float* qnw;
    const float* knw;
    const float* rope_cs;
    float eps;
    __half* kc;
    __half* vc;
    // split-K over the key range (≤ kExactRows decode rows, long contexts): partial (m, l, Σp·v) per (row, KV head, split)
    // and an arrival counter per (row, KV head), zero between launches (kAttnSplitScratch sizes them); nullptr = one
    // workgroup per (row, KV head)
    float* part = nullptr;
    int* cnt = nullptr;
    int part_rows = kExactRows;   // rows part / cnt are sized for
    // the row-invariant decode (Session batch invariance): the 64-key chunk kernel whatever the row count, so a row's
    // result is the bits of a 1-row step (many-row launches otherwise take the 32-key chunks)
    bool fixed_chunk = false;
    // ranges up to split_min keys stay in one workgroup; longer ones get pieces of ≥ split_keys keys
    // (tools/graph_cost.py, profiles/r2_attn_split_min_sweep.jsonl: 300 / 400 keys 9.7 → 8.0 / 8.2 µs at 256)
    int split_min = 256;
    int split_keys = 128;
};
constexpr int kAttnSplitMax = 16;      // workgroups per (row, KV head) at most
// scratch floats / counters for up to `rows` split decode rows of a model (G query heads per KV head, hd 128)
inline size_t attn_split_floats(int rows, int nkv, int G) { return (size_t)rows * nkv * kAttnSplitMax * G * (2 + 128); }
void attention_decode_fused(const QkFuse& fz, int ldkv, const int* kv_start, const int* kv_len, int rows, int nh,
                            int nkv, int hd, float scale, int8_t* oq, float* od, hipStream_t s, int64_t total_keys = 0);
void attention(const __half* Q, int ldq, const __half* K, const __half* V, int ldkv, const int* kv_start,
               const int* kv_len, int rows, int nh, int nkv, int hd, float scale, float* o, int8_t* oq, float* od,
               hipStream_t s, int64_t total_keys = 0, bool dense = false);

// ---- the ≤ 32-row decode linears as per-phase launches (kernels_xr.hip): exact-row arithmetic, bit-identical
// to gemm_exact_rows / the 1-row GEMVs.  src != nullptr (≤ 8 rows, K ≤ 2,048): the input rows are RMSNorm(src)·nw
// quantised inside the launch (rmsnorm_q8's arithmetic) instead of xq / xd.
bool xr_ok(int R, int K);
// the vocabulary projection of 1–16 rows (K 1,024 / 2,048) with the exact-row arithmetic (the 1-row GEMV's bits per
// row): a grid of every resident workgroup, each staging the rows once and walking the 16-column fragments
bool xr_vocab_ok(int R, int K, int N);
void xr_vocab(const int8_t* xq, const float* xd, int R, const Q8Mat& W, float* y, int ldy, hipStream_t s);
// norm (residual launches of whole rows, N = H ∈ {1,024, 2,048}): RMSNorm(y)·w → Q8 rows q / d inside the launch
// (rmsnorm_q8's arithmetic, by the last workgroups to finish); cnt: 3 words, zero between launches
struct XrNorm {
    const float* w = nullptr;
    float eps = 0.f;
    int8_t* q = nullptr;
    float* d = nullptr;
    unsigned* cnt = nullptr;
};
// the leaf split's scratch (k_xr_linear XS = 2): two workgroups per 16-column fragment; the second to arrive adds the
// first's partial tree (write-through, one arrival counter per fragment and row slice, zero between launches)
struct XrSplit {
    float* part = nullptr;      // [items][kXrSplitPart] floats: [2][RF·256], RF ≤ 2
    unsigned* cnt = nullptr;    // [items]
    int items = 0;
};
constexpr int kXrSplitItems = 256;
constexpr int kXrSplitPart = 2 * 2 * 256;   // floats per item
size_t xr_split_bytes();        // part + counters for kXrSplitItems items (counters zeroed by the owner)
XrSplit xr_split_view(void* mem);   // the layout of one xr_split_bytes() allocation
void xr_linear(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps, int R, const Q8Mat& W,
               float* y, int ldy, bool resid, hipStream_t s, const XrNorm* norm = nullptr,
               const XrSplit* split = nullptr);
// interleaved gate/up (N = 2F) + SwiGLU + Q8 → hq [R][F] / hd [R][F/32]
void xr_gu_swiglu(const int8_t* xq, const float* xd, const float* src, const float* nw, float eps, int R,
                  const Q8Mat& W, int8_t* hq, float* hd, hipStream_t s);

// ---- device-resident decode state (kernels_decode.hip)
struct DecState {
    int* last_tok;   // [U] token fed at the next step
    int* gen;        // [U] tokens generated so far
    int* done;       // [U]
    const int* budget, *n_prompt, *base;  // [U]
    int* out;        // [U][params[5]] generated tokens
    const int* params;  // U, dummy KV slot, forced, eos0, eos1, ld_out
    int* counters;   // rows this step, active after accept, bound violated
};
void dec_plan(const DecState& st, int M_max, int* ids, int* pos, int* slot, int* kvs, int* kvl, int* row_utt,
              hipStream_t s);
// dec_plan followed, in the same single-workgroup launch, by embed_rows of the planned ids (no alternative rows) into
// x [M_max][E.K]: one launch fewer per step (small steps: the one workgroup writes every row)
void dec_plan_embed(const DecState& st, int M_max, int* ids, int* pos, int* slot, int* kvs, int* kvl, int* row_utt,
                    const Q8Mat& E, float* x, hipStream_t s);
constexpr int kPlanEmbedRows = 64;   // decode steps of up to this many rows take dec_plan_embed
void force_tokens(const DecState& st, int M_max, const int* row_utt, const int* ids, int ld, int* tok, hipStream_t s);
void dec_accept(const DecState& st, int M_max, const int* row_utt, const int* tok, hipStream_t s);
// argmax_rows' final stage (over argmax_rows_partial's keys) fused with dec_accept: tok[i] as argmax_rows gives it
void argmax_accept(const DecState& st, int M_max, const void* part, const int* row_utt, int* tok, hipStream_t s);
void copy_kv_prefix(__half* kc, __half* vc, int layers, int64_t kv_slots, int kvd, int64_t src, int P0,
                    const int* bases, int count, hipStream_t s);

}  // namespace qasr
