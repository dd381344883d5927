// Session: the ASR pipeline for one device — log-mel → conv stack → windowed encoder → projector →
// prompt splice → packed prefill → continuous-batching greedy decode with an f16 KV cache → detokenise.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "kernels_audio.h"
#include "model.h"

namespace qasr {

// grow-only device scratch buffers
struct Scratch {
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    std::vector<Buf> bufs;
    uint64_t epoch = 0;  // bumped on every reallocation (captured graphs hold the old pointers)
    bool capturing = false;  // a graph capture is in progress: growth would be a bug (throws)
    void* get(int slot, size_t bytes);
    ~Scratch();
};

struct UttResult {
    std::vector<int32_t> tokens;
    std::string raw, text, language;
    int n_audio = 0, n_prompt = 0;
    bool truncated = false;   // stopped at the token budget, not at EOS (natural mode)
};

struct StageTimes {
    double mel = 0, encoder = 0, prefill = 0, decode = 0;
};

class Session {
   public:
    Session(Model* m, int n_ctx);
    ~Session();
    Session(const Session&) = delete;
    Session& operator=(const Session&) = delete;

    // audio on the device, packed; per-utterance offsets/lengths on the host
    void run_batch(const float* dpcm, const std::vector<int64_t>& off, const std::vector<int64_t>& len,
                   int max_new, int force_tps, std::vector<UttResult>& out, StageTimes* times);
    // host audio convenience
    void run_host(const std::vector<const float*>& pcm, const std::vector<int64_t>& len, int max_new, int force_tps,
                  std::vector<UttResult>& out, StageTimes* times);

    // stages (parity tests)
    void mel_host(const float* pcm, int64_t n, std::vector<float>& mel, int& t_valid, int& t_pad);
    void encode_host(const float* mel, int t_pad, int t_valid, std::vector<float>& emb, std::vector<float>* enc,
                     int& n_tok);
    void prefill_logits_host(const float* embeds, int n, std::vector<float>& logits);
    // one_pass: the forced continuation in ONE draft verify pass (n_forced ≤ kDraftRows) instead of one step each
    void forced_logits_host(const float* pcm, int64_t n, const int32_t* forced, int n_forced,
                            std::vector<float>& logits, bool one_pass = false);
    // teacher forcing through the BATCHED path (run_batch: packed prefill, continuous-batching decode steps with the
    // batch's GEMMs — in MXFP8 precision the block-scaled MFMA GEMMs): every utterance is fed forced[u][0..n_forced)
    // instead of its argmax, and the logits of the utterances in `want` are returned, [n_want][n_forced + 1][V]
    // (row j: after the prompt and forced[u][0..j)).  Eager steps (no step graphs); a test / parity hook.
    void forced_logits_batch_host(const std::vector<const float*>& pcm, const std::vector<int64_t>& len,
                                  const int32_t* forced, int n_forced, const std::vector<int>& want, float* out);

    Model& model() { return *m_; }
    int n_ctx() const { return n_ctx_; }
    // system-prompt context tokens for the following runs (hot-word biasing; empty = the reference's prompt)
    void set_context(const std::vector<int32_t>& ids) { context_ = ids; }
    // streaming decode: single-utterance runs draft their continuation from the session's previous
    // transcripts (prompt-lookup: the tokens that followed the same bigram last time) and verify a whole draft in one
    // teacher-forced pass; the accepted tokens are exactly greedy's (up to near-ties of f32 summation order)
    void set_draft(bool on) { draft_ = on; }
    // batch invariance (round 4): a batch's decode rows each run the 1-row decode step's arithmetic (the exact-row
    // linears, the fixed-chunk split attention, the exact-row vocabulary projection) and its front end / encoder /
    // decoder prefill the row-count-independent GEMM order, so an utterance's tokens are the bits of its own
    // single-utterance run whatever else shares the batch (or the GPU count).  Q8 precision only.
    // Default: QASR_BATCH_INVARIANT=1 in the environment.
    void set_batch_invariant(bool on) { batch_inv_ = on; }
    bool batch_invariant() const { return batch_inv_; }
    // benchmark / test hook: each proposed draft token is replaced by a random id with probability `rate` (draft
    // acceptance below the degenerate 100 % of synthetic weights; the output stays greedy's, only the speed changes)
    void set_draft_noise(float rate, uint64_t seed) {
        draft_noise_ = rate;
        noise_state_ = seed;
    }
    struct DraftStats {
        int64_t passes = 0, proposed = 0, accepted = 0, tokens = 0;
    };
    const DraftStats& draft_stats() const { return dstats_; }
    // streaming encoder cache: a single-utterance run whose samples extend the previous run's (the
    // app's growing interim window) reuses the audio-embedding rows of the previous run's complete 8-chunk attention
    // windows when the window's mel maximum is unchanged — those rows are then a function of the same samples
    void set_enc_cache(bool on) {
        enc_cache_ = on;
        ec_windows_ = 0;
    }
    struct EncCacheStats {
        int64_t runs = 0, windows_reused = 0, windows_computed = 0;
    };
    const EncCacheStats& enc_cache_stats() const { return ecstats_; }
    // prompt rows whose K/V a single-utterance run took from the previous run instead of prefilling them
    struct PromptKvStats {
        int64_t rows_reused = 0;
    };
    const PromptKvStats& prompt_kv_stats() const { return kvp_stats_; }
    // the audio-embedding rows (projector output, [tokens][H]) of the last single-utterance run (tests)
    std::vector<float> last_audio_embeds();
    hipStream_t stream() const { return st_; }

   private:
    struct FrontEnd {
        int total_chunks = 0, total_tokens = 0;
        int skip_tokens = 0;   // leading audio tokens taken from the encoder cache (not encoded)
        std::vector<int> n_tok, tok_base;
    };
    void front_end(const float* dpcm, const std::vector<int64_t>& off, const std::vector<int64_t>& len, FrontEnd& fe,
                   float* enc_out_dbg);
    void encoder(FrontEnd& fe, float* enc_out_dbg);
    // rows_share_kv: rows are consecutive positions of ONE utterance (a draft verify pass), so row i attends the K/V
    // rows 0…i-1 write in the same layer — the K/V write then runs as its own launch before the attention (the
    // fused decode attention writes each row's K/V in its own workgroup, unordered against the others)
    void decoder_layers(float* x, int rows, const int* d_pos, const int* d_slot, const int* d_kvs, const int* d_kvl,
                        int64_t total_keys, bool dense = false, bool rows_share_kv = false);
    void ensure_kv(int64_t slots);
    void enc_cache_store(int64_t n, int total_tokens);
    // keys: Σ key-range lengths of the step's rows when known on the host (profiling's algorithmic bytes), else 0
    void decode_step(const DecState& ds, int B, bool sizing, int64_t keys = 0);
    // one verify pass of B rows (last accepted token + draft, padded): tables in S_DTAB, argmax → pinned host
    void draft_step(int B);
    void draft_pass(int B);
    void draft_graphs_refresh();
    void draft_decode(int n_prompt, int base, int budget, int dummy, std::vector<int32_t>& toks, bool& eos,
                      bool forced);
    // exact: every row with the 1-row arithmetic (verify passes; ≤ 4 rows always are)
    void lm_head_rows(const float* x, int rows, int ldx, float* logits, bool exact = false);
    // diagnosis (QASR_DUMP_DIR set): a decode-sized stage's output rows to $QASR_DUMP_DIR/<seq>_<what>_L<l>_r<rows>.bin
    void dump_rows(const char* what, int l, int rows, const void* p, size_t bytes);
    void mx_ws(int64_t rows, int64_t kmax);
    template <class T>
    T* upload(int slot, const std::vector<T>& v);

    Model* m_;
    int n_ctx_;
    std::vector<int32_t> context_;
    hipStream_t st_ = nullptr;
    Scratch sc_;
    __half* kc_ = nullptr;
    __half* vc_ = nullptr;
    int64_t kv_slots_ = 0;
    float* rope_ = nullptr;
    int rope_n_ = 0;
    // pinned host staging for per-step uploads / downloads
    void* pin_ = nullptr;
    size_t pin_cap_ = 0;
    void* pinned(size_t bytes);
    // decode loop: pinned active-count word, per-step events, step graphs per row bucket
    void* pin_cnt_ = nullptr;
    hipEvent_t step_ev_[2] = {nullptr, nullptr};
    std::map<int, hipGraphExec_t> graphs_;
    std::map<int, hipGraphExec_t> draft_graphs_;
    uint64_t draft_key_[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    bool draft_ = false;
    float draft_noise_ = 0.f;
    uint64_t noise_state_ = 0;
    // 1–4-row decode: norms / SwiGLU fused into the GEMV prologues (QASR_NO_DEC_FUSE=1: the separate launches,
    // for A/B parity and timing; read once per session, so captured step graphs stay consistent)
    bool dec_fuse_ = getenv("QASR_NO_DEC_FUSE") == nullptr;
    // ≤ 4-row decode attention over > QkFuse::split_min keys split over workgroups (QASR_NO_ATTN_SPLIT=1: one per row and
    // KV head); the scratch is the session's own (allocated with it, counters zeroed)
    bool attn_split_ = getenv("QASR_NO_ATTN_SPLIT") == nullptr;
    float* attn_part_ = nullptr;
    int* attn_cnt_ = nullptr;
    int attn_rows_ = 0;          // rows attn_part_ / attn_cnt_ are sized for
    uint64_t attn_epoch_ = 0;    // bumped when they are reallocated (captured step graphs hold the pointers)
    void ensure_attn_split(int rows);
    bool batch_inv_ = [] {
        const char* e = getenv("QASR_BATCH_INVARIANT");
        return e && atoi(e) != 0;
    }();
    // batched teacher forcing (forced_logits_batch_host): device table of forced ids [count][ld] (-1: keep argmax),
    // the wanted utterances' output slots, the step counter
    struct TeacherForce {
        int* d_ids = nullptr;
        int ld = 0, n_forced = 0, step = 0;
        std::vector<int> want;   // utterance → output index (-1: not wanted)
        float* out = nullptr;
    };
    TeacherForce* tf_ = nullptr;
    void tf_capture(const float* logits, int rows, const int* row_utt);
    void* xr_split_mem_ = nullptr;   // the xr launches' leaf-split scratch (kernels.h XrSplit)
    XrSplit xr_split_{};
    unsigned* xr_cnt_ = nullptr;   // the residual xr launches' fused-norm counters (3 words, zero between launches)
    void xr_check();
    // split-K fix-up workspace of the decode-step GEMMs (≤ 256 rows; QASR_NO_FIXUP=1: f32 atomics instead): partial
    // tiles + per-tile arrival counters (zeroed once; the kernels leave them zero)
    float* fix_part_ = nullptr;
    size_t fix_floats_ = 0;
    unsigned* fix_cnt_ = nullptr;
    // draft length control: decayed counts of accepted draft tokens and of rejections (the per-token acceptance
    // estimate a = S / (S + F)), kept across requests; the prior a ≈ 0.89
    double draft_s_ = 4.0, draft_f_ = 0.5;
    std::vector<int32_t> history_;   // previous transcripts (the lookup corpus), oldest first
    int hist_last_ = 0;              // where the latest transcript starts in history_
    DraftStats dstats_;
    // encoder cache: the previous single-utterance run's samples, mel maximum, precision generation and the
    // embedding rows of its ec_windows_ complete windows (ec_emb_, device); ec_cand_ = windows the current run's
    // sample prefix allows (run_host → front_end)
    bool enc_cache_ = false;
    std::vector<float> ec_pcm_;
    unsigned ec_umax_ = 0;
    uint64_t ec_prec_ = 0;
    int ec_windows_ = 0, ec_cand_ = 0;
    bool ec_run_ = false;
    float* ec_emb_ = nullptr;
    size_t ec_cap_ = 0;
    EncCacheStats ecstats_;
    PromptKvStats kvp_stats_;
    int last_audio_tokens_ = 0;
    // prompt-KV reuse (run_batch): rows [0, kvp_rows_) of the KV cache hold the last completed single-utterance run's
    // prompt K/V, valid while kvp_key_ (KV epoch, precision, determinism) and the prompt prefix still match
    int kvp_rows_ = 0;
    uint64_t kvp_key_[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    std::vector<int32_t> kvp_prefix_;
    bool kv_reuse_ = getenv("QASR_NO_PROMPT_KV_REUSE") == nullptr;
    // scratch epoch, KV epoch, precision gen, determinism gen, split-attention scratch epoch + batch invariance
    uint64_t graph_key_[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    uint64_t kv_epoch_ = 0;
    int ucap_ = 0;
};
int row_bucket(int m);
// rows of a draft verify pass at most (the last accepted token + up to kDraftRows − 1 proposed tokens)
constexpr int kDraftRows = 32;

// the chat prompt of one utterance (processing_qwen3_asr.py:534-553, empty system prompt); audio
// placeholders are returned as -(audio_row + 1)
std::vector<int32_t> build_prompt(const qasr_hparams& hp, int n_audio, int audio_row0);
extern const int kPromptPrefix;   // prompt tokens before the audio, shared by every utterance
int audio_token_count(int t_valid);
void mel_dims(int64_t n, int& t_valid, int& t_pad);

}  // namespace qasr
