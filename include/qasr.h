/*
 * qasr.h — C ABI of libqasr, the MI355X-native (gfx950) Qwen3-ASR + FireRedVAD engine.
 *
 * This is the drop-in boundary for the light-whisper local ASR hot path.  Each entry point replaces one
 * interface the reference binds (paths relative to sypsyp97/light-whisper):
 *
 *   qasr_model_open        ← transcribe_cpp.Model(path, backend=)          src-tauri/resources/qwen3_asr_server.py:122
 *   qasr_session_open      ← Model.session(kv_type="f16", n_ctx=32768)     qwen3_asr_server.py:123
 *   qasr_session_run       ← Session.run(audio, timestamps="none")         qwen3_asr_server.py:144,321
 *                            (result.text / result.language, :326-327)
 *   qasr_session_close /
 *   qasr_model_close       ← Session.close() / Model.close()               qwen3_asr_server.py:100-112
 *   qasr_run_batch         ← (new) VAD-split batch of utterances, one call
 *   qasr_vad_open          ← FireRedVad.__init__ (knf fbank + ORT session) firered_vad.py:41-85
 *   qasr_vad_probabilities ← FireRedVad.probabilities                      firered_vad.py:106-111
 *   qasr_vad_speech_timestamps ← FireRedVad.speech_timestamps              firered_vad.py:116-119
 *   qasr_vad_timestamps_from_probabilities ← FireRedVad._timestamps_from_probabilities firered_vad.py:121-191
 *   qasr_decode_pcm_s16le  ← decode_inline_audio (pcm_s16le branch)        server_common.py:145-170
 *   qasr_resample_linear   ← Qwen3ASRServer._resample                      qwen3_asr_server.py:230-243
 *
 * Conventions: every function returns an int status (0 = OK); on failure qasr_last_error() returns a
 * thread-local UTF-8 message.  No C++ exception crosses the ABI.  Host buffers are plain pointers + sizes.
 * The qasr_op_* functions are the kernel-level entry points used by the parity tests: their pointer
 * arguments are DEVICE pointers and `stream` is a hipStream_t (NULL = default stream).
 * Only backend "hip" (alias "auto") exists: there is no CPU or Vulkan fallback; other names fail with
 * QASR_E_BACKEND, mirroring how transcribe_cpp rejects an unavailable backend (qwen3_asr_server.py:117-133).
 */
#ifndef QASR_H
#define QASR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QASR_API __attribute__((visibility("default")))

enum {
    QASR_OK = 0,
    QASR_E_INVALID = 1,
    QASR_E_IO = 2,
    QASR_E_FORMAT = 3,
    QASR_E_BACKEND = 4,
    QASR_E_HIP = 5,
    QASR_E_CAPACITY = 6,
    QASR_E_INTERNAL = 7,
};

typedef struct qasr_model qasr_model;
typedef struct qasr_session qasr_session;
typedef struct qasr_vad qasr_vad;

/* Model hyper-parameters (GGUF metadata "qwen3-asr.*"; see DESIGN.md §tensor names). */
typedef struct {
    int32_t n_mels, conv_ch, enc_d, enc_layers, enc_heads, enc_ffn, n_window, n_window_infer, proj_out;
    int32_t txt_h, txt_layers, txt_heads, txt_kv_heads, head_dim, txt_ffn, vocab;
    float rope_theta, rms_eps, ln_eps;
    /* special tokens of the chat prompt (defaults: Qwen2 tokenizer ids) */
    int32_t tok_im_start, tok_im_end, tok_system, tok_user, tok_assistant, tok_newline;
    int32_t tok_audio_start, tok_audio_end, tok_audio_pad, tok_eos0, tok_eos1, tok_asr_text;
} qasr_hparams;

typedef struct {
    char* text;         /* UTF-8, after "<asr_text>" (reference applies .strip() itself) */
    char* language;     /* the "language X" prefix, "" when absent */
    char* raw;          /* full detokenised output */
    int32_t* tokens;    /* generated ids (EOS excluded) */
    int32_t n_tokens;
    int32_t n_audio_tokens;
    int32_t n_prompt;
    double ms_mel, ms_encoder, ms_prefill, ms_decode;
    int32_t truncated;  /* 1: decoding stopped at the token budget, not at EOS (natural mode only) */
} qasr_result;

typedef struct {
    int32_t max_new_tokens;      /* 0 → until EOS or n_ctx for one utterance (the reference's session.run);
                                    a batch of several: 64 + 32·seconds each */
    int32_t force_tokens_per_s;  /* >0: throughput mode, exactly round(k·seconds)+1 tokens, EOS ignored */
    int32_t return_logits;       /* reserved */
} qasr_run_opts;

/* -------------------------------------------------------------------------------------------- errors */
QASR_API const char* qasr_last_error(void);
QASR_API const char* qasr_version(void);
QASR_API int qasr_device_info(char* name, size_t name_cap, double* mem_total_gb, int* n_devices);
QASR_API int qasr_set_device(int device);

/* -------------------------------------------------------------------------------------------- model */
QASR_API int qasr_model_open(const char* gguf_path, const char* backend, qasr_model** out);
/* Synthetic weights with the exact tensor shapes of `arch` ("qwen3-asr-0.6b" | "qwen3-asr-1.7b"), or of a
   custom qasr_hparams when arch == NULL; generated on the device from `seed` by the generator shared with
   the oracle.  Used when the GGUF weights are not provisioned. */
QASR_API int qasr_model_open_synthetic(const char* arch, const qasr_hparams* hp, uint64_t seed, qasr_model** out);
/* One-time weight broadcast (north_star "RCCL ... only to broadcast Q8 weights"): a model keeps every
   weight and table in ONE device blob whose offsets depend only on the hyper-parameters, so rank 0 loads (or
   generates) the model, every other rank opens a shell — the same layout allocated, nothing read or generated —
   and one collective over the blob (torch.distributed / RCCL, bench.py) makes the shells identical to rank 0's
   model.  gguf_path != NULL: hyper-parameters and tokenizer from the file's metadata (no tensor data read);
   otherwise arch / hp as qasr_model_open_synthetic.  Sessions refuse a shell until
   qasr_model_weights_received. */
QASR_API int qasr_model_open_shell(const char* gguf_path, const char* arch, const qasr_hparams* hp, qasr_model** out);
QASR_API int qasr_model_weight_blob(qasr_model* m, void** dev, size_t* bytes);
QASR_API int qasr_model_weights_received(qasr_model* m);
/* Precision of the model's GEMMs: "q8" (default — the reference's Q8_0 W8A8 arithmetic) or "mxfp8" (SURVEY §8(d)
   C5: the weights' OCP MXFP8 image — e4m3 + e8m0 per 32 — multiplied on the block-scaled fp8 matrix cores, the
   activations converted per GEMM; tolerance parity only).  Set it before opening sessions. */
QASR_API int qasr_model_set_precision(qasr_model* m, const char* mode);
QASR_API int qasr_model_hparams(const qasr_model* m, qasr_hparams* out);
QASR_API int64_t qasr_model_weight_bytes(const qasr_model* m);
/* copy one tensor back to host in its GGUF storage form (Q8_0 blocks / f32 / f16) — for parity tests */
QASR_API int qasr_model_export_tensor(const qasr_model* m, const char* name, void* dst, size_t cap, size_t* written);
/* JSON {name: [ggml type, rows, cols, conv_cin]} of every GGUF tensor the model holds (rows × cols in GGUF terms:
   Q8_0 matrices N × K; f32 vectors n × 1; f16 conv kernels Cout·Cin·9 × 1 with conv_cin = Cin).  buf == NULL:
   only *needed is set. */
QASR_API int qasr_model_tensor_table(const qasr_model* m, char* buf, size_t cap, size_t* needed);
QASR_API void qasr_model_close(qasr_model* m);

/* -------------------------------------------------------------------------------------------- session */
QASR_API int qasr_session_open(qasr_model* m, const char* kv_type, int32_t n_ctx, qasr_session** out);
QASR_API int qasr_session_run(qasr_session* s, const float* pcm16k, size_t n, int32_t timestamps, qasr_result* out);
/* Hot-word context (opt-in — the reference ignores hot_words): token ids placed in the system turn
   of the chat prompt (HF Qwen3-ASR `prompt=`, processing_qwen3_asr.py:513-538) for the session's following runs;
   n = 0 restores the reference's prompt.  qasr_model_tokenize: UTF-8 → ids as Qwen2Tokenizer.encode(text,
   add_special_tokens=False) (tokenization_qwen2.py: the Qwen2 pre-tokenizer regex, GPT-2 byte-level alphabet, the
   GGUF's tokenizer.ggml.merges by rank; NFC input assumed), or by greedy longest match when the vocabulary has no
   merges (synthetic models).  qasr_tokenizer_*: the same encoder on a given vocabulary + merge list. */
QASR_API int qasr_session_set_context(qasr_session* s, const int32_t* ids, int32_t n);
typedef struct qasr_tokenizer qasr_tokenizer;
QASR_API int qasr_tokenizer_open(const char* const* pieces, int32_t n_pieces, const uint8_t* is_special /* or NULL */,
                                 const char* const* merges, int32_t n_merges, qasr_tokenizer** out);
QASR_API int qasr_tokenizer_encode(const qasr_tokenizer* t, const char* text, size_t len, int32_t* ids, size_t cap,
                                   size_t* n_out);
QASR_API void qasr_tokenizer_close(qasr_tokenizer* t);
/* Streaming decode (the app's interim loop re-sends the last ≤ 12 s every 140-460 ms, interim.rs:
   135-156): on = 1 makes the session's single-utterance runs draft their continuation from its earlier transcripts
   (prompt lookup: the tokens that followed the same bigram before) and verify each draft in one teacher-forced pass
   whose every row runs the arithmetic of a 1-row decode step, so the accepted tokens are greedy's BIT FOR BIT (the
   transcript does not depend on the session's history).  stats: passes, draft tokens proposed, draft tokens
   accepted, tokens emitted.  set_draft_noise (benchmark / test hook, not in the reference): each proposed token is
   replaced by a random id with probability rate (acceptance below the 100 % of degenerate synthetic transcripts). */
QASR_API int qasr_session_set_draft(qasr_session* s, int32_t on);
QASR_API int qasr_session_set_draft_noise(qasr_session* s, float rate, uint64_t seed);
QASR_API int qasr_session_draft_stats(const qasr_session* s, int64_t* stats /* [4] */);
/* Batch invariance (opt-in; QASR_BATCH_INVARIANT=1 in the environment sets the default): on = 1 makes every
   utterance of a batch run (qasr_run_batch*) decode with the arithmetic of its own single-utterance run — the decode
   rows on the exact-row linears and attention chunking of a 1-row step, the front end, encoder and decoder prefill
   in the row-count-independent GEMM order — so its tokens are the same bits whatever else shares the batch or how
   many GPUs the job is sharded over (the reference decodes each request alone, qwen3_asr_server.py:321).  Q8
   precision only (ignored in MXFP8 mode).  Its cost on the C4 batch is measured in DESIGN.md §2. */
QASR_API int qasr_session_set_batch_invariant(qasr_session* s, int32_t on);
/* Streaming encoder cache: every single-utterance run encodes in a row-count-independent GEMM
   order (cache on or off), so a complete 8-chunk attention window's audio-embedding rows are a function of its
   samples and the request's log-mel maximum (Whisper-style normalisation; the conv stack is per 1 s chunk, the
   encoder attention per window).  on = 1 keeps the complete windows of each run (≥ one window) and reuses the
   previous run's (104 tokens each) whose frames lie in the samples both share bitwise (the interim loop's growing
   window, interim.rs:135-156) when the mel maximum is the same bits — encoding only the rest, bit-identical to the
   cache-off result.  A sliding window shares no prefix and reuses nothing.  stats: runs that took part, windows
   reused, windows encoded by them. */
QASR_API int qasr_session_set_encoder_cache(qasr_session* s, int32_t on);
QASR_API int qasr_session_encoder_cache_stats(const qasr_session* s, int64_t* stats /* [3] */);
/* With the encoder cache on, a run that reused the previous run's leading windows also keeps that run's K/V of the
   prompt rows they cover (the chat prefix + the reused audio tokens: same tokens, same positions, bit-identical —
   single-utterance prefill runs the row-count-independent GEMM order) and prefills only the rows after them
   (interim.rs:135-146's growing window).  *rows_reused: prompt rows taken over so far. */
QASR_API int qasr_session_prompt_kv_stats(const qasr_session* s, int64_t* rows_reused);
/* The audio-embedding rows (projector output, [tokens][text hidden] f32) of the session's last run — a test /
   debugging hook (transcribe.cpp exposes no equivalent).  out = NULL: *n_out = the float count only. */
QASR_API int qasr_session_audio_embeds(qasr_session* s, float* out, size_t cap, size_t* n_out);
QASR_API int qasr_model_tokenize(const qasr_model* m, const char* text, size_t len, int32_t* ids, size_t cap,
                                size_t* n_out);
/* ids → UTF-8 text (the transcript decoder: byte-level pieces, invalid sequences replaced as Python does) */
QASR_API int qasr_model_detokenize(const qasr_model* m, const int32_t* ids, int32_t n, char* out, size_t cap,
                                  size_t* written);
QASR_API int qasr_session_run_opts(qasr_session* s, const float* pcm16k, size_t n, const qasr_run_opts* opts,
                                   qasr_result* out);
/* Batched: `count` utterances (16 kHz f32 host buffers) encoded/prefilled/decoded together on this device. */
QASR_API int qasr_run_batch(qasr_session* s, const float* const* pcm, const size_t* n, int32_t count,
                            const qasr_run_opts* opts, qasr_result* out);
/* Same, audio already resident on the device: one packed f32 buffer, per-utterance offsets/lengths (host
   arrays).  This is the bench's timed entry point (inputs resident in HBM). */
QASR_API int qasr_run_batch_device(qasr_session* s, const float* dev_pcm, const int64_t* offsets,
                                   const int64_t* lengths, int32_t count, const qasr_run_opts* opts,
                                   qasr_result* out);
QASR_API void qasr_result_free(qasr_result* r);
QASR_API void qasr_session_close(qasr_session* s);
/* teacher-forced logits for parity tests: prompt (with audio placeholders) + forced continuation, one decode step
   per token; _verify: the continuation (≤ 32 tokens) in ONE draft verify pass of the streaming decode (same output
   layout) — the exact-row contract says both are the same bits */
QASR_API int qasr_session_forced_logits(qasr_session* s, const float* pcm16k, size_t n, const int32_t* forced,
                                        int32_t n_forced, float* logits_out /* [n_forced+1][vocab] */);
QASR_API int qasr_session_forced_logits_verify(qasr_session* s, const float* pcm16k, size_t n, const int32_t* forced,
                                               int32_t n_forced, float* logits_out /* [n_forced+1][vocab] */);
/* teacher forcing through the BATCHED path (packed prefill + continuous-batching decode steps with the batch's
   GEMMs; in MXFP8 precision the block-scaled MFMA GEMMs): utterance u is fed forced[u][0..n_forced) instead of its
   argmax; the logits of the utterances listed in want[0..n_want) are written [n_want][n_forced+1][vocab] (row j: after
   the prompt and forced[u][0..j)).  Eager steps; a parity-test hook (tests/test_model_real_gpu.py C5 test). */
QASR_API int qasr_session_forced_logits_batch(qasr_session* s, const float* const* pcm, const size_t* n,
                                              int32_t count, const int32_t* forced /* [count][n_forced] */,
                                              int32_t n_forced, const int32_t* want, int32_t n_want,
                                              float* logits_out);
/* the stages of one utterance, for layer-level parity tests (host outputs) */
QASR_API int qasr_session_mel(qasr_session* s, const float* pcm16k, size_t n, float* mel_out /*[n_mels][t_pad]*/,
                              int32_t* t_valid, int32_t* t_pad);
QASR_API int qasr_session_encode(qasr_session* s, const float* mel, int32_t t_pad, int32_t t_valid,
                                 float* audio_emb /*[n_tok][proj_out]*/, float* enc_out /*[n_tok][enc_d] or NULL*/,
                                 int32_t* n_tok);
QASR_API int qasr_session_prefill_logits(qasr_session* s, const float* embeds, int32_t n, float* logits /*[n][V]*/);

/* -------------------------------------------------------------------------------------------- VAD */
typedef struct {
    float threshold;               /* 0.5 */
    int32_t smooth_window_frames;  /* 5 */
    int32_t min_speech_duration_ms;  /* 150 */
    int32_t min_silence_duration_ms; /* 300 */
    int32_t speech_pad_ms;         /* 120 */
} qasr_vad_options;

typedef struct {
    int64_t start, end;  /* samples */
} qasr_segment;

QASR_API void qasr_vad_default_options(qasr_vad_options* o);
QASR_API int qasr_vad_open(const char* weights_path /* .qvad; NULL = bundled asset */, qasr_vad** out);
/* pcm: f32 in [-1,1) at 16 kHz (scaled ×32768 and clipped internally, firered_vad.py:89) */
QASR_API int qasr_vad_probabilities(qasr_vad* v, const float* pcm, size_t n, float* probs, size_t cap,
                                    size_t* n_frames);
QASR_API int qasr_vad_features(qasr_vad* v, const float* pcm, size_t n, float* feats /*[T][80] log-fbank*/,
                               size_t cap_frames, size_t* n_frames);
QASR_API int qasr_vad_speech_timestamps(qasr_vad* v, const float* pcm, size_t n, const qasr_vad_options* o,
                                        qasr_segment* out, size_t cap, size_t* n_out);
QASR_API int qasr_vad_timestamps_from_probabilities(const float* probs, size_t n_frames, int64_t audio_len,
                                                    const qasr_vad_options* o, qasr_segment* out, size_t cap,
                                                    size_t* n_out);
QASR_API void qasr_vad_close(qasr_vad* v);

/* -------------------------------------------------------------------------------------------- audio io */
/* returns the f32 sample count; base64 of pcm_s16le → f32 = s/32768 (server_common.py:145-170) */
/* Detokenised bytes → valid UTF-8 exactly as Python's bytes.decode("utf-8", errors="replace") (the Qwen2
   tokenizer's decode): every transcript string the library returns has been through it.  out may be NULL to size. */
QASR_API int qasr_utf8_replace_invalid(const char* in, size_t n, char* out, size_t cap, size_t* written);
QASR_API int qasr_decode_pcm_s16le(const char* b64, size_t len, float* out, size_t cap, size_t* n_out);
/* source_rate is the request's rate as given (a float rate is not truncated: `sample_rate or 16_000` feeds
   np.interp directly, qwen3_asr_server.py:252-253) */
QASR_API int qasr_resample_linear(const float* x, size_t n, double source_rate, float* out, size_t cap,
                                  size_t* n_out);

/* Path-mode input: Qwen3ASRServer._load_audio's file branch (qwen3_asr_server.py:256-267: sf.read float32 →
   channel mean → _resample) for WAV files (PCM 8/16/24/32, float32) → 16 kHz mono f32.  out == NULL: size only. */
QASR_API int qasr_audio_load_path(const char* path, float* out, size_t cap, size_t* n_out);
/* The model output's (language, transcription) split that session.run's result.language / result.text carry
   (qwen3_asr_server.py:326-327): restates the Qwen3-ASR reference parser (transformers processing_qwen3_asr.py:
   159-196, incl. its repetition fix); language "" = none.  Buffers may be NULL to size. */
QASR_API int qasr_parse_transcript(const char* raw, size_t n, char* language, size_t lang_cap, size_t* lang_len,
                                   char* text, size_t text_cap, size_t* text_len);

/* -------------------------------------------------------------------------------------------- kernel ops */
QASR_API int qasr_op_quant_rows(const float* x, int32_t M, int32_t K, int32_t ldx, int8_t* q, float* d, void* stream);
QASR_API int qasr_op_repack_q8(const uint8_t* blocks, int64_t nblk, int8_t* qs, void* sc, void* stream);
/* path: 0 auto, 1 GEMV (M <= 8), 2 MFMA GEMM, 3 / 4 / 5 GEMV with 1 / 2 / 4 columns per wave;
 * 16 + cfg + 32*splits: MFMA GEMM with a forced configuration (kernels_q8.hip kGemmCfgs, 0..15; 31 = heuristic)
 * and split-K count (0 heuristic) — tuning only.  epi: 0 store, 1 residual, 2 gelu */
QASR_API int qasr_op_linear_q8(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                               int32_t N, int32_t K, const float* bias, const float* res, float* y, int32_t ldy,
                               int32_t epi, int32_t path, void* stream);
QASR_API int qasr_op_rmsnorm_q8(const float* x, int32_t M, int32_t H, const float* w, float eps, int8_t* q, float* d,
                                void* stream);
QASR_API int qasr_op_layernorm_q8(const float* x, int32_t M, int32_t H, const float* w, const float* b, float eps,
                                  int8_t* q, float* d, float* y, void* stream);
QASR_API int qasr_op_swiglu_q8(const float* gu, int32_t M, int32_t F, int8_t* q, float* d, void* stream);
/* gate|up Q8 matrix [2F][K] (split planes) → rows interleaved by 16 in place (32j+t: t<16 gate 16j+t, else up
 * 16j+t-16), the layout the fused SwiGLU GEMM and qasr_op_swiglu_q8_interleaved read */
QASR_API int qasr_op_interleave_gate_up(int8_t* qs, void* sc, int32_t N, int32_t K, void* stream);
/* h = silu(x·Wgᵀ)·(x·Wuᵀ) quantised to Q8 rows (hq [M][N/2], hd [M][N/64]) in the GEMM epilogue; W interleaved */
QASR_API int qasr_op_gemm_swiglu_q8(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                    int32_t N, int32_t K, int8_t* hq, float* hd, void* stream);
/* Q8 GEMM with a fused output epilogue (M > 8, the MFMA path): epi 4 = erf-GELU(acc + bias) quantised to Q8 rows
   (yq [M][N] int8, yd [M][N/32] f32 block scales; y unused), epi 5 = f16(acc + bias) into y (__half, row stride
   ldy).  cfg: GEMM configuration (-1 = heuristic). */
/* MXFP8 precision mode: Q8 blocks (q int8, d f32 or f16) → OCP MXFP8 (e4m3 elements q·d·2^-E
   rounded to nearest even, e8m0 byte E+127 with E the smallest exponent putting the block maximum ≤ 448). */
QASR_API int qasr_op_q8_to_mx(const int8_t* q, const void* d, int32_t d_is_f16, int64_t nblk, uint8_t* q8,
                             uint8_t* s8, void* stream);
/* y = epi(X·Wᵀ) on MXFP8 operands (v_mfma_scale_f32_16x16x128_f8f6f4); epi as qasr_op_linear_q8 (0-2), 3 SwiGLU
   (yq/yd), 4 GELU+Q8 (yq/yd); cfg -1 auto, 0 128×128, 1 64×64, 2 64×128, 3 128×128 3-stage ring, 4 128×64.  K % 128 == 0. */
QASR_API int qasr_op_gemm_mx(const uint8_t* x8, const uint8_t* xs, int32_t M, const uint8_t* w8, const uint8_t* ws,
                             int32_t N, int32_t K, const float* bias, const float* res, float* y, int32_t ldy,
                             int32_t epi, int8_t* yq, float* yd, int32_t cfg, void* stream);
QASR_API int qasr_op_linear_q8_ex(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                  int32_t N, int32_t K, const float* bias, void* y, int32_t ldy, int32_t epi,
                                  int8_t* yq, float* yd, int32_t cfg, void* stream);
QASR_API int qasr_op_swiglu_q8_interleaved(const float* gu, int32_t M, int32_t F, int8_t* q, float* d, void* stream);
/* The 1–4-row decoder GEMV (about one workgroup per CU) with the row operations around it fused; bit-identical to
   the separate launches.  pro 0: activations = the Q8 rows xq [M][K] / xd [M][K/32], K ≤ 6144; pro 1: activations
   = Q8(RMSNorm(src)·nw), src rows of K floats at stride ld_src, K ≤ 4096.  epi 0 store / 1 residual into y (y may
   alias res), or 3 (pro 1 only): W = gate/up interleaved by 16 (qasr_op_interleave_gate_up), N % 64 == 0, output
   h = Q8(silu(g)·u) rows hq [M][N/2] / hd [M][N/64].  M ≤ 4. */
QASR_API int qasr_op_gemv_fused(int32_t pro, const float* src, int32_t ld_src, const float* nw, float eps, int32_t M,
                                const int8_t* xq, const float* xd, const int8_t* wqs, const void* wsc, int32_t N,
                                int32_t K, const float* res, float* y, int32_t ldy, int32_t epi, int8_t* hq,
                                float* hd, void* stream);
/* The draft verify passes' exact-row linear on the matrix core (engine.cpp, ≥ 5 rows): y = X·Wᵀ (epi 0) or y = res +
   X·Wᵀ (epi 1, y may alias res) with bit for bit the arithmetic of qasr_op_gemv_fused(pro 0) on each row alone — the
   exact-row contract that makes drafted decoding emit greedy's tokens (qwen3_asr_server.py:321's session.run is one
   greedy decode; the batch-invariant decode's linears).  M ≥ 1 (32-row chunks in one launch), K a multiple of 1,024
   (K/1024 ∈ {1,2,3,4,6}). */
QASR_API int qasr_op_gemm_exact_rows(const int8_t* xq, const float* xd, int32_t M, const int8_t* wqs, const void* wsc,
                                     int32_t N, int32_t K, const float* res, float* y, int32_t ldy, int32_t epi,
                                     void* stream);
QASR_API int qasr_op_qk_norm_rope(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                  const int32_t* pos, const int32_t* slot, const float* qnw, const float* knw,
                                  const float* rope_cs, float eps, void* qout, void* kc, void* vc, void* stream);
/* decode attention with the q/k norm + RoPE and the KV-cache write fused in (hd 128): qkv f32 rows as for
   qasr_op_qk_norm_rope, K/V caches as for qasr_op_attention (ld = nkv·hd); output Q8 rows (oq, od).  Same
   results as qasr_op_qk_norm_rope followed by qasr_op_attention. */
QASR_API int qasr_op_attention_decode_fused(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                            const int32_t* pos, const int32_t* slot, const float* qnw,
                                            const float* knw, const float* rope_cs, float eps, void* kc, void* vc,
                                            const int32_t* kv_start, const int32_t* kv_len, float scale, int8_t* oq,
                                            float* od, void* stream);
/* The same for ≤ 4 rows with key ranges longer than 768 split over up to 16 workgroups per (row, KV head): part =
   4·nkv·16·G·130 floats of scratch, cnt = 4·nkv int32 counters, zero before the first call (left zero by every call).
   Same math up to the f32 order of the pieces' merge (flash-decoding). */
QASR_API int qasr_op_attention_decode_split(const float* qkv, int32_t rows, int32_t nh, int32_t nkv, int32_t hd,
                                            const int32_t* pos, const int32_t* slot, const float* qnw,
                                            const float* knw, const float* rope_cs, float eps, void* kc, void* vc,
                                            const int32_t* kv_start, const int32_t* kv_len, float scale, int8_t* oq,
                                            float* od, float* part, int32_t* cnt, void* stream);
QASR_API int qasr_op_attention(const void* q, int32_t ldq, const void* k, const void* v, int32_t ldkv,
                               const int32_t* kv_start, const int32_t* kv_len, int32_t rows, int32_t nh, int32_t nkv,
                               int32_t hd, float scale, float* o, int8_t* oq, float* od, void* stream);
/* Same contract; dense != 0 selects the MFMA tile kernel (runs of 16 consecutive rows sharing their key range:
   prefill prompt rows, encoder windows); P·V in f16 (see DESIGN.md §2 for the tolerance). */
QASR_API int qasr_op_attention_dense(const void* q, int32_t ldq, const void* k, const void* v, int32_t ldkv,
                                     const int32_t* kv_start, const int32_t* kv_len, int32_t rows, int32_t nh,
                                     int32_t nkv, int32_t hd, float scale, float* o, int8_t* oq, float* od,
                                     int32_t dense, void* stream);
QASR_API int qasr_op_argmax(const float* x, int32_t M, int32_t V, int32_t* out, void* stream);
QASR_API int qasr_op_embed_rows(const int32_t* ids, int32_t n, const int8_t* wqs, const void* wsc, int32_t K,
                                const float* alt, float* out, void* stream);
QASR_API int qasr_op_synth_q8(uint64_t seed, const char* name, int64_t N, int64_t K, float sigma, int8_t* qs, void* sc,
                              void* stream);
QASR_API int qasr_op_rope_table(int32_t n_ctx, int32_t head_dim, float theta, float* host_out /*[n_ctx][hd/2][2]*/);
QASR_API int qasr_op_mel(const float* pcm, int64_t n, int32_t n_mels, float* mel /*[n_mels][t_pad]*/, void* stream);
/* conv 3×3 stride 2 pad 1 + GELU (audio encoder conv2/conv3): in f16 [n_chunks][Hi][Wi][C] channel-last, w f16
 * [Cout=C][9][Cin=C] (tap-major), out_mode 0: f16 [chunk][Ho][Wo][C]; 1: f32 [chunk][Wo][C][Ho] */
QASR_API int qasr_op_conv3x3_gelu(const void* in, int32_t n_chunks, int32_t Hi, int32_t Wi, const void* w,
                                  const float* bias, int32_t C, void* out, int32_t out_mode, void* stream);
QASR_API int qasr_op_fbank(const float* pcm, int64_t n, float* feats /*[T][80]*/, void* stream);
QASR_API int qasr_stream_sync(void* stream);

/* Deterministic mode (process-wide, DEFAULT ON; QASR_ATOMICS=1 in the environment starts the process with it off):
   GEMMs never add split-K partial sums with float atomics (whose landing order varies run to run, a last-ulp
   difference that can flip a near-tie) — splits go through the ordered fix-up or do not happen — so every run of
   the same input gives bit-identical logits and tokens.  on = 0 is a throughput A/B knob only.  Sessions
   re-capture their step graphs after a switch.  qasr_get_deterministic reports the current mode. */
QASR_API int qasr_set_deterministic(int32_t on);
QASR_API int qasr_get_deterministic(int32_t* on);

/* -------------------------------------------------------------------------------------------- multi-GPU */
/* Native RCCL collectives (north_star: "RCCL over xGMI used only to broadcast Q8 weights and gather
   token streams"), so a host without PyTorch (the Rust app) drives the N-GPU path over this ABI.
   One process per GPU.  Rank 0 calls qasr_dist_unique_id and hands the 128 bytes to every rank out of band (a pipe,
   a file, a TCP store); each rank calls qasr_dist_init with its rank, the world size and its device.
   qasr_dist_broadcast_weights: ONE broadcast of the model's weight blob from `root` (which loaded or generated it)
   into the other ranks' shells (qasr_model_open_shell: identical layout), then every rank's wrapping 64-bit blob
   checksum all-gathered and compared (error if any differs); the shells then accept sessions.
   qasr_dist_broadcast: the same collective on any device buffer (send NULL = in place).
   qasr_dist_gather_tokens: every rank's segments' token ids ([n_seg] lengths + the flat ids, host arrays) to every
   rank, in rank order: rank_segs [world] = segments per rank; with all_lens / all_tokens NULL only the totals are
   reported (*n_segs_out, *n_tokens_out), then call again with buffers of that size.  Not in the reference (it runs
   one process, one device, one utterance).
   qasr_dist_agree: status agreement before a collective — every rank passes its local status (0 = this rank's
   previous step succeeded, anything else = it failed) and gets *any_failed = 1 on every rank if any rank's was
   nonzero (one all-gather of an int32).  A host calls it before each collective after the communicator exists
   (weight broadcast, probability gather, token gather): a rank whose VAD or batch failed then makes every rank
   return an error instead of leaving the others blocked inside the next collective (the reference's crash
   detection, funasr_service.rs:1367-1385, sees one process exit; engine_longform.cpp is the worked example). */
typedef struct qasr_comm qasr_comm;
typedef struct {
    uint64_t bytes;      /* blob bytes broadcast */
    double ms;           /* wall time of the broadcast */
    uint64_t checksum;   /* the root's wrapping 64-bit blob sum */
    int32_t checksums_agree;
} qasr_dist_info;
QASR_API int qasr_dist_unique_id(uint8_t* out /* 128 bytes */, size_t cap);
QASR_API int qasr_dist_init(const uint8_t* id /* 128 bytes */, int32_t rank, int32_t world, int32_t device,
                            qasr_comm** out);
/* qasr_dist_init with an explicit deadline (ms; <= 0: QASR_DIST_TIMEOUT_MS from the environment, else 300,000) for
   the init and for every later collective on the communicator: a rank that never calls init (it crashed before it) or
   never enters a collective makes the others return QASR_E_BACKEND at the deadline instead of blocking forever (an
   init that timed out is abandoned on a helper thread; a collective's communicator is aborted and every later call
   on it fails at once).  After such an error the host is expected to exit, as the reference's engine does; after an init
   timeout it should leave with _exit (the abandoned thread is still inside RCCL, and runtime teardown at a normal exit
   may fault — seen from a Python host; the C++ `engine longform` exits 1 cleanly).  qasr_dist_init = this with timeout_ms 0.  RCCL may print its version banner on stdout during
   qasr_dist_unique_id / init: a host whose stdout is a protocol channel points fd 1 elsewhere around these calls
   (the library does not touch process-wide file descriptors; engine_longform.cpp and qasr/dist.py do it). */
QASR_API int qasr_dist_init_deadline(const uint8_t* id /* 128 bytes */, int32_t rank, int32_t world, int32_t device,
                                     double timeout_ms, qasr_comm** out);
QASR_API void qasr_dist_close(qasr_comm* c);
QASR_API int qasr_dist_broadcast(qasr_comm* c, const void* send, void* recv, size_t bytes, int32_t root);
QASR_API int qasr_dist_broadcast_weights(qasr_comm* c, qasr_model* m, int32_t root, qasr_dist_info* info);
QASR_API int qasr_dist_gather_tokens(qasr_comm* c, const int32_t* lens, int32_t n_seg, const int32_t* tokens,
                                     int32_t* rank_segs /* [world] */, int32_t* all_lens, size_t lens_cap,
                                     int32_t* all_tokens, size_t tokens_cap, size_t* n_segs_out, size_t* n_tokens_out);
QASR_API int qasr_dist_agree(qasr_comm* c, int32_t local_status, int32_t* any_failed);

/* -------------------------------------------------------------------------------------------- profiling */
/* live per-kernel-class timing (hipEvents on each instrumented launch's stream) + algorithmic FLOPs/bytes;
   report = JSON {"gemm_q8": {"count", "ms", "flops", "bytes"}, ...}.  Used by bench.py for its roofline. */
QASR_API int qasr_prof_enable(int on);
QASR_API int qasr_prof_reset(void);
QASR_API int qasr_prof_report(char* buf, size_t cap, size_t* needed);

#ifdef __cplusplus
}
#endif

/* Engine-internal tuning and A/B hooks (forced GEMM configurations, split-K fix-up workspace, weight-streaming row
   limit, stage-scale registration) live in qasr_tune.h: they are not part of the drop-in boundary. */
#endif /* QASR_H */
