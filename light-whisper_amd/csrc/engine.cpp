// Host orchestration of the ASR hot path on one MI355X (see engine.h).  All compute is HIP kernels on
// one stream; the host only builds index tables (prompt layout, window ranges, KV slots) and reads back
// one int32 per active utterance per decode step.
#include "engine.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <climits>
#include <cstdio>
#include <map>
#include <chrono>

#include "capi_util.h"
#include "kernels.h"

namespace qasr {

namespace {
enum SlotId {
    S_UTTS, S_WORK, S_CHUNK_UTT, S_UMAX, S_LM, S_MELX, S_A1, S_A2, S_A3, S_XQ, S_XD, S_PROJ, S_VALID, S_HS,
    S_QKV, S_QKVH, S_FF, S_KVS, S_KVL, S_EMB, S_IDS, S_POS, S_SLOT, S_X, S_QH, S_GU, S_LAST, S_XN, S_LOGITS,
    S_TOK, S_PCM, S_ENC, S_DSTATE, S_DOUT, S_DTAB, S_ARGP, S_HQ, S_HD, S_MX, S_COUNT
};

inline int post_cnn_len(int l) {
    for (int i = 0; i < 3; i++) l = l > 0 ? (l - 1) / 2 + 1 : 0;
    return l;
}

struct Timer {
    hipEvent_t a, b;
    hipStream_t s;
    double* out;
    Timer(hipStream_t st, double* o) : s(st), out(o) {
        if (!out) return;
        QASR_HIP(hipEventCreate(&a));
        QASR_HIP(hipEventCreate(&b));
        QASR_HIP(hipEventRecord(a, s));
    }
    ~Timer() {
        if (!out) return;
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        *out += ms;
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
    }
};

__global__ void k_gather_rows(const float* __restrict__ x, const int* __restrict__ idx, int n, int H,
                              float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * H) return;
    const int r = (int)(i / H), c = (int)(i % H);
    y[i] = x[(size_t)idx[r] * H + c];
}
}  // namespace

int audio_token_count(int t_valid) { return (t_valid / 100) * 13 + post_cnn_len(t_valid % 100); }

void mel_dims(int64_t n, int& t_valid, int& t_pad) {
    const int64_t nn = std::max<int64_t>(n, 8000);  // min_length (feature_extraction_qwen3_asr.py:192-196)
    t_valid = (int)((nn + 159) / 160);
    t_pad = (t_valid + 99) / 100 * 100;
}

const int kPromptPrefix = 9;   // prefix tokens before the audio without a system context

// chat prompt (processing_qwen3_asr.py:534-553): the optional system context (hot words, SURVEY §8(f) 4: opt-in,
// the reference sends none) sits between "system\n" and its <|im_end|>, like HF's `prompt=` system message
std::vector<int32_t> build_prompt(const qasr_hparams& h, int n_audio, int audio_row0,
                                  const std::vector<int32_t>& context = {}) {
    std::vector<int32_t> p = {h.tok_im_start, h.tok_system, h.tok_newline};
    p.insert(p.end(), context.begin(), context.end());
    const int32_t pre[] = {h.tok_im_end, h.tok_newline, h.tok_im_start, h.tok_user, h.tok_newline, h.tok_audio_start};
    p.insert(p.end(), pre, pre + 6);
    for (int i = 0; i < n_audio; i++) p.push_back(-(audio_row0 + i + 1));
    const int32_t tail[] = {h.tok_audio_end, h.tok_im_end, h.tok_newline, h.tok_im_start, h.tok_assistant,
                            h.tok_newline};
    p.insert(p.end(), tail, tail + 6);
    return p;
}

void* Scratch::get(int slot, size_t bytes) {
    if ((int)bufs.size() <= slot) bufs.resize(slot + 1);
    Buf& b = bufs[slot];
    bytes = std::max<size_t>(bytes, 256);
    if (b.cap < bytes) {
        QASR_CHECK(!capturing, QASR_E_INTERNAL, "scratch growth during graph capture");
        if (b.p) {
            QASR_HIP(hipDeviceSynchronize());  // queued kernels may still use the old buffer
            QASR_HIP(hipFree(b.p));
        }
        b.p = nullptr;
        epoch++;
        const size_t cap = bytes + bytes / 4;
        QASR_HIP(hipMalloc(&b.p, cap));
        b.cap = cap;
    }
    return b.p;
}
Scratch::~Scratch() {
    for (auto& b : bufs)
        if (b.p) (void)hipFree(b.p);
}

Session::Session(Model* m, int n_ctx) : m_(m), n_ctx_(n_ctx) {
    QASR_CHECK(n_ctx > 32, QASR_E_INVALID, "n_ctx too small");
    QASR_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    // counters [0, 8), draft tokens [8, 8 + kDraftRows), the encoder cache's mel-maximum read-back [60]
    QASR_HIP(hipHostMalloc(&pin_cnt_, 256, hipHostMallocDefault));
    for (auto& e : step_ev_) QASR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    rope_n_ = n_ctx;
    std::vector<float> tab((size_t)n_ctx * m->hp.head_dim);
    rope_table(n_ctx, m->hp.head_dim, m->hp.rope_theta, tab.data());
    QASR_HIP(hipMalloc(&rope_, tab.size() * sizeof(float)));
    QASR_HIP(hipMemcpy(rope_, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice));
    // the reference session reserves the full f16 KV for n_ctx (qwen3_asr_server.py:123); + the dummy slot
    ensure_kv(n_ctx + 1);
    // split-K decode attention scratch (≤ 4 rows over long key ranges): partial states + zeroed arrival counters
    const int nkv = m->hp.txt_kv_heads, G = nkv > 0 ? m->hp.txt_heads / nkv : 1;
    if (m->hp.head_dim == 128 && nkv > 0) {
        ensure_attn_split(kExactRows);
    }
    // split-K fix-up of the decode GEMMs: up to kFixSplits partial tiles of 256 rows × the widest decoder weight
    const qasr_hparams& hp = m->hp;
    const size_t widest = (size_t)std::max(std::max(2 * hp.txt_ffn, hp.txt_h),
                                           (hp.txt_heads + 2 * hp.txt_kv_heads) * hp.head_dim);
    QASR_HIP(hipMalloc(&xr_cnt_, 4 * sizeof(unsigned)));
    QASR_HIP(hipMemset(xr_cnt_, 0, 4 * sizeof(unsigned)));
    // the xr launches' leaf split (two workgroups per 16-column fragment): partial trees + arrival counters
    QASR_HIP(hipMalloc(&xr_split_mem_, xr_split_bytes()));
    QASR_HIP(hipMemset(xr_split_mem_, 0, xr_split_bytes()));
    xr_split_ = xr_split_view(xr_split_mem_);
    const char* nofix = getenv("QASR_NO_FIXUP");
    if (!nofix || atoi(nofix) == 0) {
        fix_floats_ = (size_t)256 * ((widest + 127) / 128 * 128) * kFixSplits;
        QASR_HIP(hipMalloc(&fix_part_, fix_floats_ * sizeof(float)));
        QASR_HIP(hipMalloc(&fix_cnt_, (size_t)kFixCounters * sizeof(unsigned)));
        QASR_HIP(hipMemset(fix_cnt_, 0, (size_t)kFixCounters * sizeof(unsigned)));
    }
}

Session::~Session() {
    if (kc_) (void)hipFree(kc_);
    if (vc_) (void)hipFree(vc_);
    if (rope_) (void)hipFree(rope_);
    if (attn_part_) (void)hipFree(attn_part_);
    if (attn_cnt_) (void)hipFree(attn_cnt_);
    if (fix_part_) (void)hipFree(fix_part_);
    if (ec_emb_) (void)hipFree(ec_emb_);
    if (fix_cnt_) (void)hipFree(fix_cnt_);
    if (xr_cnt_) (void)hipFree(xr_cnt_);
    if (xr_split_mem_) (void)hipFree(xr_split_mem_);
    if (pin_) (void)hipHostFree(pin_);
    for (auto& g : graphs_) (void)hipGraphExecDestroy(g.second);
    for (auto& g : draft_graphs_) (void)hipGraphExecDestroy(g.second);
    for (auto& e : step_ev_)
        if (e) (void)hipEventDestroy(e);
    if (pin_cnt_) (void)hipHostFree(pin_cnt_);
    if (st_) (void)hipStreamDestroy(st_);
}

void* Session::pinned(size_t bytes) {
    if (pin_cap_ < bytes) {
        if (pin_) QASR_HIP(hipHostFree(pin_));
        pin_cap_ = std::max<size_t>(bytes, 1 << 16);
        QASR_HIP(hipHostMalloc(&pin_, pin_cap_, hipHostMallocDefault));
    }
    return pin_;
}

template <class T>
T* Session::upload(int slot, const std::vector<T>& v) {
    T* d = (T*)sc_.get(slot, v.size() * sizeof(T));
    if (!v.empty()) {
        // host vectors are transient: complete the copy before returning
        QASR_HIP(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st_));
        QASR_HIP(hipStreamSynchronize(st_));
    }
    return d;
}

void Session::ensure_kv(int64_t slots) {
    if (slots <= kv_slots_) return;
    QASR_HIP(hipStreamSynchronize(st_));
    if (kc_) QASR_HIP(hipFree(kc_));
    if (vc_) QASR_HIP(hipFree(vc_));
    kc_ = vc_ = nullptr;
    const qasr_hparams& h = m_->hp;
    const size_t per = (size_t)h.txt_layers * (size_t)slots * h.txt_kv_heads * h.head_dim * sizeof(__half);
    QASR_HIP(hipMalloc(&kc_, per));
    QASR_HIP(hipMalloc(&vc_, per));
    kv_slots_ = slots;
    kv_epoch_++;
}

// ------------------------------------------------------------------------------------------ front end
void Session::front_end(const float* dpcm, const std::vector<int64_t>& off, const std::vector<int64_t>& len,
                        FrontEnd& fe, float* enc_out_dbg) {
    (void)enc_out_dbg;
    const qasr_hparams& h = m_->hp;
    const int count = (int)len.size();
    std::vector<MelUtt> utts(count);
    std::vector<int2> work;
    std::vector<int> chunk_utt;
    int frames = 0, chunks = 0;
    fe.n_tok.assign(count, 0);
    fe.tok_base.assign(count, 0);
    std::vector<int> valid_idx;
    for (int u = 0; u < count; u++) {
        MelUtt& U = utts[u];
        U.pcm_off = off[u];
        U.n = len[u];
        const int64_t nn = std::max<int64_t>(len[u], 8000);
        U.P = std::max<int64_t>(nn, 480000);
        U.t_all = (int)(U.P / 160);
        int tv, tp;
        mel_dims(len[u], tv, tp);
        U.t_valid = tv;
        U.t_comp = std::min(tv + 3, U.t_all);
        U.frame0 = frames;
        U.chunk0 = chunks;
        U.n_chunks = tp / 100;
        for (int t0 = 0; t0 < U.t_comp; t0 += 16) work.push_back(make_int2(u, t0));
        for (int c = 0; c < U.n_chunks; c++) {
            chunk_utt.push_back(u);
            const int clen = std::max(0, std::min(100, tv - c * 100));
            const int v = post_cnn_len(clen);
            for (int t = 0; t < v; t++) valid_idx.push_back((chunks + c) * 13 + t);
        }
        fe.tok_base[u] = fe.total_tokens;
        fe.n_tok[u] = audio_token_count(tv);
        fe.total_tokens += fe.n_tok[u];
        frames += U.t_comp;
        chunks += U.n_chunks;
    }
    QASR_CHECK((int)valid_idx.size() == fe.total_tokens, QASR_E_INTERNAL, "audio token count mismatch");
    fe.total_chunks = chunks;
    const int C = h.conv_ch, d = h.enc_d, nm = h.n_mels, F3 = m_->audio_F3();
    MelUtt* d_utts = upload(S_UTTS, utts);
    int2* d_work = upload(S_WORK, work);
    int* d_cu = upload(S_CHUNK_UTT, chunk_utt);
    unsigned* d_umax = (unsigned*)sc_.get(S_UMAX, count * sizeof(unsigned));
    QASR_HIP(hipMemsetAsync(d_umax, 0, count * sizeof(unsigned), st_));
    float* lm = (float*)sc_.get(S_LM, (size_t)frames * nm * sizeof(float));
    float* melx = (float*)sc_.get(S_MELX, (size_t)chunks * nm * 100 * sizeof(float));
    mel_frames(dpcm, d_utts, d_work, (int)work.size(), nm, m_->dft_basis, m_->mel_filters, lm, d_umax, st_);
    mel_normalize(d_utts, count, chunks, d_cu, nm, lm, d_umax, melx, st_);
    // encoder cache (single-utterance runs of run_host): the leading windows the sample prefix allows are reused when
    // this window's mel maximum equals the cached one (then their normalised mel frames, conv chunks and windowed
    // encoder rows are functions of the same samples); the conv stack and the encoder run on the remaining chunks
    fe.skip_tokens = 0;
    if (ec_run_) {
        // the mel maximum reaches the pinned word with the stream (run_host keeps it once the run has synchronised);
        // only a run with reusable windows waits for it here
        QASR_HIP(hipMemcpyAsync((unsigned*)pin_cnt_ + 60, d_umax, sizeof(unsigned), hipMemcpyDeviceToHost, st_));
        if (ec_cand_ > 0) QASR_HIP(hipStreamSynchronize(st_));
        const unsigned umax_new = ((volatile const unsigned*)pin_cnt_)[60];
        // (ec_cand_ ≤ the windows the previous run stored; run_host marks them invalid while this run overwrites them)
        const int reuse = ec_cand_ > 0 && umax_new == ec_umax_ && m_->precision_gen == ec_prec_ ? ec_cand_ : 0;
        const int per = h.n_window_infer / 100;   // chunks per attention window
        if (reuse > 0 && per * reuse < chunks) {
            const int c0 = per * reuse;
            fe.skip_tokens = 13 * c0;
            melx += (size_t)c0 * nm * 100;
            chunks -= c0;
            valid_idx.erase(valid_idx.begin(), valid_idx.begin() + fe.skip_tokens);
            for (int& v : valid_idx) v -= fe.skip_tokens;
        }
    }
    const int n_out = fe.total_tokens - fe.skip_tokens;
    // conv stack
    const int H1 = (nm + 1) / 2, W1 = 50, H2 = (H1 + 1) / 2, W2 = 25;
    __half* a1 = (__half*)sc_.get(S_A1, (size_t)chunks * H1 * W1 * C * sizeof(__half));
    __half* a2 = (__half*)sc_.get(S_A2, (size_t)chunks * H2 * W2 * C * sizeof(__half));
    float* a3 = (float*)sc_.get(S_A3, (size_t)chunks * 13 * C * F3 * sizeof(float));
    conv1_gelu(melx, chunks, nm, m_->conv_w[0], m_->conv_b[0], C, a1, st_);
    conv3x3_gelu(a1, chunks, H1, W1, m_->conv_w[1], m_->conv_b[1], C, a2, 0, st_);
    conv3x3_gelu(a2, chunks, H2, W2, m_->conv_w[2], m_->conv_b[2], C, a3, 1, st_);
    const int rows = chunks * 13, K = C * F3;
    // the row-count-independent GEMM order for every run (round 5: batches too): one utterance's audio-embedding rows
    // are the same bits whether a window is computed in this run or reused from the encoder cache, and in a batch of
    // any composition.  At batch sizes (M > 256) it is the table's own 128×128 tile without split: no cost.
    StableOrderScope order(true);
    int8_t* xq = (int8_t*)sc_.get(S_XQ, (size_t)rows * K);
    float* xd = (float*)sc_.get(S_XD, (size_t)rows * (K / QK) * sizeof(float));
    quant_rows(a3, rows, K, K, xq, xd, st_);
    float* proj = (float*)sc_.get(S_PROJ, (size_t)rows * d * sizeof(float));
    mx_ws(rows, K);
    linear_q8(xq, xd, rows, m_->conv_out, nullptr, nullptr, proj, d, EPI_STORE, st_);
    int* d_valid = upload(S_VALID, valid_idx);
    float* hs = (float*)sc_.get(S_HS, (size_t)n_out * d * sizeof(float));
    add_posemb_gather(proj, chunks, 13, d, m_->pos_emb, d_valid, n_out, hs, st_);
    QASR_HIP(hipGetLastError());
}

// windowed bidirectional encoder + ln_post + projector → S_EMB [tokens][H]
void Session::encoder(FrontEnd& fe, float* enc_out_dbg) {
    const qasr_hparams& h = m_->hp;
    // fe.skip_tokens (one utterance): its leading cached rows are not encoded; the rest starts on a window boundary,
    // so encoding it as an utterance of its own gives the same windows
    const int skip = fe.skip_tokens, N = fe.total_tokens - skip, d = h.enc_d, F = h.enc_ffn, H = h.txt_h;
    QASR_CHECK(skip == 0 || fe.n_tok.size() == 1, QASR_E_INTERNAL, "encoder cache: one utterance");
    // rows independent of the row count, for every run (front_end)
    StableOrderScope order(true);
    // attention windows (get_audio_cu_seqlens, modeling_qwen3_asr.py:276-315)
    std::vector<int> kvs(N), kvl(N);
    for (size_t u = 0; u < fe.n_tok.size(); u++) {
        const int n = fe.n_tok[u] - skip;
        // all chunks but the last are full → max post-CNN length is 13 unless the utterance is one partial chunk
        const int maxlen = n >= 13 ? 13 : n;
        const int window = maxlen * (h.n_window_infer / 100);
        for (int i = 0; i < n; i++) {
            const int w0 = (i / window) * window;
            kvs[fe.tok_base[u] + i] = fe.tok_base[u] + w0;
            kvl[fe.tok_base[u] + i] = std::min(window, n - w0);
        }
    }
    int* d_kvs = upload(S_KVS, kvs);
    int* d_kvl = upload(S_KVL, kvl);
    int64_t total_keys = 0;
    for (int v : kvl) total_keys += v;
    float* hs = (float*)sc_.get(S_HS, (size_t)N * d * sizeof(float));
    const int kmax = std::max(d, F);
    int8_t* xq = (int8_t*)sc_.get(S_XQ, (size_t)N * kmax);
    float* xd = (float*)sc_.get(S_XD, (size_t)N * (kmax / QK) * sizeof(float));
    float* qkv = (float*)sc_.get(S_QKV, (size_t)N * 3 * d * sizeof(float));
    __half* qkvh = (__half*)sc_.get(S_QKVH, (size_t)N * 3 * d * sizeof(__half));
    float* ff = (float*)sc_.get(S_FF, (size_t)N * std::max(F, d) * sizeof(float));
    const float scale = 1.0f / sqrtf((float)(d / h.enc_heads));
    // MFMA-GEMM row counts (> kGemvRows) take the fused epilogues: QKV written as f16 for the attention,
    // up-projection GELU quantised to the down-projection's Q8 rows in place; GEMV row counts keep separate passes
    const bool fused = N > kGemvRows;
    mx_ws(N, std::max(F, d));
    int8_t* hq = fused ? (int8_t*)sc_.get(S_HQ, (size_t)N * std::max(F, d)) : nullptr;
    float* hdq = fused ? (float*)sc_.get(S_HD, (size_t)N * (std::max(F, d) / QK) * sizeof(float)) : nullptr;
    for (int l = 0; l < h.enc_layers; l++) {
        const EncLayer& e = m_->enc[l];
        layernorm_q8(hs, N, d, e.ln1_w, e.ln1_b, h.ln_eps, xq, xd, nullptr, st_);
        if (fused) {
            gemm_q8(xq, xd, N, e.qkv, e.qkv_b, nullptr, (float*)qkvh, 3 * d, EPI_STORE_F16, st_);
        } else {
            linear_q8(xq, xd, N, e.qkv, e.qkv_b, nullptr, qkv, 3 * d, EPI_STORE, st_);
            to_f16(qkv, N, 3 * d, 3 * d, qkvh, 3 * d, st_);
        }
        attention(qkvh, 3 * d, qkvh + d, qkvh + 2 * d, 3 * d, d_kvs, d_kvl, N, h.enc_heads, h.enc_heads, d / h.enc_heads,
                  scale, nullptr, xq, xd, st_, total_keys, /*dense=*/true);
        linear_q8(xq, xd, N, e.o, e.o_b, hs, hs, d, EPI_RESID, st_);
        layernorm_q8(hs, N, d, e.ln2_w, e.ln2_b, h.ln_eps, xq, xd, nullptr, st_);
        if (fused) {
            gemm_q8(xq, xd, N, e.up, e.up_b, nullptr, nullptr, F, EPI_GELU_Q8, st_, -1, 0, hq, hdq);
            linear_q8(hq, hdq, N, e.down, e.down_b, hs, hs, d, EPI_RESID, st_);
        } else {
            linear_q8(xq, xd, N, e.up, e.up_b, nullptr, ff, F, EPI_GELU, st_);
            quant_rows(ff, N, F, F, xq, xd, st_);
            linear_q8(xq, xd, N, e.down, e.down_b, hs, hs, d, EPI_RESID, st_);
        }
    }
    layernorm_q8(hs, N, d, m_->ln_post_w, m_->ln_post_b, h.ln_eps, xq, xd, enc_out_dbg, st_);
    if (fused) {
        gemm_q8(xq, xd, N, m_->proj1, m_->proj1_b, nullptr, nullptr, d, EPI_GELU_Q8, st_, -1, 0, hq, hdq);
        std::swap(xq, hq);
        std::swap(xd, hdq);
    } else {
        linear_q8(xq, xd, N, m_->proj1, m_->proj1_b, nullptr, ff, d, EPI_GELU, st_);
        quant_rows(ff, N, d, d, xq, xd, st_);
    }
    float* emb = (float*)sc_.get(S_EMB, (size_t)(skip + N) * H * sizeof(float));
    linear_q8(xq, xd, N, m_->proj2, m_->proj2_b, nullptr, emb + (size_t)skip * H, H, EPI_STORE, st_);
    if (skip > 0)
        QASR_HIP(hipMemcpyAsync(emb, ec_emb_, (size_t)skip * H * sizeof(float), hipMemcpyDeviceToDevice, st_));
    last_audio_tokens_ = skip + N;
    QASR_HIP(hipGetLastError());
}

// encoder cache update after a single-utterance run of n samples: keep the embedding rows of its complete windows
// (every frame of their chunks inside the samples: frame t reads samples up to 160·t + 199)
void Session::enc_cache_store(int64_t n, int total_tokens) {
    const qasr_hparams& h = m_->hp;
    const int per = h.n_window_infer / 100;
    int w = 0;
    while (16000LL * (per * (w + 1) - 1) + 16040 <= n && 13 * per * (w + 1) <= total_tokens) w++;
    const size_t bytes = (size_t)w * 13 * per * h.txt_h * sizeof(float);
    if (bytes > ec_cap_) {
        QASR_HIP(hipStreamSynchronize(st_));   // this run's reuse copy may still read the old buffer
        if (ec_emb_) QASR_HIP(hipFree(ec_emb_));
        ec_emb_ = nullptr;
        ec_cap_ = 0;
        QASR_HIP(hipMalloc(&ec_emb_, bytes));
        ec_cap_ = bytes;
    }
    if (bytes) QASR_HIP(hipMemcpyAsync(ec_emb_, sc_.get(S_EMB, 0), bytes, hipMemcpyDeviceToDevice, st_));
    ec_windows_ = w;   // (ec_umax_: run_host, once the run has synchronised)
    ec_prec_ = m_->precision_gen;
}

std::vector<float> Session::last_audio_embeds() {
    std::vector<float> out((size_t)last_audio_tokens_ * m_->hp.txt_h);
    if (!out.empty()) {
        QASR_HIP(hipMemcpyAsync(out.data(), sc_.get(S_EMB, 0), out.size() * sizeof(float), hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipStreamSynchronize(st_));
    }
    return out;
}

// ------------------------------------------------------------------------------------------ decoder
static const bool g_dump = getenv("QASR_DUMP_DIR") != nullptr;

void Session::dump_rows(const char* what, int l, int rows, const void* p, size_t bytes) {
    static int seq = 0;
    // a pass being captured into a step graph cannot synchronise its stream (the capture would fail): dumps come
    // from eager passes only (the diagnosis tools set QASR_NO_GRAPH)
    if (sc_.capturing) return;
    std::vector<char> h(bytes);
    QASR_HIP(hipStreamSynchronize(st_));
    QASR_HIP(hipMemcpy(h.data(), p, bytes, hipMemcpyDeviceToHost));
    const char* dir = getenv("QASR_DUMP_DIR");
    if (!dir) return;
    char fn[1024];
    snprintf(fn, sizeof fn, "%s/%06d_%s_L%02d_r%d.bin", dir, seq++, what, l, rows);
    if (FILE* f = fopen(fn, "wb")) {
        fwrite(h.data(), 1, bytes, f);
        fclose(f);
    }
}

// the split decode attention's partial states + zeroed arrival counters for `rows` rows (grow-only; never while a step
// graph is being captured — the eager sizing step of the largest bucket runs first)
void Session::ensure_attn_split(int rows) {
    if (rows <= attn_rows_) return;
    QASR_CHECK(!sc_.capturing, QASR_E_INTERNAL, "split attention scratch growth during graph capture");
    const int nkv = m_->hp.txt_kv_heads, G = m_->hp.txt_heads / nkv;
    if (attn_part_) {
        QASR_HIP(hipDeviceSynchronize());   // queued steps may still use the old buffers
        QASR_HIP(hipFree(attn_part_));
        QASR_HIP(hipFree(attn_cnt_));
    }
    QASR_HIP(hipMalloc(&attn_part_, attn_split_floats(rows, nkv, G) * sizeof(float)));
    QASR_HIP(hipMalloc(&attn_cnt_, (size_t)rows * nkv * sizeof(int)));
    QASR_HIP(hipMemset(attn_cnt_, 0, (size_t)rows * nkv * sizeof(int)));
    attn_rows_ = rows;
    attn_epoch_++;
}

// the fused-norm residual launches flag a wait that timed out (never with the grid resident) in xr_cnt_[2]
void Session::xr_check() {
    unsigned e = 0;
    QASR_HIP(hipMemcpy(&e, xr_cnt_ + 2, sizeof e, hipMemcpyDeviceToHost));
    if (e != 0) {
        QASR_HIP(hipMemset(xr_cnt_, 0, 4 * sizeof(unsigned)));
        throw Error(QASR_E_INTERNAL, "decoder: a fused-norm wait timed out (workgroups not co-resident)");
    }
}

void Session::decoder_layers(float* x, int rows, const int* d_pos, const int* d_slot, const int* d_kvs,
                             const int* d_kvl, int64_t total_keys, bool dense, bool rows_share_kv) {
    const qasr_hparams& h = m_->hp;
    const int H = h.txt_h, F = h.txt_ffn, nh = h.txt_heads, nkv = h.txt_kv_heads, hd = h.head_dim;
    const int QD = nh * hd, KD = nkv * hd;
    const int kmax = std::max(std::max(H, QD), F);
    FixupScope fixup(rows <= 256 ? fix_part_ : nullptr, fix_floats_, fix_cnt_, kFixCounters);
    int8_t* xq = (int8_t*)sc_.get(S_XQ, (size_t)rows * kmax);
    float* xd = (float*)sc_.get(S_XD, (size_t)rows * (kmax / QK) * sizeof(float));
    float* qkv = (float*)sc_.get(S_QKV, (size_t)rows * (QD + 2 * KD) * sizeof(float));
    __half* qh = (__half*)sc_.get(S_QH, (size_t)rows * QD * sizeof(__half));
    const bool fused = rows > kGemvRows;
    mx_ws(rows, kmax);
    float* gu = fused ? nullptr : (float*)sc_.get(S_GU, (size_t)rows * 2 * F * sizeof(float));
    // the fused gate-up epilogue writes the SwiGLU rows into a second Q8 buffer (its input xq is still being read)
    int8_t* hq = fused ? (int8_t*)sc_.get(S_HQ, (size_t)rows * F) : nullptr;
    float* hd_ = fused ? (float*)sc_.get(S_HD, (size_t)rows * (F / QK) * sizeof(float)) : nullptr;
    const float scale = 1.0f / sqrtf((float)hd);
    const size_t layer_kv = (size_t)kv_slots_ * KD;
    const bool fuse_qk = !dense && hd == 128 && (nh / nkv == 2 || nh / nkv == 4) && !getenv("QASR_NO_QK_FUSE");
    // exact rows (a draft verify pass): every row runs the arithmetic of a 1-row decode step — the fused GEMVs in
    // row groups against the same weight registers, the same per-row decode attention (split over the key range like a
    // single row) — so the accepted tokens are greedy's bit for bit, whatever the draft
    // batch invariance (set_batch_invariant): a batch's decode rows (different utterances) take the exact-row path too
    const bool inv = batch_inv_ && !dense && !rows_share_kv && !m_->mx();
    const bool exact = (rows_share_kv && rows <= kExactRows) || inv;
    const bool gv_shapes = gemv_fused_ok(GV_RMS, rows, H) && gemv_fused_ok(GV_NONE, rows, F) &&
                           gemv_fused_ok(GV_NONE, rows, QD);
    // GEMV row counts: the norms and the SwiGLU run inside the GEMVs' prologues (5 launches per layer, not 8)
    // exact rows from exact_mfma_rows() up: the same arithmetic on the matrix core (gemm_exact_rows: the block dots by
    // MFMA, the GEMV's fma chains and wave-sum tree in-lane), with the norms and the SwiGLU as their own launches
    // (rmsnorm_q8 / swiglu_q8 are the fused prologue's / epilogue's arithmetic) — 8 launches per layer, each near a
    // 1-row launch's time, where the GEMV's v_dot4 rows cost ~10× a 1-row step at 32 rows
    const bool xm = exact && rows >= exact_mfma_rows() && gemm_exact_rows_ok(rows, m_->dec[0].qkv) &&
                    gemm_exact_rows_ok(rows, m_->dec[0].down) && gemm_exact_rows_ok(rows, m_->dec[0].gu);
    const bool gv = !xm && gv_shapes && (exact || (rows <= gemv_layer_rows() && dec_fuse_));
    QASR_CHECK(!rows_share_kv || (exact && (gv || xm)), QASR_E_INTERNAL,
               "decoder: a verify pass needs the exact-row path (≤ kExactRows rows, GEMV shapes)");
    QASR_CHECK(!inv || gv || xm, QASR_E_INTERNAL, "decoder: batch invariance needs the exact-row linears");
    if (inv && fuse_qk && attn_split_) ensure_attn_split(rows);
    // batched decode rows (the table path) of few rows: the exact-row kernel where it is the faster launch (cold
    // weights, deterministic table: QKV 5.6 / 7.5 against 7.2 / 9.6 µs at 16 / 32 rows, O-projection 6.7–8.6 against
    // 10.2–10.9 µs at 16–64 rows, down 12.9 against 15.0 µs at 16 rows; profiles/r4_exact_cost_*.json) — the strong-
    // scaling regime (32 segments per GPU at N = 8); round 5: down to 32 rows too (the xr launch, 13.0 against the table's
    // 13.6 µs at 32 rows, profiles/r5_xr_cost.log).  QASR_XR_ROWS=q,o,d overrides the row limits (0 = never).
    static const std::array<int, 3> xr_lim = [] {
        std::array<int, 3> v{32, 64, 32};
        if (const char* e = getenv("QASR_XR_ROWS")) sscanf(e, "%d,%d,%d", &v[0], &v[1], &v[2]);
        return v;
    }();
    const bool xr = !dense && !gv && !xm && !m_->mx();
    const bool xr_qkv = xr && rows <= xr_lim[0] && gemm_exact_rows_ok(rows, m_->dec[0].qkv);
    const bool xr_o = xr && rows <= xr_lim[1] && gemm_exact_rows_ok(rows, m_->dec[0].o);
    const bool xr_down = xr && rows <= xr_lim[2] && gemm_exact_rows_ok(rows, m_->dec[0].down);
    // ≤ 32 rows: the exact-row linears as the per-phase launches (xr_linear: weights loaded up front, rows staged in
    // LDS; bit-identical to gemm_exact_rows — tests/test_ops_gpu.py::test_xr_linear_bit_identical_to_exact_rows),
    // faster at 2-32 rows on O / down and from 24 rows on QKV (profiles/r5_xr_cost.log); QASR_NO_XR=1 keeps
    // gemm_exact_rows (read per call, like QASR_XR_NORM below: tests switch it between sessions)
    const bool no_xr = getenv("QASR_NO_XR") != nullptr;
    auto xr_path = [&](const Q8Mat& W) { return !no_xr && xr_ok(rows, W.K) && W.N % 16 == 0; };
    auto exact_linear = [&](const int8_t* q, const float* d, const Q8Mat& W, const float* res, float* y, int ldy,
                            int epi) {
        if (xr_path(W)) xr_linear(q, d, nullptr, nullptr, 0.f, rows, W, y, ldy, epi == EPI_RESID, st_, nullptr, &xr_split_);
        else gemm_exact_rows(q, d, rows, W, res, y, ldy, epi, st_);
    };
    // a residual exact-row launch that also leaves RMSNorm(x)·nw as the next launch's Q8 rows in (nq, nd) — the norm
    // fused into its tail (xr_norm_tail: no separate rmsnorm_q8 launch).  Returns false (and runs the plain residual
    // launch) where the fused form does not apply.  Opt-in (QASR_XR_NORM=1): bit-identical, but the tail's wait for
    // the last column tile plus one row per norm workgroup costs more than the rmsnorm_q8 launch it replaces — 32-
    // segment share 1137 vs 1183 audio-s/s with it off (profiles/r5_seg32_xrnorm.json).
    const bool no_xr_norm = getenv("QASR_XR_NORM") == nullptr;
    auto resid_norm = [&](const int8_t* q, const float* d, const Q8Mat& W, const float* nw, int8_t* nq, float* nd) {
        if (!no_xr_norm && nw && rows >= 5 && xr_path(W) && (H == 1024 || H == 2048) && xr_cnt_) {
            const XrNorm nm{nw, h.rms_eps, nq, nd, xr_cnt_};
            xr_linear(q, d, nullptr, nullptr, 0.f, rows, W, x, H, true, st_, &nm);
            return true;
        }
        exact_linear(q, d, W, x, x, H, EPI_RESID);
        return false;
    };
    bool normed = false;   // xq / xd already hold this layer's RMSNorm(x)·attn_norm (fused into the last down launch)
    int8_t* hq2 = gv || xm ? (int8_t*)sc_.get(S_HQ, (size_t)rows * F) : nullptr;   // the SwiGLU Q8 rows
    float* hd2 = gv || xm ? (float*)sc_.get(S_HD, (size_t)rows * (F / QK) * sizeof(float)) : nullptr;
    float* gux = xm ? (float*)sc_.get(S_GU, (size_t)rows * 2 * F * sizeof(float)) : nullptr;
    for (int l = 0; l < h.txt_layers; l++) {
        const DecLayer& L = m_->dec[l];
        __half* kc = kc_ + (size_t)l * layer_kv;
        __half* vc = vc_ + (size_t)l * layer_kv;
        // decode-sized steps: the norm launch also clears the QKV output, so the split-K QKV GEMM needs no memset —
        // only with f32-atomic split-K (deterministic mode splits through the fix-up, which stores every output)
        const bool zq = rows <= 256 && !deterministic();
        const bool dmp = g_dump && rows <= kExactRows;
        if (dmp) dump_rows("x_in", l, rows, x, (size_t)rows * H * sizeof(float));
        const float* next_norm = l + 1 < h.txt_layers ? m_->dec[l + 1].attn_norm : nullptr;
        if (xm) {
            if (!normed) rmsnorm_q8(x, rows, H, H, L.attn_norm, h.rms_eps, xq, xd, st_);
            exact_linear(xq, xd, L.qkv, nullptr, qkv, QD + 2 * KD, EPI_STORE);
        } else if (gv) {
            gemv_fused(GV_RMS, nullptr, nullptr, x, H, L.attn_norm, h.rms_eps, rows, L.qkv, nullptr, qkv, QD + 2 * KD,
                       EPI_STORE, nullptr, nullptr, st_);
        } else if (xr_qkv) {
            if (!normed) rmsnorm_q8(x, rows, H, H, L.attn_norm, h.rms_eps, xq, xd, st_);
            exact_linear(xq, xd, L.qkv, nullptr, qkv, QD + 2 * KD, EPI_STORE);
        } else {
            QASR_CHECK(!normed, QASR_E_INTERNAL, "decoder: a fused norm feeds the table QKV path");
            rmsnorm_q8(x, rows, H, H, L.attn_norm, h.rms_eps, xq, xd, st_, zq ? qkv : nullptr,
                       zq ? (int64_t)rows * (QD + 2 * KD) : 0);
            linear_q8(xq, xd, rows, L.qkv, nullptr, nullptr, qkv, QD + 2 * KD, EPI_STORE, st_, zq);
        }
        if (dmp) dump_rows("qkv", l, rows, qkv, (size_t)rows * (QD + 2 * KD) * sizeof(float));
        if (fuse_qk) {   // decode rows: q/k norm + RoPE + KV write inside the attention kernel
            // a verify pass's row i attends the K/V rows 0…i-1 write in this layer: all rows' K/V go to the cache in a
            // launch of their own first; the fused kernel then rewrites each row's own K/V with the same bits
            if (rows_share_kv)
                qk_norm_rope(qkv, rows, nh, nkv, hd, d_pos, d_slot, L.q_norm, L.k_norm, rope_, h.rms_eps, qh, kc, vc,
                             st_);
            QkFuse fz{qkv, d_pos, d_slot, L.q_norm, L.k_norm, rope_, h.rms_eps, kc, vc};
            if ((rows <= 4 || exact) && attn_part_ && attn_split_ && rows <= attn_rows_) {   // long key ranges split
                fz.part = attn_part_;                                                         // over workgroups
                fz.cnt = attn_cnt_;
                fz.part_rows = attn_rows_;
            }
            fz.fixed_chunk = inv;   // the 1-row step's chunking for every row
            attention_decode_fused(fz, KD, d_kvs, d_kvl, rows, nh, nkv, hd, scale, xq, xd, st_, total_keys);
        } else {
            qk_norm_rope(qkv, rows, nh, nkv, hd, d_pos, d_slot, L.q_norm, L.k_norm, rope_, h.rms_eps, qh, kc, vc, st_);
            attention(qh, QD, kc, vc, KD, d_kvs, d_kvl, rows, nh, nkv, hd, scale, nullptr, xq, xd, st_, total_keys,
                      dense);
        }
        if (dmp) {
            dump_rows("att_q", l, rows, xq, (size_t)rows * QD);
            dump_rows("att_d", l, rows, xd, (size_t)rows * (QD / QK) * sizeof(float));
        }
        if (xm) {   // the same steps with the exact-row linears (≤ 32 rows: the xr launches, norms fused in)
            if (!resid_norm(xq, xd, L.o, L.ffn_norm, xq, xd)) rmsnorm_q8(x, rows, H, H, L.ffn_norm, h.rms_eps, xq, xd, st_);
            if (dmp) dump_rows("x_mid", l, rows, x, (size_t)rows * H * sizeof(float));
            if (xr_path(L.gu) && L.gu.K <= 2048) {   // gate/up + SwiGLU + Q8 in one exact launch
                xr_gu_swiglu(xq, xd, nullptr, nullptr, 0.f, rows, L.gu, hq2, hd2, st_);
            } else {
                exact_linear(xq, xd, L.gu, nullptr, gux, 2 * F, EPI_STORE);
                swiglu_q8(gux, rows, F, hq2, hd2, st_, /*interleaved=*/true);
            }
            if (dmp) {
                dump_rows("h_q", l, rows, hq2, (size_t)rows * F);
                dump_rows("h_d", l, rows, hd2, (size_t)rows * (F / QK) * sizeof(float));
            }
            // under QASR_DUMP_DIR the launch still runs, only its fused norm is dropped (the dump reads x_in)
            normed = resid_norm(hq2, hd2, L.down, g_dump ? nullptr : next_norm, xq, xd);
            continue;
        }
        if (gv) {   // O-projection + residual; norm + gate/up + SwiGLU + Q8; down-projection + residual
            gemv_fused(GV_NONE, xq, xd, nullptr, 0, nullptr, 0.f, rows, L.o, x, x, H, EPI_RESID, nullptr, nullptr, st_);
            if (dmp) dump_rows("x_mid", l, rows, x, (size_t)rows * H * sizeof(float));
            gemv_fused(GV_RMS, nullptr, nullptr, x, H, L.ffn_norm, h.rms_eps, rows, L.gu, nullptr, nullptr, 0,
                       EPI_SWIGLU, hq2, hd2, st_);
            if (dmp) {
                dump_rows("h_q", l, rows, hq2, (size_t)rows * F);
                dump_rows("h_d", l, rows, hd2, (size_t)rows * (F / QK) * sizeof(float));
            }
            gemv_fused(GV_NONE, hq2, hd2, nullptr, 0, nullptr, 0.f, rows, L.down, x, x, H, EPI_RESID, nullptr, nullptr,
                       st_);
            continue;
        }
        bool o_normed = false;
        if (xr_o)
            o_normed = resid_norm(xq, xd, L.o, L.ffn_norm, xq, xd);
        else
            linear_q8(xq, xd, rows, L.o, nullptr, x, x, H, EPI_RESID, st_);
        if (!o_normed) rmsnorm_q8(x, rows, H, H, L.ffn_norm, h.rms_eps, xq, xd, st_);
        if (fused) {  // SwiGLU + Q8 in the gate-up GEMM epilogue (rows interleaved at load)
            gemm_q8(xq, xd, rows, L.gu, nullptr, nullptr, nullptr, 2 * F, EPI_SWIGLU, st_, -1, 0, hq, hd_);
            std::swap(xq, hq);
            std::swap(xd, hd_);
        } else {
            linear_q8(xq, xd, rows, L.gu, nullptr, nullptr, gu, 2 * F, EPI_STORE, st_);
            swiglu_q8(gu, rows, F, xq, xd, st_, true);
        }
        // the next layer's QKV reads the fused norm only on its exact-row path (xr_qkv)
        if (xr_down)
            normed = resid_norm(xq, xd, L.down, xr_qkv && !g_dump ? next_norm : nullptr, fused ? hq : xq,
                                fused ? hd_ : xd);
        else
            linear_q8(xq, xd, rows, L.down, nullptr, x, x, H, EPI_RESID, st_);
        if (fused) {
            std::swap(xq, hq);
            std::swap(xd, hd_);
        }
    }
    QASR_HIP(hipGetLastError());
}

// MXFP8 precision mode: the activations' fp8 image for GEMMs of up to rows × kmax (thread-local registration)
void Session::mx_ws(int64_t rows, int64_t kmax) {
    if (!m_->mx()) return;
    const size_t bytes = mx_workspace_bytes(rows, kmax);
    set_mx_workspace(sc_.get(S_MX, bytes), bytes);
}

void Session::lm_head_rows(const float* x, int rows, int ldx, float* logits, bool exact) {
    const qasr_hparams& h = m_->hp;
    int8_t* xq = (int8_t*)sc_.get(S_XQ, (size_t)std::max(rows, 1) * std::max(h.txt_h, std::max(h.txt_ffn, h.txt_heads * h.head_dim)));
    float* xd = (float*)sc_.get(S_XD, (size_t)std::max(rows, 1) * (std::max(h.txt_h, std::max(h.txt_ffn, h.txt_heads * h.head_dim)) / QK) * sizeof(float));
    rmsnorm_q8(x, rows, h.txt_h, ldx, m_->out_norm, h.rms_eps, xq, xd, st_);
    mx_ws(rows, h.txt_h);
    // ≤ 4 rows (1-row decode steps) and exact rows (verify passes): the weight-streaming GEMV, one per-row arithmetic
    // for any row count (k_gemv_wide's row groups); more rows: the MFMA GEMM
    // round 6: 5–16 rows — the N = 8 share's later decode steps, short draft verify passes, a small batch's first
    // tokens — through k_xr_vocab (the 1-row GEMV's bits per row, in default and exact modes alike: 72–74 against the
    // table's 79–86 µs, profiles/r6n_lmhead_cost.log); QASR_XR_VOCAB=0 restores the table GEMM / exact kernel
    const bool xv = rows > kGemvRows && !m_->mx() && xr_vocab_ok(rows, h.txt_h, h.vocab) &&
                    !(getenv("QASR_XR_VOCAB") && atoi(getenv("QASR_XR_VOCAB")) == 0);
    if (xv)
        xr_vocab(xq, xd, rows, m_->lm_head, logits, h.vocab, st_);
    else if (exact && rows >= exact_mfma_rows() && gemm_exact_rows_ok(rows, m_->lm_head))
        gemm_exact_rows(xq, xd, rows, m_->lm_head, nullptr, logits, h.vocab, EPI_STORE, st_);
    else if ((rows <= kGemvRows || exact) && gemv_fused_ok(GV_NONE, rows, h.txt_h))
        gemv_fused(GV_NONE, xq, xd, nullptr, 0, nullptr, 0.f, rows, m_->lm_head, nullptr, logits, h.vocab, EPI_STORE,
                   nullptr, nullptr, st_);
    else
        linear_q8(xq, xd, rows, m_->lm_head, nullptr, nullptr, logits, h.vocab, EPI_STORE, st_);
}

// row bucket of a decode step: 1/2/4 rows (GEMV path), 8, then steps of 16 / 32 / 64 / 128 rows
int row_bucket(int m) {
    if (m <= 1) return 1;
    if (m <= 2) return 2;
    if (m <= 4) return 4;
    if (m <= 8) return 8;
    if (m <= 64) return (m + 15) / 16 * 16;
    if (m <= 256) return (m + 31) / 32 * 32;
    if (m <= 1024) return (m + 63) / 64 * 64;
    return (m + 127) / 128 * 128;
}

// one decode step over B rows, fully on the device: plan → embed → 28 layers → lm_head → argmax → accept →
// active count to the pinned host word.  Capturable (no allocation once the scratch is sized, no sync).
void Session::decode_step(const DecState& ds, int B, bool sizing, int64_t keys) {
    (void)sizing;
    const qasr_hparams& h = m_->hp;
    const int H = h.txt_h, V = h.vocab;
    int* tab = (int*)sc_.get(S_DTAB, (size_t)6 * B * sizeof(int));
    float* x = (float*)sc_.get(S_X, (size_t)B * H * sizeof(float));
    if (B <= kPlanEmbedRows) {   // plan + embedding in one launch
        dec_plan_embed(ds, B, tab, tab + B, tab + 2 * B, tab + 3 * B, tab + 4 * B, tab + 5 * B, m_->tok_embd, x, st_);
    } else {
        dec_plan(ds, B, tab, tab + B, tab + 2 * B, tab + 3 * B, tab + 4 * B, tab + 5 * B, st_);
        embed_rows(tab, B, m_->tok_embd, nullptr, x, st_);
    }
    decoder_layers(x, B, tab + B, tab + 2 * B, tab + 3 * B, tab + 4 * B, keys);
    float* logits = (float*)sc_.get(S_LOGITS, (size_t)B * V * sizeof(float));
    lm_head_rows(x, B, H, logits, batch_inv_ && !m_->mx());
    int* d_tok = (int*)sc_.get(S_TOK, (size_t)B * sizeof(int));
    void* argp = sc_.get(S_ARGP, argmax_scratch_bytes(B));
    if (tf_) {
        argmax_rows(logits, B, V, d_tok, st_, argp);
        force_tokens(ds, B, tab + 5 * B, tf_->d_ids, tf_->ld, d_tok, st_);
        tf_capture(logits, B, tab + 5 * B);
        dec_accept(ds, B, tab + 5 * B, d_tok, st_);
    } else {   // the argmax's final stage and the accept in one launch
        argmax_rows_partial(logits, B, V, argp, st_);
        argmax_accept(ds, B, argp, tab + 5 * B, d_tok, st_);
    }
    QASR_HIP(hipMemcpyAsync(pin_cnt_, ds.counters, 4 * sizeof(int), hipMemcpyDeviceToHost, st_));
}

// teacher forcing: the wanted utterances' logits rows of this step → out[w][step][V] (eager steps, host sync)
void Session::tf_capture(const float* logits, int rows, const int* row_utt) {
    const int V = m_->hp.vocab;
    std::vector<int> ru(rows);
    if (row_utt) {
        QASR_HIP(hipMemcpyAsync(ru.data(), row_utt, (size_t)rows * sizeof(int), hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipStreamSynchronize(st_));
    } else {
        for (int r = 0; r < rows; r++) ru[r] = r;   // the prefill's first-token rows: row u = utterance u
    }
    const int j = tf_->step++;
    if (j > tf_->n_forced) return;
    for (int r = 0; r < rows; r++) {
        const int u = ru[r];
        if (u < 0 || u >= (int)tf_->want.size() || tf_->want[u] < 0) continue;
        float* dst = tf_->out + ((size_t)tf_->want[u] * (tf_->n_forced + 1) + j) * V;
        QASR_HIP(hipMemcpyAsync(dst, logits + (size_t)r * V, (size_t)V * sizeof(float), hipMemcpyDeviceToHost, st_));
    }
    QASR_HIP(hipStreamSynchronize(st_));
}

// ------------------------------------------------------------------------------------------ draft decode
// One verify pass over B rows whose ids / positions / KV slots / key ranges sit in S_DTAB (5 tables of 16): embed →
// 28 layers (the decode path: fused q/k-norm + RoPE + KV write, per-row attention over each row's own causal range)
// → lm_head → argmax → token ids to the pinned host words [8, 8 + B).  Capturable like decode_step.
void Session::draft_step(int B) {
    const qasr_hparams& h = m_->hp;
    constexpr int R = kDraftRows;
    int* tab = (int*)sc_.get(S_DTAB, (size_t)6 * R * sizeof(int));
    float* x = (float*)sc_.get(S_X, (size_t)R * h.txt_h * sizeof(float));
    embed_rows(tab, B, m_->tok_embd, nullptr, x, st_);
    decoder_layers(x, B, tab + R, tab + 2 * R, tab + 3 * R, tab + 4 * R, 0, /*dense=*/false, /*rows_share_kv=*/B > 1);
    float* logits = (float*)sc_.get(S_LOGITS, (size_t)R * h.vocab * sizeof(float));
    lm_head_rows(x, B, h.txt_h, logits, /*exact=*/true);
    int* d_tok = (int*)sc_.get(S_TOK, (size_t)R * sizeof(int));
    argmax_rows(logits, B, h.vocab, d_tok, st_, sc_.get(S_ARGP, argmax_scratch_bytes(R)));
    QASR_HIP(hipMemcpyAsync((int*)pin_cnt_ + 8, d_tok, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, st_));
}

// bucket graphs hold scratch / KV / weight pointers: retire them whenever any of those moved
void Session::draft_graphs_refresh() {
    const uint64_t key[5] = {sc_.epoch, kv_epoch_, m_->precision_gen, deterministic_gen(), attn_epoch_};
    if (memcmp(key, draft_key_, sizeof key) != 0) {
        for (auto& g : draft_graphs_) (void)hipGraphExecDestroy(g.second);
        draft_graphs_.clear();
        memcpy(draft_key_, key, sizeof key);
    }
}

// one verify pass of bucket B (the tables already in S_DTAB): the bucket's captured graph, or an eager pass that also
// sizes the scratch, then captured for the next time
void Session::draft_pass(int B) {
    const bool graphs = !prof_enabled() && !getenv("QASR_NO_GRAPH");
    auto it = draft_graphs_.find(B);
    if (graphs && it != draft_graphs_.end()) {
        QASR_HIP(hipGraphLaunch(it->second, st_));
        return;
    }
    draft_step(B);            // eager: also sizes the scratch this bucket needs before its graph is captured
    draft_graphs_refresh();   // (a growth retires the other buckets' graphs)
    if (!graphs) return;
    QASR_HIP(hipStreamSynchronize(st_));
    hipGraph_t g;
    QASR_HIP(hipStreamBeginCapture(st_, hipStreamCaptureModeRelaxed));
    sc_.capturing = true;
    try {
        draft_step(B);
    } catch (...) {
        sc_.capturing = false;
        (void)hipStreamEndCapture(st_, &g);
        throw;
    }
    sc_.capturing = false;
    QASR_HIP(hipStreamEndCapture(st_, &g));
    hipGraphExec_t ex;
    QASR_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    draft_graphs_.emplace(B, ex);
}

// Prompt-lookup decoding of one utterance (toks holds the first, prefill-chosen token).  Each pass feeds the last
// accepted token and a draft — the tokens that followed the most recent earlier occurrence of the last two (else one)
// accepted tokens in the session's history — and accepts greedy's tokens up to and including the first that departs
// from the draft.  Row i's logits predict the token after row i's input, so an accepted prefix is exactly what one
// greedy step per token would emit; KV rows written for rejected draft tokens sit past the accepted length and are
// rewritten by the next pass.  A draft that keeps failing at its first token shrinks (to none: a plain greedy step).
// forced: a fixed token count (force_tokens_per_s): EOS is emitted like any token, as by the batch loop.
void Session::draft_decode(int n_prompt, int base, int budget, int dummy, std::vector<int32_t>& toks, bool& eos,
                           bool forced) {
    const qasr_hparams& h = m_->hp;
    constexpr int RMAX = kDraftRows;
    // Draft length: with per-token acceptance a, a pass of k drafted tokens yields 1 + a + … + a^k tokens and costs
    // kPassCost[bucket] (kernel time of one verify pass of 1/2/4/8/16/32 rows relative to a 1-row pass, 1.7B:
    // profiles/r3u_pass_cost.log — the GEMV rows up to 4, the exact-row MFMA linears from 5); k fills a row bucket
    // (1, 3, 7, 15, 31) and is the one with the most tokens per unit cost at the current estimate of a — never worse
    // than plain greedy steps in expectation, long drafts only while they keep being accepted
    static constexpr double kPassCost[6] = {1.0, 1.24, 1.71, 1.93, 2.04, 2.66};
    auto draft_len = [&](int cap) {
        const double a = draft_s_ / (draft_s_ + draft_f_);
        int best = 0;
        double best_rate = 1.0 / kPassCost[0];
        double y = 1.0, p = 1.0;
        for (int k = 1, b = 1; k <= std::min(cap, RMAX - 1); k++) {
            p *= a;
            y += p;
            if (k + 1 == 1 << b) {   // k + 1 rows fill bucket b
                const double rate = y / kPassCost[b];
                if (rate > best_rate) best_rate = rate, best = k;
                b++;
            }
        }
        return best;
    };
    int* tab = (int*)sc_.get(S_DTAB, (size_t)6 * RMAX * sizeof(int));
    int* hb = (int*)pinned((size_t)6 * RMAX * sizeof(int));
    draft_graphs_refresh();
    // the continuation of the last bigram (else unigram) in the previous transcripts.  Within the latest transcript —
    // the previous window of the same speech, in step with this decode (a few tokens ahead where the window's start
    // moved) — the occurrence nearest the current position, so a repeated n-gram does not cut the draft short at its
    // last occurrence; else the most recent occurrence anywhere.
    auto lookup = [&](std::vector<int32_t>& draft, int cap) {
        draft.clear();
        if (cap <= 0 || history_.empty()) return;
        const int n = (int)toks.size(), H = (int)history_.size();
        for (int order = std::min(2, n); order >= 1 && draft.empty(); order--) {
            auto match = [&](int j) {
                for (int k = 0; k < order; k++)
                    if (history_[j + k] != toks[n - order + k]) return false;
                return true;
            };
            int best = -1, bd = INT_MAX;
            for (int j = hist_last_; j + order < H; j++) {   // leaves ≥ 1 token to propose
                const int d = std::abs(j - hist_last_ + order - n);
                if (d < bd && match(j)) bd = d, best = j;
            }
            for (int j = H - order - 1; best < 0 && j >= 0; j--)
                if (match(j)) best = j;
            if (best >= 0)
                for (int k = best + order; k < H && (int)draft.size() < cap; k++) draft.push_back(history_[k]);
        }
        if (draft_noise_ > 0.f) {   // set_draft_noise: corrupt proposals (splitmix64 stream)
            for (int32_t& t : draft) {
                const uint64_t r = smix(noise_state_++);
                if ((double)(r >> 11) * 0x1.0p-53 < draft_noise_) t = (int32_t)(smix(r) % (uint64_t)h.vocab);
            }
        }
    };
    std::vector<int32_t> draft;
    eos = false;
    while ((int)toks.size() < budget) {
        const int pos = n_prompt + (int)toks.size() - 1;   // position of the last accepted token
        lookup(draft, draft_len(budget - (int)toks.size() - 1));
        const int R = 1 + (int)draft.size();
        const int B = R <= 1 ? 1 : R <= 2 ? 2 : R <= 4 ? 4 : R <= 8 ? 8 : R <= 16 ? 16 : 32;
        for (int i = 0; i < B; i++) {
            const bool real = i < R;
            hb[i] = real ? (i == 0 ? toks.back() : draft[i - 1]) : 0;
            hb[RMAX + i] = real ? pos + i : 0;
            hb[2 * RMAX + i] = real ? base + pos + i : dummy;
            hb[3 * RMAX + i] = real ? base : dummy;
            hb[4 * RMAX + i] = real ? pos + i + 1 : 1;
        }
        QASR_HIP(hipMemcpyAsync(tab, hb, (size_t)5 * RMAX * sizeof(int), hipMemcpyHostToDevice, st_));
        draft_pass(B);
        QASR_HIP(hipStreamSynchronize(st_));
        const int* got = (const int*)pin_cnt_ + 8;
        dstats_.passes++;
        dstats_.proposed += R - 1;
        int acc = 0;
        bool rejected = false;   // the pass ended on a drafted token greedy did not choose (not on EOS / the budget)
        for (int i = 0; i < R; i++) {
            const int t = got[i];
            if (!forced && (t == h.tok_eos0 || t == h.tok_eos1)) {
                eos = true;
                break;
            }
            toks.push_back(t);
            if ((int)toks.size() >= budget) break;
            if (i < R - 1 && t != draft[i]) {   // row i + 1 was fed a token greedy did not choose
                rejected = true;
                break;
            }
            if (i < R - 1) acc++;
        }
        dstats_.accepted += acc;
        if (R > 1) {   // acc successes, then one rejection if a drafted token was refused — a pass cut short by EOS
                       // or the token budget rejected nothing, so it leaves the failure count alone
            draft_s_ = 0.8 * draft_s_ + acc;
            draft_f_ = 0.8 * draft_f_ + (rejected ? 1.0 : 0.0);
        } else {       // a plain step: the estimate relaxes toward the prior, so drafting is tried again later
            draft_s_ = 0.95 * draft_s_ + 0.05 * 4.0;
            draft_f_ = 0.95 * draft_f_ + 0.05 * 0.5;
        }
        if (eos) break;
    }
}

// ------------------------------------------------------------------------------------------ batch run
void Session::run_batch(const float* dpcm, const std::vector<int64_t>& off, const std::vector<int64_t>& len,
                        int max_new, int force_tps, std::vector<UttResult>& out, StageTimes* times) {
    const qasr_hparams& h = m_->hp;
    const int count = (int)len.size();
    out.assign(count, UttResult());
    if (count == 0) return;
    for (int u = 0; u < count; u++) QASR_CHECK(len[u] > 0, QASR_E_INVALID, "empty utterance");
    FrontEnd fe;
    {
        Timer t(st_, times ? &times->mel : nullptr);
        front_end(dpcm, off, len, fe, nullptr);
    }
    {
        Timer t(st_, times ? &times->encoder : nullptr);
        encoder(fe, nullptr);
    }
    if (ec_run_) {
        ecstats_.runs++;
        const int per = h.n_window_infer / 100;
        ecstats_.windows_reused += fe.skip_tokens / (13 * per);
        ecstats_.windows_computed += (fe.total_tokens - fe.skip_tokens + 13 * per - 1) / (13 * per);
        enc_cache_store(len[0], fe.total_tokens);
    }
    // prompts, KV slots, generation budgets
    std::vector<int> n_prompt(count), base(count), row0(count), budget(count);
    std::vector<int32_t> ids;
    // the prompt prefix before the audio (im_start system \n im_end \n im_start user \n audio_start) is the same
    // tokens at the same positions for every utterance, so its K/V is computed once and copied into each
    // utterance's slots; the packed prefill then starts at position P0
    const int P0 = kPromptPrefix + (int)context_.size();
    const int shared = count >= 4 ? P0 : 0;
    // prompt-KV reuse (round 4; a growing interim window, interim.rs:135-146): a single-utterance run whose encoder
    // reused the previous run's leading windows (fe.skip_tokens audio rows, bit-identical embeddings) has the same
    // prompt rows [0, P0 + skip_tokens) at the same positions as that run; single-utterance prefill runs the
    // row-count-independent order, so their K/V — still in slots [0, …) of this session's cache, which nothing since
    // has written — are the bits a recomputation would give: the prefill starts after them
    int reuse = 0;
    {
        const uint64_t key[4] = {kv_epoch_, m_->precision_gen, deterministic_gen(), 0};
        const std::vector<int32_t> head = build_prompt(h, 0, 0, context_);
        const bool same = kvp_rows_ > 0 && !memcmp(key, kvp_key_, sizeof key) && count == 1 && ec_run_ &&
                          kvp_prefix_ == std::vector<int32_t>(head.begin(), head.begin() + P0) && kv_reuse_;
        if (same && fe.skip_tokens > 0) reuse = std::min(P0 + fe.skip_tokens, kvp_rows_);
        kvp_rows_ = 0;   // valid again only once this run has completed (below)
    }
    // a completed single-utterance run leaves its prompt rows' K/V in slots [0, n_prompt) for the next run
    auto remember_prompt_kv = [&]() {
        if (count != 1 || m_->mx()) return;
        const std::vector<int32_t> head = build_prompt(h, 0, 0, context_);
        kvp_prefix_.assign(head.begin(), head.begin() + P0);
        const uint64_t key[4] = {kv_epoch_, m_->precision_gen, deterministic_gen(), 0};
        memcpy(kvp_key_, key, sizeof key);
        kvp_rows_ = n_prompt[0];
    };
    int64_t slots = 0;
    std::vector<std::vector<int32_t>> prompts(count);
    for (int u = 0; u < count; u++) {
        prompts[u] = build_prompt(h, fe.n_tok[u], fe.tok_base[u], context_);
        n_prompt[u] = (int)prompts[u].size();
        const double secs = (double)len[u] / 16000.0;
        // one utterance decodes until EOS or n_ctx, like the reference's session.run; a batch caps each utterance
        // (its KV slot range is reserved up front)
        if (tf_) budget[u] = tf_->n_forced + 1;   // teacher forcing: n_forced + 1 logits rows
        else if (force_tps > 0) budget[u] = std::max(1, (int)lround(force_tps * secs) + 1);
        else budget[u] = max_new > 0 ? max_new : count == 1 ? n_ctx_ : 64 + (int)ceil(32.0 * secs);
        budget[u] = std::min(budget[u], n_ctx_ - n_prompt[u]);
        QASR_CHECK(budget[u] > 0, QASR_E_CAPACITY, "utterance exceeds n_ctx");
        base[u] = (int)slots;
        slots += n_prompt[u] + budget[u];
        out[u].n_audio = fe.n_tok[u];
        out[u].n_prompt = n_prompt[u];
    }
    const int64_t pref = slots + 1;          // slots: utterances, the dummy slot, the shared prefix
    const uint64_t kv_ep = kv_epoch_;
    ensure_kv(slots + 1 + (shared ? P0 : 0));
    if (kv_epoch_ != kv_ep) reuse = 0;   // a reallocated cache holds none of the previous run's rows: prefill them all
    const int skip = shared ? shared : reuse;
    for (int u = 0; u < count; u++) {
        row0[u] = (int)ids.size();
        ids.insert(ids.end(), prompts[u].begin() + skip, prompts[u].end());
    }
    kvp_stats_.rows_reused += reuse;
    const int T = (int)ids.size(), H = h.txt_h, V = h.vocab;
    std::vector<int> pos(T), slot(T), kvs(T), kvl(T), last(count);
    for (int u = 0; u < count; u++) {
        for (int i = skip; i < n_prompt[u]; i++) {
            const int r = row0[u] + i - skip;
            pos[r] = i;
            slot[r] = base[u] + i;
            kvs[r] = base[u];
            kvl[r] = i + 1;
        }
        last[u] = row0[u] + n_prompt[u] - skip - 1;
    }
    // device-resident decode state (kernels_decode.hip): one int32 block, laid out by a grow-only capacity so
    // the pointers captured in the step graphs stay valid across calls
    int ld = 1;
    for (int u = 0; u < count; u++) ld = std::max(ld, budget[u]);
    if (ucap_ < count) {
        ucap_ = 64;
        while (ucap_ < count) ucap_ *= 2;
    }
    int* blk = (int*)sc_.get(S_DSTATE, (size_t)(6 * ucap_ + 16) * sizeof(int));
    DecState ds;
    ds.last_tok = blk;
    ds.gen = blk + ucap_;
    ds.done = blk + 2 * ucap_;
    ds.budget = blk + 3 * ucap_;
    ds.n_prompt = blk + 4 * ucap_;
    ds.base = blk + 5 * ucap_;
    int* params = blk + 6 * ucap_;
    ds.params = params;
    ds.counters = params + 8;
    ds.out = (int*)sc_.get(S_DOUT, (size_t)count * ld * sizeof(int));
    {
        std::vector<int> hb((size_t)6 * ucap_ + 16, 0);
        for (int u = 0; u < count; u++) {
            hb[3 * ucap_ + u] = budget[u];
            hb[4 * ucap_ + u] = n_prompt[u];
            hb[5 * ucap_ + u] = base[u];
        }
        int* hp = hb.data() + 6 * ucap_;
        hp[0] = count;
        hp[1] = (int)slots;  // the dummy KV slot (reserved by ensure_kv below)
        hp[2] = force_tps > 0 || tf_;
        hp[3] = h.tok_eos0;
        hp[4] = h.tok_eos1;
        hp[5] = ld;
        QASR_HIP(hipMemcpyAsync(blk, hb.data(), hb.size() * sizeof(int), hipMemcpyHostToDevice, st_));
        QASR_HIP(hipStreamSynchronize(st_));
    }
    {
        Timer t(st_, times ? &times->prefill : nullptr);
        // every decoder prefill in the row-count-independent GEMM order (every output one block chain in K order), and
        // the first token's vocabulary projection with the 1-row GEMV's per-row arithmetic: a prompt row and the
        // prompt's first token are the same bits in any batch as in the segment's single run (round 5: batches too —
        // the default batch's first tokens had flipped against the single runs' at 0.3-1 % logit margins, the
        // synthetic model's spread between GEMM orders; at C4's row counts the stable tiles are the table's own)
        StableOrderScope order(true);
        sc_.get(S_X, (size_t)std::max(T, P0) * H * sizeof(float));
        if (shared) {
            const std::vector<int32_t> full = build_prompt(h, 0, 0, context_);
            std::vector<int32_t> pid(full.begin(), full.begin() + P0);
            std::vector<int> ppos(P0), pslot(P0), pkvs(P0, (int)pref), pkvl(P0);
            for (int i = 0; i < P0; i++) {
                ppos[i] = i;
                pslot[i] = (int)pref + i;
                pkvl[i] = i + 1;
            }
            float* xp = (float*)sc_.get(S_X, (size_t)P0 * H * sizeof(float));
            int* dpi = upload(S_IDS, pid);
            embed_rows(dpi, P0, m_->tok_embd, nullptr, xp, st_);
            decoder_layers(xp, P0, upload(S_POS, ppos), upload(S_SLOT, pslot), upload(S_KVS, pkvs),
                           upload(S_KVL, pkvl), (int64_t)P0 * (P0 + 1) / 2, /*dense=*/true);
            copy_kv_prefix(kc_, vc_, h.txt_layers, kv_slots_, h.txt_kv_heads * h.head_dim, pref, P0,
                           upload(S_LAST, base), count, st_);
            QASR_HIP(hipStreamSynchronize(st_));   // the small tables above are reused by the main prefill
        }
        int* d_ids = upload(S_IDS, ids);
        int* d_pos = upload(S_POS, pos);
        int* d_slot = upload(S_SLOT, slot);
        int* d_kvs = upload(S_KVS, kvs);
        int* d_kvl = upload(S_KVL, kvl);
        float* x = (float*)sc_.get(S_X, (size_t)T * H * sizeof(float));
        float* emb = (float*)sc_.get(S_EMB, (size_t)fe.total_tokens * H * sizeof(float));
        embed_rows(d_ids, T, m_->tok_embd, emb, x, st_);
        int64_t keys = 0;
        for (int v : kvl) keys += v;
        decoder_layers(x, T, d_pos, d_slot, d_kvs, d_kvl, keys, /*dense=*/true);
        int* d_last = upload(S_LAST, last);
        float* xn = (float*)sc_.get(S_XN, (size_t)count * H * sizeof(float));
        k_gather_rows<<<(unsigned)cdiv64((int64_t)count * H, 256), 256, 0, st_>>>(x, d_last, count, H, xn);
        float* logits = (float*)sc_.get(S_LOGITS, (size_t)count * V * sizeof(float));
        lm_head_rows(xn, count, H, logits, !m_->mx());
        int* d_tok = (int*)sc_.get(S_TOK, count * sizeof(int));
        argmax_rows(logits, count, V, d_tok, st_, sc_.get(S_ARGP, argmax_scratch_bytes(count)));
        // the first generated token of every utterance: plan (identity rows) + accept on the device
        int* tab = (int*)sc_.get(S_DTAB, (size_t)6 * count * sizeof(int));
        dec_plan(ds, count, tab, tab + count, tab + 2 * count, tab + 3 * count, tab + 4 * count, tab + 5 * count, st_);
        if (tf_) {
            force_tokens(ds, count, tab + 5 * count, tf_->d_ids, tf_->ld, d_tok, st_);
            tf_capture(logits, count, nullptr);
        }
        dec_accept(ds, count, tab + 5 * count, d_tok, st_);
        QASR_HIP(hipMemcpyAsync(pin_cnt_, ds.counters, 4 * sizeof(int), hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipStreamSynchronize(st_));
    }
    if (count == 1 && draft_ && !tf_) {   // streaming: prompt-lookup drafts from earlier transcripts
        std::vector<int32_t> toks;
        bool eos = false;
        {
            Timer tdd(st_, times ? &times->decode : nullptr);
            int* hs = (int*)pinned(4 * sizeof(int));
            QASR_HIP(hipMemcpyAsync(hs, ds.out, sizeof(int), hipMemcpyDeviceToHost, st_));
            QASR_HIP(hipMemcpyAsync(hs + 1, ds.gen, sizeof(int), hipMemcpyDeviceToHost, st_));
            QASR_HIP(hipMemcpyAsync(hs + 2, ds.done, sizeof(int), hipMemcpyDeviceToHost, st_));
            QASR_HIP(hipStreamSynchronize(st_));
            const int first = hs[0], gen = hs[1], done = hs[2];
            if (gen > 0) toks.push_back(first);
            eos = gen == 0;   // the prompt's first choice was EOS (natural mode)
            if (!done) draft_decode(n_prompt[0], base[0], budget[0], (int)slots, toks, eos, force_tps > 0);
        }
        out[0].tokens = toks;
        out[0].truncated = force_tps <= 0 && !eos && (int)toks.size() >= budget[0];
        hist_last_ = (int)history_.size();
        history_.insert(history_.end(), toks.begin(), toks.end());
        if (history_.size() > 8192) {
            const int cut = (int)history_.size() - 8192;
            history_.erase(history_.begin(), history_.begin() + cut);
            hist_last_ = std::max(0, hist_last_ - cut);
        }
        dstats_.tokens += (int64_t)toks.size();
        UttResult& r = out[0];
        xr_check();
        r.raw = m_->tok.decode(r.tokens.data(), (int)r.tokens.size());
        Tokenizer::parse(r.raw, r.language, r.text);
        remember_prompt_kv();
        return;
    }
    // continuous-batching greedy decode: rows = a bucket of the active count (padding rows are dummies); the
    // bound is the active count read back one step late, which never undercounts because it only decreases
    Timer td(st_, times ? &times->decode : nullptr);
    int bound = ((volatile int*)pin_cnt_)[1];
    const bool graphs = !prof_enabled() && !getenv("QASR_NO_GRAPH") && !tf_;
    if (bound > 0) {
        // size every scratch slot for the largest bucket eagerly, before any capture
        const int bmax = row_bucket(bound);
        sc_.get(S_DTAB, (size_t)6 * bmax * sizeof(int));
        sc_.get(S_X, (size_t)bmax * H * sizeof(float));
        sc_.get(S_LOGITS, (size_t)bmax * V * sizeof(float));
        sc_.get(S_TOK, (size_t)bmax * sizeof(int));
        sc_.get(S_ARGP, argmax_scratch_bytes(bmax));
        sc_.get(S_GU, (size_t)kGemvRows * 2 * h.txt_ffn * sizeof(float));  // the unfused (GEMV-row) SwiGLU
        decode_step(ds, bmax, true);  // also sizes the layer scratch
        QASR_HIP(hipEventRecord(step_ev_[0], st_));
    }
    // captured step graphs hold scratch, KV and weight pointers: any reallocation or precision change retires them;
    // so does a switch of the per-call launch-path variables (QASR_NO_XR / QASR_XR_NORM, read in decoder_layers)
    const uint64_t launch_path = (getenv("QASR_NO_XR") ? 1 : 0) + (getenv("QASR_XR_NORM") ? 2 : 0) +
                                 (getenv("QASR_XR_VOCAB") && atoi(getenv("QASR_XR_VOCAB")) == 0 ? 4 : 0);
    const uint64_t key[5] = {sc_.epoch, kv_epoch_, m_->precision_gen, deterministic_gen(),
                             attn_epoch_ * 64 + launch_path * 4 + (batch_inv_ ? 1 : 0)};
    if (memcmp(key, graph_key_, sizeof key) != 0) {
        for (auto& g : graphs_) (void)hipGraphExecDestroy(g.second);
        graphs_.clear();
        memcpy(graph_key_, key, sizeof key);
    }
    int step = 1;
    // QASR_STEP_HIST=1: decode steps per row bucket on stderr (tuning aid for the decode GEMM shapes)
    static const bool hist = getenv("QASR_STEP_HIST") != nullptr;
    std::map<int, int> steps_per_bucket;
    while (bound > 0) {
        const int B = row_bucket(bound);
        if (hist) steps_per_bucket[B]++;
        if (graphs) {
            auto it = graphs_.find(B);
            if (it == graphs_.end()) {
                hipGraph_t g;
                QASR_HIP(hipStreamBeginCapture(st_, hipStreamCaptureModeRelaxed));
                sc_.capturing = true;
                try {
                    decode_step(ds, B, false);
                } catch (...) {
                    sc_.capturing = false;
                    (void)hipStreamEndCapture(st_, &g);
                    throw;
                }
                sc_.capturing = false;
                QASR_HIP(hipStreamEndCapture(st_, &g));
                hipGraphExec_t ex;
                QASR_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
                (void)hipGraphDestroy(g);
                it = graphs_.emplace(B, ex).first;
            }
            QASR_HIP(hipGraphLaunch(it->second, st_));
        } else {
            // eager steps (profiling runs): the keys the step's rows attend, for the attention's algorithmic bytes —
            // known on the host only with a forced token count (utterance u is active while step < budget[u])
            int64_t keys = 0;
            if (force_tps > 0)
                for (int u = 0; u < count; u++)
                    if (budget[u] > step) keys += n_prompt[u] + step;
            decode_step(ds, B, false, keys);
        }
        QASR_HIP(hipEventRecord(step_ev_[step & 1], st_));
        QASR_HIP(hipEventSynchronize(step_ev_[(step - 1) & 1]));
        const int seen = ((volatile int*)pin_cnt_)[1];
        bound = std::min(bound, seen);
        step++;
    }
    QASR_HIP(hipStreamSynchronize(st_));
    xr_check();
    if (hist) {
        fprintf(stderr, "decode steps per row bucket:");
        for (auto& kv : steps_per_bucket) fprintf(stderr, " %d:%d", kv.first, kv.second);
        fprintf(stderr, "\n");
    }
    {
        std::vector<int> hb((size_t)6 * ucap_ + 16), ho((size_t)count * ld);
        QASR_HIP(hipMemcpyAsync(hb.data(), blk, hb.size() * sizeof(int), hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipMemcpyAsync(ho.data(), ds.out, ho.size() * sizeof(int), hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipStreamSynchronize(st_));
        QASR_CHECK(hb[6 * ucap_ + 8 + 2] == 0, QASR_E_INTERNAL, "decode: row bound violated");
        for (int u = 0; u < count; u++) {
            const int g = hb[ucap_ + u];
            out[u].tokens.assign(ho.begin() + (size_t)u * ld, ho.begin() + (size_t)u * ld + g);
            out[u].truncated = force_tps <= 0 && g >= budget[u];
        }
    }
    for (int u = 0; u < count; u++) {
        UttResult& r = out[u];
        r.raw = m_->tok.decode(r.tokens.data(), (int)r.tokens.size());
        Tokenizer::parse(r.raw, r.language, r.text);
    }
    remember_prompt_kv();
}

void Session::run_host(const std::vector<const float*>& pcm, const std::vector<int64_t>& len, int max_new,
                       int force_tps, std::vector<UttResult>& out, StageTimes* times) {
    std::vector<int64_t> off(len.size());
    int64_t total = 0;
    for (size_t i = 0; i < len.size(); i++) {
        off[i] = total;
        total += len[i];
    }
    float* d = (float*)sc_.get(S_PCM, (size_t)std::max<int64_t>(total, 1) * sizeof(float));
    for (size_t i = 0; i < len.size(); i++)
        QASR_HIP(hipMemcpyAsync(d + off[i], pcm[i], (size_t)len[i] * sizeof(float), hipMemcpyHostToDevice, st_));
    // encoder cache: every single-utterance run encodes in the row-count-independent order (front_end), so each of
    // its complete windows is a function of the window's samples and the request's mel maximum; the run stores them,
    // and the next run reuses those its sample prefix shares bitwise (the app's growing interim window before it
    // reaches 12 s) when its mel maximum is the same bits.  A sliding window shares no prefix and reuses nothing.
    const bool single = enc_cache_ && len.size() == 1;
    ec_run_ = false;
    ec_cand_ = 0;
    if (single) {
        const int64_t m = std::min<int64_t>(len[0], (int64_t)ec_pcm_.size());
        int64_t L = 0;
        const size_t B = 4096;
        while (L + (int64_t)B <= m && !memcmp(pcm[0] + L, ec_pcm_.data() + L, B * sizeof(float))) L += B;
        while (L < m && !memcmp(pcm[0] + L, ec_pcm_.data() + L, sizeof(float))) L++;
        const int per = m_->hp.n_window_infer / 100;
        const auto frames_in = [&](int w, int64_t n) { return 16000LL * (per * w - 1) + 16040 <= n; };
        // (Q8 precision only: the MXFP8 GEMMs have no row-count-independent order)
        ec_run_ = !m_->mx() && frames_in(1, len[0]);
        // windows whose chunks' frames all lie in the samples this run shares with the previous one (bitwise)
        while (ec_run_ && ec_cand_ < ec_windows_ && frames_in(ec_cand_ + 1, L)) ec_cand_++;
        ec_windows_ = 0;   // invalid until this run stores its own (an exception leaves it empty)
    }
    try {
        run_batch(d, off, len, max_new, force_tps, out, times);
    } catch (...) {
        ec_run_ = false;
        ec_windows_ = 0;
        ec_pcm_.clear();
        throw;
    }
    if (single) ec_pcm_.assign(pcm[0], pcm[0] + len[0]);
    if (ec_run_) ec_umax_ = ((volatile const unsigned*)pin_cnt_)[60];   // this run's mel maximum (the stream is idle)
    ec_run_ = false;
}

// ------------------------------------------------------------------------------------------ test stages
void Session::mel_host(const float* pcm, int64_t n, std::vector<float>& mel, int& t_valid, int& t_pad) {
    const qasr_hparams& h = m_->hp;
    float* d = (float*)sc_.get(S_PCM, (size_t)n * sizeof(float));
    QASR_HIP(hipMemcpyAsync(d, pcm, (size_t)n * sizeof(float), hipMemcpyHostToDevice, st_));
    FrontEnd fe;
    std::vector<int64_t> off = {0}, len = {n};
    front_end(d, off, len, fe, nullptr);
    mel_dims(n, t_valid, t_pad);
    std::vector<float> chunked((size_t)h.n_mels * t_pad);
    QASR_HIP(hipMemcpyAsync(chunked.data(), sc_.get(S_MELX, 0), chunked.size() * sizeof(float), hipMemcpyDeviceToHost, st_));
    QASR_HIP(hipStreamSynchronize(st_));
    mel.assign(chunked.size(), 0.f);
    const int nch = t_pad / 100;
    for (int c = 0; c < nch; c++)
        for (int m = 0; m < h.n_mels; m++)
            for (int t = 0; t < 100; t++) mel[(size_t)m * t_pad + c * 100 + t] = chunked[((size_t)c * h.n_mels + m) * 100 + t];
}

void Session::encode_host(const float* mel, int t_pad, int t_valid, std::vector<float>& emb, std::vector<float>* enc,
                          int& n_tok) {
    // bypass the log-mel stage: feed the given mel into the conv stack
    const qasr_hparams& h = m_->hp;
    const int nch = t_pad / 100, nm = h.n_mels, C = h.conv_ch, d = h.enc_d, F3 = m_->audio_F3();
    std::vector<float> chunked((size_t)nch * nm * 100);
    for (int c = 0; c < nch; c++)
        for (int m = 0; m < nm; m++)
            for (int t = 0; t < 100; t++) chunked[((size_t)c * nm + m) * 100 + t] = mel[(size_t)m * t_pad + c * 100 + t];
    float* melx = (float*)sc_.get(S_MELX, chunked.size() * sizeof(float));
    QASR_HIP(hipMemcpyAsync(melx, chunked.data(), chunked.size() * sizeof(float), hipMemcpyHostToDevice, st_));
    FrontEnd fe;
    fe.total_chunks = nch;
    fe.n_tok = {audio_token_count(t_valid)};
    fe.tok_base = {0};
    fe.total_tokens = fe.n_tok[0];
    std::vector<int> valid_idx;
    for (int c = 0; c < nch; c++) {
        const int v = post_cnn_len(std::max(0, std::min(100, t_valid - c * 100)));
        for (int t = 0; t < v; t++) valid_idx.push_back(c * 13 + t);
    }
    const int H1 = (nm + 1) / 2, H2 = (H1 + 1) / 2;
    __half* a1 = (__half*)sc_.get(S_A1, (size_t)nch * H1 * 50 * C * sizeof(__half));
    __half* a2 = (__half*)sc_.get(S_A2, (size_t)nch * H2 * 25 * C * sizeof(__half));
    float* a3 = (float*)sc_.get(S_A3, (size_t)nch * 13 * C * F3 * sizeof(float));
    conv1_gelu(melx, nch, nm, m_->conv_w[0], m_->conv_b[0], C, a1, st_);
    conv3x3_gelu(a1, nch, H1, 50, m_->conv_w[1], m_->conv_b[1], C, a2, 0, st_);
    conv3x3_gelu(a2, nch, H2, 25, m_->conv_w[2], m_->conv_b[2], C, a3, 1, st_);
    const int rows = nch * 13, K = C * F3;
    int8_t* xq = (int8_t*)sc_.get(S_XQ, (size_t)rows * K);
    float* xd = (float*)sc_.get(S_XD, (size_t)rows * (K / QK) * sizeof(float));
    quant_rows(a3, rows, K, K, xq, xd, st_);
    float* proj = (float*)sc_.get(S_PROJ, (size_t)rows * d * sizeof(float));
    mx_ws(rows, K);
    linear_q8(xq, xd, rows, m_->conv_out, nullptr, nullptr, proj, d, EPI_STORE, st_);
    int* d_valid = upload(S_VALID, valid_idx);
    float* hs = (float*)sc_.get(S_HS, (size_t)fe.total_tokens * d * sizeof(float));
    add_posemb_gather(proj, nch, 13, d, m_->pos_emb, d_valid, fe.total_tokens, hs, st_);
    float* encd = enc ? (float*)sc_.get(S_ENC, (size_t)fe.total_tokens * d * sizeof(float)) : nullptr;
    encoder(fe, encd);
    n_tok = fe.total_tokens;
    emb.resize((size_t)n_tok * h.txt_h);
    QASR_HIP(hipMemcpyAsync(emb.data(), sc_.get(S_EMB, 0), emb.size() * sizeof(float), hipMemcpyDeviceToHost, st_));
    if (enc) {
        enc->resize((size_t)n_tok * d);
        QASR_HIP(hipMemcpyAsync(enc->data(), encd, enc->size() * sizeof(float), hipMemcpyDeviceToHost, st_));
    }
    QASR_HIP(hipStreamSynchronize(st_));
}

void Session::prefill_logits_host(const float* embeds, int n, std::vector<float>& logits) {
    kvp_rows_ = 0;   // writes K/V rows from slot 0 (no prompt-KV reuse after it)
    const qasr_hparams& h = m_->hp;
    QASR_CHECK(n > 0 && n <= n_ctx_, QASR_E_CAPACITY, "prefill length exceeds n_ctx");
    ensure_kv(n);
    std::vector<int> pos(n), slot(n), kvs(n, 0), kvl(n);
    for (int i = 0; i < n; i++) {
        pos[i] = i;
        slot[i] = i;
        kvl[i] = i + 1;
    }
    float* x = (float*)sc_.get(S_X, (size_t)n * h.txt_h * sizeof(float));
    QASR_HIP(hipMemcpyAsync(x, embeds, (size_t)n * h.txt_h * sizeof(float), hipMemcpyHostToDevice, st_));
    int* d_pos = upload(S_POS, pos);
    int* d_slot = upload(S_SLOT, slot);
    int* d_kvs = upload(S_KVS, kvs);
    int* d_kvl = upload(S_KVL, kvl);
    decoder_layers(x, n, d_pos, d_slot, d_kvs, d_kvl, (int64_t)n * (n + 1) / 2, /*dense=*/true);
    float* lg = (float*)sc_.get(S_LOGITS, (size_t)n * h.vocab * sizeof(float));
    lm_head_rows(x, n, h.txt_h, lg);
    logits.resize((size_t)n * h.vocab);
    QASR_HIP(hipMemcpyAsync(logits.data(), lg, logits.size() * sizeof(float), hipMemcpyDeviceToHost, st_));
    QASR_HIP(hipStreamSynchronize(st_));
}

// prompt from the audio, then the forced continuation one token per step (the decode path, M = 1):
// logits [n_forced + 1][V]
void Session::forced_logits_host(const float* pcm, int64_t n, const int32_t* forced, int n_forced,
                                 std::vector<float>& logits, bool one_pass) {
    kvp_rows_ = 0;   // writes K/V rows from slot 0 (no prompt-KV reuse after it)
    const qasr_hparams& h = m_->hp;
    const int H = h.txt_h, V = h.vocab;
    float* d = (float*)sc_.get(S_PCM, (size_t)n * sizeof(float));
    QASR_HIP(hipMemcpyAsync(d, pcm, (size_t)n * sizeof(float), hipMemcpyHostToDevice, st_));
    FrontEnd fe;
    std::vector<int64_t> off = {0}, len = {n};
    front_end(d, off, len, fe, nullptr);
    encoder(fe, nullptr);
    std::vector<int32_t> ids = build_prompt(h, fe.n_tok[0], 0, context_);
    const int P = (int)ids.size();
    // the one-pass verify needs one more KV slot (the dummy slot of its bucket's padding rows); the step-by-step
    // path accepts a sequence that exactly fills n_ctx
    const int extra = one_pass ? 1 : 0;
    QASR_CHECK(P + n_forced + extra <= n_ctx_, QASR_E_CAPACITY, "forced sequence exceeds n_ctx");
    ensure_kv(P + n_forced + 1 + extra);
    logits.assign((size_t)(n_forced + 1) * V, 0.f);
    std::vector<int> pos(P), slot(P), kvs(P, 0), kvl(P);
    for (int i = 0; i < P; i++) {
        pos[i] = i;
        slot[i] = i;
        kvl[i] = i + 1;
    }
    int* d_ids = upload(S_IDS, ids);
    float* x = (float*)sc_.get(S_X, (size_t)std::max(P, 1) * H * sizeof(float));
    float* emb = (float*)sc_.get(S_EMB, (size_t)fe.total_tokens * H * sizeof(float));
    embed_rows(d_ids, P, m_->tok_embd, emb, x, st_);
    {
        StableOrderScope order(true);   // the prefill of run_batch: row 0's logits are the run's first-token logits
        decoder_layers(x, P, upload(S_POS, pos), upload(S_SLOT, slot), upload(S_KVS, kvs), upload(S_KVL, kvl),
                       (int64_t)P * (P + 1) / 2, /*dense=*/true);
    }
    float* lg = (float*)sc_.get(S_LOGITS, (size_t)V * sizeof(float));
    lm_head_rows(x + (size_t)(P - 1) * H, 1, H, lg);
    QASR_HIP(hipMemcpyAsync(logits.data(), lg, (size_t)V * sizeof(float), hipMemcpyDeviceToHost, st_));
    if (one_pass && n_forced > 0) {
        // the whole continuation as one verify pass of the streaming decode (draft_step): row i feeds forced[i] at
        // position P + i and its logits predict the token after it — the rows a drafted decode accepts from
        QASR_CHECK(n_forced <= kDraftRows, QASR_E_INVALID, "one-pass forced logits: at most kDraftRows tokens");
        QASR_HIP(hipStreamSynchronize(st_));
        // (the row bucket of the streaming decode, padded with dummy rows, through the same captured graphs)
        constexpr int R = kDraftRows;
        const int B = n_forced <= 1 ? 1 : n_forced <= 2 ? 2 : n_forced <= 4 ? 4 : n_forced <= 8 ? 8 : n_forced <= 16 ? 16 : 32;
        const int dummy = P + n_forced + 1;
        std::vector<int> hb((size_t)5 * R, 0);
        for (int i = 0; i < B; i++) {
            const bool real = i < n_forced;
            hb[i] = real ? forced[i] : 0;
            hb[R + i] = real ? P + i : 0;
            hb[2 * R + i] = real ? P + i : dummy;
            hb[3 * R + i] = real ? 0 : dummy;
            hb[4 * R + i] = real ? P + i + 1 : 1;
        }
        int* tab = (int*)sc_.get(S_DTAB, (size_t)6 * R * sizeof(int));
        QASR_HIP(hipMemcpyAsync(tab, hb.data(), hb.size() * sizeof(int), hipMemcpyHostToDevice, st_));
        sc_.get(S_X, (size_t)R * H * sizeof(float));
        sc_.get(S_LOGITS, (size_t)R * V * sizeof(float));
        draft_graphs_refresh();
        draft_pass(B);
        QASR_HIP(hipMemcpyAsync(logits.data() + V, sc_.get(S_LOGITS, 0), (size_t)n_forced * V * sizeof(float),
                                hipMemcpyDeviceToHost, st_));
        QASR_HIP(hipStreamSynchronize(st_));
        return;
    }
    for (int i = 0; i < n_forced; i++) {
        const int p = P + i;
        std::vector<int> one_id = {forced[i]}, one_pos = {p}, one_slot = {p}, one_kvs = {0}, one_kvl = {p + 1};
        int* di = upload(S_IDS, one_id);
        embed_rows(di, 1, m_->tok_embd, nullptr, x, st_);
        decoder_layers(x, 1, upload(S_POS, one_pos), upload(S_SLOT, one_slot), upload(S_KVS, one_kvs),
                       upload(S_KVL, one_kvl), p + 1);
        lm_head_rows(x, 1, H, lg);
        QASR_HIP(hipMemcpyAsync(logits.data() + (size_t)(i + 1) * V, lg, (size_t)V * sizeof(float),
                                hipMemcpyDeviceToHost, st_));
    }
    QASR_HIP(hipStreamSynchronize(st_));
}

void Session::forced_logits_batch_host(const std::vector<const float*>& pcm, const std::vector<int64_t>& len,
                                       const int32_t* forced, int n_forced, const std::vector<int>& want, float* out) {
    const int count = (int)len.size();
    QASR_CHECK(count > 0 && n_forced >= 0 && (n_forced == 0 || forced) && out, QASR_E_INVALID, "bad arguments");
    TeacherForce tf;
    tf.n_forced = n_forced;
    tf.ld = n_forced + 1;
    tf.want.assign(count, -1);
    for (size_t w = 0; w < want.size(); w++) {
        QASR_CHECK(want[w] >= 0 && want[w] < count && tf.want[want[w]] < 0, QASR_E_INVALID, "want: bad or repeated index");
        tf.want[want[w]] = (int)w;
    }
    tf.out = out;
    std::vector<int> ids((size_t)count * tf.ld, -1);
    for (int u = 0; u < count; u++)
        for (int j = 0; j < n_forced; j++) ids[(size_t)u * tf.ld + j] = forced[(size_t)u * n_forced + j];
    QASR_HIP(hipMalloc(&tf.d_ids, ids.size() * sizeof(int)));
    struct Reset {
        Session* s;
        TeacherForce* t;
        ~Reset() {
            (void)hipStreamSynchronize(s->st_);
            (void)hipFree(t->d_ids);
            s->tf_ = nullptr;
        }
    } reset{this, &tf};
    QASR_HIP(hipMemcpy(tf.d_ids, ids.data(), ids.size() * sizeof(int), hipMemcpyHostToDevice));
    tf_ = &tf;
    std::vector<UttResult> res;
    run_host(pcm, len, 0, 0, res, nullptr);
    // (the loop may run one more, empty step: the host reads the active count one step late)
    QASR_CHECK(tf.step >= n_forced + 1, QASR_E_INTERNAL, "teacher forcing: step count");
    for (int u = 0; u < count; u++)
        for (int j = 0; j < n_forced; j++)
            QASR_CHECK(res[u].tokens[j] == forced[(size_t)u * n_forced + j], QASR_E_INTERNAL,
                       "teacher forcing: a forced token was not accepted");
}

}  // namespace qasr
