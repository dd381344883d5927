// extern "C": model / session / batch / VAD / audio-io entry points (include/qasr.h).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qasr.h"
#include "capi_util.h"
#include "engine.h"
#include "kernels_audio.h"
#include "vad.h"

using namespace qasr;

#include "capi_handles.h"

namespace {

void check_backend(const char* backend) {
    const std::string b = backend ? backend : "hip";
    QASR_CHECK(b == "hip" || b == "auto", QASR_E_BACKEND,
               "backend '" + b + "' is not available: this engine runs on HIP (MI355X) only");
    int n = 0;
    QASR_HIP(hipGetDeviceCount(&n));
    QASR_CHECK(n > 0, QASR_E_BACKEND, "no HIP device visible");
}

char* dup(const std::string& s) {
    char* p = (char*)malloc(s.size() + 1);
    memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    return p;
}

void fill_result(const UttResult& u, const StageTimes& t, qasr_result* r) {
    memset(r, 0, sizeof(*r));
    r->text = dup(u.text);
    r->language = dup(u.language);
    r->raw = dup(u.raw);
    r->n_tokens = (int32_t)u.tokens.size();
    r->tokens = (int32_t*)malloc(sizeof(int32_t) * std::max<size_t>(1, u.tokens.size()));
    if (!u.tokens.empty()) memcpy(r->tokens, u.tokens.data(), u.tokens.size() * sizeof(int32_t));
    r->n_audio_tokens = u.n_audio;
    r->n_prompt = u.n_prompt;
    r->ms_mel = t.mel;
    r->ms_encoder = t.encoder;
    r->ms_prefill = t.prefill;
    r->ms_decode = t.decode;
    r->truncated = u.truncated ? 1 : 0;
}

}  // namespace

#include <dlfcn.h>

static std::string lib_dir() {
    Dl_info info;
    if (dladdr((void*)&qasr_version, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t s = p.rfind('/');
        return s == std::string::npos ? "." : p.substr(0, s);
    }
    return ".";
}

extern "C" {

// ------------------------------------------------------------------------------------------------ model
QASR_API int qasr_model_open(const char* gguf_path, const char* backend, qasr_model** out) {
    return guard([&] {
        QASR_CHECK(gguf_path && out, QASR_E_INVALID, "null argument");
        check_backend(backend);
        auto h = std::make_unique<qasr_model>();
        h->m = load_gguf_model(gguf_path);
        *out = h.release();
    });
}

QASR_API int qasr_model_open_synthetic(const char* arch, const qasr_hparams* hp, uint64_t seed, qasr_model** out) {
    return guard([&] {
        QASR_CHECK(out, QASR_E_INVALID, "null argument");
        check_backend("hip");
        qasr_hparams h;
        if (arch) default_hparams(arch, &h);
        else {
            QASR_CHECK(hp, QASR_E_INVALID, "either arch or hparams");
            h = *hp;
        }
        auto m = std::make_unique<qasr_model>();
        m->m = make_synthetic_model(h, seed, arch ? arch : "custom");
        *out = m.release();
    });
}

QASR_API int qasr_model_open_shell(const char* gguf_path, const char* arch, const qasr_hparams* hp, qasr_model** out) {
    return guard([&] {
        QASR_CHECK(out, QASR_E_INVALID, "null argument");
        check_backend("hip");
        auto m = std::make_unique<qasr_model>();
        if (gguf_path) {
            m->m = load_gguf_model(gguf_path, true);
        } else {
            qasr_hparams h;
            if (arch) default_hparams(arch, &h);
            else {
                QASR_CHECK(hp, QASR_E_INVALID, "either a GGUF path, arch or hparams");
                h = *hp;
            }
            m->m = make_synthetic_shell(h, arch ? arch : "custom");
        }
        *out = m.release();
    });
}

QASR_API int qasr_model_weight_blob(qasr_model* m, void** dev, size_t* bytes) {
    return guard([&] {
        QASR_CHECK(m && dev && bytes, QASR_E_INVALID, "null argument");
        *dev = m->m->mem.base;
        *bytes = m->m->mem.bytes;
    });
}

QASR_API int qasr_model_weights_received(qasr_model* m) {
    return guard([&] {
        QASR_CHECK(m, QASR_E_INVALID, "null argument");
        QASR_HIP(hipDeviceSynchronize());
        m->m->weights_pending = false;
    });
}

QASR_API int qasr_model_set_precision(qasr_model* m, const char* mode) {
    return guard([&] {
        QASR_CHECK(m && mode, QASR_E_INVALID, "null argument");
        set_precision(*m->m, mode);
    });
}

QASR_API int qasr_model_hparams(const qasr_model* m, qasr_hparams* out) {
    return guard([&] {
        QASR_CHECK(m && out, QASR_E_INVALID, "null argument");
        *out = m->m->hp;
    });
}

QASR_API int64_t qasr_model_weight_bytes(const qasr_model* m) { return m ? m->m->weight_bytes() : 0; }

QASR_API int qasr_model_export_tensor(const qasr_model* m, const char* name, void* dst, size_t cap, size_t* written) {
    return guard([&] {
        QASR_CHECK(m && name && dst && written, QASR_E_INVALID, "null argument");
        export_tensor(*m->m, name, dst, cap, written);
    });
}

QASR_API int qasr_model_tensor_table(const qasr_model* m, char* buf, size_t cap, size_t* needed) {
    return guard([&] {
        QASR_CHECK(m && needed, QASR_E_INVALID, "null argument");
        std::string j = "{";
        for (const auto& kv : m->m->slots) {
            const TensorSlot& t = kv.second;
            char b[256];
            snprintf(b, sizeof b, "%s\"%s\": [%u, %lld, %lld, %d]", j.size() > 1 ? ", " : "", kv.first.c_str(), t.type,
                     (long long)t.rows, (long long)t.cols, t.conv_cin);
            j += b;
        }
        j += "}";
        *needed = j.size() + 1;
        if (buf && cap >= j.size() + 1) memcpy(buf, j.c_str(), j.size() + 1);
        else if (buf) QASR_CHECK(false, QASR_E_CAPACITY, "buffer too small");
    });
}

QASR_API void qasr_model_close(qasr_model* m) { delete m; }

// ------------------------------------------------------------------------------------------------ session
QASR_API int qasr_session_open(qasr_model* m, const char* kv_type, int32_t n_ctx, qasr_session** out) {
    return guard([&] {
        QASR_CHECK(m && out, QASR_E_INVALID, "null argument");
        QASR_CHECK(!kv_type || std::string(kv_type) == "f16", QASR_E_INVALID, "kv_type must be \"f16\"");
        QASR_CHECK(!m->m->weights_pending, QASR_E_INVALID,
                   "model is a shell whose weights have not arrived (qasr_model_weights_received)");
        ensure_stage_scales(*m->m);
        auto s = std::make_unique<qasr_session>();
        s->s = std::make_unique<Session>(m->m.get(), n_ctx > 0 ? n_ctx : 32768);
        *out = s.release();
    });
}

QASR_API int qasr_model_tokenize(const qasr_model* m, const char* text, size_t len, int32_t* ids, size_t cap,
                                size_t* n_out) {
    return guard([&] {
        QASR_CHECK(m && (text || len == 0) && n_out, QASR_E_INVALID, "null argument");
        const std::vector<int32_t> v = m->m->tok.encode(std::string(text ? text : "", len));
        *n_out = v.size();
        QASR_CHECK(!ids || cap >= v.size(), QASR_E_CAPACITY, "id buffer too small");
        if (ids && !v.empty()) memcpy(ids, v.data(), v.size() * sizeof(int32_t));
    });
}

// a stand-alone byte-level BPE tokenizer (pieces + merges), the model tokenizer's encoder without a model
struct qasr_tokenizer {
    qasr::Tokenizer t;
};

QASR_API int qasr_tokenizer_open(const char* const* pieces, int32_t n_pieces, const uint8_t* is_special,
                                 const char* const* merges, int32_t n_merges, qasr_tokenizer** out) {
    return guard([&] {
        QASR_CHECK(pieces && n_pieces > 0 && n_merges >= 0 && (merges || n_merges == 0) && out, QASR_E_INVALID,
                   "bad arguments");
        auto t = std::make_unique<qasr_tokenizer>();
        t->t.pieces.assign(pieces, pieces + n_pieces);
        t->t.is_special.assign(n_pieces, 0);
        if (is_special) t->t.is_special.assign(is_special, is_special + n_pieces);
        t->t.merges.assign(merges, merges + n_merges);
        *out = t.release();
    });
}

QASR_API int qasr_tokenizer_encode(const qasr_tokenizer* t, const char* text, size_t len, int32_t* ids, size_t cap,
                                   size_t* n_out) {
    return guard([&] {
        QASR_CHECK(t && (text || len == 0) && n_out, QASR_E_INVALID, "null argument");
        const std::vector<int32_t> v = t->t.encode(std::string(text ? text : "", len));
        *n_out = v.size();
        QASR_CHECK(!ids || cap >= v.size(), QASR_E_CAPACITY, "id buffer too small");
        if (ids && !v.empty()) memcpy(ids, v.data(), v.size() * sizeof(int32_t));
    });
}

QASR_API void qasr_tokenizer_close(qasr_tokenizer* t) { delete t; }

QASR_API int qasr_model_detokenize(const qasr_model* m, const int32_t* ids, int32_t n, char* out, size_t cap,
                                  size_t* written) {
    return guard([&] {
        QASR_CHECK(m && (ids || n == 0) && n >= 0 && written, QASR_E_INVALID, "null argument");
        const std::string t = m->m->tok.decode(ids, n);
        *written = t.size();
        QASR_CHECK(!out || cap >= t.size(), QASR_E_CAPACITY, "text buffer too small");
        if (out && !t.empty()) memcpy(out, t.data(), t.size());
    });
}

QASR_API int qasr_session_set_context(qasr_session* s, const int32_t* ids, int32_t n) {
    return guard([&] {
        QASR_CHECK(s && n >= 0 && (ids || n == 0), QASR_E_INVALID, "bad arguments");
        s->s->set_context(std::vector<int32_t>(ids, ids + n));
    });
}

QASR_API int qasr_session_set_draft(qasr_session* s, int32_t on) {
    return guard([&] {
        QASR_CHECK(s, QASR_E_INVALID, "null argument");
        s->s->set_draft(on != 0);
    });
}

QASR_API int qasr_session_set_batch_invariant(qasr_session* s, int32_t on) {
    return guard([&] {
        QASR_CHECK(s, QASR_E_INVALID, "null argument");
        s->s->set_batch_invariant(on != 0);
    });
}

QASR_API int qasr_session_set_draft_noise(qasr_session* s, float rate, uint64_t seed) {
    return guard([&] {
        QASR_CHECK(s && rate >= 0.f && rate <= 1.f, QASR_E_INVALID, "bad arguments");
        s->s->set_draft_noise(rate, seed);
    });
}

QASR_API int qasr_session_draft_stats(const qasr_session* s, int64_t* stats) {
    return guard([&] {
        QASR_CHECK(s && stats, QASR_E_INVALID, "null argument");
        const Session::DraftStats& d = s->s->draft_stats();
        stats[0] = d.passes, stats[1] = d.proposed, stats[2] = d.accepted, stats[3] = d.tokens;
    });
}

QASR_API int qasr_session_set_encoder_cache(qasr_session* s, int32_t on) {
    return guard([&] {
        QASR_CHECK(s, QASR_E_INVALID, "null argument");
        s->s->set_enc_cache(on != 0);
    });
}

QASR_API int qasr_session_encoder_cache_stats(const qasr_session* s, int64_t* stats) {
    return guard([&] {
        QASR_CHECK(s && stats, QASR_E_INVALID, "null argument");
        const Session::EncCacheStats& e = s->s->enc_cache_stats();
        stats[0] = e.runs, stats[1] = e.windows_reused, stats[2] = e.windows_computed;
    });
}

QASR_API int qasr_session_prompt_kv_stats(const qasr_session* s, int64_t* rows_reused) {
    return guard([&] {
        QASR_CHECK(s && rows_reused, QASR_E_INVALID, "null argument");
        *rows_reused = s->s->prompt_kv_stats().rows_reused;
    });
}

QASR_API int qasr_session_audio_embeds(qasr_session* s, float* out, size_t cap, size_t* n_out) {
    return guard([&] {
        QASR_CHECK(s && n_out, QASR_E_INVALID, "null argument");
        const std::vector<float> e = s->s->last_audio_embeds();
        *n_out = e.size();
        QASR_CHECK(!out || cap >= e.size(), QASR_E_CAPACITY, "audio_embeds: buffer too small");
        if (out) std::copy(e.begin(), e.end(), out);
    });
}

QASR_API int qasr_session_run_opts(qasr_session* s, const float* pcm16k, size_t n, const qasr_run_opts* opts,
                                   qasr_result* out) {
    return guard([&] {
        QASR_CHECK(s && pcm16k && out && n > 0, QASR_E_INVALID, "bad arguments");
        std::vector<UttResult> res;
        StageTimes t;
        s->s->run_host({pcm16k}, {(int64_t)n}, opts ? opts->max_new_tokens : 0, opts ? opts->force_tokens_per_s : 0,
                       res, &t);
        fill_result(res[0], t, out);
    });
}

QASR_API int qasr_session_run(qasr_session* s, const float* pcm16k, size_t n, int32_t timestamps, qasr_result* out) {
    (void)timestamps;  // only timestamps="none" is used by the reference (qwen3_asr_server.py:144,321)
    return qasr_session_run_opts(s, pcm16k, n, nullptr, out);
}

QASR_API int qasr_run_batch(qasr_session* s, const float* const* pcm, const size_t* n, int32_t count,
                            const qasr_run_opts* opts, qasr_result* out) {
    return guard([&] {
        QASR_CHECK(s && pcm && n && out && count >= 0, QASR_E_INVALID, "bad arguments");
        std::vector<const float*> p(pcm, pcm + count);
        std::vector<int64_t> len(count);
        for (int i = 0; i < count; i++) len[i] = (int64_t)n[i];
        std::vector<UttResult> res;
        StageTimes t;
        s->s->run_host(p, len, opts ? opts->max_new_tokens : 0, opts ? opts->force_tokens_per_s : 0, res, &t);
        for (int i = 0; i < count; i++) fill_result(res[i], t, &out[i]);
    });
}

QASR_API int qasr_run_batch_device(qasr_session* s, const float* dev_pcm, const int64_t* offsets,
                                   const int64_t* lengths, int32_t count, const qasr_run_opts* opts,
                                   qasr_result* out) {
    return guard([&] {
        QASR_CHECK(s && dev_pcm && offsets && lengths && count >= 0, QASR_E_INVALID, "bad arguments");
        std::vector<int64_t> off(offsets, offsets + count), len(lengths, lengths + count);
        std::vector<UttResult> res;
        StageTimes t;
        s->s->run_batch(dev_pcm, off, len, opts ? opts->max_new_tokens : 0, opts ? opts->force_tokens_per_s : 0, res,
                        &t);
        if (out)
            for (int i = 0; i < count; i++) fill_result(res[i], t, &out[i]);
    });
}

QASR_API void qasr_result_free(qasr_result* r) {
    if (!r) return;
    free(r->text);
    free(r->language);
    free(r->raw);
    free(r->tokens);
    memset(r, 0, sizeof(*r));
}

QASR_API void qasr_session_close(qasr_session* s) { delete s; }

QASR_API int qasr_session_forced_logits(qasr_session* s, const float* pcm16k, size_t n, const int32_t* forced,
                                        int32_t n_forced, float* logits_out) {
    return guard([&] {
        QASR_CHECK(s && pcm16k && logits_out && n_forced >= 0, QASR_E_INVALID, "bad arguments");
        std::vector<float> lg;
        s->s->forced_logits_host(pcm16k, (int64_t)n, forced, n_forced, lg);
        memcpy(logits_out, lg.data(), lg.size() * sizeof(float));
    });
}

QASR_API int qasr_session_forced_logits_batch(qasr_session* s, const float* const* pcm, const size_t* n,
                                              int32_t count, const int32_t* forced, int32_t n_forced,
                                              const int32_t* want, int32_t n_want, float* logits_out) {
    return guard([&] {
        QASR_CHECK(s && pcm && n && count > 0 && n_forced >= 0 && (want || n_want == 0) && n_want >= 0 &&
                       (logits_out || n_want == 0),
                   QASR_E_INVALID, "bad arguments");
        std::vector<const float*> p(pcm, pcm + count);
        std::vector<int64_t> len(count);
        for (int i = 0; i < count; i++) len[i] = (int64_t)n[i];
        std::vector<int> w(want, want + n_want);
        s->s->forced_logits_batch_host(p, len, forced, n_forced, w, logits_out);
    });
}

QASR_API int qasr_session_forced_logits_verify(qasr_session* s, const float* pcm16k, size_t n, const int32_t* forced,
                                               int32_t n_forced, float* logits_out) {
    return guard([&] {
        QASR_CHECK(s && pcm16k && logits_out && n_forced >= 0 && n_forced <= kDraftRows, QASR_E_INVALID,
                   "bad arguments (n_forced ≤ 32)");
        std::vector<float> lg;
        s->s->forced_logits_host(pcm16k, (int64_t)n, forced, n_forced, lg, /*one_pass=*/true);
        memcpy(logits_out, lg.data(), lg.size() * sizeof(float));
    });
}

QASR_API int qasr_session_mel(qasr_session* s, const float* pcm16k, size_t n, float* mel_out, int32_t* t_valid,
                              int32_t* t_pad) {
    return guard([&] {
        QASR_CHECK(s && pcm16k && n > 0, QASR_E_INVALID, "bad arguments");
        std::vector<float> mel;
        int tv, tp;
        s->s->mel_host(pcm16k, (int64_t)n, mel, tv, tp);
        if (mel_out) memcpy(mel_out, mel.data(), mel.size() * sizeof(float));
        if (t_valid) *t_valid = tv;
        if (t_pad) *t_pad = tp;
    });
}

QASR_API int qasr_session_encode(qasr_session* s, const float* mel, int32_t t_pad, int32_t t_valid,
                                 float* audio_emb, float* enc_out, int32_t* n_tok) {
    return guard([&] {
        QASR_CHECK(s && mel && t_pad > 0 && t_pad % 100 == 0 && t_valid > 0 && t_valid <= t_pad, QASR_E_INVALID,
                   "bad arguments");
        std::vector<float> emb, enc;
        int nt = 0;
        s->s->encode_host(mel, t_pad, t_valid, emb, enc_out ? &enc : nullptr, nt);
        if (audio_emb) memcpy(audio_emb, emb.data(), emb.size() * sizeof(float));
        if (enc_out) memcpy(enc_out, enc.data(), enc.size() * sizeof(float));
        if (n_tok) *n_tok = nt;
    });
}

QASR_API int qasr_session_prefill_logits(qasr_session* s, const float* embeds, int32_t n, float* logits) {
    return guard([&] {
        QASR_CHECK(s && embeds && logits && n > 0, QASR_E_INVALID, "bad arguments");
        std::vector<float> lg;
        s->s->prefill_logits_host(embeds, n, lg);
        memcpy(logits, lg.data(), lg.size() * sizeof(float));
    });
}

// ------------------------------------------------------------------------------------------------ VAD
QASR_API void qasr_vad_default_options(qasr_vad_options* o) {
    if (!o) return;
    o->threshold = 0.5f;  // FireRedVadOptions, firered_vad.py:25-31
    o->smooth_window_frames = 5;
    o->min_speech_duration_ms = 150;
    o->min_silence_duration_ms = 300;
    o->speech_pad_ms = 120;
}

QASR_API int qasr_vad_open(const char* weights_path, qasr_vad** out) {
    return guard([&] {
        QASR_CHECK(out, QASR_E_INVALID, "null argument");
        check_backend("hip");
        std::string p = weights_path ? weights_path : "";
        if (p.empty()) {
            const char* e = getenv("QASR_VAD_WEIGHTS");
            p = e ? e : lib_dir() + "/../assets/fireredvad_dfsmn.qvad";
        }
        auto v = std::make_unique<qasr_vad>();
        v->v = std::make_unique<Vad>(p);
        *out = v.release();
    });
}

QASR_API int qasr_vad_features(qasr_vad* v, const float* pcm, size_t n, float* feats, size_t cap_frames,
                               size_t* n_frames) {
    return guard([&] {
        QASR_CHECK(v && (pcm || n == 0), QASR_E_INVALID, "bad arguments");
        std::vector<float> f;
        v->v->features(pcm, (int64_t)n, f);
        const size_t T = f.size() / 80;
        if (n_frames) *n_frames = T;
        QASR_CHECK(!feats || cap_frames >= T, QASR_E_CAPACITY, "feature buffer too small");
        if (feats && T) memcpy(feats, f.data(), f.size() * sizeof(float));
    });
}

QASR_API int qasr_vad_probabilities(qasr_vad* v, const float* pcm, size_t n, float* probs, size_t cap,
                                    size_t* n_frames) {
    return guard([&] {
        QASR_CHECK(v && (pcm || n == 0), QASR_E_INVALID, "bad arguments");
        std::vector<float> p;
        v->v->probabilities(pcm, (int64_t)n, p);
        if (n_frames) *n_frames = p.size();
        QASR_CHECK(!probs || cap >= p.size(), QASR_E_CAPACITY, "probability buffer too small");
        if (probs && !p.empty()) memcpy(probs, p.data(), p.size() * sizeof(float));
    });
}

QASR_API int qasr_vad_timestamps_from_probabilities(const float* probs, size_t n_frames, int64_t audio_len,
                                                    const qasr_vad_options* o, qasr_segment* out, size_t cap,
                                                    size_t* n_out) {
    return guard([&] {
        qasr_vad_options opt;
        qasr_vad_default_options(&opt);
        if (o) opt = *o;
        auto seg = timestamps_from_probabilities(probs, (int64_t)n_frames, audio_len, opt);
        if (n_out) *n_out = seg.size();
        QASR_CHECK(!out || cap >= seg.size(), QASR_E_CAPACITY, "segment buffer too small");
        if (out)
            for (size_t i = 0; i < seg.size(); i++) out[i] = qasr_segment{seg[i].first, seg[i].second};
    });
}

QASR_API int qasr_vad_speech_timestamps(qasr_vad* v, const float* pcm, size_t n, const qasr_vad_options* o,
                                        qasr_segment* out, size_t cap, size_t* n_out) {
    return guard([&] {
        QASR_CHECK(v && (pcm || n == 0), QASR_E_INVALID, "bad arguments");
        std::vector<float> p;
        v->v->probabilities(pcm, (int64_t)n, p);
        qasr_vad_options opt;
        qasr_vad_default_options(&opt);
        if (o) opt = *o;
        auto seg = timestamps_from_probabilities(p.data(), (int64_t)p.size(), (int64_t)n, opt);
        if (n_out) *n_out = seg.size();
        QASR_CHECK(!out || cap >= seg.size(), QASR_E_CAPACITY, "segment buffer too small");
        if (out)
            for (size_t i = 0; i < seg.size(); i++) out[i] = qasr_segment{seg[i].first, seg[i].second};
    });
}

QASR_API void qasr_vad_close(qasr_vad* v) { delete v; }

// ------------------------------------------------------------------------------------------------ audio io
// base64 with Python's b64decode(validate=True) acceptance rules and error texts (server_common.py:155-158)
QASR_API int qasr_utf8_replace_invalid(const char* in, size_t n, char* out, size_t cap, size_t* written) {
    return guard([&] {
        QASR_CHECK((in || n == 0) && written, QASR_E_INVALID, "null argument");
        const std::string r = utf8_replace_invalid(std::string(in ? in : "", n));
        *written = r.size();
        QASR_CHECK(out && cap >= r.size(), QASR_E_CAPACITY, "output buffer too small");
        memcpy(out, r.data(), r.size());
    });
}

QASR_API int qasr_parse_transcript(const char* raw, size_t n, char* language, size_t lang_cap, size_t* lang_len,
                                   char* text, size_t text_cap, size_t* text_len) {
    return guard([&] {
        QASR_CHECK((raw || n == 0) && lang_len && text_len, QASR_E_INVALID, "null argument");
        std::string lang, txt;
        Tokenizer::parse(utf8_replace_invalid(std::string(raw ? raw : "", n)), lang, txt);
        *lang_len = lang.size();
        *text_len = txt.size();
        QASR_CHECK((!language || lang_cap >= lang.size()) && (!text || text_cap >= txt.size()), QASR_E_CAPACITY,
                   "output buffer too small");
        if (language && !lang.empty()) memcpy(language, lang.data(), lang.size());
        if (text && !txt.empty()) memcpy(text, txt.data(), txt.size());
    });
}

namespace {
struct B64Table {
    int8_t v[256];
    constexpr B64Table() : v() {
        for (int i = 0; i < 256; i++) v[i] = -1;
        for (int i = 0; i < 26; i++) v['A' + i] = (int8_t)i, v['a' + i] = (int8_t)(26 + i);
        for (int i = 0; i < 10; i++) v['0' + i] = (int8_t)(52 + i);
        v['+'] = 62;
        v['/'] = 63;
    }
};
constexpr B64Table kB64{};
}  // namespace

QASR_API int qasr_decode_pcm_s16le(const char* b64, size_t len, float* out, size_t cap, size_t* n_out) {
    return guard([&] {
        QASR_CHECK(b64 || len == 0, QASR_E_INVALID, "null argument");
        const unsigned char* u = (const unsigned char*)b64;
        // table-driven (branch-free on the data: a 12 s window is 512 KB of random-looking characters)
        size_t q = 0;
        while (q < len && kB64.v[u[q]] >= 0) q++;
        size_t p = 0;
        while (q + p < len && b64[q + p] == '=') p++;
        QASR_CHECK(q + p == len && p <= 2, QASR_E_FORMAT, "Non-base64 digit found");
        QASR_CHECK(q % 4 != 1, QASR_E_FORMAT,
                   "Invalid base64-encoded string: number of data characters (" + std::to_string(q) +
                       ") cannot be 1 more than a multiple of 4");
        QASR_CHECK(q % 4 == 0 || (q % 4) + p >= 4, QASR_E_FORMAT, "Incorrect padding");
        const size_t nbytes = q / 4 * 3 + (q % 4 ? q % 4 - 1 : 0);
        // odd byte count: distinct code (QASR_E_INVALID) so callers can order it after the sample-rate check
        QASR_CHECK(nbytes % 2 == 0, QASR_E_INVALID, "PCM s16le 数据字节数必须为偶数");
        const size_t ns = nbytes / 2;
        if (n_out) *n_out = ns;
        QASR_CHECK(!out || cap >= ns, QASR_E_CAPACITY, "sample buffer too small");
        if (!out) return;
        std::vector<uint8_t> bytes(nbytes + 3);
        size_t o = 0, i = 0;
        for (; i + 4 <= q; i += 4, o += 3) {
            const uint32_t v = (uint32_t)kB64.v[u[i]] << 18 | (uint32_t)kB64.v[u[i + 1]] << 12 |
                               (uint32_t)kB64.v[u[i + 2]] << 6 | (uint32_t)kB64.v[u[i + 3]];
            bytes[o] = (uint8_t)(v >> 16);
            bytes[o + 1] = (uint8_t)(v >> 8);
            bytes[o + 2] = (uint8_t)v;
        }
        if (i < q) {   // 2 or 3 trailing characters → 1 or 2 bytes
            uint32_t v = 0;
            for (size_t k = 0; k < 4; k++) v = v << 6 | (uint32_t)(i + k < q ? kB64.v[u[i + k]] : 0);
            bytes[o] = (uint8_t)(v >> 16);
            bytes[o + 1] = (uint8_t)(v >> 8);
        }
        for (size_t k = 0; k < ns; k++) out[k] = (float)(int16_t)(bytes[2 * k] | (bytes[2 * k + 1] << 8)) / 32768.0f;
    });
}

// np.interp(np.linspace(0, N-1, round(N·16000/sr)), arange(N), x) in float64, cast to f32
QASR_API int qasr_resample_linear(const float* x, size_t n, double source_rate, float* out, size_t cap,
                                  size_t* n_out) {
    return guard([&] {
        QASR_CHECK(source_rate > 0 && std::isfinite(source_rate), QASR_E_INVALID, "bad sample rate");
        if (source_rate == 16000.0) {
            if (n_out) *n_out = n;
            QASR_CHECK(!out || cap >= n, QASR_E_CAPACITY, "buffer too small");
            if (out && n) memcpy(out, x, n * sizeof(float));
            return;
        }
        const double tl = nearbyint((double)n * 16000.0 / source_rate);
        const int64_t target = (int64_t)tl;
        if (n_out) *n_out = target > 0 ? (size_t)target : 0;
        if (target <= 0) return;
        QASR_CHECK(!out || cap >= (size_t)target, QASR_E_CAPACITY, "buffer too small");
        if (!out) return;
        const double stop = n > 0 ? (double)(n - 1) : 0.0;
        const double step = target > 1 ? stop / (double)(target - 1) : 0.0;
        for (int64_t i = 0; i < target; i++) {
            double xv = target > 1 ? (double)i * step : 0.0;
            if (i == target - 1 && target > 1) xv = stop;
            double r;
            if (n == 0) r = 0.0;
            else if (xv >= (double)(n - 1)) r = x[n - 1];
            else {
                const int64_t j = (int64_t)floor(xv);
                if (xv == (double)j) r = x[j];
                else {
                    const double slope = (double)x[j + 1] - (double)x[j];
                    r = slope * (xv - (double)j) + (double)x[j];
                }
            }
            out[i] = (float)r;
        }
    });
}

// ------------------------------------------------------------------------------------------------ front-end ops
static std::once_flag g_tab_once;
static float *g_basis = nullptr, *g_filt = nullptr, *g_win = nullptr, *g_banks = nullptr;
static int g_filt_mels = 0;

static void ensure_tables(int n_mels) {
    std::call_once(g_tab_once, [&] {
        std::vector<float> basis, filt((size_t)201 * n_mels), win(400), banks(80 * 256);
        dft_basis_table(basis);
        mel_filter_table(n_mels, filt.data());
        povey_window(win.data());
        kaldi_mel_banks(banks.data());
        QASR_HIP(hipMalloc(&g_basis, basis.size() * 4));
        QASR_HIP(hipMalloc(&g_filt, filt.size() * 4));
        QASR_HIP(hipMalloc(&g_win, win.size() * 4));
        QASR_HIP(hipMalloc(&g_banks, banks.size() * 4));
        QASR_HIP(hipMemcpy(g_basis, basis.data(), basis.size() * 4, hipMemcpyHostToDevice));
        QASR_HIP(hipMemcpy(g_filt, filt.data(), filt.size() * 4, hipMemcpyHostToDevice));
        QASR_HIP(hipMemcpy(g_win, win.data(), win.size() * 4, hipMemcpyHostToDevice));
        QASR_HIP(hipMemcpy(g_banks, banks.data(), banks.size() * 4, hipMemcpyHostToDevice));
        g_filt_mels = n_mels;
    });
    QASR_CHECK(g_filt_mels == n_mels, QASR_E_INVALID, "qasr_op_mel supports one n_mels per process");
}

// single-utterance log-mel into [n_mels][t_pad] (device in/out)
QASR_API int qasr_op_mel(const float* pcm, int64_t n, int32_t n_mels, float* mel, void* stream) {
    return guard([&] {
        QASR_CHECK(pcm && mel && n > 0, QASR_E_INVALID, "bad arguments");
        ensure_tables(n_mels);
        hipStream_t s = (hipStream_t)stream;
        MelUtt U{};
        int tv, tp;
        mel_dims(n, tv, tp);
        U.pcm_off = 0;
        U.n = n;
        U.P = std::max<int64_t>(std::max<int64_t>(n, 8000), 480000);
        U.t_all = (int)(U.P / 160);
        U.t_valid = tv;
        U.t_comp = std::min(tv + 3, U.t_all);
        U.n_chunks = tp / 100;
        std::vector<int2> work;
        for (int t0 = 0; t0 < U.t_comp; t0 += 16) work.push_back(make_int2(0, t0));
        std::vector<int> cu(U.n_chunks, 0);
        MelUtt* du;
        int2* dw;
        int* dcu;
        unsigned* dmax;
        float *lm, *x;
        QASR_HIP(hipMalloc(&du, sizeof(MelUtt)));
        QASR_HIP(hipMalloc(&dw, work.size() * sizeof(int2)));
        QASR_HIP(hipMalloc(&dcu, cu.size() * sizeof(int)));
        QASR_HIP(hipMalloc(&dmax, 4));
        QASR_HIP(hipMalloc(&lm, (size_t)U.t_comp * n_mels * 4));
        QASR_HIP(hipMalloc(&x, (size_t)U.n_chunks * n_mels * 100 * 4));
        QASR_HIP(hipMemcpy(du, &U, sizeof(MelUtt), hipMemcpyHostToDevice));
        QASR_HIP(hipMemcpy(dw, work.data(), work.size() * sizeof(int2), hipMemcpyHostToDevice));
        QASR_HIP(hipMemcpy(dcu, cu.data(), cu.size() * sizeof(int), hipMemcpyHostToDevice));
        QASR_HIP(hipMemsetAsync(dmax, 0, 4, s));
        mel_frames(pcm, du, dw, (int)work.size(), n_mels, g_basis, g_filt, lm, dmax, s);
        mel_normalize(du, 1, U.n_chunks, dcu, n_mels, lm, dmax, x, s);
        // [chunk][m][100] → [m][t_pad]
        for (int c = 0; c < U.n_chunks; c++)
            QASR_HIP(hipMemcpy2DAsync(mel + c * 100, (size_t)tp * 4, x + (size_t)c * n_mels * 100, 100 * 4, 100 * 4,
                                      (size_t)n_mels, hipMemcpyDeviceToDevice, s));
        QASR_HIP(hipStreamSynchronize(s));
        for (void* p : {(void*)du, (void*)dw, (void*)dcu, (void*)dmax, (void*)lm, (void*)x}) (void)hipFree(p);
    });
}

QASR_API int qasr_op_conv3x3_gelu(const void* in, int32_t n_chunks, int32_t Hi, int32_t Wi, const void* w,
                                  const float* bias, int32_t C, void* out, int32_t out_mode, void* stream) {
    return guard([&] {
        QASR_CHECK(n_chunks >= 0 && Hi > 0 && Wi > 0 && C % 32 == 0 && (out_mode == 0 || out_mode == 1),
                   QASR_E_INVALID, "conv3x3_gelu: bad arguments");
        conv3x3_gelu((const __half*)in, n_chunks, Hi, Wi, (const __half*)w, bias, C, out, out_mode,
                     (hipStream_t)stream);
        QASR_HIP(hipGetLastError());
    });
}

QASR_API int qasr_op_fbank(const float* pcm, int64_t n, float* feats, void* stream) {
    return guard([&] {
        ensure_tables(128);
        const int T = Vad::n_frames(n);
        kaldi_fbank(pcm, n, T, g_win, g_banks, feats, (hipStream_t)stream);
        QASR_HIP(hipGetLastError());
    });
}

}  // extern "C"
