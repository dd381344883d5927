// `engine` — the native drop-in for the reference's bundled ASR sidecar.
//
// Spawned exactly like the reference's `engine.exe serve --engine <id>` (engine.py:39-57, funasr_service.rs:
// 917-972), it speaks the same stdio protocol as BaseASRServer.run (server_common.py:339-437) with the
// Qwen3ASRServer semantics (qwen3_asr_server.py:33-402): one JSON object per line in, one per line out,
// `request_id` echoed, replies byte-compatible with Python's json.dumps(ensure_ascii=False).  stdout carries
// only protocol lines; logs go to stderr and <LIGHT_WHISPER_DATA_DIR>/logs/qwen3_asr_server.log.
//
// Model resolution follows hf_cache_utils.find_hf_snapshot_file (hf_cache_utils.py:73-117).  Test hooks
// (never used by the app): QASR_SYNTHETIC=1 loads seeded synthetic weights when no GGUF is provisioned;
// QASR_PROTOCOL_TEST_FAKE=1 replaces model + VAD by the reference tests' fakes (test_qwen3_asr_server.py:15-57);
// QASR_FORCE_TOKENS_PER_S=k fixes the decode length at round(k·seconds)+1 tokens (benchmarks: deterministic work
// on synthetic weights, SURVEY §8(d) "decode length control"); QASR_MAX_NEW_TOKENS=n caps the natural-EOS decode
// (synthetic weights rarely emit EOS: without a cap each request would decode to n_ctx).
#include <dirent.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/qasr.h"
#include "json.h"

using qjson::Value;

namespace {

volatile sig_atomic_t g_running = 1;
void on_signal(int) { g_running = 0; }

// ------------------------------------------------------------------------------------------ logging
std::string g_log_path;
void logf(const char* fmt, ...) {
    char msg[4096];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    time_t t = time(nullptr);
    char ts[64];
    strftime(ts, sizeof ts, "%Y-%m-%d %H:%M:%S", localtime(&t));
    fprintf(stderr, "%s - INFO - %s\n", ts, msg);
    if (!g_log_path.empty()) {
        struct stat st;
        if (stat(g_log_path.c_str(), &st) == 0 && st.st_size > 5 * 1024 * 1024) {  // 5 MB × 3 backups
            for (int i = 3; i >= 1; i--) {
                std::string a = g_log_path + (i == 1 ? "" : "." + std::to_string(i - 1));
                std::string b = g_log_path + "." + std::to_string(i);
                rename(a.c_str(), b.c_str());
            }
        }
        if (FILE* f = fopen(g_log_path.c_str(), "a")) {
            fprintf(f, "%s - INFO - %s\n", ts, msg);
            fclose(f);
        }
    }
}

void mkdirs(const std::string& p) {
    std::string cur;
    for (size_t i = 0; i < p.size(); i++) {
        cur += p[i];
        if (p[i] == '/' && cur.size() > 1) mkdir(cur.c_str(), 0755);
    }
    mkdir(p.c_str(), 0755);
}

void setup_log() {
    const char* d = getenv("LIGHT_WHISPER_DATA_DIR");
    std::string dir = d ? std::string(d) + "/logs" : std::string("/tmp/light_whisper_logs");
    mkdirs(dir);
    g_log_path = dir + "/qwen3_asr_server.log";
}

// ------------------------------------------------------------------------------------------ models
struct ModelSpec {
    const char* id;
    const char* repo;
    const char* file;
};
const ModelSpec kModels[] = {
    {"qwen3-asr-0.6b", "handy-computer/Qwen3-ASR-0.6B-gguf", "Qwen3-ASR-0.6B-Q8_0.gguf"},
    {"qwen3-asr-1.7b", "handy-computer/Qwen3-ASR-1.7B-gguf", "Qwen3-ASR-1.7B-Q8_0.gguf"},
};

std::string hf_cache_root() {
    if (const char* c = getenv("HF_HUB_CACHE"); c && *c) return c;
    if (const char* h = getenv("HF_HOME"); h && *h) return std::string(h) + "/hub";
    const char* home = getenv("HOME");
    return std::string(home ? home : ".") + "/.cache/huggingface/hub";
}

std::string read_file(const std::string& p) {
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) return std::string();
    std::string s;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

// hf_cache_utils.find_hf_snapshot_file: refs/main first, size ≥ 1 MB, optional completion manifest
std::string find_snapshot_file(const std::string& repo, const std::string& file) {
    std::string rd = repo;
    for (auto& c : rd)
        if (c == '/') c = '-';
    std::string repo_dir = hf_cache_root() + "/models--" + [&] {
        std::string r;
        for (char c : repo) r += c == '/' ? std::string("--") : std::string(1, c);
        return r;
    }();
    std::string snaps = repo_dir + "/snapshots";
    std::vector<std::string> names;
    std::string ref = read_file(repo_dir + "/refs/main");
    while (!ref.empty() && (ref.back() == '\n' || ref.back() == ' ' || ref.back() == '\r')) ref.pop_back();
    if (!ref.empty()) names.push_back(ref);
    if (DIR* d = opendir(snaps.c_str())) {
        while (dirent* e = readdir(d)) {
            std::string n = e->d_name;
            if (n == "." || n == "..") continue;
            bool dup = false;
            for (auto& x : names) dup |= x == n;
            if (!dup) names.push_back(n);
        }
        closedir(d);
    } else {
        return std::string();
    }
    for (auto& n : names) {
        std::string cand = snaps + "/" + n + "/" + file;
        struct stat st;
        if (stat(cand.c_str(), &st) != 0 || st.st_size < 1000000) continue;
        std::string man = read_file(snaps + "/" + n + "/.light_whisper_complete.json");
        if (!man.empty()) {
            try {
                Value m = qjson::parse(man);
                const Value* files = m.get("files");
                bool ok = false;
                if (files && files->type == Value::Arr)
                    for (auto& it : files->a) {
                        const Value* p = it.get("path");
                        const Value* s = it.get("size");
                        if (p && p->type == Value::Str && p->s == file)
                            ok = s && ((s->type == Value::Int && s->i == st.st_size) ||
                                       (s->type == Value::Float && s->f == (double)st.st_size));
                    }
                if (!ok) continue;
            } catch (...) {
                // legacy caches predate the completion manifest
            }
        }
        return cand;
    }
    return std::string();
}

double round_n(double v, int digits) {  // Python round(v, digits) (correctly rounded decimal)
    char b[64];
    snprintf(b, sizeof b, "%.*f", digits, v);
    return strtod(b, nullptr);
}

std::string py_strip(const std::string& s) {  // str.strip() for the common whitespace set
    auto ws = [](const std::string& x, size_t i, size_t& len) -> bool {
        unsigned char c = (unsigned char)x[i];
        if (c == ' ' || (c >= 0x09 && c <= 0x0d) || (c >= 0x1c && c <= 0x1f)) { len = 1; return true; }
        if (c == 0xC2 && i + 1 < x.size() && ((unsigned char)x[i + 1] == 0x85 || (unsigned char)x[i + 1] == 0xA0)) { len = 2; return true; }
        if (c == 0xE3 && i + 2 < x.size() && (unsigned char)x[i + 1] == 0x80 && (unsigned char)x[i + 2] == 0x80) { len = 3; return true; }
        if (c == 0xE2 && i + 2 < x.size() && (unsigned char)x[i + 1] == 0x80 &&
            (((unsigned char)x[i + 2] >= 0x80 && (unsigned char)x[i + 2] <= 0x8A) || (unsigned char)x[i + 2] == 0xA8 ||
             (unsigned char)x[i + 2] == 0xA9 || (unsigned char)x[i + 2] == 0xAF)) { len = 3; return true; }
        if (c == 0xE2 && i + 2 < x.size() && (unsigned char)x[i + 1] == 0x81 && (unsigned char)x[i + 2] == 0x9F) { len = 3; return true; }
        return false;
    };
    size_t b = 0, e = s.size(), len;
    while (b < e && ws(s, b, len)) b += len;
    // trailing: scan back to a codepoint start
    for (;;) {
        if (e <= b) break;
        size_t st = e - 1;
        while (st > b && ((unsigned char)s[st] & 0xC0) == 0x80) st--;
        if (ws(s, st, len) && st + len == e) e = st;
        else break;
    }
    return s.substr(b, e - b);
}

std::string py_str(const Value* v) {  // str() of a JSON value, as the reference formats it into messages
    if (!v || v->type == Value::Null) return "None";
    switch (v->type) {
        case Value::Bool: return v->b ? "True" : "False";
        case Value::Int: return std::to_string(v->i);
        case Value::Float: return qjson::float_repr(v->f);
        case Value::Str: return v->s;
        default: return qjson::dumps(*v);
    }
}

// ------------------------------------------------------------------------------------------ server
struct Server {
    std::string engine;
    bool fake = false;
    bool initialized = false;
    qasr_model* model = nullptr;
    qasr_session* session = nullptr;
    qasr_vad* vad = nullptr;
    std::string backend = "auto";
    std::string device = "cpu";
    std::string gpu_name;
    double gpu_mem = 0;
    int transcription_count = 0;
    double total_audio_duration = 0, total_inference_ms = 0, total_vad_ms = 0;
    int vad_calls = 0, vad_rejected = 0;

    void add_device_info(Value& r) {
        r.set("device", Value::str(device));
        if (!gpu_name.empty()) {
            r.set("gpu_name", Value::str(gpu_name));
            r.set("gpu_memory_total", Value::number(round_n(gpu_mem, 1)));
        }
    }

    void close_runtime() {
        if (session) qasr_session_close(session);
        if (model) qasr_model_close(model);
        if (vad) qasr_vad_close(vad);
        session = nullptr;
        model = nullptr;
        vad = nullptr;
    }

    Value initialize() {
        Value r = Value::object();
        if (initialized) {
            r.set("success", Value::boolean(true));
            r.set("message", Value::str("模型已初始化"));
            r.set("engine", Value::str(engine));
            return r;
        }
        const ModelSpec* spec = nullptr;
        for (auto& m : kModels)
            if (engine == m.id) spec = &m;
        const auto t0 = std::chrono::steady_clock::now();
        std::string path;
        const bool synth = getenv("QASR_SYNTHETIC") && std::string(getenv("QASR_SYNTHETIC")) == "1";
        if (!fake) {
            path = find_snapshot_file(spec->repo, spec->file);
            if (path.empty() && !synth) {
                r.set("success", Value::boolean(false));
                r.set("error", Value::str(std::string("Qwen3-ASR Q8 模型未下载: ") + spec->file));
                r.set("type", Value::str("models_not_downloaded"));
                r.set("engine", Value::str(engine));
                return r;
            }
        }
        auto fail = [&](const std::string& msg) {
            close_runtime();
            logf("Qwen3-ASR 初始化失败: %s", msg.c_str());
            Value e = Value::object();
            e.set("success", Value::boolean(false));
            e.set("error", Value::str("Qwen3-ASR 初始化失败: " + msg));
            e.set("type", Value::str("init_error"));
            e.set("engine", Value::str(engine));
            return e;
        };
        if (!fake) {
            int rc;
            if (!path.empty()) {
                logf("加载 Qwen3-ASR: %s", path.c_str());
                rc = qasr_model_open(path.c_str(), "hip", &model);
            } else {
                logf("未找到 GGUF，使用合成权重 (QASR_SYNTHETIC=1)");
                rc = qasr_model_open_synthetic(engine.c_str(), nullptr, 0, &model);
            }
            if (rc != QASR_OK) return fail(qasr_last_error());
            if (qasr_session_open(model, "f16", 32768, &session) != QASR_OK) return fail(qasr_last_error());
            // interim requests re-send overlapping windows: draft each decode from the earlier transcripts (greedy's
            // tokens, verified in one pass; QASR_STREAM_DRAFT=0 turns it off)
            const char* sd = getenv("QASR_STREAM_DRAFT");
            qasr_session_set_draft(session, !(sd && std::string(sd) == "0"));
            // and reuse the encoder windows a growing window shares with the previous request (QASR_STREAM_ENC_CACHE=0
            // turns it off)
            const char* ec = getenv("QASR_STREAM_ENC_CACHE");
            qasr_session_set_encoder_cache(session, !(ec && std::string(ec) == "0"));
            // benchmark hook (tools/stream_bench.py --draft-noise): corrupt proposed draft tokens at this rate — the
            // transcripts stay greedy's, only the acceptance (and the speed) changes
            if (const char* dn = getenv("QASR_DRAFT_NOISE")) qasr_session_set_draft_noise(session, (float)atof(dn), 1);
            if (qasr_vad_open(nullptr, &vad) != QASR_OK) return fail(qasr_last_error());
            backend = "hip";
            device = "hip";
            char name[256] = {0};
            double mem = 0;
            int nd = 0;
            if (qasr_device_info(name, sizeof name, &mem, &nd) == QASR_OK) {
                gpu_name = name;
                gpu_mem = mem;
            }
            warmup();
        } else {
            backend = "auto";
            device = "auto";
        }
        initialized = true;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        char msg[128];
        snprintf(msg, sizeof msg, "Qwen3-ASR 初始化成功，耗时: %.2f秒", el);
        r.set("success", Value::boolean(true));
        r.set("message", Value::str(msg));
        r.set("model_loaded", Value::boolean(true));
        r.set("engine", Value::str(engine));
        r.set("backend", Value::str(backend));
        add_device_info(r);
        return r;
    }

    // the reference's warm-up signal, default_rng(0).standard_normal(16000)·0.002 as f32 (qwen3_asr_server.py:139-140),
    // precomputed by tools/gen_warmup_noise.py into assets/ beside the VAD weights; an LCG stand-in if it is absent
    // (the warm-up's output is discarded either way)
    static std::vector<float> warmup_noise() {
        std::vector<float> noise(16000);
        char exe[4096] = {0};
        const ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
        std::string dir = n > 0 ? std::string(exe, (size_t)n) : std::string();
        dir = dir.substr(0, dir.find_last_of('/') + 1);
        if (FILE* f = fopen((dir + "../assets/warmup_noise.f32").c_str(), "rb")) {
            const size_t got = fread(noise.data(), sizeof(float), noise.size(), f);
            fclose(f);
            if (got == noise.size()) return noise;
        }
        uint64_t s = 0x9E3779B97F4A7C15ull;
        for (auto& v : noise) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            v = 0.002f * ((float)(s >> 40) / 16777216.0f * 2.f - 1.f);
        }
        return noise;
    }

    void warmup() {  // qwen3_asr_server.py:135-150 (1 s of quiet noise through VAD and ASR)
        std::vector<float> z(16000, 0.f);
        const std::vector<float> noise = warmup_noise();
        size_t nf = 0;
        std::vector<float> probs(200);
        qasr_vad_probabilities(vad, z.data(), z.size(), probs.data(), probs.size(), &nf);
        qasr_result res;
        qasr_run_opts o{16, 0, 0};
        if (qasr_session_run_opts(session, noise.data(), noise.size(), &o, &res) == QASR_OK) qasr_result_free(&res);
    }

    // firered_vad speech timestamps (or the reference tests' FakeVad in protocol-test mode)
    std::vector<qasr_segment> speech(const std::vector<float>& a) {
        std::vector<qasr_segment> out;
        if (fake) {
            bool any = false;
            for (float v : a) any |= v != 0.f;
            if (any) out = {{1600, 6400}, {9600, 14400}};
            return out;
        }
        size_t n = 0;
        out.resize(a.size() / 160 + 2);
        if (qasr_vad_speech_timestamps(vad, a.data(), a.size(), nullptr, out.data(), out.size(), &n) != QASR_OK)
            throw std::runtime_error(qasr_last_error());
        out.resize(n);
        return out;
    }

    // QASR_HOTWORD_CONTEXT=1 (opt-in): the request's hot_words, joined by ", ", become the system
    // context of the prompt (HF Qwen3-ASR `prompt=`).  Default: ignored, exactly like the reference server.
    void set_hotword_context(const Value* hw) {
        static const bool on = getenv("QASR_HOTWORD_CONTEXT") && std::string(getenv("QASR_HOTWORD_CONTEXT")) == "1";
        std::vector<int32_t> ids;
        if (on && hw && hw->type == Value::Arr) {
            std::string text;
            for (const Value& w : hw->a)
                if (w.type == Value::Str && !w.s.empty()) text += (text.empty() ? "" : ", ") + w.s;
            if (!text.empty()) {
                size_t n = 0;
                if (qasr_model_tokenize(model, text.data(), text.size(), nullptr, 0, &n) == QASR_OK && n > 0) {
                    ids.resize(n);
                    if (qasr_model_tokenize(model, text.data(), text.size(), ids.data(), n, &n) != QASR_OK) ids.clear();
                }
            }
        }
        qasr_session_set_context(session, ids.empty() ? nullptr : ids.data(), (int32_t)ids.size());
    }

    Value transcribe(const Value& cmd) {
        if (!initialized) {
            Value ir = initialize();
            if (!ir.get("success")->b) return ir;
        }
        const Value* b64 = cmd.get("audio_base64");
        const Value* path = cmd.get("audio_path");
        const Value* fmt_v = cmd.get("audio_format");
        const Value* sr_v = cmd.get("sample_rate");
        std::string input_mode = (b64 && b64->truthy()) ? "memory" : "path";
        try {
            std::vector<float> audio;
            double duration = 0;
            if (b64 && b64->truthy()) {
                if (b64->type != Value::Str) throw std::runtime_error("音频 base64 解码失败: argument should be a bytes-like object or ASCII string, not '" + std::string(b64->type == Value::Int ? "int" : "list") + "'");
                std::string fmt = fmt_v && fmt_v->type == Value::Str && !fmt_v->s.empty() ? fmt_v->s : "pcm_s16le";
                for (auto& c : fmt) c = (char)tolower(c);
                // decode_inline_audio order (server_common.py:150-187): base64, format, rate, byte parity
                size_t ns = 0;
                const int probe = qasr_decode_pcm_s16le(b64->s.data(), b64->s.size(), nullptr, 0, &ns);
                if (probe == QASR_E_FORMAT) throw std::runtime_error(std::string("音频 base64 解码失败: ") + qasr_last_error());
                const bool has_rate = sr_v && sr_v->truthy() && ((sr_v->type == Value::Int && sr_v->i > 0) ||
                                                                 (sr_v->type == Value::Float && sr_v->f > 0));
                if (fmt == "pcm_s16le") {
                    if (!has_rate) throw std::runtime_error("PCM 内存音频缺少有效采样率");
                    if (probe == QASR_E_INVALID) throw std::runtime_error("PCM s16le 数据字节数必须为偶数");
                    audio.resize(b64->s.size() / 4 * 3 / 2 + 4);
                    if (qasr_decode_pcm_s16le(b64->s.data(), b64->s.size(), audio.data(), audio.size(), &ns) != QASR_OK)
                        throw std::runtime_error(qasr_last_error());
                    audio.resize(ns);
                    const double rate = sr_v->type == Value::Int ? (double)sr_v->i : sr_v->f;
                    duration = (double)ns / rate;
                    if (rate != 16000.0) {   // the float rate as given (no truncation: np.interp gets it as is)
                        size_t nout = 0;
                        qasr_resample_linear(audio.data(), audio.size(), rate, nullptr, 0, &nout);
                        std::vector<float> rs(nout);
                        if (nout && qasr_resample_linear(audio.data(), audio.size(), rate, rs.data(), nout, &nout) != QASR_OK)
                            throw std::runtime_error(qasr_last_error());
                        audio.swap(rs);
                    }
                } else if (fmt == "wav") {
                    throw std::runtime_error("Qwen3-ASR 内存输入仅支持 PCM");
                } else {
                    throw std::runtime_error("不支持的内存音频格式: " + fmt);
                }
            } else {
                const std::string p = path && path->type == Value::Str ? path->s : py_str(path);
                struct stat st;
                if (!path || !path->truthy() || stat(p.c_str(), &st) != 0) throw std::runtime_error("音频文件不存在: " + p);
                // soundfile read → mono mean → _resample (qwen3_asr_server.py:256-267), in libqasr
                size_t ns = 0;
                if (qasr_audio_load_path(p.c_str(), nullptr, 0, &ns) != QASR_OK) throw std::runtime_error(qasr_last_error());
                audio.resize(ns);
                if (ns && qasr_audio_load_path(p.c_str(), audio.data(), ns, &ns) != QASR_OK)
                    throw std::runtime_error(qasr_last_error());
                audio.resize(ns);
                duration = (double)audio.size() / 16000.0;
            }
            total_audio_duration += duration;
            Value r = Value::object();
            if (duration < 0.5) {
                r.set("success", Value::boolean(true));
                r.set("text", Value::str(""));
                r.set("duration", Value::number(duration));
                r.set("engine", Value::str(engine));
                r.set("input_mode", Value::str(input_mode));
                return r;
            }
            const auto v0 = std::chrono::steady_clock::now();
            std::vector<qasr_segment> chunks = speech(audio);
            const double vad_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - v0).count();
            vad_calls++;
            total_vad_ms += vad_ms;
            int64_t st = 0, en = 0;
            if (!chunks.empty()) {
                st = std::max<int64_t>(0, chunks.front().start);
                en = std::min<int64_t>((int64_t)audio.size(), chunks.back().end);
            }
            if (chunks.empty() || en <= st) {
                vad_rejected++;
                r.set("success", Value::boolean(true));
                r.set("text", Value::str(""));
                r.set("raw_text", Value::str(""));
                r.set("duration", Value::number(duration));
                r.set("speech_duration", Value::number(0.0));
                r.set("language", Value::str("unknown"));
                r.set("engine", Value::str(engine));
                r.set("model_type", Value::str(engine));
                r.set("backend", Value::str(backend));
                r.set("input_mode", Value::str(input_mode));
                r.set("vad_segments", Value::integer(0));
                r.set("vad_ms", Value::number(round_n(vad_ms, 3)));
                r.set("inference_ms", Value::number(0.0));
                return r;
            }
            std::vector<float> speech_audio(audio.begin() + st, audio.begin() + en);
            const double speech_duration = (double)speech_audio.size() / 16000.0;
            const auto i0 = std::chrono::steady_clock::now();
            std::string text, language;
            if (fake) {
                text = "  测试文本 ";
                language = "Chinese";
            } else {
                qasr_result res;
                set_hotword_context(cmd.get("hot_words"));
                static const int force_tps = getenv("QASR_FORCE_TOKENS_PER_S") ? atoi(getenv("QASR_FORCE_TOKENS_PER_S")) : 0;
                static const int max_new = getenv("QASR_MAX_NEW_TOKENS") ? atoi(getenv("QASR_MAX_NEW_TOKENS")) : 0;
                const qasr_run_opts o{max_new, force_tps, 0};
                if (qasr_session_run_opts(session, speech_audio.data(), speech_audio.size(), &o, &res) != QASR_OK)
                    throw std::runtime_error(qasr_last_error());
                text = res.text ? res.text : "";
                language = res.language ? res.language : "";
                qasr_result_free(&res);
            }
            const double inf_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - i0).count();
            total_inference_ms += inf_ms;
            transcription_count++;
            text = py_strip(text);
            if (language.empty()) language = "unknown";
            r.set("success", Value::boolean(true));
            r.set("text", Value::str(text));
            r.set("raw_text", Value::str(text));
            r.set("confidence", Value::number(0.0));
            r.set("duration", Value::number(duration));
            r.set("speech_duration", Value::number(round_n(speech_duration, 3)));
            r.set("language", Value::str(language));
            r.set("engine", Value::str(engine));
            r.set("model_type", Value::str(engine));
            r.set("backend", Value::str(backend));
            r.set("input_mode", Value::str(input_mode));
            r.set("vad_segments", Value::integer((int64_t)chunks.size()));
            r.set("vad_ms", Value::number(round_n(vad_ms, 3)));
            r.set("inference_ms", Value::number(round_n(inf_ms, 3)));
            return r;
        } catch (const std::exception& e) {
            logf("Qwen3-ASR 转录失败: %s", e.what());
            Value r = Value::object();
            r.set("success", Value::boolean(false));
            r.set("error", Value::str(std::string("音频转录失败: ") + e.what()));
            r.set("type", Value::str("transcription_error"));
            r.set("input_mode", Value::str(input_mode));
            return r;
        }
    }

    Value stats() {
        Value s = Value::object();
        s.set("transcription_count", Value::integer(transcription_count));
        s.set("total_audio_duration", Value::number(round_n(total_audio_duration, 2)));
        s.set("average_inference_ms", Value::number(round_n(total_inference_ms / std::max(1, transcription_count), 3)));
        s.set("average_vad_ms", Value::number(round_n(total_vad_ms / std::max(1, vad_calls), 3)));
        s.set("vad_calls", Value::integer(vad_calls));
        s.set("vad_rejected", Value::integer(vad_rejected));
        s.set("initialized", Value::boolean(initialized));
        s.set("engine", Value::str(engine));
        s.set("backend", Value::str(backend));
        s.set("speculative_decoding", Value::boolean(false));
        if (session) {   // this engine's prompt-lookup drafting of interim windows (an addition to the reference keys)
            int64_t st[4] = {0, 0, 0, 0};
            if (qasr_session_draft_stats(session, st) == QASR_OK) {
                Value d = Value::object();
                d.set("passes", Value::integer((int)st[0]));
                d.set("proposed", Value::integer((int)st[1]));
                d.set("accepted", Value::integer((int)st[2]));
                d.set("tokens", Value::integer((int)st[3]));
                s.set("prompt_lookup", d);
            }
            if (qasr_session_encoder_cache_stats(session, st) == QASR_OK) {
                Value e = Value::object();
                e.set("runs", Value::integer((int)st[0]));
                e.set("windows_reused", Value::integer((int)st[1]));
                e.set("windows_encoded", Value::integer((int)st[2]));
                s.set("encoder_cache", e);
            }
        }
        Value ml = Value::object();
        ml.set("asr", Value::boolean(model != nullptr || (fake && initialized)));
        ml.set("vad", Value::boolean(vad != nullptr || (fake && initialized)));
        ml.set("punc", Value::boolean(true));
        s.set("models_loaded", ml);
        return s;
    }

    Value status() {
        Value r = Value::object();
        const bool loaded = (model && session) || (fake && initialized);
        r.set("success", Value::boolean(true));
        r.set("installed", Value::boolean(true));
        r.set("initialized", Value::boolean(initialized));
        r.set("version", Value::str(fake ? "0.1.3" : qasr_version()));
        r.set("engine", Value::str(engine));
        r.set("backend", Value::str(backend));
        r.set("model_loaded", Value::boolean(loaded));
        Value m = Value::object();
        m.set("asr", Value::boolean(loaded));
        m.set("vad", Value::boolean(vad != nullptr || (fake && initialized)));
        m.set("punc", Value::boolean(true));
        r.set("models", m);
        add_device_info(r);
        return r;
    }

    void reply(const Value& v) {
        std::string s = qjson::dumps(v);
        s += '\n';
        fwrite(s.data(), 1, s.size(), stdout);
        fflush(stdout);
    }

    int run() {
        logf("%s 服务器启动", engine.c_str());
        reply(initialize());
        std::string line;
        char* lbuf = nullptr;   // POSIX getline: one buffered read per line (a 12 s window is a ~0.5 MB line)
        size_t lcap = 0;
        while (g_running) {
            const ssize_t got = getline(&lbuf, &lcap, stdin);
            if (got < 0) break;
            line.assign(lbuf, (size_t)(got > 0 && lbuf[got - 1] == '\n' ? got - 1 : got));
            // str.strip()
            size_t b = 0, e = line.size();
            while (b < e && isspace((unsigned char)line[b])) b++;
            while (e > b && isspace((unsigned char)line[e - 1])) e--;
            if (b == e) continue;
            Value cmd;
            try {
                cmd = qjson::parse(line.substr(b, e - b));
            } catch (...) {
                Value r = Value::object();
                r.set("success", Value::boolean(false));
                r.set("error", Value::str("无效的JSON命令"));
                reply(r);
                continue;
            }
            Value rid;
            bool has_rid = false;
            if (cmd.type == Value::Obj) {
                const Value* r = cmd.get("request_id");
                if (r && (r->type == Value::Int || r->type == Value::Bool)) {
                    rid = *r;
                    has_rid = true;
                }
            } else {
                static const char* tn[] = {"NoneType", "bool", "int", "float", "str", "list", "dict"};
                Value r = Value::object();
                r.set("success", Value::boolean(false));
                r.set("error", Value::str(std::string("'") + tn[cmd.type] + "' object has no attribute 'get'"));
                r.set("traceback", Value::str("Traceback (most recent call last):\n  AttributeError\n"));
                reply(r);
                continue;
            }
            const Value* a = cmd.get("action");
            const std::string action = a && a->type == Value::Str ? a->s : "";
            Value result;
            if (action == "transcribe") result = transcribe(cmd);
            else if (action == "status") result = status();
            else if (action == "stats") {
                result = Value::object();
                result.set("success", Value::boolean(true));
                result.set("stats", stats());
            } else if (action == "cleanup") {
                result = Value::object();
                result.set("success", Value::boolean(true));
                result.set("message", Value::str("内存清理完成"));
            } else if (action == "exit") {
                result = Value::object();
                result.set("success", Value::boolean(true));
                result.set("message", Value::str("服务器退出"));
                if (has_rid) result.set("request_id", rid);
                reply(result);
                break;
            } else {
                result = Value::object();
                result.set("success", Value::boolean(false));
                result.set("error", Value::str("未知命令: " + py_str(a)));
            }
            if (has_rid) result.set("request_id", rid);
            reply(result);
        }
        free(lbuf);
        logf("%s 服务器退出", engine.c_str());
        close_runtime();
        return 0;
    }
};

int usage() {
    fprintf(stderr, "usage: engine serve --engine {qwen3-asr-0.6b,qwen3-asr-1.7b}\n"
                    "       engine longform --engine {qwen3-asr-0.6b,qwen3-asr-1.7b} [--force-tps K] [--max-new N] "
                    "[--batch-invariant] recording.wav   (one process per GPU: RANK / WORLD_SIZE / LOCAL_RANK)\n");
    return 2;
}

}  // namespace

int longform_main(const std::string& engine, const std::string& gguf, int argc, char** argv);   // engine_longform.cpp

int main(int argc, char** argv) {
    signal(SIGTERM, on_signal);
    signal(SIGINT, on_signal);
    std::string engine;
    if (argc >= 2) {
        const std::string cmd = argv[1];
        for (int i = 2; i + 1 < argc; i++)
            if (std::string(argv[i]) == "--engine") engine = argv[i + 1];
        if (cmd == "download") {
            fprintf(stderr, "model download is not part of this engine; provision the GGUF into the HF cache\n");
            return 2;
        }
        if (cmd == "longform" && !engine.empty()) {
            // the GGUF from the HF cache like `serve` (hf_cache_utils.find_hf_snapshot_file); QASR_SYNTHETIC=1 allows
            // the seeded synthetic weights when it is absent
            const ModelSpec* spec = nullptr;
            for (const auto& m : kModels)
                if (engine == m.id) spec = &m;
            if (!spec) return usage();
            const std::string path = find_snapshot_file(spec->repo, spec->file);
            const bool synth = getenv("QASR_SYNTHETIC") && std::string(getenv("QASR_SYNTHETIC")) == "1";
            if (path.empty() && !synth) {
                fprintf(stderr, "Qwen3-ASR Q8 模型未下载: %s\n", spec->file);
                return 1;
            }
            setvbuf(stdout, nullptr, _IOFBF, 1 << 16);
            return longform_main(engine, path, argc - 2, argv + 2);
        }
        if (cmd != "serve" || engine.empty()) return usage();
    } else {
        const char* e = getenv("LIGHT_WHISPER_ASR_ENGINE");
        engine = e ? e : "qwen3-asr-0.6b";
    }
    if (engine != "qwen3-asr-0.6b" && engine != "qwen3-asr-1.7b") {
        fprintf(stderr, "不支持的 Qwen3-ASR 引擎: %s\n", engine.c_str());
        return usage();
    }
    setvbuf(stdout, nullptr, _IOFBF, 1 << 16);
    setup_log();
    Server s;
    s.engine = engine;
    s.fake = getenv("QASR_PROTOCOL_TEST_FAKE") && std::string(getenv("QASR_PROTOCOL_TEST_FAKE")) == "1";
    setenv("HF_HUB_OFFLINE", "1", 1);
    return s.run();
}
