// Model construction: HBM layout, GGUF loading (tensor-name table validated by shape) and the on-device
// synthetic weight generator (same values as oracle/qasr_oracle.c orc_model_synth).
#include "model.h"

#include <math.h>
#include <string.h>

#include "gguf.h"
#include "kernels.h"
#include "kernels_audio.h"

namespace qasr {

void DevAlloc::reserve(size_t n) {
    QASR_CHECK(!base && !counting, QASR_E_INVALID, "weight arena reserved twice");
    QASR_HIP(hipMalloc((void**)&base, n));
    QASR_HIP(hipMemset(base, 0, n));   // padding bytes too: equal layouts hold equal images (broadcast checksum)
    cap = n;
}
void* DevAlloc::alloc(size_t n) {
    n = (n + 255) / 256 * 256;
    const size_t off = bytes;
    bytes += n;
    if (counting) return (void*)(uintptr_t)(off + 256);   // distinct non-null placeholders, never dereferenced
    QASR_CHECK(base && bytes <= cap, QASR_E_INVALID, "weight arena overflow");
    return base + off;
}
DevAlloc::~DevAlloc() {
    if (base) (void)hipFree(base);
}

static void set_special_defaults(qasr_hparams* hp) {
    hp->tok_im_start = 151644;
    hp->tok_im_end = 151645;
    hp->tok_system = 8948;
    hp->tok_user = 872;
    hp->tok_assistant = 77091;
    hp->tok_newline = 198;
    hp->tok_audio_start = 151669;
    hp->tok_audio_end = 151670;
    hp->tok_audio_pad = 151676;
    hp->tok_eos0 = 151645;
    hp->tok_eos1 = 151643;
    hp->tok_asr_text = 151704;
}

// Dimensions of the two pinned checkpoints (hf_cache_utils.py:11-26).
void default_hparams(const char* arch, qasr_hparams* hp) {
    memset(hp, 0, sizeof(*hp));
    const std::string a = arch ? arch : "qwen3-asr-1.7b";
    hp->n_mels = 128;
    hp->conv_ch = 480;
    hp->n_window = 50;
    hp->n_window_infer = 800;
    hp->txt_layers = 28;
    hp->txt_heads = 16;
    hp->txt_kv_heads = 8;
    hp->head_dim = 128;
    hp->vocab = 151936;
    hp->rope_theta = 1000000.0f;
    hp->rms_eps = 1e-6f;
    hp->ln_eps = 1e-5f;
    if (a == "qwen3-asr-0.6b") {
        hp->enc_d = 896; hp->enc_layers = 18; hp->enc_heads = 14; hp->enc_ffn = 3584;
        hp->txt_h = 1024; hp->txt_ffn = 3072;
    } else if (a == "qwen3-asr-1.7b") {
        hp->enc_d = 1024; hp->enc_layers = 24; hp->enc_heads = 16; hp->enc_ffn = 4096;
        hp->txt_h = 2048; hp->txt_ffn = 6144;
    } else {
        throw Error(QASR_E_INVALID, "unknown architecture: " + a);
    }
    hp->proj_out = hp->txt_h;
    set_special_defaults(hp);
}

static void validate(const qasr_hparams& h) {
    QASR_CHECK(h.n_mels == 128, QASR_E_FORMAT, "n_mels must be 128");
    QASR_CHECK(h.conv_ch > 0 && h.conv_ch % 32 == 0, QASR_E_FORMAT, "conv channels must be a multiple of 32");
    QASR_CHECK(h.enc_d % 64 == 0 && h.enc_heads > 0 && h.enc_d / h.enc_heads == 64, QASR_E_FORMAT,
               "encoder head_dim must be 64");
    QASR_CHECK(h.enc_ffn % 32 == 0 && h.txt_ffn % 32 == 0 && h.txt_h % 32 == 0, QASR_E_FORMAT, "dims % 32");
    QASR_CHECK(h.head_dim == 128, QASR_E_FORMAT, "decoder head_dim must be 128");
    QASR_CHECK(h.txt_kv_heads > 0 && h.txt_heads % h.txt_kv_heads == 0, QASR_E_FORMAT, "bad GQA head counts");
    QASR_CHECK(h.proj_out == h.txt_h, QASR_E_FORMAT, "projector output must equal the text hidden size");
    QASR_CHECK(h.n_window * 2 == 100 && h.n_window_infer % 100 == 0, QASR_E_FORMAT, "n_window must be 50");
    QASR_CHECK(h.enc_layers > 0 && h.txt_layers > 0 && h.vocab > 0, QASR_E_FORMAT, "empty model");
}

// ----------------------------------------------------------------------------------------------- layout
namespace {

Q8Mat alloc_q8(Model& m, int N, int K) {
    Q8Mat w;
    w.N = N;
    w.K = K;
    w.qs = (int8_t*)m.mem.alloc((size_t)N * K);
    w.sc = (__half*)m.mem.alloc((size_t)N * (K / QK) * sizeof(__half));
    return w;
}

void reg_q8(Model& m, const std::string& name, const Q8Mat& w, int64_t row0, int64_t rows) {
    TensorSlot s{};
    s.type = 8;
    s.base = w.qs;
    s.sc = w.sc;
    s.rows = rows;
    s.cols = w.K;
    s.row0 = row0;
    s.ld = w.K;
    m.slots[name] = s;
}

float* alloc_f32(Model& m, const std::string& name, int64_t n) {
    float* p = (float*)m.mem.alloc((size_t)n * sizeof(float));
    TensorSlot s{};
    s.type = 0;
    s.base = p;
    s.rows = n;
    s.cols = 1;
    m.slots[name] = s;
    return p;
}

__half* alloc_conv(Model& m, const std::string& name, int cout, int cin) {
    __half* p = (__half*)m.mem.alloc((size_t)cout * cin * 9 * sizeof(__half));
    TensorSlot s{};
    s.type = 1;
    s.base = p;
    s.rows = (int64_t)cout * cin * 9;
    s.cols = 1;
    s.conv_cin = cin;
    m.slots[name] = s;
    return p;
}

std::string nm(const char* fmt, int l) {
    char b[128];
    snprintf(b, sizeof b, fmt, l);
    return b;
}

void build_layout(Model& m) {
    const qasr_hparams& h = m.hp;
    const int C = h.conv_ch, d = h.enc_d, H = h.txt_h, F3 = m.audio_F3();
    const int QD = h.txt_heads * h.head_dim, KD = h.txt_kv_heads * h.head_dim;
    m.conv_w[0] = alloc_conv(m, "a.conv1.weight", C, 1);
    m.conv_w[1] = alloc_conv(m, "a.conv2.weight", C, C);
    m.conv_w[2] = alloc_conv(m, "a.conv3.weight", C, C);
    for (int i = 0; i < 3; i++) m.conv_b[i] = alloc_f32(m, nm("a.conv%d.bias", i + 1), C);
    m.conv_out = alloc_q8(m, d, C * F3);
    reg_q8(m, "a.conv_out.weight", m.conv_out, 0, d);
    m.enc.resize(h.enc_layers);
    for (int l = 0; l < h.enc_layers; l++) {
        EncLayer& e = m.enc[l];
        e.ln1_w = alloc_f32(m, nm("a.blk.%d.ln1.weight", l), d);
        e.ln1_b = alloc_f32(m, nm("a.blk.%d.ln1.bias", l), d);
        e.ln2_w = alloc_f32(m, nm("a.blk.%d.ln2.weight", l), d);
        e.ln2_b = alloc_f32(m, nm("a.blk.%d.ln2.bias", l), d);
        e.qkv = alloc_q8(m, 3 * d, d);
        reg_q8(m, nm("a.blk.%d.attn_q.weight", l), e.qkv, 0, d);
        reg_q8(m, nm("a.blk.%d.attn_k.weight", l), e.qkv, d, d);
        reg_q8(m, nm("a.blk.%d.attn_v.weight", l), e.qkv, 2 * d, d);
        e.qkv_b = (float*)m.mem.alloc((size_t)3 * d * sizeof(float));
        for (int j = 0; j < 3; j++) {
            TensorSlot s{};
            s.type = 0;
            s.base = e.qkv_b + j * d;
            s.rows = d;
            s.cols = 1;
            m.slots[nm(j == 0 ? "a.blk.%d.attn_q.bias" : j == 1 ? "a.blk.%d.attn_k.bias" : "a.blk.%d.attn_v.bias", l)] = s;
        }
        e.o = alloc_q8(m, d, d);
        reg_q8(m, nm("a.blk.%d.attn_out.weight", l), e.o, 0, d);
        e.o_b = alloc_f32(m, nm("a.blk.%d.attn_out.bias", l), d);
        e.up = alloc_q8(m, h.enc_ffn, d);
        reg_q8(m, nm("a.blk.%d.ffn_up.weight", l), e.up, 0, h.enc_ffn);
        e.up_b = alloc_f32(m, nm("a.blk.%d.ffn_up.bias", l), h.enc_ffn);
        e.down = alloc_q8(m, d, h.enc_ffn);
        reg_q8(m, nm("a.blk.%d.ffn_down.weight", l), e.down, 0, d);
        e.down_b = alloc_f32(m, nm("a.blk.%d.ffn_down.bias", l), d);
    }
    m.ln_post_w = alloc_f32(m, "a.ln_post.weight", d);
    m.ln_post_b = alloc_f32(m, "a.ln_post.bias", d);
    m.proj1 = alloc_q8(m, d, d);
    reg_q8(m, "a.proj1.weight", m.proj1, 0, d);
    m.proj1_b = alloc_f32(m, "a.proj1.bias", d);
    m.proj2 = alloc_q8(m, h.proj_out, d);
    reg_q8(m, "a.proj2.weight", m.proj2, 0, h.proj_out);
    m.proj2_b = alloc_f32(m, "a.proj2.bias", h.proj_out);
    m.tok_embd = alloc_q8(m, h.vocab, H);
    reg_q8(m, "token_embd.weight", m.tok_embd, 0, h.vocab);
    m.lm_head = m.tok_embd;  // tied (tie_word_embeddings); an "output.weight" in the GGUF replaces it
    m.out_norm = alloc_f32(m, "output_norm.weight", H);
    m.dec.resize(h.txt_layers);
    for (int l = 0; l < h.txt_layers; l++) {
        DecLayer& L = m.dec[l];
        L.attn_norm = alloc_f32(m, nm("blk.%d.attn_norm.weight", l), H);
        L.ffn_norm = alloc_f32(m, nm("blk.%d.ffn_norm.weight", l), H);
        L.q_norm = alloc_f32(m, nm("blk.%d.attn_q_norm.weight", l), h.head_dim);
        L.k_norm = alloc_f32(m, nm("blk.%d.attn_k_norm.weight", l), h.head_dim);
        L.qkv = alloc_q8(m, QD + 2 * KD, H);
        reg_q8(m, nm("blk.%d.attn_q.weight", l), L.qkv, 0, QD);
        reg_q8(m, nm("blk.%d.attn_k.weight", l), L.qkv, QD, KD);
        reg_q8(m, nm("blk.%d.attn_v.weight", l), L.qkv, QD + KD, KD);
        L.o = alloc_q8(m, H, QD);
        reg_q8(m, nm("blk.%d.attn_output.weight", l), L.o, 0, H);
        L.gu = alloc_q8(m, 2 * h.txt_ffn, H);
        reg_q8(m, nm("blk.%d.ffn_gate.weight", l), L.gu, 0, h.txt_ffn);
        reg_q8(m, nm("blk.%d.ffn_up.weight", l), L.gu, h.txt_ffn, h.txt_ffn);
        L.down = alloc_q8(m, H, h.txt_ffn);
        reg_q8(m, nm("blk.%d.ffn_down.weight", l), L.down, 0, H);
    }
}

constexpr size_t DFT_BASIS_FLOATS = (size_t)400 * 402;

// the whole device layout: weights, the untied vocabulary projection when the checkpoint has one, and the
// fixed tables — the probe pass (mem.counting) sizes the arena, the second pass carves it
void layout_all(Model& m, bool untied) {
    build_layout(m);
    if (untied) {
        m.lm_head = alloc_q8(m, m.hp.vocab, m.hp.txt_h);
        reg_q8(m, "output.weight", m.lm_head, 0, m.hp.vocab);
    }
    m.pos_emb = (float*)m.mem.alloc((size_t)13 * m.hp.enc_d * sizeof(float));
    m.mel_filters = (float*)m.mem.alloc((size_t)201 * m.hp.n_mels * sizeof(float));
    m.dft_basis = (float*)m.mem.alloc(DFT_BASIS_FLOATS * sizeof(float));
}

void make_layout(Model& m, bool untied) {
    Model probe;
    probe.hp = m.hp;
    probe.mem.counting = true;
    layout_all(probe, untied);
    m.mem.reserve(probe.mem.bytes);
    layout_all(m, untied);
    QASR_CHECK(m.mem.bytes == probe.mem.bytes, QASR_E_INVALID, "layout probe mismatch");
}

// fixed tables: sinusoid position embedding (SinusoidsPositionEmbedding, modeling_qwen3_asr.py:245-263),
// Slaney mel filters (feature_extraction_qwen3_asr.py:94-102) and the windowed DFT basis of the STFT
void build_tables(Model& m, hipStream_t s) {
    const int d = m.hp.enc_d, nmel = m.hp.n_mels;
    std::vector<float> pe((size_t)13 * d);
    const float inc = logf(10000.f) / (float)(d / 2 - 1);
    for (int t = 0; t < 13; t++)
        for (int i = 0; i < d / 2; i++) {
            float st = (float)t * expf(-inc * (float)i);
            pe[(size_t)t * d + i] = sinf(st);
            pe[(size_t)t * d + d / 2 + i] = cosf(st);
        }
    QASR_HIP(hipMemcpyAsync(m.pos_emb, pe.data(), pe.size() * sizeof(float), hipMemcpyHostToDevice, s));
    std::vector<float> filt((size_t)201 * nmel), basis;
    mel_filter_table(nmel, filt.data());
    QASR_HIP(hipMemcpyAsync(m.mel_filters, filt.data(), filt.size() * sizeof(float), hipMemcpyHostToDevice, s));
    dft_basis_table(basis);
    QASR_CHECK(basis.size() == DFT_BASIS_FLOATS, QASR_E_INVALID, "DFT basis size");
    QASR_HIP(hipMemcpyAsync(m.dft_basis, basis.data(), basis.size() * sizeof(float), hipMemcpyHostToDevice, s));
    QASR_HIP(hipStreamSynchronize(s));
}

void make_tokenizer_synthetic(Model& m) {
    const qasr_hparams& h = m.hp;
    const int32_t ids[] = {h.tok_im_start, h.tok_im_end, h.tok_audio_start, h.tok_audio_end, h.tok_audio_pad,
                           h.tok_eos1, h.tok_asr_text};
    const char* txt[] = {"<|im_start|>", "<|im_end|>", "<|audio_start|>", "<|audio_end|>", "<|audio_pad|>",
                         "<|endoftext|>", "<asr_text>"};
    m.tok.make_synthetic(h.vocab, ids, txt, 7);
}

}  // namespace

// ----------------------------------------------------------------------------------------------- synthetic
// The per-tensor (sigma | center, scale) table mirrors orc_model_synth in oracle/qasr_oracle.c.
// device layouts the kernels want, applied once after load: decoder gate|up rows interleaved by 16 so the
// gate-up GEMM epilogue computes SwiGLU and its Q8 blocks in registers (kernels_q8.hip EPI_SWIGLU)
// (a shell receives the blob already interleaved: it only records the slot layout)
void finalize_layout(Model& m, hipStream_t s, bool data = true) {
    for (int l = 0; l < m.hp.txt_layers; l++) {
        if (data) interleave_gate_up(m.dec[l].gu, s);
        for (const char* n : {"blk.%d.ffn_gate.weight", "blk.%d.ffn_up.weight"}) m.slots.at(nm(n, l)).il16_F = m.hp.txt_ffn;
    }
}

std::unique_ptr<Model> make_synthetic_model(const qasr_hparams& hp, uint64_t seed, const std::string& arch) {
    validate(hp);
    auto mp = std::make_unique<Model>();
    Model& m = *mp;
    m.hp = hp;
    m.arch = arch;
    make_layout(m, false);
    hipStream_t s = nullptr;
    const int C = hp.conv_ch, d = hp.enc_d, H = hp.txt_h, F3 = m.audio_F3();
    const int QD = hp.txt_heads * hp.head_dim;
    auto base = [&](const std::string& name) { return smix(seed ^ fnv1a(name.c_str())); };
    auto q8 = [&](const std::string& name, float sigma) {
        const TensorSlot& t = m.slots.at(name);
        synth_q8(base(name), t.rows * (t.cols / QK), sigma / 73.6f, (int8_t*)t.base + t.row0 * t.ld,
                 t.sc + t.row0 * (t.ld / QK), s, name == "token_embd.weight" ? t.cols / QK : 0);
    };
    auto f32 = [&](const std::string& name, float center, float scale) {
        const TensorSlot& t = m.slots.at(name);
        synth_f32(base(name), t.rows, center, scale, (float*)t.base, s);
    };
    auto conv = [&](const std::string& name, float scale) {
        const TensorSlot& t = m.slots.at(name);
        __half* tmp = nullptr;
        QASR_HIP(hipMalloc(&tmp, (size_t)t.rows * sizeof(__half)));
        synth_f16(base(name), t.rows, scale, tmp, s);
        reorder_conv_weight(tmp, C, t.conv_cin, (__half*)t.base, s);
        QASR_HIP(hipStreamSynchronize(s));
        QASR_HIP(hipFree(tmp));
    };
    conv("a.conv1.weight", 1.0f / 3.0f * 1.7320508f);
    conv("a.conv2.weight", 1.7320508f / sqrtf((float)C * 9));
    conv("a.conv3.weight", 1.7320508f / sqrtf((float)C * 9));
    for (int i = 1; i <= 3; i++) f32(nm("a.conv%d.bias", i), 0.f, 0.05f);
    q8("a.conv_out.weight", 1.0f / sqrtf((float)C * F3));
    for (int l = 0; l < hp.enc_layers; l++) {
        f32(nm("a.blk.%d.ln1.weight", l), 1.f, 0.1f);
        f32(nm("a.blk.%d.ln1.bias", l), 0.f, 0.05f);
        f32(nm("a.blk.%d.ln2.weight", l), 1.f, 0.1f);
        f32(nm("a.blk.%d.ln2.bias", l), 0.f, 0.05f);
        const char* lin[6] = {"attn_q", "attn_k", "attn_v", "attn_out", "ffn_up", "ffn_down"};
        const int KK[6] = {d, d, d, d, d, hp.enc_ffn};
        for (int i = 0; i < 6; i++) {
            char b[128];
            snprintf(b, sizeof b, "a.blk.%d.%s.weight", l, lin[i]);
            q8(b, 0.5f / sqrtf((float)KK[i]));
            snprintf(b, sizeof b, "a.blk.%d.%s.bias", l, lin[i]);
            f32(b, 0.f, 0.02f);
        }
    }
    f32("a.ln_post.weight", 1.f, 0.1f);
    f32("a.ln_post.bias", 0.f, 0.05f);
    q8("a.proj1.weight", 1.0f / sqrtf((float)d));
    f32("a.proj1.bias", 0.f, 0.02f);
    q8("a.proj2.weight", 1.0f / sqrtf((float)d));
    f32("a.proj2.bias", 0.f, 0.02f);
    q8("token_embd.weight", 1.0f);
    f32("output_norm.weight", 1.f, 0.1f);
    for (int l = 0; l < hp.txt_layers; l++) {
        f32(nm("blk.%d.attn_norm.weight", l), 1.f, 0.1f);
        f32(nm("blk.%d.ffn_norm.weight", l), 1.f, 0.1f);
        f32(nm("blk.%d.attn_q_norm.weight", l), 1.f, 0.1f);
        f32(nm("blk.%d.attn_k_norm.weight", l), 1.f, 0.1f);
        q8(nm("blk.%d.attn_q.weight", l), 1.0f / sqrtf((float)H));
        q8(nm("blk.%d.attn_k.weight", l), 1.0f / sqrtf((float)H));
        q8(nm("blk.%d.attn_v.weight", l), 1.0f / sqrtf((float)H));
        q8(nm("blk.%d.attn_output.weight", l), 0.5f / sqrtf((float)QD));
        q8(nm("blk.%d.ffn_gate.weight", l), 1.0f / sqrtf((float)H));
        q8(nm("blk.%d.ffn_up.weight", l), 1.0f / sqrtf((float)H));
        q8(nm("blk.%d.ffn_down.weight", l), 0.5f / sqrtf((float)hp.txt_ffn));
    }
    QASR_HIP(hipGetLastError());
    finalize_layout(m, s);
    build_tables(m, s);
    make_tokenizer_synthetic(m);
    return mp;
}

std::unique_ptr<Model> make_synthetic_shell(const qasr_hparams& hp, const std::string& arch) {
    validate(hp);
    auto mp = std::make_unique<Model>();
    Model& m = *mp;
    m.hp = hp;
    m.arch = arch;
    make_layout(m, false);
    finalize_layout(m, nullptr, false);
    build_tables(m, nullptr);
    make_tokenizer_synthetic(m);
    m.weights_pending = true;
    return mp;
}

// ----------------------------------------------------------------------------------------------- GGUF
// The pinned checkpoints (Qwen3-ASR-{0.6B,1.7B}-Q8_0.gguf, hf_cache_utils.py:11-26, opened by transcribe_cpp.Model at
// qwen3_asr_server.py:122) are not in this container, so their tensor names and metadata keys are unknown.  The
// loader therefore resolves every logical tensor through a table of candidate names — this engine's exporter
// (llama.cpp-style text names, "a." audio prefix), the original qwen_asr / HF state-dict names ("thinker.audio_tower.*",
// "thinker.model.*", "model.language_model.*", "model.multi_modal_projector.linear_{1,2}") and llama.cpp mtmd-style
// audio names — validates each one's shape, derives every hyper-parameter a shape determines from the shapes, and fails
// loudly (QASR_E_FORMAT, the server's init_error) on a tensor it cannot map, a tensor it needs but cannot find, a
// shape or type it does not support, and missing required metadata (RoPE base, RMSNorm epsilon).
namespace {

bool starts(const std::string& s, const char* p) { return s.compare(0, strlen(p), p) == 0; }

std::vector<std::string> name_candidates(const std::string& canon) {
    std::vector<std::string> out = {canon};
    static const char* AP[] = {"thinker.audio_tower.", "model.audio_tower.", "audio_tower.", "audio."};
    static const char* TP[] = {"thinker.model.", "model.language_model.", "language_model.model.", "model.",
                               "language_model."};
    auto audio = [&](const std::string& tail) {
        for (const char* p : AP) out.push_back(p + tail);
    };
    auto text = [&](const std::string& tail) {
        for (const char* p : TP) out.push_back(p + tail);
    };
    const size_t dot = canon.rfind('.');
    const std::string leaf = canon.substr(dot + 1);   // weight / bias
    int l = -1, i = -1;
    char part[64] = {0};
    if (sscanf(canon.c_str(), "a.conv%d.%*s", &i) == 1 && canon.compare(0, 7, "a.conv_") != 0) {
        audio("conv2d" + std::to_string(i) + "." + leaf);
        out.push_back("a.conv2d." + std::to_string(i) + "." + leaf);
    } else if (canon == "a.conv_out.weight") {
        audio("conv_out.weight");
        out.push_back("a.conv_out.weight");
    } else if (sscanf(canon.c_str(), "a.blk.%d.%63[^.]", &l, part) == 2) {
        const std::string p = part, L = "layers." + std::to_string(l) + ".";
        static const std::pair<const char*, const char*> m[] = {
            {"ln1", "self_attn_layer_norm"}, {"ln2", "final_layer_norm"}, {"attn_q", "self_attn.q_proj"},
            {"attn_k", "self_attn.k_proj"}, {"attn_v", "self_attn.v_proj"}, {"attn_out", "self_attn.out_proj"},
            {"ffn_up", "fc1"}, {"ffn_down", "fc2"}};
        for (auto& kv : m)
            if (p == kv.first) audio(L + kv.second + "." + leaf);
        if (p == "attn_out") out.push_back("a.blk." + std::to_string(l) + ".attn_output." + leaf);
    } else if (starts(canon, "a.ln_post.")) {
        audio("ln_post." + leaf);
        out.push_back("a.post_ln." + leaf);
    } else if (starts(canon, "a.proj1.") || starts(canon, "a.proj2.")) {
        const char k = canon[6];
        audio(std::string("proj") + k + "." + leaf);
        out.push_back(std::string("model.multi_modal_projector.linear_") + k + "." + leaf);
        out.push_back(std::string("multi_modal_projector.linear_") + k + "." + leaf);
        out.push_back(std::string("mm.a.mlp.") + k + "." + leaf);
    } else if (canon == "token_embd.weight") {
        text("embed_tokens.weight");
    } else if (canon == "output_norm.weight") {
        text("norm.weight");
    } else if (canon == "output.weight") {
        out.push_back("thinker.lm_head.weight");
        out.push_back("lm_head.weight");
    } else if (sscanf(canon.c_str(), "blk.%d.%63[^.]", &l, part) == 2) {
        const std::string p = part, L = "layers." + std::to_string(l) + ".";
        static const std::pair<const char*, const char*> m[] = {
            {"attn_norm", "input_layernorm"}, {"ffn_norm", "post_attention_layernorm"},
            {"attn_q_norm", "self_attn.q_norm"}, {"attn_k_norm", "self_attn.k_norm"}, {"attn_q", "self_attn.q_proj"},
            {"attn_k", "self_attn.k_proj"}, {"attn_v", "self_attn.v_proj"}, {"attn_output", "self_attn.o_proj"},
            {"ffn_gate", "mlp.gate_proj"}, {"ffn_up", "mlp.up_proj"}, {"ffn_down", "mlp.down_proj"}};
        for (auto& kv : m)
            if (p == kv.first) text(L + kv.second + "." + leaf);
    }
    return out;
}

// Tensors a checkpoint may carry that the engine recomputes (the encoder's sinusoid position table, modeling_
// qwen3_asr.py:245-263, a non-persistent buffer some exporters still write; llama.cpp's RoPE frequency table)
bool ignorable_tensor(const std::string& n) {
    return n.find("positional_embedding") != std::string::npos || n == "rope_freqs.weight" ||
           n.find("rotary_emb.inv_freq") != std::string::npos;
}

struct GgufResolver {
    const GgufFile& f;
    std::map<std::string, std::string> used;   // file name → logical name
    explicit GgufResolver(const GgufFile& g) : f(g) {}
    const GgufTensor* find(const std::string& canon) {
        for (const std::string& c : name_candidates(canon))
            if (const GgufTensor* t = f.tensor(c)) {
                auto it = used.find(c);
                QASR_CHECK(it == used.end() || it->second == canon, QASR_E_FORMAT,
                           "GGUF tensor " + c + " maps to both " + it->second + " and " + canon);
                used[c] = canon;
                return t;
            }
        return nullptr;
    }
    const GgufTensor* need(const std::string& canon) {
        const GgufTensor* t = find(canon);
        QASR_CHECK(t, QASR_E_FORMAT, "GGUF is missing tensor " + canon + " (looked for: " + join(name_candidates(canon)) + ")");
        return t;
    }
    static std::string join(const std::vector<std::string>& v) {
        std::string s;
        for (auto& x : v) s += (s.empty() ? "" : ", ") + x;
        return s;
    }
    int count_layers(const char* fmt) {
        int n = 0;
        while (find(nm(fmt, n))) n++;
        return n;
    }
};

int64_t nelem(const GgufTensor* t) {
    int64_t n = 1;
    for (auto d : t->dims) n *= d;
    return n;
}

// metadata value by exact key (any of `keys`) or by unique suffix; nullptr when absent
const GgufValue* meta(const GgufFile& f, std::initializer_list<const char*> keys, std::initializer_list<const char*> suffixes) {
    for (const char* k : keys)
        if (const GgufValue* v = f.get(k)) return v;
    const GgufValue* hit = nullptr;
    std::string hit_key;
    for (const auto& kv : f.metadata())
        for (const char* sfx : suffixes) {
            const size_t n = strlen(sfx);
            if (kv.first.size() >= n && kv.first.compare(kv.first.size() - n, n, sfx) == 0) {
                QASR_CHECK(!hit || hit_key == kv.first, QASR_E_FORMAT,
                           "GGUF metadata is ambiguous: " + hit_key + " and " + kv.first);
                hit = &kv.second, hit_key = kv.first;
            }
        }
    return hit;
}
bool numeric(const GgufValue* v) { return v && v->type != 8 && v->type != 9; }

}  // namespace

std::unique_ptr<Model> load_gguf_model(const std::string& path, bool shell) {
    GgufFile f(path);
    GgufResolver R(f);
    const std::string A = f.get_str("general.architecture", "qwen3-asr");
    qasr_hparams hp;
    memset(&hp, 0, sizeof hp);
    // ---- hyper-parameters from the tensor shapes (GGUF dims: ne0 = row length K, ne1 = rows N)
    const GgufTensor* conv1 = R.need("a.conv1.weight");
    hp.conv_ch = (int)(nelem(conv1) / 9);
    const GgufTensor* co = R.need("a.conv_out.weight");
    QASR_CHECK(co->dims.size() == 2, QASR_E_FORMAT, "conv_out weight must be 2-D");
    hp.enc_d = (int)co->dims[1];
    const int F3 = (int)(co->dims[0] / std::max(1, hp.conv_ch));
    hp.enc_layers = R.count_layers("a.blk.%d.attn_q.weight");
    hp.enc_ffn = (int)R.need("a.blk.0.ffn_up.weight")->dims[1];
    hp.proj_out = (int)R.need("a.proj2.weight")->dims[1];
    const GgufTensor* te = R.need("token_embd.weight");
    QASR_CHECK(te->dims.size() == 2, QASR_E_FORMAT, "token embedding must be 2-D");
    hp.txt_h = (int)te->dims[0];
    hp.vocab = (int)te->dims[1];
    hp.txt_layers = R.count_layers("blk.%d.attn_q.weight");
    hp.head_dim = (int)nelem(R.need("blk.0.attn_q_norm.weight"));
    hp.txt_heads = (int)(R.need("blk.0.attn_q.weight")->dims[1] / std::max(1, hp.head_dim));
    hp.txt_kv_heads = (int)(R.need("blk.0.attn_k.weight")->dims[1] / std::max(1, hp.head_dim));
    hp.txt_ffn = (int)R.need("blk.0.ffn_gate.weight")->dims[1];
    // ---- scalars no shape determines
    std::string assumed;
    auto get_i = [&](const char* what, std::initializer_list<const char*> keys, std::initializer_list<const char*> sfx,
                     int arch_value) {
        const GgufValue* v = meta(f, keys, sfx);
        if (numeric(v)) return (int)v->i;
        assumed += std::string(assumed.empty() ? "" : ", ") + what + "=" + std::to_string(arch_value);
        return arch_value;
    };
    auto need_f = [&](const char* what, std::initializer_list<const char*> keys, std::initializer_list<const char*> sfx) {
        const GgufValue* v = meta(f, keys, sfx);
        QASR_CHECK(numeric(v), QASR_E_FORMAT, std::string("GGUF metadata is missing ") + what);
        return (float)v->f;
    };
    // the Qwen3-ASR audio encoder's fixed architecture (configuration_qwen3_asr.py: head_dim 64, n_window 50,
    // n_window_infer 800, nn.LayerNorm eps 1e-5, 128 mel bins ⇔ 16 conv_out frequency rows) when the file is silent
    hp.n_mels = get_i("n_mels", {}, {"audio.n_mels", "audio.num_mel_bins", "num_mel_bins"}, F3 == 16 ? 128 : 0);
    hp.enc_heads = get_i("enc_heads", {}, {"audio.attention.head_count", "audio.encoder_attention_heads",
                                           "encoder_attention_heads"}, hp.enc_d / 64);
    hp.n_window = get_i("n_window", {}, {"audio.n_window", ".n_window"}, 50);
    hp.n_window_infer = get_i("n_window_infer", {}, {"audio.n_window_infer", ".n_window_infer"}, 800);
    hp.rope_theta = need_f("the RoPE base (*.rope.freq_base)", {}, {".rope.freq_base", ".rope_theta"});
    hp.rms_eps = need_f("the RMSNorm epsilon (*.attention.layer_norm_rms_epsilon)", {},
                        {".attention.layer_norm_rms_epsilon", ".rms_norm_eps"});
    {
        const GgufValue* v = meta(f, {}, {"audio.attention.layer_norm_epsilon", "audio.layer_norm_epsilon"});
        if (numeric(v)) hp.ln_eps = (float)v->f;
        else hp.ln_eps = 1e-5f, assumed += std::string(assumed.empty() ? "" : ", ") + "ln_eps=1e-5";
    }
    if (!assumed.empty())
        fprintf(stderr, "qasr: %s: architecture values assumed (no metadata key): %s\n", path.c_str(), assumed.c_str());
    QASR_CHECK(F3 * hp.conv_ch == co->dims[0] && (((hp.n_mels + 1) / 2 + 1) / 2 + 1) / 2 == F3, QASR_E_FORMAT,
               "conv_out input width does not match the conv stack");
    // ---- special tokens: metadata ids, else the canonical pieces of the Qwen2 vocabulary
    const GgufValue* toks = f.get("tokenizer.ggml.tokens");
    QASR_CHECK(toks && toks->arr_type == 8 && (int)toks->arr_s.size() >= hp.vocab, QASR_E_FORMAT,
               "GGUF has no tokenizer vocabulary (tokenizer.ggml.tokens) covering the embedding rows");
    std::map<std::string, int> piece_id;
    for (int id = (int)toks->arr_s.size() - 1; id >= 0; id--) piece_id[toks->arr_s[id]] = id;   // lowest id wins
    auto tok = [&](const char* key, const char* piece) {
        const GgufValue* v = meta(f, {(A + ".token." + key).c_str()}, {});
        if (numeric(v)) return (int)v->i;
        auto it = piece_id.find(piece);
        QASR_CHECK(it != piece_id.end(), QASR_E_FORMAT,
                   std::string("GGUF vocabulary has no ") + piece + " token (nor metadata " + A + ".token." + key + ")");
        return it->second;
    };
    hp.tok_im_start = tok("im_start", "<|im_start|>");
    hp.tok_im_end = tok("im_end", "<|im_end|>");
    hp.tok_system = tok("system", "system");
    hp.tok_user = tok("user", "user");
    hp.tok_assistant = tok("assistant", "assistant");
    hp.tok_newline = tok("newline", "\xC4\x8A");   // "Ċ": the byte-level piece of "\n"
    hp.tok_audio_start = tok("audio_start", "<|audio_start|>");
    hp.tok_audio_end = tok("audio_end", "<|audio_end|>");
    hp.tok_audio_pad = tok("audio_pad", "<|audio_pad|>");
    hp.tok_eos0 = tok("eos0", "<|im_end|>");
    hp.tok_eos1 = tok("eos1", "<|endoftext|>");
    hp.tok_asr_text = tok("asr_text", "<asr_text>");
    validate(hp);

    auto mp = std::make_unique<Model>();
    Model& m = *mp;
    m.hp = hp;
    m.arch = f.get_str("general.name", "qwen3-asr");
    const GgufTensor* out = R.find("output.weight");   // untied checkpoints carry their own vocabulary projection
    make_layout(m, out != nullptr);
    // ---- every slot: resolve, check type and shape, upload
    hipStream_t s = nullptr;
    uint8_t* staging = nullptr;
    size_t staging_cap = 0;
    for (auto& kv : m.slots) {
        const std::string& name = kv.first;
        const TensorSlot& t = kv.second;
        const GgufTensor* g = R.need(name);
        if (t.type == 8) {
            QASR_CHECK(g->type == GGML_Q8_0, QASR_E_FORMAT,
                       name + ": linear stored as ggml type " + std::to_string(g->type) + "; only Q8_0 linears are supported");
            QASR_CHECK(g->dims.size() == 2 && g->dims[0] == t.cols && g->dims[1] == t.rows, QASR_E_FORMAT,
                       name + ": shape mismatch");
        } else if (t.type == 0) {
            QASR_CHECK((g->type == GGML_F32 || g->type == GGML_F16) && nelem(g) == t.rows, QASR_E_FORMAT,
                       name + ": expected an f32 / f16 vector of " + std::to_string(t.rows));
        } else {
            QASR_CHECK(g->type == GGML_F16 && nelem(g) == t.rows, QASR_E_FORMAT, name + ": expected an f16 conv kernel");
        }
        if (shell) continue;
        if (t.type == 8) {
            if (g->nbytes > staging_cap) {
                if (staging) QASR_HIP(hipFree(staging));
                staging_cap = g->nbytes;
                QASR_HIP(hipMalloc(&staging, staging_cap));
            }
            QASR_HIP(hipMemcpy(staging, g->data, g->nbytes, hipMemcpyHostToDevice));
            repack_q8(staging, t.rows * (t.cols / QK), (int8_t*)t.base + t.row0 * t.ld, t.sc + t.row0 * (t.ld / QK), s);
            QASR_HIP(hipStreamSynchronize(s));
        } else if (t.type == 0) {
            std::vector<float> v((size_t)t.rows);
            if (g->type == GGML_F32) memcpy(v.data(), g->data, v.size() * 4);
            else
                for (size_t i = 0; i < v.size(); i++) v[i] = __half2float(((const __half*)g->data)[i]);   // exact
            QASR_HIP(hipMemcpy(t.base, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        } else {
            __half* tmp = nullptr;
            QASR_HIP(hipMalloc(&tmp, g->nbytes));
            QASR_HIP(hipMemcpy(tmp, g->data, g->nbytes, hipMemcpyHostToDevice));
            reorder_conv_weight(tmp, hp.conv_ch, t.conv_cin, (__half*)t.base, s);
            QASR_HIP(hipStreamSynchronize(s));
            QASR_HIP(hipFree(tmp));
        }
    }
    if (staging) QASR_HIP(hipFree(staging));
    for (const auto& kv : f.tensors())
        QASR_CHECK(R.used.count(kv.first) || ignorable_tensor(kv.first), QASR_E_FORMAT,
                   "GGUF tensor " + kv.first + " is not mapped to any Qwen3-ASR tensor");
    finalize_layout(m, s, !shell);
    build_tables(m, s);
    m.weights_pending = shell;
    m.tok.pieces = toks->arr_s;
    // byte-level BPE merges ("a b", by rank) for hot-word context encoding (tokenizer.cpp Tokenizer::encode)
    if (const GgufValue* mg = f.get("tokenizer.ggml.merges"))
        if (mg->arr_type == 8) m.tok.merges = mg->arr_s;
    m.tok.is_special.assign(m.tok.pieces.size(), 0);
    if (const GgufValue* tt = f.get("tokenizer.ggml.token_type"))
        for (size_t i = 0; i < tt->arr_i.size() && i < m.tok.is_special.size(); i++)
            m.tok.is_special[i] = tt->arr_i[i] == 3 || tt->arr_i[i] == 4;  // CONTROL / USER_DEFINED
    return mp;
}

// ----------------------------------------------------------------------------------------------- precision
namespace {
template <typename F>
void for_each_gemm_weight(Model& m, F f) {
    f(m.conv_out);
    for (auto& e : m.enc) f(e.qkv), f(e.o), f(e.up), f(e.down);
    f(m.proj1);
    f(m.proj2);
    for (auto& L : m.dec) f(L.qkv), f(L.o), f(L.gu), f(L.down);
    f(m.lm_head);   // tied: a copy of tok_embd's pointers; the embedding lookup keeps reading the Q8 rows
}
}  // namespace

void set_precision(Model& m, const std::string& mode) {
    QASR_CHECK(mode == "q8" || mode == "mxfp8", QASR_E_INVALID, "precision must be \"q8\" or \"mxfp8\"");
    QASR_CHECK(!m.weights_pending, QASR_E_INVALID, "set_precision: the model's weights have not arrived");
    if (mode == "q8") {
        if (!m.mx()) return;
        QASR_HIP(hipDeviceSynchronize());   // queued GEMMs may still read the fp8 images
        for_each_gemm_weight(m, [](Q8Mat& w) { w.mx = nullptr, w.mxs = nullptr; });
        m.mx_mem.reset();
        m.precision_gen++;
        return;
    }
    if (m.mx()) return;
    auto mem = std::make_unique<DevAlloc>();
    DevAlloc probe;
    probe.counting = true;
    for_each_gemm_weight(m, [&](Q8Mat& w) {
        if (w.K % 128 == 0) probe.alloc((size_t)w.N * w.K), probe.alloc((size_t)w.N * (w.K / QK));
    });
    mem->reserve(probe.bytes);
    hipStream_t s = nullptr;
    for_each_gemm_weight(m, [&](Q8Mat& w) {
        if (w.K % 128 != 0) return;   // stays on the Q8 GEMM
        w.mx = (uint8_t*)mem->alloc((size_t)w.N * w.K);
        w.mxs = (uint8_t*)mem->alloc((size_t)w.N * (w.K / QK));
        q8w_to_mx(w.qs, w.sc, (int64_t)w.N * (w.K / QK), w.mx, w.mxs, s);
    });
    QASR_HIP(hipStreamSynchronize(s));
    m.mx_mem = std::move(mem);
    m.precision_gen++;
}

void ensure_stage_scales(Model& m) {
    std::lock_guard<std::mutex> lk(m.s4_mu);
    if (m.s4_mem) return;
    auto each = [&](auto f) {
        for (auto& L : m.dec) f(L.qkv), f(L.o), f(L.gu), f(L.down);
        f(m.lm_head);
    };
    auto ok = [](const Q8Mat& w) { return w.qs && w.K % 128 == 0 && w.N % 2 == 0; };
    DevAlloc probe;
    probe.counting = true;
    each([&](Q8Mat& w) {
        if (ok(w)) probe.alloc((size_t)w.N * (w.K / QK) * sizeof(__half));
    });
    auto mem = std::make_unique<DevAlloc>();
    mem->reserve(std::max<size_t>(probe.bytes, 256));
    hipStream_t s = nullptr;
    each([&](Q8Mat& w) {
        if (!ok(w)) return;
        __half* o = (__half*)mem->alloc((size_t)w.N * (w.K / QK) * sizeof(__half));
        q8_stage_scales(w.sc, w.N, w.K, o, s);
        w.sc4 = o;
    });
    QASR_HIP(hipStreamSynchronize(s));
    m.s4_mem = std::move(mem);
}

// ----------------------------------------------------------------------------------------------- export
void export_tensor(const Model& m, const std::string& name, void* dst, size_t cap, size_t* written) {
    auto it = m.slots.find(name);
    QASR_CHECK(it != m.slots.end(), QASR_E_INVALID, "unknown tensor " + name);
    const TensorSlot& t = it->second;
    if (t.type == 8) {
        const int64_t nb = t.cols / QK;
        const size_t bytes = (size_t)(t.rows * nb * QBYTES);
        QASR_CHECK(cap >= bytes, QASR_E_CAPACITY, "export buffer too small");
        std::vector<int8_t> qs((size_t)(t.rows * t.cols));
        std::vector<uint16_t> sc((size_t)(t.rows * nb));
        if (t.il16_F > 0) {
            const int64_t N = 2 * t.il16_F;
            std::vector<int8_t> aq((size_t)(N * t.cols));
            std::vector<uint16_t> as((size_t)(N * nb));
            QASR_HIP(hipMemcpy(aq.data(), t.base, aq.size(), hipMemcpyDeviceToHost));
            QASR_HIP(hipMemcpy(as.data(), t.sc, as.size() * 2, hipMemcpyDeviceToHost));
            for (int64_t r = 0; r < t.rows; r++) {
                const int64_t p = gate_up_interleaved_row(t.row0 + r, t.il16_F);
                memcpy(&qs[(size_t)(r * t.cols)], &aq[(size_t)(p * t.cols)], (size_t)t.cols);
                memcpy(&sc[(size_t)(r * nb)], &as[(size_t)(p * nb)], (size_t)nb * 2);
            }
        } else {
            QASR_HIP(hipMemcpy(qs.data(), (int8_t*)t.base + t.row0 * t.ld, qs.size(), hipMemcpyDeviceToHost));
            QASR_HIP(hipMemcpy(sc.data(), t.sc + t.row0 * nb, sc.size() * 2, hipMemcpyDeviceToHost));
        }
        uint8_t* o = (uint8_t*)dst;
        for (int64_t b = 0; b < t.rows * nb; b++) {
            memcpy(o + b * QBYTES, &sc[(size_t)b], 2);
            memcpy(o + b * QBYTES + 2, &qs[(size_t)b * QK], QK);
        }
        *written = bytes;
    } else if (t.type == 0) {
        QASR_CHECK(cap >= (size_t)t.rows * 4, QASR_E_CAPACITY, "export buffer too small");
        QASR_HIP(hipMemcpy(dst, t.base, (size_t)t.rows * 4, hipMemcpyDeviceToHost));
        *written = (size_t)t.rows * 4;
    } else {
        // conv weights back in GGUF order [Cout][Cin][3][3]
        const int cin = t.conv_cin, cout = (int)(t.rows / (cin * 9));
        QASR_CHECK(cap >= (size_t)t.rows * 2, QASR_E_CAPACITY, "export buffer too small");
        std::vector<uint16_t> r((size_t)t.rows);
        QASR_HIP(hipMemcpy(r.data(), t.base, r.size() * 2, hipMemcpyDeviceToHost));
        uint16_t* o = (uint16_t*)dst;
        for (int co = 0; co < cout; co++)
            for (int k = 0; k < 9; k++)
                for (int ci = 0; ci < cin; ci++) o[((size_t)co * cin + ci) * 9 + k] = r[((size_t)co * 9 + k) * cin + ci];
        *written = (size_t)t.rows * 2;
    }
}

}  // namespace qasr
