// FireRedVAD on the GPU (firered_vad.py:38-191): weights from the repo's .qvad container, Kaldi fbank +
// CMVN + DFSMN as HIP kernels, the sequential segmenter on the host.
#include "vad.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "kernels_audio.h"

namespace qasr {

namespace {
const char* kOrder[] = {"mean", "istd", "w1", "b1", "w2", "b2", "lb0", "lb1", "lb2", "lb3", "lb4", "lb5", "lb6",
                        "lb7", "la0", "la1", "la2", "la3", "la4", "la5", "la6", "la7", "wa0", "wa1", "wa2", "wa3",
                        "wa4", "wa5", "wa6", "ba0", "ba1", "ba2", "ba3", "ba4", "ba5", "ba6", "wb0", "wb1", "wb2",
                        "wb3", "wb4", "wb5", "wb6", "wd", "bd", "wo", "bo"};
}

// .qvad: "QVADF32\0", u32 version, u32 count, count × {char name[32], u32 ndim, u32 dims[4]}, pad to 16,
// then each array's f32 data padded to 16 bytes (writer: tools/convert_vad.py)
Vad::Vad(const std::string& path) {
    FILE* f = fopen(path.c_str(), "rb");
    QASR_CHECK(f, QASR_E_IO, "cannot open VAD weights: " + path);
    std::vector<uint8_t> data;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    data.resize((size_t)sz);
    size_t got = fread(data.data(), 1, data.size(), f);
    fclose(f);
    QASR_CHECK(got == data.size() && sz > 16 && memcmp(data.data(), "QVADF32\0", 8) == 0, QASR_E_FORMAT,
               "not a .qvad file: " + path);
    uint32_t ver, n;
    memcpy(&ver, &data[8], 4);
    memcpy(&n, &data[12], 4);
    QASR_CHECK(ver == 1 && n == 47, QASR_E_FORMAT, "unexpected .qvad layout");
    size_t pos = 16;
    std::vector<std::pair<std::string, size_t>> meta;
    for (uint32_t i = 0; i < n; i++) {
        QASR_CHECK(pos + 52 <= data.size(), QASR_E_FORMAT, "truncated .qvad");
        std::string name((const char*)&data[pos], strnlen((const char*)&data[pos], 32));
        uint32_t dims[5];
        memcpy(dims, &data[pos + 32], 20);
        size_t cnt = 1;
        for (uint32_t k = 0; k < dims[0]; k++) cnt *= dims[1 + k];
        meta.emplace_back(name, cnt);
        pos += 52;
    }
    pos = (pos + 15) / 16 * 16;
    std::vector<float> win(400), banks(80 * 256);
    {   // one device allocation for every array + the two fbank tables (256-B granules, as DevAlloc hands out)
        size_t total = 0;
        for (const auto& mi : meta) total += (mi.second * 4 + 255) / 256 * 256;
        total += (win.size() * 4 + 255) / 256 * 256 + (banks.size() * 4 + 255) / 256 * 256;
        mem_.reserve(total);
    }
    for (uint32_t i = 0; i < n; i++) {
        QASR_CHECK(meta[i].first == kOrder[i], QASR_E_FORMAT, "unexpected .qvad array " + meta[i].first);
        const size_t bytes = meta[i].second * 4;
        QASR_CHECK(pos + bytes <= data.size(), QASR_E_FORMAT, "truncated .qvad data");
        if (meta[i].first == "bo") memcpy(&bo_, &data[pos], 4);
        float* d = (float*)mem_.alloc(bytes);
        QASR_HIP(hipMemcpy(d, &data[pos], bytes, hipMemcpyHostToDevice));
        arr_[meta[i].first] = d;
        pos += (bytes + 15) / 16 * 16;
    }
    povey_window(win.data());
    kaldi_mel_banks(banks.data());
    win_ = (float*)mem_.alloc(win.size() * 4);
    banks_ = (float*)mem_.alloc(banks.size() * 4);
    QASR_HIP(hipMemcpy(win_, win.data(), win.size() * 4, hipMemcpyHostToDevice));
    QASR_HIP(hipMemcpy(banks_, banks.data(), banks.size() * 4, hipMemcpyHostToDevice));
    QASR_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
}

Vad::~Vad() {
    for (auto& b : bufs_)
        if (b) (void)hipFree(b);
    if (st_) (void)hipStreamDestroy(st_);
}

float* Vad::buf(int i, size_t bytes) {
    if ((int)bufs_.size() <= i) {
        bufs_.resize(i + 1, nullptr);
        caps_.resize(i + 1, 0);
    }
    if (caps_[i] < bytes) {
        if (bufs_[i]) {
            QASR_HIP(hipStreamSynchronize(st_));
            QASR_HIP(hipFree(bufs_[i]));
        }
        caps_[i] = std::max<size_t>(bytes + bytes / 4, 4096);
        QASR_HIP(hipMalloc(&bufs_[i], caps_[i]));
    }
    return (float*)bufs_[i];
}

int Vad::n_frames(int64_t n) { return n >= 400 ? (int)(1 + (n - 400) / 160) : 0; }

void Vad::features_device(const float* pcm_host, int64_t n, float** d_feats, int* T_out) {
    const int T = n_frames(n);
    *T_out = T;
    if (T == 0) return;
    std::vector<float> scaled((size_t)n);
    for (int64_t i = 0; i < n; i++) {  // firered_vad.py:89 — x·32768 clipped, not rounded
        float v = pcm_host[i] * 32768.0f;
        scaled[(size_t)i] = v < -32768.f ? -32768.f : (v > 32767.f ? 32767.f : v);
    }
    float* dp = buf(0, (size_t)n * 4);
    QASR_HIP(hipMemcpyAsync(dp, scaled.data(), (size_t)n * 4, hipMemcpyHostToDevice, st_));
    float* feats = buf(1, (size_t)T * 80 * 4);
    kaldi_fbank(dp, n, T, win_, banks_, feats, st_);
    QASR_HIP(hipStreamSynchronize(st_));
    *d_feats = feats;
}

void Vad::features(const float* pcm, int64_t n, std::vector<float>& feats) {
    float* d = nullptr;
    int T = 0;
    features_device(pcm, n, &d, &T);
    feats.assign((size_t)T * 80, 0.f);
    if (T) QASR_HIP(hipMemcpy(feats.data(), d, feats.size() * 4, hipMemcpyDeviceToHost));
}

void Vad::probabilities(const float* pcm, int64_t n, std::vector<float>& probs) {
    float* feats = nullptr;
    int T = 0;
    features_device(pcm, n, &feats, &T);
    probs.assign((size_t)T, 0.f);
    if (T == 0) return;
    auto A = [&](const char* k) { return arr_.at(k); };
    float* x = buf(2, (size_t)T * 80 * 4);
    float* h = buf(3, (size_t)T * 256 * 4);
    float* p = buf(4, (size_t)T * 128 * 4);
    float* s = buf(5, (size_t)T * 128 * 4);
    float* s2 = buf(6, (size_t)T * 128 * 4);
    float* pr = buf(7, (size_t)T * 4);
    cmvn(feats, T, A("mean"), A("istd"), x, st_);
    dense_f32(x, T, 80, A("w1"), A("b1"), 256, 1, h, st_);
    dense_f32(h, T, 256, A("w2"), A("b2"), 128, 1, p, st_);
    fsmn_block(p, T, A("lb0"), A("la0"), nullptr, s, st_);
    char k1[8], k2[8], k3[8], k4[8], k5[8];
    for (int k = 0; k < 7; k++) {
        snprintf(k1, sizeof k1, "wa%d", k);
        snprintf(k2, sizeof k2, "ba%d", k);
        snprintf(k3, sizeof k3, "wb%d", k);
        snprintf(k4, sizeof k4, "lb%d", k + 1);
        snprintf(k5, sizeof k5, "la%d", k + 1);
        dense_f32(s, T, 128, A(k1), A(k2), 256, 1, h, st_);
        dense_f32(h, T, 256, A(k3), nullptr, 128, 0, p, st_);
        fsmn_block(p, T, A(k4), A(k5), s, s2, st_);
        std::swap(s, s2);
    }
    dense_f32(s, T, 128, A("wd"), A("bd"), 256, 1, h, st_);
    vad_head(h, T, A("wo"), bo_, pr, st_);
    QASR_HIP(hipGetLastError());
    QASR_HIP(hipMemcpyAsync(probs.data(), pr, (size_t)T * 4, hipMemcpyDeviceToHost, st_));
    QASR_HIP(hipStreamSynchronize(st_));
}

// firered_vad.py:121-191
std::vector<std::pair<int64_t, int64_t>> timestamps_from_probabilities(const float* probs, int64_t T,
                                                                       int64_t audio_len, const qasr_vad_options& o) {
    std::vector<std::pair<int64_t, int64_t>> out;
    if (T <= 0) return out;
    std::vector<float> sm((size_t)T);
    const int win = o.smooth_window_frames > 1 ? o.smooth_window_frames : 1;
    if (win > 1) {
        const float kv = 1.0f / (float)win;
        for (int64_t t = 0; t < T; t++) {
            double acc = 0.0;
            for (int j = 0; j < win; j++)
                if (t - j >= 0) acc += (double)probs[t - j] * (double)kv;
            sm[(size_t)t] = (float)acc;
        }
        for (int64_t t = 0; t < std::min<int64_t>(win - 1, T); t++) {
            double a = 0.0;
            for (int64_t j = 0; j <= t; j++) a += probs[j];
            sm[(size_t)t] = (float)(a / (double)(t + 1));
        }
    } else {
        for (int64_t t = 0; t < T; t++) sm[(size_t)t] = probs[t];
    }
    const int64_t min_sp = std::max(1, o.min_speech_duration_ms / 10);
    const int64_t min_si = std::max(1, o.min_silence_duration_ms / 10);
    const int64_t pad = std::max<int64_t>(0, (int64_t)o.speech_pad_ms * 16000 / 1000);
    std::vector<std::pair<int64_t, int64_t>> seg;
    int64_t cand = -1, sp = -1, si = -1;
    for (int64_t i = 0; i < T; i++) {
        const bool is_sp = sm[(size_t)i] >= o.threshold;
        if (sp < 0) {
            if (is_sp) {
                if (cand < 0) cand = i;
                if (i - cand + 1 >= min_sp) {
                    sp = cand;
                    si = -1;
                }
            } else {
                cand = -1;
            }
            continue;
        }
        if (is_sp) {
            si = -1;
            continue;
        }
        if (si < 0) {
            si = i;
            continue;
        }
        if (i - si + 1 >= min_si) {
            seg.emplace_back(sp, si);
            sp = cand = si = -1;
        }
    }
    if (sp >= 0) seg.emplace_back(sp, T);
    for (auto& s : seg) {
        const int64_t st = std::max<int64_t>(0, s.first * 160 - pad);
        const int64_t en = std::min<int64_t>(audio_len, s.second * 160 + pad);
        if (en <= st) continue;
        if (!out.empty() && st <= out.back().second) out.back().second = std::max(out.back().second, en);
        else out.emplace_back(st, en);
    }
    return out;
}

}  // namespace qasr
