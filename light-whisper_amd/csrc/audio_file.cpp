// Path-mode audio input: Qwen3ASRServer._load_audio's file branch (qwen3_asr_server.py:256-267) —
// sf.read(path, dtype="float32", always_2d=True) → audio.mean(axis=1, dtype=float32) → _resample(audio, rate).
// soundfile / libsndfile are not part of this image; the WAV container and libsndfile's float normalisation of
// integer PCM (int16 / 2^15, int24 / 2^23, int32 / 2^31, unsigned 8-bit (x − 128) / 2^7) are restated here for PCM
// 8/16/24/32, IEEE float32 / float64 (doubles narrowed to float) and G.711 µ-law / A-law (libsndfile's 16-bit
// decode tables — Sun g711.c ulaw2linear / alaw2linear — times 1/0x8000), WAVE_FORMAT_EXTENSIBLE included.  Other
// codecs (ADPCM, GSM …) and containers (FLAC, OGG …) are refused with an error reply (INTEGRATION.md lists them).
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/qasr.h"
#include "capi_util.h"

namespace {

std::string slurp(const char* path) {
    std::string s;
    FILE* f = fopen(path, "rb");
    if (!f) return s;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

// G.711 code → 16-bit linear (libsndfile ulaw_decode / alaw_decode)
int ulaw_linear(unsigned char c) {
    const int u = ~c & 0xFF;
    const int t = (((u & 0x0F) << 3) + 0x84) << ((u & 0x70) >> 4);
    return (u & 0x80) ? 0x84 - t : t - 0x84;
}
int alaw_linear(unsigned char c) {
    const int a = c ^ 0x55, seg = (a & 0x70) >> 4;
    int t = (a & 0x0F) << 4;
    t = seg == 0 ? t + 8 : (t + 0x108) << (seg - 1);
    return (a & 0x80) ? t : -t;
}

uint16_t u16(const std::string& d, size_t at) { return (uint16_t)((uint8_t)d[at] | ((uint8_t)d[at + 1] << 8)); }
uint32_t u32(const std::string& d, size_t at) {
    return (uint32_t)(uint8_t)d[at] | ((uint32_t)(uint8_t)d[at + 1] << 8) | ((uint32_t)(uint8_t)d[at + 2] << 16) |
           ((uint32_t)(uint8_t)d[at + 3] << 24);
}

// RIFF/WAVE → mono f32 (channel mean) at the file's rate; soundfile's error texts where it has one
void read_wav(const std::string& path, std::vector<float>& mono, int& rate) {
    const std::string d = slurp(path.c_str());
    const std::string open_err = "Error opening '" + path + "': ";
    QASR_CHECK(d.size() >= 12 && d.compare(0, 4, "RIFF") == 0 && d.compare(8, 4, "WAVE") == 0, QASR_E_FORMAT,
               open_err + "Format not recognised.");
    int fmt = 0, ch = 0, bits = 0;
    rate = 0;
    for (size_t pos = 12; pos + 8 <= d.size();) {
        const std::string id = d.substr(pos, 4);
        const uint64_t sz = u32(d, pos + 4);
        const size_t body = pos + 8;
        if (id == "fmt " && sz >= 16 && body + 16 <= d.size()) {
            fmt = u16(d, body);
            ch = u16(d, body + 2);
            rate = (int)u32(d, body + 4);
            bits = u16(d, body + 14);
            if (fmt == 0xFFFE && sz >= 26 && body + 26 <= d.size()) fmt = u16(d, body + 24);   // extensible sub-format
        } else if (id == "data") {
            QASR_CHECK(ch > 0 && rate > 0, QASR_E_FORMAT, open_err + "Format not recognised.");
            const bool pcm = fmt == 1 && (bits == 8 || bits == 16 || bits == 24 || bits == 32);
            const bool flt = fmt == 3 && (bits == 32 || bits == 64), g711 = (fmt == 6 || fmt == 7) && bits == 8;
            QASR_CHECK(pcm || flt || g711, QASR_E_FORMAT, open_err + "Unsupported WAV sample format");
            const size_t n = (size_t)std::min<uint64_t>(sz, d.size() - body);
            const size_t bps = (size_t)bits / 8, frames = n / (bps * (size_t)ch);
            mono.assign(frames, 0.f);
            const unsigned char* base = (const unsigned char*)d.data() + body;
            for (size_t i = 0; i < frames; i++) {
                float acc = 0.f;
                for (int c = 0; c < ch; c++) {
                    const unsigned char* p = base + (i * (size_t)ch + (size_t)c) * bps;
                    float v;
                    if (fmt == 3 && bits == 64) {
                        double dv;
                        memcpy(&dv, p, 8);
                        v = (float)dv;
                    } else if (fmt == 3) memcpy(&v, p, 4);
                    else if (fmt == 7) v = (float)ulaw_linear(p[0]) * (1.f / 32768.f);
                    else if (fmt == 6) v = (float)alaw_linear(p[0]) * (1.f / 32768.f);
                    else if (bits == 16) v = (float)(int16_t)(p[0] | (p[1] << 8)) / 32768.f;
                    else if (bits == 24)
                        v = (float)((int32_t)(((uint32_t)p[0] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 24)) >> 8) /
                            8388608.f;
                    else if (bits == 32)
                        v = (float)(int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                                             ((uint32_t)p[3] << 24)) / 2147483648.f;
                    else v = ((float)p[0] - 128.f) / 128.f;
                    acc += v;   // numpy's float32 mean over axis 1: a running f32 sum, then one division
                }
                mono[i] = acc / (float)ch;
            }
            return;
        }
        QASR_CHECK(sz <= d.size() - body, QASR_E_FORMAT, open_err + "Format not recognised.");
        pos = body + (size_t)sz + (size_t)(sz & 1);
    }
    throw qasr::Error(QASR_E_FORMAT, open_err + "Format not recognised.");
}

}  // namespace

extern "C" {

QASR_API int qasr_audio_load_path(const char* path, float* out, size_t cap, size_t* n_out) {
    return qasr::guard([&] {
        QASR_CHECK(path && n_out, QASR_E_INVALID, "null argument");
        std::vector<float> mono;
        int rate = 0;
        read_wav(path, mono, rate);
        size_t n = 0;
        if (qasr_resample_linear(mono.data(), mono.size(), (double)rate, nullptr, 0, &n) != QASR_OK)
            throw qasr::Error(QASR_E_FORMAT, qasr_last_error());
        *n_out = n;
        if (!out) return;
        QASR_CHECK(cap >= n, QASR_E_CAPACITY, "sample buffer too small");
        if (n && qasr_resample_linear(mono.data(), mono.size(), (double)rate, out, cap, &n) != QASR_OK)
            throw qasr::Error(QASR_E_FORMAT, qasr_last_error());
    });
}

}  // extern "C"
