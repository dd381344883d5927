// Device-resident Qwen3-ASR model (audio encoder + projector + Qwen3 decoder) for gfx950.
//
// HBM layout: every 2-D linear is Q8_0 repacked SoA (int8 [N][K] + f16 [N][K/32]);
// attention q/k/v (and the encoder's biases) and the decoder's gate/up are concatenated along N so one
// W8A8 launch produces them together.  Conv kernels are f16, reordered to [Cout][ky][kx][Cin] for the
// channel-last implicit GEMM.  Norm weights and biases are f32.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "tokenizer.h"

namespace qasr {

struct DevAlloc {
    std::vector<void*> ptrs;
    size_t bytes = 0;
    void* alloc(size_t n);
    ~DevAlloc();
};

struct EncLayer {
    float *ln1_w, *ln1_b, *ln2_w, *ln2_b;
    Q8Mat qkv, o, up, down;
    float *qkv_b, *o_b, *up_b, *down_b;
};

struct DecLayer {
    float *attn_norm, *q_norm, *k_norm, *ffn_norm;
    Q8Mat qkv, o, gu, down;
};

// where a GGUF tensor lives on the device (for export / parity tests)
struct TensorSlot {
    uint32_t type;      // GGML_F32 / GGML_F16 / GGML_Q8_0
    void* base;         // f32/f16 data, or Q8 qs
    __half* sc;         // Q8 scales
    int64_t rows, cols; // Q8: N, K (the slice [row0, row0+rows) of the concatenated matrix); f32/f16: n, 1
    int64_t row0;
    int64_t ld;         // Q8: K
    int conv_cin;       // f16 conv weights stored reordered (0 = plain)
    int64_t il16_F;     // Q8 gate|up rows stored interleaved by 16 (interleave_gate_up), F = half the rows
};

struct Model {
    qasr_hparams hp{};
    std::string arch;
    DevAlloc mem;
    // audio tower
    __half* conv_w[3]{};   // [Cout][9][Cin] (conv1: Cin = 1)
    float* conv_b[3]{};
    Q8Mat conv_out;
    std::vector<EncLayer> enc;
    float *ln_post_w = nullptr, *ln_post_b = nullptr;
    Q8Mat proj1, proj2;
    float *proj1_b = nullptr, *proj2_b = nullptr;
    float* pos_emb = nullptr;      // [13][enc_d] sinusoids
    float* mel_filters = nullptr;  // [201][n_mels]
    float* dft_basis = nullptr;    // [400][402] periodic-Hann-windowed cos/sin (mel STFT)
    // text decoder
    Q8Mat tok_embd, lm_head;
    float* out_norm = nullptr;
    std::vector<DecLayer> dec;
    Tokenizer tok;
    std::map<std::string, TensorSlot> slots;

    int audio_F3() const { return (((hp.n_mels + 1) / 2 + 1) / 2 + 1) / 2; }
    int64_t weight_bytes() const { return (int64_t)mem.bytes; }
};

void default_hparams(const char* arch, qasr_hparams* hp);
std::unique_ptr<Model> load_gguf_model(const std::string& path);
std::unique_ptr<Model> make_synthetic_model(const qasr_hparams& hp, uint64_t seed, const std::string& arch);
void export_tensor(const Model& m, const std::string& name, void* dst, size_t cap, size_t* written);

}  // namespace qasr
