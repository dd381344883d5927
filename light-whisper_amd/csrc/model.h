// Device-resident Qwen3-ASR model (audio encoder + projector + Qwen3 decoder) for gfx950.
//
// HBM layout: every 2-D linear is Q8_0 repacked SoA (int8 [N][K] + f16 [N][K/32]);
// attention q/k/v (and the encoder's biases) and the decoder's gate/up are concatenated along N so one
// W8A8 launch produces them together.  Conv kernels are f16, reordered to [Cout][ky][kx][Cin] for the
// channel-last implicit GEMM.  Norm weights and biases are f32.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "tokenizer.h"

namespace qasr {

// Every weight and table of a model lives in ONE device allocation whose offsets depend only on the
// hyper-parameters (and on whether the checkpoint has an untied output.weight): the blob a rank-0 load fills
// and one RCCL broadcast copies into every other rank's identically laid-out shell.
struct DevAlloc {
    char* base = nullptr;
    size_t cap = 0, bytes = 0;
    bool counting = false;   // layout probe: hands out offsets only, touches no memory
    void reserve(size_t n);
    void* alloc(size_t n);
    DevAlloc() = default;
    DevAlloc(const DevAlloc&) = delete;
    DevAlloc& operator=(const DevAlloc&) = delete;
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

    bool weights_pending = false;   // a shell: layout allocated, weights still to arrive (broadcast)
    // precision mode "mxfp8" (SURVEY §8(d) C5): MXFP8 images of the GEMM weights in their own allocation
    std::unique_ptr<DevAlloc> mx_mem;
    bool mx() const { return mx_mem != nullptr; }
    // bumped by every precision change: sessions' captured decode graphs hold the GEMM weight pointers of the
    // precision they were captured in, so a change invalidates them (engine.cpp run_batch)
    uint64_t precision_gen = 0;
    // the decoder matrices' regrouped stage scales (Q8Mat::sc4), derived once the weights are in place
    std::unique_ptr<DevAlloc> s4_mem;
    std::mutex s4_mu;

    int audio_F3() const { return (((hp.n_mels + 1) / 2 + 1) / 2 + 1) / 2; }
    int64_t weight_bytes() const { return (int64_t)mem.bytes; }
};

void default_hparams(const char* arch, qasr_hparams* hp);
// shell = true: hyper-parameters and tokenizer from the GGUF metadata, the device layout allocated, no tensor
// data read (the receiving side of the weight broadcast)
std::unique_ptr<Model> load_gguf_model(const std::string& path, bool shell = false);
std::unique_ptr<Model> make_synthetic_model(const qasr_hparams& hp, uint64_t seed, const std::string& arch);
std::unique_ptr<Model> make_synthetic_shell(const qasr_hparams& hp, const std::string& arch);
void export_tensor(const Model& m, const std::string& name, void* dst, size_t cap, size_t* written);
// "q8" (default: the reference's W8A8 arithmetic) or "mxfp8" (block-scaled fp8 GEMMs; tolerance parity only).
// Open sessions re-capture their decode graphs on their next run (precision_gen).
void set_precision(Model& m, const std::string& mode);
// derive Q8Mat::sc4 for the decoder layers' matrices and the vocabulary projection (K % 128 == 0), once; called
// when a session opens (the weights are final then: loaded, generated or received by broadcast, gate|up interleaved)
void ensure_stage_scales(Model& m);

}  // namespace qasr
