// Audio front-end kernels: Qwen3-ASR log-mel + conv stack (encoder input) and the FireRedVAD front end.
#pragma once
#include <vector>

#include "common.h"
#include "prof.h"

namespace qasr {

// host tables
void mel_filter_table(int n_mels, float* out /*[201][n_mels]*/);       // Slaney, like HF mel_filter_bank
void dft_basis_table(std::vector<float>& out /*[400][402]*/);          // periodic Hann × (cos, -sin)
void kaldi_mel_banks(float* out /*[80][256]*/);                        // kaldi-native-fbank MelBanks
void povey_window(float* out /*[400]*/);

// One utterance of a batched front end (device array of these).
struct MelUtt {
    int64_t pcm_off;   // offset into the packed pcm buffer
    int64_t n;         // samples (before the 8000-sample minimum pad)
    int64_t P;         // padded length (max(n', 480000))
    int t_all;         // P / 160
    int t_comp;        // frames computed explicitly (the rest are pure zero padding)
    int t_valid;
    int chunk0;        // first 100-frame chunk index in the batch
    int n_chunks;
    int frame0;        // first row in the log-mel scratch
};

// log10 mel power of frames; writes lm [frame0+t][n_mels] and the per-utterance max (ordered-uint encoded)
void mel_frames(const float* pcm, const MelUtt* utts, const int2* work /*(utt, t0)*/, int n_work, int n_mels,
                const float* basis, const float* filt, float* lm, unsigned* umax, hipStream_t s);
// normalise + lay out per chunk: x [chunk][n_mels][100] f32 (conv1 input)
void mel_normalize(const MelUtt* utts, int n_utts, int total_chunks, const int* chunk_utt, int n_mels, const float* lm,
                   const unsigned* umax, float* x, hipStream_t s);
// conv1 (Cin = 1, 3×3 s2 p1) + GELU → f16 channel-last [chunk][H1][W1][C]
void conv1_gelu(const float* x, int n_chunks, int n_mels, const __half* w /*[C][9]*/, const float* b, int C,
                __half* y, hipStream_t s);
// conv 3×3 s2 p1 as implicit GEMM on f16 MFMA: in [chunk][Hi][Wi][C] f16 → GELU →
//   out_mode 0: f16 [chunk][Ho][Wo][C];  out_mode 1: f32 [chunk][Wo][C][Ho] (conv_out input rows)
void conv3x3_gelu(const __half* in, int n_chunks, int Hi, int Wi, const __half* w /*[C][9][C]*/, const float* b,
                  int C, void* out, int out_mode, hipStream_t s);
void reorder_conv_weight(const __half* src /*[Cout][Cin][9]*/, int cout, int cin, __half* dst /*[Cout][9][Cin]*/,
                         hipStream_t s);

// FireRedVAD: Kaldi fbank (LDS radix-2 FFT, 512 points) on int16-scaled samples → log-fbank [T][80]
void kaldi_fbank(const float* pcm, int64_t n, int T, const float* window, const float* banks, float* feats,
                 hipStream_t s);
// f32 dense layer y[T][N] = act(x[T][K]·W[K][N] + b) (+ skip); act 1 = ReLU
void dense_f32(const float* x, int T, int K, const float* W, const float* b, int N, int relu, float* y,
               hipStream_t s);
// CMVN then dense: x' = (x - mean)·istd
void cmvn(const float* x, int T, const float* mean, const float* istd, float* y, hipStream_t s);
// FSMN memory block: y = x + lookback(x) + lookahead(x) (+ skip), 128 channels, 20+20 taps
void fsmn_block(const float* x, int T, const float* lb, const float* la, const float* skip, float* y, hipStream_t s);
// final 256→1 + sigmoid
void vad_head(const float* h, int T, const float* wo, float bo, float* probs, hipStream_t s);

}  // namespace qasr
