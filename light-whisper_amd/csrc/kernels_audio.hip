// Audio front ends for gfx950:
//   * Qwen3-ASR log-mel (feature_extraction_qwen3_asr.py:104-127 + the padding rules of __call__:189-228):
//     windowed 400-point DFT per frame against an L2-resident basis (16 frames per workgroup share every
//     basis load), |X|², Slaney mel, log10, per-utterance max via ordered-uint atomics, then clamp/normalise
//     into the per-chunk conv1 layout.
//   * encoder conv stack (modeling_qwen3_asr.py:344-346,407-409): conv1 direct (Cin = 1), conv2/conv3 as
//     channel-last implicit GEMMs on v_mfma_f32_16x16x32_f16 (f16 operands — the ggml im2col convention —
//     f32 accumulation) with fused bias + GELU.
//   * FireRedVAD (firered_vad.py:87-111): Kaldi fbank with a per-wave LDS radix-2 FFT (512 points),
//     DFSMN dense layers (f32), FSMN memory blocks and the sigmoid head.
#include <math.h>
#include <stdlib.h>

#include <utility>

#include "kernels_audio.h"
#include "lds_dma.h"

namespace qasr {

// ================================================================================================ tables
static double slaney_h2m(double f) {
    if (f >= 1000.0) return 15.0 + log(f / 1000.0) * (27.0 / log(6.4));
    return 3.0 * f / 200.0;
}
static double slaney_m2h(double m) {
    if (m >= 15.0) return 1000.0 * exp((log(6.4) / 27.0) * (m - 15.0));
    return 200.0 * m / 3.0;
}

void mel_filter_table(int n_mels, float* out) {
    std::vector<double> ff((size_t)n_mels + 2);
    const double mmin = slaney_h2m(0.0), mmax = slaney_h2m(8000.0);
    for (int i = 0; i < n_mels + 2; i++) {
        double mel = mmin + (mmax - mmin) * (double)i / (double)(n_mels + 1);
        if (i == n_mels + 1) mel = mmax;
        ff[(size_t)i] = slaney_m2h(mel);
    }
    for (int k = 0; k < 201; k++) {
        double fk = 8000.0 * (double)k / 200.0;
        for (int m = 0; m < n_mels; m++) {
            double down = -(ff[m] - fk) / (ff[m + 1] - ff[m]);
            double up = (ff[m + 2] - fk) / (ff[m + 2] - ff[m + 1]);
            double v = down < up ? down : up;
            if (v < 0.0) v = 0.0;
            v *= 2.0 / (ff[m + 2] - ff[m]);
            out[k * n_mels + m] = (float)v;
        }
    }
}

void dft_basis_table(std::vector<float>& out) {
    out.assign((size_t)400 * 402, 0.f);
    for (int i = 0; i < 400; i++) {
        const double w = 0.5 - 0.5 * cos(2.0 * M_PI * i / 400.0);  // periodic Hann (torch.hann_window)
        for (int k = 0; k < 201; k++) {
            const double a = -2.0 * M_PI * (double)((k * i) % 400) / 400.0;
            out[(size_t)i * 402 + 2 * k] = (float)(w * cos(a));
            out[(size_t)i * 402 + 2 * k + 1] = (float)(w * sin(a));
        }
    }
}

static double kaldi_mel(double f) { return 1127.0 * log(1.0 + f / 700.0); }

void kaldi_mel_banks(float* banks) {
    const double fft_bin_width = 16000.0 / 512;
    const double mel_low = kaldi_mel(20.0), mel_high = kaldi_mel(8000.0);
    const double delta = (mel_high - mel_low) / 81;
    for (int b = 0; b < 80; b++) {
        double left = mel_low + b * delta, center = left + delta, right = center + delta;
        for (int i = 0; i < 256; i++) {
            double mel = kaldi_mel(fft_bin_width * i);
            float w = 0.f;
            if (mel > left && mel < right)
                w = (float)(mel <= center ? (mel - left) / (center - left) : (right - mel) / (right - center));
            banks[b * 256 + i] = w;
        }
    }
}

void povey_window(float* out) {
    for (int i = 0; i < 400; i++) out[i] = (float)pow(0.5 - 0.5 * cos(2.0 * M_PI * i / 399.0), 0.85);
}

// ================================================================================================ log-mel
__device__ __forceinline__ unsigned f2ord(float f) {
    unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

constexpr int MFR = 16;  // frames per workgroup

__global__ __launch_bounds__(256) void k_mel_frames(const float* __restrict__ pcm, const MelUtt* __restrict__ utts,
                                                    const int2* __restrict__ work, int n_mels,
                                                    const float* __restrict__ basis, const float* __restrict__ filt,
                                                    float* __restrict__ lm, unsigned* __restrict__ umax) {
    __shared__ float xs[MFR][400];
    __shared__ float ps[MFR][201];
    const int2 wk = work[blockIdx.x];
    const MelUtt U = utts[wk.x];
    const int t0 = wk.y;
    const int nf = min(MFR, U.t_comp - t0);
    const float* x = pcm + U.pcm_off;
    for (int idx = threadIdx.x; idx < MFR * 400; idx += 256) {
        const int f = idx / 400, i = idx % 400;
        float v = 0.f;
        if (f < nf) {
            int64_t sidx = (int64_t)(t0 + f) * 160 - 200 + i;
            if (sidx < 0) sidx = -sidx;                         // reflect (center=True)
            if (sidx >= U.P) sidx = 2 * U.P - 2 - sidx;
            v = sidx < U.n ? x[sidx] : 0.f;                     // beyond the clip: zero padding
        }
        xs[f][i] = v;
    }
    __syncthreads();
    const int k = threadIdx.x;
    if (k < 201) {
        float re[MFR], im[MFR];
#pragma unroll
        for (int f = 0; f < MFR; f++) re[f] = im[f] = 0.f;
        const float2* b2 = (const float2*)basis;
        for (int i = 0; i < 400; i++) {
            const float2 b = b2[i * 201 + k];
#pragma unroll
            for (int f = 0; f < MFR; f++) {
                const float xv = xs[f][i];
                re[f] += xv * b.x;
                im[f] += xv * b.y;
            }
        }
#pragma unroll
        for (int f = 0; f < MFR; f++) ps[f][k] = re[f] * re[f] + im[f] * im[f];
    }
    __syncthreads();
    for (int m = threadIdx.x; m < n_mels; m += 256) {
        // the filter's nonzero band [lo, hi): outside it every term is +0 (finite powers), so summing only the band
        // gives the same bits as the full 201-bin sum (acc starts at +0 and never turns -0)
        int lo = 201, hi = 0;
        for (int kk = 0; kk < 201; kk++)
            if (filt[kk * n_mels + m] != 0.f) lo = min(lo, kk), hi = kk + 1;
        float lmax = -INFINITY;
        for (int f = 0; f < nf; f++) {
            float acc = 0.f;
            for (int kk = lo; kk < hi; kk++) acc += filt[kk * n_mels + m] * ps[f][kk];
            const float l = log10f(fmaxf(acc, 1e-10f));
            lm[(size_t)(U.frame0 + t0 + f) * n_mels + m] = l;
            lmax = fmaxf(lmax, l);
        }
        if (nf > 0) atomicMax(umax + wk.x, f2ord(lmax));
    }
}

void mel_frames(const float* pcm, const MelUtt* utts, const int2* work, int n_work, int n_mels, const float* basis,
                const float* filt, float* lm, unsigned* umax, hipStream_t s) {
    if (n_work <= 0) return;
    ProfScope ps(s, "mel_frames", (double)n_work * 16 * (400.0 * 402 * 2 + 201.0 * n_mels * 2), (double)n_work * 16 * (640 + 4.0 * n_mels));
    k_mel_frames<<<n_work, 256, 0, s>>>(pcm, utts, work, n_mels, basis, filt, lm, umax);
}

__global__ void k_mel_normalize(const MelUtt* __restrict__ utts, int total_chunks, const int* __restrict__ chunk_utt,
                                int n_mels, const float* __restrict__ lm, const unsigned* __restrict__ umax,
                                float* __restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)total_chunks * n_mels * 100) return;
    const int t = (int)(i % 100);
    const int m = (int)((i / 100) % n_mels);
    const int c = (int)(i / (100 * n_mels));
    const int u = chunk_utt[c];
    const MelUtt U = utts[u];
    float gmax = ord2f(umax[u]);
    if (U.t_all > U.t_comp) gmax = fmaxf(gmax, -10.f);  // pure zero-padding frames: log10(1e-10)
    const int frame = (c - U.chunk0) * 100 + t;
    float v = 0.f;                                      // np.pad of the mel axis
    if (frame < U.t_all) {
        float l = frame < U.t_comp ? lm[(size_t)(U.frame0 + frame) * n_mels + m] : -10.f;
        l = fmaxf(l, gmax - 8.f);
        v = (l + 4.f) / 4.f;
    }
    x[i] = v;
}

void mel_normalize(const MelUtt* utts, int n_utts, int total_chunks, const int* chunk_utt, int n_mels, const float* lm,
                   const unsigned* umax, float* x, hipStream_t s) {
    (void)n_utts;
    const int64_t n = (int64_t)total_chunks * n_mels * 100;
    if (n <= 0) return;
    k_mel_normalize<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(utts, total_chunks, chunk_utt, n_mels, lm, umax, x);
}

// ================================================================================================ conv stack
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// conv1 (Cin = 1, 3×3, stride 2, pad 1) + GELU: one workgroup per (chunk, output row).  The three input rows
// (f16-rounded, zero-padded) sit in LDS and are read as broadcasts; each thread keeps one output channel's 9
// taps and bias in registers and walks the 50 output columns, so every store instruction writes 256
// consecutive channels of one position (channel-last f16 output).
__global__ __launch_bounds__(256) void k_conv1_gelu(const float* __restrict__ x, int n_chunks, int H0,
                                                    const __half* __restrict__ w, const float* __restrict__ b, int C,
                                                    __half* __restrict__ y) {
    constexpr int W0 = 100, W1 = 50;
    const int H1 = (H0 + 1) / 2;
    const int oy = blockIdx.x, ch = blockIdx.y;
    __shared__ float xs[3][W0 + 2];
    const float* xc = x + (size_t)ch * H0 * W0;
    for (int i = threadIdx.x; i < 3 * (W0 + 2); i += 256) {
        const int ky = i / (W0 + 2), ix = i % (W0 + 2) - 1, iy = 2 * oy - 1 + ky;
        xs[ky][ix + 1] = (iy >= 0 && iy < H0 && ix >= 0 && ix < W0) ? __half2float(f2h(xc[iy * W0 + ix])) : 0.f;
    }
    __syncthreads();
    __half* yr = y + ((size_t)ch * H1 + oy) * W1 * C;
    // two adjacent channels per thread (C even): one 4-byte store per position instead of two 2-byte ones; each
    // output's arithmetic is unchanged
    for (int c2 = threadIdx.x; 2 * c2 < C; c2 += 256) {
        const int co = 2 * c2;
        float k9[2][9];
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int t = 0; t < 9; t++) k9[h][t] = __half2float(w[(co + h) * 9 + t]);
        const float bias0 = b[co], bias1 = b[co + 1];
        for (int ox = 0; ox < W1; ox++) {
            float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
            for (int ky = 0; ky < 3; ky++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) {
                    const float xv = xs[ky][2 * ox + kx];
                    acc0 += k9[0][ky * 3 + kx] * xv;
                    acc1 += k9[1][ky * 3 + kx] * xv;
                }
            *(__half2*)(yr + (size_t)ox * C + co) = __halves2half2(f2h(gelu_f(acc0 + bias0)), f2h(gelu_f(acc1 + bias1)));
        }
    }
}

void conv1_gelu(const float* x, int n_chunks, int n_mels, const __half* w, const float* b, int C, __half* y,
                hipStream_t s) {
    const int64_t n = (int64_t)n_chunks * ((n_mels + 1) / 2) * 50 * C;
    if (n <= 0) return;
    QASR_CHECK(C % 2 == 0, QASR_E_INVALID, "conv1: channel count must be even");
    ProfScope ps(s, "conv1", (double)n * 18, (double)n * 2);
    k_conv1_gelu<<<dim3((n_mels + 1) / 2, n_chunks), 256, 0, s>>>(x, n_chunks, n_mels, w, b, C, y);
}

typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// generic-width fallback (channels a multiple of 32, e.g. the tiny test configs): 64×64 tiles, K step 32
constexpr int CT = 64;     // output tile (positions × channels)
constexpr int CLD = 40;    // LDS row stride in halves (80 B)

__global__ __launch_bounds__(256) void k_conv3x3_gelu_c32(const __half* __restrict__ in, int n_chunks, int Hi, int Wi,
                                                      const __half* __restrict__ w, const float* __restrict__ bias,
                                                      int C, void* __restrict__ out, int out_mode) {
    __shared__ __attribute__((aligned(16))) _Float16 As[CT * CLD];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[CT * CLD];
    const int Ho = (Hi + 1) / 2, Wo = (Wi + 1) / 2;
    const int M = n_chunks * Ho * Wo;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int n0 = blockIdx.x * CT, m0 = blockIdx.y * CT;
    // staging: row t>>2, 8 halves at (t&3)*8
    const int srow = tid >> 2, sseg = (tid & 3) * 8;
    const int am = m0 + srow;
    int a_ch = 0, a_oy = 0, a_ox = 0;
    const bool a_ok = am < M;
    if (a_ok) {
        a_ch = am / (Ho * Wo);
        const int rem = am % (Ho * Wo);
        a_oy = rem / Wo;
        a_ox = rem % Wo;
    }
    const int bn = n0 + srow;
    const bool b_ok = bn < C;
    const int cblk = C / 32;
    const int steps = 9 * cblk;
    v4f acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

    int4 ra, rb;
    auto gload = [&](int st) {
        const int tap = st / cblk, ci0 = (st % cblk) * 32 + sseg;
        const int ky = tap / 3, kx = tap % 3;
        const int iy = 2 * a_oy - 1 + ky, ix = 2 * a_ox - 1 + kx;
        ra = (a_ok && iy >= 0 && iy < Hi && ix >= 0 && ix < Wi)
                 ? *(const int4*)(in + (((size_t)a_ch * Hi + iy) * Wi + ix) * C + ci0)
                 : make_int4(0, 0, 0, 0);
        rb = b_ok ? *(const int4*)(w + ((size_t)bn * 9 + tap) * C + ci0) : make_int4(0, 0, 0, 0);
    };
    auto lstore = [&]() {
        *(int4*)(As + srow * CLD + sseg) = ra;
        *(int4*)(Bs + srow * CLD + sseg) = rb;
    };
    const int fr = lane & 15, fk = 8 * (lane >> 4);
    gload(0);
    lstore();
    __syncthreads();
    for (int st = 0; st < steps; st++) {
        const bool more = st + 1 < steps;
        if (more) gload(st + 1);
        v8h a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; i++) a[i] = *(const v8h*)(As + (wr * 32 + i * 16 + fr) * CLD + fk);
#pragma unroll
        for (int j = 0; j < 2; j++) b[j] = *(const v8h*)(Bs + (wc * 32 + j * 16 + fr) * CLD + fk);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        __syncthreads();
        if (more) {
            lstore();
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int col = n0 + wc * 32 + j * 16 + fr;
            if (col >= C) continue;
            const float bv = bias[col];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wr * 32 + i * 16 + 4 * (lane >> 4) + r;
                if (row >= M) continue;
                const float v = gelu_f(acc[i][j][r] + bv);
                if (out_mode == 0) {
                    ((__half*)out)[(size_t)row * C + col] = f2h(v);
                } else {
                    const int ch = row / (Ho * Wo), rem = row % (Ho * Wo), oy = rem / Wo, ox = rem % Wo;
                    ((float*)out)[(((size_t)ch * Wo + ox) * C + col) * Ho + oy] = v;
                }
            }
        }
    }
}

// conv 3×3 stride 2 pad 1 as an implicit GEMM on v_mfma_f32_16x16x32_f16: rows = output positions (chunk, oy, ox),
// columns = output channels, K = (tap, input channel) with channel-last f16 activations so each (position, tap)
// contributes one contiguous 2·BK-byte run.  Tile 256 positions × 160 channels (C = 480: three column tiles, so
// each gathered activation panel is re-read 3×, not 5× as with 96-channel tiles — the kernel is bound by these
// L2/Infinity-Cache re-reads, ≈120 GB per C4 step at 96×128), 8 waves of 64×80, K step 96 (three 32-deep MFMA
// slices), one LDS buffer (78 KB) refilled from a register prefetch of the next step between two barriers, and
// unconditional clamped staging loads (padding taps and tails zeroed by masks at the LDS write).  128×96 → 128×160 →
// 256×160: 20.6 → 16.1 → 15.0 ms per C4 step.  LDS image: 192-B rows (no pad), 16-B chunk c of row r at chunk
// c ^ ((r >> 1) & 3): every ds_read_b128 fragment lane group ({0–3,12–15,20–27}, … — MI355X_MICROARCH.md §LDS) and
// every ds_write_b128 8-lane group hits distinct banks (the previous 208-B padded rows were 2-way on both; r2 PMC:
// 3.6 conflict cycles per LDS instruction).  Two LDS buffers (156 KB, one workgroup per CU as the 216 VGPRs allow
// anyway): step st+1's registers go into the other buffer right after step st's MFMAs, so one barrier per step
// instead of two; the MFMA order is unchanged (same bits).
// Tile order: the ⌈C/160⌉ column tiles of one position tile are consecutive logical tiles, and logical tiles are
// dealt to the XCDs in contiguous ranges (workgroup b runs on XCD b mod 8), so the column tiles that gather the same
// activation panel run side by side behind one L2 instead of on three XCDs that each fetch it.
#ifndef QASR_CONV_XCD
#define QASR_CONV_XCD 1
#endif
constexpr int CV_BM = 256, CV_BN = 160, CV_BK = 96, CV_LD = CV_BK, CV_TJ = CV_BN / 32, CV_NT = 512;
__device__ __forceinline__ int cv_swz(int row) { return (row >> 1) & 3; }
constexpr int CV_ACH = CV_BM * (CV_BK / 8) / CV_NT;                  // 6 A chunks of 16 B per thread
constexpr int CV_BCH = (CV_BN * (CV_BK / 8) + CV_NT - 1) / CV_NT;            // B chunks per thread (last partial)

__global__ __launch_bounds__(CV_NT) void k_conv3x3_gelu(const __half* __restrict__ in, int n_chunks, int Hi, int Wi,
                                                      const __half* __restrict__ w, const float* __restrict__ bias,
                                                      int C, void* __restrict__ out, int out_mode) {
    __shared__ __attribute__((aligned(16))) _Float16 As[2][CV_BM * CV_LD];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[2][CV_BN * CV_LD];
    const int Ho = (Hi + 1) / 2, Wo = (Wi + 1) / 2;
    const int M = n_chunks * Ho * Wo;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int nct = (C + CV_BN - 1) / CV_BN;
#if QASR_CONV_XCD
    const int total = gridDim.x, xcd = blockIdx.x % 8, q = total / 8, r = total % 8;
    const int t = xcd * q + min(xcd, r) + blockIdx.x / 8;   // a bijection: XCD x holds q (+1 if x < r) tiles
#else
    const int t = blockIdx.x;
#endif
    const int n0 = (t % nct) * CV_BN, m0 = (t / nct) * CV_BM;
    constexpr int SEG = CV_BK / 8;   // 16-byte chunks per row per step
    // per staged A chunk: its output position, decoded once
    int a_base[CV_ACH], a_oy[CV_ACH], a_ox[CV_ACH];
    bool a_in[CV_ACH];
#pragma unroll
    for (int c = 0; c < CV_ACH; c++) {
        const int ch = tid + CV_NT * c, row = m0 + ch / SEG;
        a_in[c] = row < M;
        const int rr = min(row, M - 1);
        const int chn = rr / (Ho * Wo), rem = rr % (Ho * Wo);
        a_oy[c] = rem / Wo;
        a_ox[c] = rem % Wo;
        a_base[c] = chn * Hi;
    }
    const int kper = C / CV_BK, steps = 9 * kper;
    v4f acc[4][CV_TJ];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < CV_TJ; j++) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

    int4 ra[CV_ACH], rb[CV_BCH];
    unsigned oka = 0, okb = 0;
    auto gload = [&](int st) {
        const int tap = st / kper, ci0 = (st % kper) * CV_BK;
        const int ky = tap / 3, kx = tap % 3;
        oka = 0;
#pragma unroll
        for (int c = 0; c < CV_ACH; c++) {
            const int ch = tid + CV_NT * c, seg = ch % SEG;
            const int iy = 2 * a_oy[c] - 1 + ky, ix = 2 * a_ox[c] - 1 + kx;
            const bool ok = a_in[c] && iy >= 0 && iy < Hi && ix >= 0 && ix < Wi;
            oka |= (unsigned)ok << c;
            const int iyc = min(max(iy, 0), Hi - 1), ixc = min(max(ix, 0), Wi - 1);
            ra[c] = *(const int4*)(in + (((size_t)a_base[c] + iyc) * Wi + ixc) * C + ci0 + seg * 8);
        }
        okb = 0;
#pragma unroll
        for (int c = 0; c < CV_BCH; c++) {
            const int ch = tid + CV_NT * c, row = ch / SEG, seg = ch % SEG;
            const bool ok = ch < CV_BN * SEG && n0 + row < C;
            okb |= (unsigned)ok << c;
            const int co = min(n0 + row, C - 1);
            rb[c] = *(const int4*)(w + ((size_t)co * 9 + tap) * C + ci0 + seg * 8);
        }
    };
    auto masked = [](int4 v, unsigned ok) {
        const int mk = -(int)(ok & 1u);
        return make_int4(v.x & mk, v.y & mk, v.z & mk, v.w & mk);
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int c = 0; c < CV_ACH; c++) {
            const int ch = tid + CV_NT * c;
            *(int4*)(&As[buf][(ch / SEG) * CV_LD + ((ch % SEG) ^ cv_swz(ch / SEG)) * 8]) = masked(ra[c], oka >> c);
        }
#pragma unroll
        for (int c = 0; c < CV_BCH; c++) {
            const int ch = tid + CV_NT * c;
            if (ch < CV_BN * SEG)
                *(int4*)(&Bs[buf][(ch / SEG) * CV_LD + ((ch % SEG) ^ cv_swz(ch / SEG)) * 8]) = masked(rb[c], okb >> c);
        }
    };
    const int fr = lane & 15, kg = lane >> 4;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int st = 0; st < steps; st++) {
        gload(min(st + 1, steps - 1));   // unconditional (the last one is a harmless repeat)
        const _Float16* as = As[st & 1];
        const _Float16* bs = Bs[st & 1];
#pragma unroll
        for (int ks = 0; ks < CV_BK / 32; ks++) {
            v8h a[4], b[CV_TJ];
            // fragment rows are fr + multiples of 16, so their swizzle is cv_swz(fr)
            const int fo = ((ks * 4 + kg) ^ cv_swz(fr)) * 8;
#pragma unroll
            for (int i = 0; i < 4; i++) a[i] = *(const v8h*)(as + (wr * 64 + i * 16 + fr) * CV_LD + fo);
#pragma unroll
            for (int j = 0; j < CV_TJ; j++) b[j] = *(const v8h*)(bs + (wc * 16 * CV_TJ + j * 16 + fr) * CV_LD + fo);
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < CV_TJ; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        // buffer (st+1)&1 was last read in step st−1, which every wave finished before the previous barrier
        if (st + 1 < steps) lstore((st + 1) & 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j < CV_TJ; j++) {
            const int col = n0 + wc * 16 * CV_TJ + j * 16 + fr;
            if (col >= C) continue;
            const float bv = bias[col];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
                if (row >= M) continue;
                const float v = gelu_f(acc[i][j][r] + bv);
                if (out_mode == 0) {
                    ((__half*)out)[(size_t)row * C + col] = f2h(v);
                } else {
                    const int ch = row / (Ho * Wo), rem = row % (Ho * Wo), oy = rem / Wo, ox = rem % Wo;
                    ((float*)out)[(((size_t)ch * Wo + ox) * C + col) * Ho + oy] = v;
                }
            }
        }
    }
}

// The same implicit GEMM (same tile 256 × 160, same 8 waves of 64×80, same MFMA order → the same bits) with the
// operands staged global → LDS by LDS-DMA (`global_load_lds_dwordx4`) into a 6-deep ring of K-32 stages instead of
// through registers and ds_write_b128 into two K-96 buffers, and the fragments in two register sets.  Round 5 PMC of
// the register-staged kernel: MFMA busy 0.25 with every LDS and fetch rate far below its ceiling — its per-step
// phases (gathered loads landing, 78 ds_write_b128 per workgroup at 13 cycles each — MI355X_MICROARCH.md §LDS — then
// the fragment reads after the barrier, then the MFMAs) ran one after another.
//  * A stage is K = 32 (one tap, 32 input channels): A [256][64 B] (16 pieces of 16 rows × 4 lanes) and B [160][64 B]
//    (10 pieces); waves 0–7 take A pieces 2w, 2w+1 and B piece w, waves 0–1 also B pieces 8, 9.
//  * Padding taps and rows past M load 16 zero bytes from `g_conv_zero` (the DMA cannot mask).
//  * Stage s+1's fragment reads are issued right after stage s's barrier, before stage s's MFMAs (which use the
//    other register set), so the LDS reads overlap the matrix work.
//  * LDS image: 64-B rows, 16-B chunk c of row r at chunk c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}: the four 16-lane
//    groups of every ds_read_b128 fragment read ({0–3,12–15,20–27}, …) then touch 16 distinct 4-bank units
//    (checked exhaustively for rows 16k + fr); the DMA's lane-linear 1-KB writes are conflict-free by construction.
// QASR_CONV_BK=64 (A/B): K-64 stages (128-B rows: whole cache lines per gathered row), a 3-deep ring, both K-32
// slices of a stage read after its barrier (the second under the first's MFMAs); LDS image 16-B chunk c of row r at
// c ^ ((r >> 1) & 7), conflict-free for the same fragment reads.
constexpr int CD_NBUF32 = 6;   // K-32: 6 × 26 KB = 159,744 B of LDS: one workgroup (8 waves, 2 per SIMD) per CU
constexpr int CD_NBUF64 = 3;   // K-64: 3 × 52 KB
__device__ __forceinline__ int cd_swz32(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int cd_swz64(int row) { return (row >> 1) & 7; }
__device__ __attribute__((aligned(16))) int4 g_conv_zero[1];
// f(integral_constant<int, U>) for U = 0 … N-1, each call its own code (compile-time ring slot and register set)
template <int... U, class F>
__device__ __forceinline__ void cd_unroll(std::integer_sequence<int, U...>, F&& f) {
    (f(std::integral_constant<int, U>{}), ...);
}

template <int BK, int NBUF, int NW = 8>
__global__ __launch_bounds__(NW * 64) void k_conv3x3_gelu_dma(const __half* __restrict__ in, int n_chunks, int Hi,
                                                          int Wi, const __half* __restrict__ w,
                                                          const float* __restrict__ bias, int C,
                                                          void* __restrict__ out, int out_mode) {
    static_assert(BK == 32 || BK == 64, "conv stage K");
    // NW waves as (NW/2) × 2 of 64×80: BM = 32·NW positions (8 waves: 256, one workgroup per CU)
    constexpr int BM = 32 * NW;
    constexpr int ROWB = BK * 2, OB = BM * ROWB, STAGE = (BM + CV_BN) * ROWB;
    static_assert(NBUF * STAGE <= 163840, "conv ring exceeds LDS");
    constexpr int RW = BK / 8, RPP = 64 / RW;            // lanes per row, rows per 1-KB piece
    constexpr int PA = BM / RPP, PB = CV_BN / RPP;   // pieces per stage: 16 + 10 (K-32, 8 waves), 32 + 20 (K-64)
    constexpr int AW = PA / NW, BW = PB / NW, BX = PB - NW * BW;   // per wave: AW A, BW B (+1 for waves < BX)
    static_assert(AW * NW == PA && BX < NW, "conv pieces");
    constexpr int KS = BK / 32;                          // K-32 MFMA slices per stage
    constexpr bool PIPE = BK == 32;                      // cross-stage fragment prefetch (two register sets)
    auto swz = [](int r) { return BK == 32 ? cd_swz32(r) : cd_swz64(r); };
    __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];
    const int Ho = (Hi + 1) / 2, Wo = (Wi + 1) / 2;
    const int M = n_chunks * Ho * Wo;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int nct = (C + CV_BN - 1) / CV_BN;
#if QASR_CONV_XCD
    const int total = gridDim.x, xcd = blockIdx.x % 8, q = total / 8, r8 = total % 8;
    const int t = xcd * q + min(xcd, r8) + blockIdx.x / 8;
#else
    const int t = blockIdx.x;
#endif
    const int n0 = (t % nct) * CV_BN, m0 = (t / nct) * BM;
    const int steps = 9 * (C / BK);
    // this lane's DMA sources: A pieces AW·w + u (row RPP·p + lane/RW, 16-B slot lane%RW ← chunk slot ^ swz(row)):
    // the address of its tap-(0, 0) pixel (never read when that tap is padding) and a 9-bit mask of the taps that
    // are inside the image — a stage then adds one wave-uniform offset and tests one bit
    const __half* a_ptr[AW];
    unsigned a_ok[AW];
#pragma unroll
    for (int u = 0; u < AW; u++) {
        const int row = RPP * (AW * wave + u) + lane / RW, pos = m0 + row;
        const int rr = min(pos, M - 1), chn = rr / (Ho * Wo), rem = rr % (Ho * Wo);
        const int iy0 = 2 * (rem / Wo) - 1, ix0 = 2 * (rem % Wo) - 1;
        unsigned ok = 0;
#pragma unroll
        for (int tp = 0; tp < 9; tp++)
            ok |= (unsigned)(pos < M && (unsigned)(iy0 + tp / 3) < (unsigned)Hi && (unsigned)(ix0 + tp % 3) < (unsigned)Wi)
                  << tp;
        a_ok[u] = ok;
        a_ptr[u] = in + (size_t)chn * Hi * Wi * C + (ptrdiff_t)(iy0 * Wi + ix0) * C + 8 * ((lane % RW) ^ swz(row));
    }
    const bool bx = wave < BX;   // this wave takes an extra B piece (wave-uniform)
    const __half* b_src[BW + 1];
    uint32_t b_dst[BW + 1];
#pragma unroll
    for (int u = 0; u <= BW; u++) {
        const int p = u < BW ? BW * wave + u : min(NW * BW + wave, PB - 1), row = RPP * p + lane / RW;
        const int co = min(n0 + row, C - 1);
        b_src[u] = w + (size_t)co * 9 * C + 8 * ((lane % RW) ^ swz(row));
        b_dst[u] = OB + 1024 * p;
    }
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const uint32_t wa = __builtin_amdgcn_readfirstlane(lds0 + 1024 * AW * wave);
    uint32_t wb[BW + 1];
#pragma unroll
    for (int u = 0; u <= BW; u++) wb[u] = __builtin_amdgcn_readfirstlane(lds0 + b_dst[u]);
    // stages are issued strictly in order: (tap, ci0) of the next one advance by counters, no division
    int it_ky = 0, it_kx = 0, it_tap = 0, it_ci = 0;
    // piece q of the next stage's DMAs: q < AW the A pieces, then BW B pieces, then the extra B piece (waves < BX)
    constexpr int NPQ = AW + BW + (BX > 0 ? 1 : 0);
    auto issue_piece = [&](int buf, int q) __attribute__((always_inline)) {
        const uint32_t so = buf * STAGE;
        if (q < AW) {
            const int aoff = (it_ky * Wi + it_kx) * C + it_ci;   // wave-uniform
            const bool ok = (a_ok[q] >> it_tap) & 1u;
            dma_lds16(ok ? (const void*)(a_ptr[q] + aoff) : (const void*)g_conv_zero, wa + so + 1024 * q);
        } else if (q < AW + BW) {
            dma_lds16(b_src[q - AW] + (it_tap * C + it_ci), wb[q - AW] + so);
        } else if (bx) {
            dma_lds16(b_src[BW] + (it_tap * C + it_ci), wb[BW] + so);
        }
    };
    auto advance = [&]() __attribute__((always_inline)) {
        it_ci += BK;
        if (it_ci == C) {
            it_ci = 0;
            it_tap++;
            it_kx++;
            if (it_kx == 3) {
                it_kx = 0;
                it_ky++;
            }
        }
    };
    auto issue = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < NPQ; q++) issue_piece(buf, q);
        advance();
    };
    const int fr = lane & 15, kg = lane >> 4;
    v4f acc[4][CV_TJ];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < CV_TJ; j++) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
    // (waves whose rows all lie past M compute on the clamped rows too; their results are not stored)
    constexpr int NSET = PIPE ? 2 : KS;
    v8h fa[NSET][4], fb[NSET][CV_TJ];
    auto frags = [&](int set, int buf, int ks) __attribute__((always_inline)) {
        const char* st = smem + buf * STAGE;
        const int fo = 16 * ((4 * ks + kg) ^ swz(fr));   // fragment rows are fr + multiples of 16
#pragma unroll
        for (int i = 0; i < 4; i++) fa[set][i] = *(const v8h*)(st + (wr * 64 + i * 16 + fr) * ROWB + fo);
#pragma unroll
        for (int j = 0; j < CV_TJ; j++)
            fb[set][j] = *(const v8h*)(st + OB + (wc * 16 * CV_TJ + j * 16 + fr) * ROWB + fo);
    };
    auto mfmas = [&](int set) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < CV_TJ; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[set][i], fb[set][j], acc[i][j], 0, 0, 0);
    };
    constexpr int NPW = AW + BW;   // DMAs per wave per stage (+1 on waves < BX)
    auto wait_ahead = [&](int ahead) __attribute__((always_inline)) {   // at most `ahead` of this wave's stages still in flight, LDS reads done
        if (BX > 0 && bx) wait_stages<NPW + 1, NBUF>(ahead);
        else wait_stages<NPW, NBUF>(ahead);
    };
    if constexpr (PIPE) {
        // the ring's NBUF stages are all issued up front; stage s frees its buffer for stage s + NBUF
#pragma unroll
        for (int s = 0; s < NBUF; s++)
            if (s < steps) issue(s);
        wait_ahead(min(NBUF - 1, steps - 1));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        frags(0, 0, 0);
        // one stage: this wave's DMAs of stage s+1 have landed and its reads of stage s are done (lgkmcnt(0)); the
        // barrier makes both true for every wave — stage s+1 is readable, stage s's buffer is free for stage s + NBUF.
        // The next stage's fragment reads are unconditional (past the last stage they re-read a stale buffer, unused):
        // a conditional read would make the compiler's own lgkmcnt wait before the MFMAs a full drain.
        auto stage = [&](int s, auto ubc) __attribute__((always_inline)) {
            constexpr int ub = decltype(ubc)::value;
            wait_ahead(max(0, min(NBUF - 2, steps - 2 - s)));
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            // (this order: the fragment reads after the DMA issue keep the kernel at 205 VGPRs; reads first spilled 5)
            if (s + NBUF < steps) issue(ub % NBUF);
            frags((ub + 1) & 1, (ub + 1) % NBUF, 0);
            mfmas(ub & 1);
        };
        // two ring trips per loop trip, so every unrolled stage's ring slot and register set are constants; the last
        // partial trip is a guarded copy
        constexpr int TRIP = 2 * NBUF;
        const int full = steps / TRIP * TRIP;
        for (int s0 = 0; s0 < full; s0 += TRIP)
            cd_unroll(std::make_integer_sequence<int, TRIP>{}, [&](auto u) { stage(s0 + u.value, u); });
        cd_unroll(std::make_integer_sequence<int, TRIP>{}, [&](auto u) {
            if (full + u.value < steps) stage(full + u.value, u);
        });
    } else {
        // NBUF-1 stages in flight; stage s's barrier frees stage s-1's buffer for stage s + NBUF - 1
        constexpr int D = NBUF - 1;
#pragma unroll
        for (int s = 0; s < D; s++)
            if (s < steps) issue(s);
        auto stage = [&](int s, auto ubc) __attribute__((always_inline)) {
            constexpr int ub = decltype(ubc)::value;
            wait_ahead(max(0, min(D - 1, steps - 1 - s)));
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (s + D < steps) issue((ub + D) % NBUF);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) frags(ks, ub, ks);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) mfmas(ks);
        };
        const int full = steps / NBUF * NBUF;
        for (int s0 = 0; s0 < full; s0 += NBUF)
            cd_unroll(std::make_integer_sequence<int, NBUF>{}, [&](auto u) { stage(s0 + u.value, u); });
        cd_unroll(std::make_integer_sequence<int, NBUF>{}, [&](auto u) {
            if (full + u.value < steps) stage(full + u.value, u);
        });
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int j = 0; j < CV_TJ; j++) {
            const int col = n0 + wc * 16 * CV_TJ + j * 16 + fr;
            if (col >= C) continue;
            const float bv = bias[col];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
                if (row >= M) continue;
                const float v = gelu_f(acc[i][j][r] + bv);
                if (out_mode == 0) {
                    ((__half*)out)[(size_t)row * C + col] = f2h(v);
                } else {
                    const int ch = row / (Ho * Wo), rem = row % (Ho * Wo), oy = rem / Wo, ox = rem % Wo;
                    ((float*)out)[(((size_t)ch * Wo + ox) * C + col) * Ho + oy] = v;
                }
            }
        }
    }
}

void conv3x3_gelu(const __half* in, int n_chunks, int Hi, int Wi, const __half* w, const float* b, int C, void* out,
                  int out_mode, hipStream_t s) {
    const int M = n_chunks * ((Hi + 1) / 2) * ((Wi + 1) / 2);
    if (M <= 0) return;
    QASR_CHECK(C % 32 == 0, QASR_E_INVALID, "conv channels must be a multiple of 32");
    ProfScope ps(s, "conv3x3_f16", 2.0 * M * C * 9.0 * C, (double)M * 9 * C * 2 / 4 + (double)M * C * 2);
    // QASR_CONV_DMA=0: the register-staged kernel (A/B; same bits)
    static const bool dma = !(getenv("QASR_CONV_DMA") && atoi(getenv("QASR_CONV_DMA")) == 0);
    static const int bk = getenv("QASR_CONV_BK") ? atoi(getenv("QASR_CONV_BK")) : 32;
    const int grid = cdiv(C, CV_BN) * cdiv(M, CV_BM);
    if (C % CV_BK == 0 && dma && bk == 64 && C % 64 == 0) {
        k_conv3x3_gelu_dma<64, CD_NBUF64><<<grid, CV_NT, 0, s>>>(in, n_chunks, Hi, Wi, w, b, C, out, out_mode);
    } else if (C % CV_BK == 0 && dma) {
        k_conv3x3_gelu_dma<32, CD_NBUF32><<<grid, CV_NT, 0, s>>>(in, n_chunks, Hi, Wi, w, b, C, out, out_mode);
    } else if (C % CV_BK == 0) {
        k_conv3x3_gelu<<<cdiv(C, CV_BN) * cdiv(M, CV_BM), CV_NT, 0, s>>>(in, n_chunks, Hi, Wi, w, b, C, out, out_mode);
    } else {
        dim3 grid(cdiv(C, CT), cdiv(M, CT));
        k_conv3x3_gelu_c32<<<grid, 256, 0, s>>>(in, n_chunks, Hi, Wi, w, b, C, out, out_mode);
    }
}

__global__ void k_reorder_conv(const __half* __restrict__ src, int cout, int cin, __half* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)cout * cin * 9) return;
    const int ci = (int)(i % cin), k = (int)((i / cin) % 9), co = (int)(i / ((int64_t)cin * 9));
    dst[i] = src[((size_t)co * cin + ci) * 9 + k];
}

void reorder_conv_weight(const __half* src, int cout, int cin, __half* dst, hipStream_t s) {
    const int64_t n = (int64_t)cout * cin * 9;
    k_reorder_conv<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(src, cout, cin, dst);
}

// ================================================================================================ FireRedVAD
// One wave per 400-sample frame: DC removal, pre-emphasis 0.97, Povey window, zero-pad to 512, in-LDS
// radix-2 FFT (bit-reversed load, 9 butterfly stages, 4 butterflies per lane), power, 80 Kaldi mel bins,
// natural log floored at FLT_EPSILON (kaldi-native-fbank 1.22.3 defaults, firered_vad.py:65-72).
__global__ __launch_bounds__(256) void k_kaldi_fbank(const float* __restrict__ pcm, int T,
                                                     const float* __restrict__ win, const float* __restrict__ banks,
                                                     float* __restrict__ feats) {
    __shared__ float sre[4][512];
    __shared__ float sim[4][512];
    __shared__ float tw[2][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 256; i += 256) {
        float sv, cv;
        sincospif((float)i / 256.0f, &sv, &cv);   // exp(-2πi·i/512) = cos(π i/256) - i sin(π i/256)
        tw[0][i] = cv;
        tw[1][i] = -sv;
    }
    __syncthreads();
    const int t = blockIdx.x * 4 + w;
    if (t >= T) return;
    float* re = sre[w];
    float* im = sim[w];
    const float* x = pcm + (size_t)t * 160;
    float v[7];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 7; j++) {
        const int i = lane + 64 * j;
        v[j] = i < 400 ? x[i] : 0.f;
        sum += v[j];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float mean = sum / 400.f;
#pragma unroll
    for (int j = 0; j < 7; j++) {
        const int i = lane + 64 * j;
        if (i < 400) re[i] = v[j] - mean;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float y[7];
#pragma unroll
    for (int j = 0; j < 7; j++) {
        const int i = lane + 64 * j;
        if (i < 400) {
            const float cur = re[i];
            const float prev = i > 0 ? re[i - 1] : cur;
            y[j] = (cur - 0.97f * prev) * win[i];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int i = lane + 64 * j;
        const int r = (int)(__brev((unsigned)i) >> 23);   // 9-bit reversal
        re[r] = (j < 7 && i < 400) ? y[j] : 0.f;
        im[r] = 0.f;
    }
    for (int half = 1; half < 512; half <<= 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int tstride = 256 / half;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int bf = lane + 64 * j;              // butterfly 0..255
            const int grp = bf / half, k = bf % half;
            const int i0 = grp * 2 * half + k, i1 = i0 + half;
            const float wr = tw[0][k * tstride], wi = tw[1][k * tstride];
            const float xr = re[i1] * wr - im[i1] * wi;
            const float xi = re[i1] * wi + im[i1] * wr;
            const float ur = re[i0], ui = im[i0];
            re[i0] = ur + xr; im[i0] = ui + xi;
            re[i1] = ur - xr; im[i1] = ui - xi;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float pw[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int i = lane + 64 * j;
        pw[j] = re[i] * re[i] + im[i] * im[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 4; j++) re[lane + 64 * j] = pw[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int m = lane; m < 80; m += 64) {
        float e = 0.f;
        const float* bk = banks + m * 256;
        for (int i = 0; i < 256; i++) e += bk[i] * re[i];
        feats[(size_t)t * 80 + m] = logf(fmaxf(e, 1.1920928955078125e-07f));
    }
}

void kaldi_fbank(const float* pcm, int64_t n, int T, const float* window, const float* banks, float* feats,
                 hipStream_t s) {
    (void)n;
    if (T <= 0) return;
    k_kaldi_fbank<<<cdiv(T, 4), 256, 0, s>>>(pcm, T, window, banks, feats);
}

__global__ void k_cmvn(const float* __restrict__ x, int T, const float* __restrict__ mean,
                       const float* __restrict__ istd, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)T * 80) return;
    const int c = (int)(i % 80);
    y[i] = (x[i] - mean[c]) * istd[c];
}

void cmvn(const float* x, int T, const float* mean, const float* istd, float* y, hipStream_t s) {
    const int64_t n = (int64_t)T * 80;
    if (n <= 0) return;
    k_cmvn<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(x, T, mean, istd, y);
}

// y[T][N] = act(x[T][K]·W[K][N] + b): 64×64 tile, 16-deep K slabs in LDS, 4×4 outputs per thread
__global__ __launch_bounds__(256) void k_dense_f32(const float* __restrict__ x, int T, int K,
                                                   const float* __restrict__ W, const float* __restrict__ b, int N,
                                                   int relu, float* __restrict__ y) {
    __shared__ float xs[16][65];
    __shared__ float ws[16][64];
    const int tid = threadIdx.x;
    const int t0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const int tr = (tid / 16) * 4, tc = (tid % 16) * 4;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 16) {
        for (int i = tid; i < 16 * 64; i += 256) {
            const int r = i / 16, kk = i % 16;   // x tile: 64 rows × 16 k
            const int tt = t0 + r, k = k0 + kk;
            xs[kk][r] = (tt < T && k < K) ? x[(size_t)tt * K + k] : 0.f;
            const int kr = i / 64, nn = i % 64;  // W tile: 16 k × 64 n
            ws[kr][nn] = (k0 + kr < K && n0 + nn < N) ? W[(size_t)(k0 + kr) * N + n0 + nn] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; kk++) {
            float a[4], bb[4];
#pragma unroll
            for (int i = 0; i < 4; i++) a[i] = xs[kk][tr + i];
#pragma unroll
            for (int j = 0; j < 4; j++) bb[j] = ws[kk][tc + j];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] += a[i] * bb[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int tt = t0 + tr + i;
        if (tt >= T) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int nn = n0 + tc + j;
            if (nn >= N) continue;
            float v = acc[i][j] + (b ? b[nn] : 0.f);
            if (relu) v = fmaxf(v, 0.f);
            y[(size_t)tt * N + nn] = v;
        }
    }
}

void dense_f32(const float* x, int T, int K, const float* W, const float* b, int N, int relu, float* y, hipStream_t s) {
    if (T <= 0) return;
    dim3 grid(cdiv(N, 64), cdiv(T, 64));
    k_dense_f32<<<grid, 256, 0, s>>>(x, T, K, W, b, N, relu, y);
}

__global__ void k_fsmn(const float* __restrict__ x, int T, const float* __restrict__ lb, const float* __restrict__ la,
                       const float* __restrict__ skip, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)T * 128) return;
    const int c = (int)(i % 128);
    const int t = (int)(i / 128);
    float ab = 0.f, aa = 0.f;
#pragma unroll
    for (int j = 0; j < 20; j++) {
        const int k = t + j - 19;
        if (k >= 0) ab += lb[c * 20 + j] * x[(size_t)k * 128 + c];
    }
    if (t < T - 1) {
#pragma unroll
        for (int j = 0; j < 20; j++) {
            const int k = t + 1 + j;
            if (k < T) aa += la[c * 20 + j] * x[(size_t)k * 128 + c];
        }
    }
    float v = x[i] + ab;
    v = v + aa;
    if (skip) v += skip[i];
    y[i] = v;
}

void fsmn_block(const float* x, int T, const float* lb, const float* la, const float* skip, float* y, hipStream_t s) {
    const int64_t n = (int64_t)T * 128;
    if (n <= 0) return;
    k_fsmn<<<(unsigned)cdiv64(n, 256), 256, 0, s>>>(x, T, lb, la, skip, y);
}

__global__ __launch_bounds__(256) void k_vad_head(const float* __restrict__ h, int T, const float* __restrict__ wo,
                                                  float bo, float* __restrict__ probs) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= T) return;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j++) acc += h[(size_t)t * 256 + lane + 64 * j] * wo[lane + 64 * j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) probs[t] = 1.f / (1.f + expf(-(acc + bo)));
}

void vad_head(const float* h, int T, const float* wo, float bo, float* probs, hipStream_t s) {
    if (T <= 0) return;
    k_vad_head<<<cdiv(T, 4), 256, 0, s>>>(h, T, wo, bo, probs);
}

}  // namespace qasr
