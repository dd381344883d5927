// Device-resident continuous-batching state for greedy decode.  Each step is planned, run and accepted on the
// device, so the host only launches (one hipGraph per row bucket) and reads back the number of rows still
// active, one step late, to pick the next bucket.  Mirrors the host loop of the reference server's
// session.run (one utterance) for a batch: a row finishes at EOS (natural mode) or when its budget is spent.
#include "kernels.h"
#include "rowops.h"

namespace qasr {

// one workgroup: compact the not-done utterances into rows [0, M), pad rows [M, M_max) with a harmless dummy
// (token 0 at position 0 writing / reading only the dummy KV slot), zero the active counter for accept
// EMBED (small steps, dec_plan_embed): the same workgroup then writes the step's input rows — token embeddings of
// the planned ids, k_embed_rows' arithmetic — after a barrier, instead of a second launch
template <bool EMBED>
__global__ __launch_bounds__(1024) void k_dec_plan(DecState st, int M_max, int* __restrict__ ids,
                                                   int* __restrict__ pos, int* __restrict__ slot,
                                                   int* __restrict__ kvs, int* __restrict__ kvl,
                                                   int* __restrict__ row_utt, const int8_t* __restrict__ eqs,
                                                   const __half* __restrict__ esc, int K, float* __restrict__ x) {
    __shared__ int part[1024];
    const int U = st.params[0], dummy = st.params[1];
    const int per = (U + 1023) / 1024;
    const int u0 = threadIdx.x * per, u1 = min(U, u0 + per);
    int c = 0;
    for (int u = u0; u < u1; u++) c += st.done[u] ? 0 : 1;
    part[threadIdx.x] = c;
    __syncthreads();
    // Hillis-Steele inclusive scan over 1024 partial counts
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int r = part[threadIdx.x] - c;
    for (int u = u0; u < u1; u++) {
        if (st.done[u]) continue;
        if (r < M_max) {
            const int p = st.n_prompt[u] + st.gen[u] - 1;
            ids[r] = st.last_tok[u];
            pos[r] = p;
            slot[r] = st.base[u] + p;
            kvs[r] = st.base[u];
            kvl[r] = p + 1;
            row_utt[r] = u;
        }
        r++;
    }
    const int M = part[1023];
    for (int i = M + threadIdx.x; i < M_max; i += 1024) {
        ids[i] = 0;
        pos[i] = 0;
        slot[i] = dummy;
        kvs[i] = dummy;
        kvl[i] = 1;
        row_utt[i] = -1;
    }
    if (threadIdx.x == 0) {
        st.counters[0] = min(M, M_max);   // rows of this step
        st.counters[1] = 0;               // active after accept
        if (M > M_max) st.counters[2] = 1;  // bound violated (the host checks)
    }
    if constexpr (EMBED) {
        __threadfence_block();
        __syncthreads();
        const int nb = K / QK;
        for (int i = threadIdx.x; i < M_max * nb; i += 1024) {
            const int r = i / nb, b = i % nb;
            dequant_block_q8(eqs, esc, K, ids[r], b, x + (size_t)r * K + b * QK);
        }
    }
}

__device__ __forceinline__ void accept_row(const DecState& st, int u, int t) {
    const int forced = st.params[2], eos0 = st.params[3], eos1 = st.params[4], ld = st.params[5];
    int still = 0;
    if (!forced && (t == eos0 || t == eos1)) {
        st.done[u] = 1;
    } else {
        const int g = st.gen[u];
        st.out[(size_t)u * ld + g] = t;
        st.gen[u] = g + 1;
        st.last_tok[u] = t;
        if (g + 1 >= st.budget[u]) st.done[u] = 1;
        else still = 1;
    }
    if (still) atomicAdd(&st.counters[1], 1);
}

__global__ void k_dec_accept(DecState st, int M_max, const int* __restrict__ row_utt, const int* __restrict__ tok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M_max || i >= st.counters[0]) return;
    const int u = row_utt[i];
    if (u < 0) return;
    accept_row(st, u, tok[i]);
}

// argmax_rows' second stage fused with k_dec_accept (one launch fewer per decode step): wave i reduces row i's
// kArgParts keys (max is order-free: the same token as k_argmax_final) and lane 0 stores it and accepts it
__global__ __launch_bounds__(256) void k_argmax_accept(DecState st, int M_max,
                                                       const unsigned long long* __restrict__ part,
                                                       const int* __restrict__ row_utt, int* __restrict__ tok) {
    const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= M_max) return;   // whole wave
    unsigned long long k = lane < kArgParts ? part[(size_t)i * kArgParts + lane] : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)k, o), hi = __shfl_xor((unsigned)(k >> 32), o);
        k = max(k, ((unsigned long long)hi << 32) | lo);
    }
    if (lane != 0) return;
    const int t = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
    tok[i] = t;
    if (i >= st.counters[0]) return;
    const int u = row_utt[i];
    if (u >= 0) accept_row(st, u, t);
}

void argmax_accept(const DecState& st, int M_max, const void* part, const int* row_utt, int* tok, hipStream_t s) {
    if (M_max <= 0) return;
    k_argmax_accept<<<cdiv(M_max, 4), 256, 0, s>>>(st, M_max, (const unsigned long long*)part, row_utt, tok);
}

// batched teacher forcing (Session::forced_logits_batch_host): row i's accepted token becomes the forced id of its
// utterance at its next position (ids [U][ld], -1 keeps the argmax); runs between the argmax and k_dec_accept
__global__ void k_force_tokens(DecState st, int M_max, const int* __restrict__ row_utt, const int* __restrict__ ids,
                               int ld, int* __restrict__ tok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M_max || i >= st.counters[0]) return;
    const int u = row_utt[i];
    if (u < 0) return;
    const int g = st.gen[u];
    const int f = g < ld ? ids[(size_t)u * ld + g] : -1;
    if (f >= 0) tok[i] = f;
}

void force_tokens(const DecState& st, int M_max, const int* row_utt, const int* ids, int ld, int* tok, hipStream_t s) {
    if (M_max <= 0) return;
    k_force_tokens<<<cdiv(M_max, 256), 256, 0, s>>>(st, M_max, row_utt, ids, ld, tok);
}

void dec_plan(const DecState& st, int M_max, int* ids, int* pos, int* slot, int* kvs, int* kvl, int* row_utt,
              hipStream_t s) {
    k_dec_plan<false><<<1, 1024, 0, s>>>(st, M_max, ids, pos, slot, kvs, kvl, row_utt, nullptr, nullptr, 0, nullptr);
}

void dec_plan_embed(const DecState& st, int M_max, int* ids, int* pos, int* slot, int* kvs, int* kvl, int* row_utt,
                    const Q8Mat& E, float* x, hipStream_t s) {
    QASR_CHECK(E.K % QK == 0, QASR_E_INVALID, "dec_plan_embed: embedding width");
    k_dec_plan<true><<<1, 1024, 0, s>>>(st, M_max, ids, pos, slot, kvs, kvl, row_utt, E.qs, E.sc, E.K, x);
}

void dec_accept(const DecState& st, int M_max, const int* row_utt, const int* tok, hipStream_t s) {
    if (M_max <= 0) return;
    k_dec_accept<<<cdiv(M_max, 256), 256, 0, s>>>(st, M_max, row_utt, tok);
}

// copy the shared prompt prefix's K/V (P0 slots from `src`, every layer) into each utterance's first slots
__global__ void k_copy_kv_prefix(__half* __restrict__ kc, __half* __restrict__ vc, int64_t kv_slots, int kvd,
                                 int64_t src, int P0, const int* __restrict__ bases) {
    const int u = blockIdx.x, l = blockIdx.y;
    const size_t n = (size_t)P0 * kvd / 8;   // int4 units
    const size_t so = ((size_t)l * kv_slots + src) * kvd, dso = ((size_t)l * kv_slots + bases[u]) * kvd;
    const int4* ks = (const int4*)(kc + so);
    const int4* vs = (const int4*)(vc + so);
    int4* kd = (int4*)(kc + dso);
    int4* vd = (int4*)(vc + dso);
    for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
        kd[i] = ks[i];
        vd[i] = vs[i];
    }
}

void copy_kv_prefix(__half* kc, __half* vc, int layers, int64_t kv_slots, int kvd, int64_t src, int P0,
                    const int* bases, int count, hipStream_t s) {
    if (count <= 0 || P0 <= 0) return;
    QASR_CHECK(kvd % 8 == 0, QASR_E_INVALID, "copy_kv_prefix: kv width must be a multiple of 8");
    k_copy_kv_prefix<<<dim3(count, layers), 256, 0, s>>>(kc, vc, kv_slots, kvd, src, P0, bases);
}

}  // namespace qasr
