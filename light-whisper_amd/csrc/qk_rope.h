// q/k RMS-norm + RoPE of one head (hd 128) held two dims per lane (2·lane, 2·lane+1) by one wave, shared by
// k_qk_norm_rope_row (kernels_nn.hip) and the fused decode attention (kernels_attn.hip).  Written with
// separately rounded operations (the build's -ffp-contract=off keeps them unfused) so that both kernels round identically
// (the fused path is tested bit for bit).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

namespace qasr {

// v: the two raw dims, g: their norm weights, cs: (cos, sin) of the pair indices e0, e0+1 (e0 = 2·lane mod 64),
// lo: 2·lane < 64 (first half of the rotate-half pairing; the partner is lane ^ 32)
__device__ __forceinline__ __half2 norm_rope_hd128(float2 v, float2 g, float4 cs, bool lo, float eps) {
    float ss = __fadd_rn(__fmul_rn(v.x, v.x), __fmul_rn(v.y, v.y));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss = __fadd_rn(ss, __shfl_xor(ss, o));
    const float inv = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(__fdiv_rn(ss, 128.0f), eps)));
    const float a = __fmul_rn(__fmul_rn(v.x, inv), g.x), b = __fmul_rn(__fmul_rn(v.y, inv), g.y);
    const float pa = __shfl_xor(a, 32), pb = __shfl_xor(b, 32);
    const float oa = lo ? __fsub_rn(__fmul_rn(a, cs.x), __fmul_rn(pa, cs.y))
                        : __fadd_rn(__fmul_rn(a, cs.x), __fmul_rn(pa, cs.y));
    const float ob = lo ? __fsub_rn(__fmul_rn(b, cs.z), __fmul_rn(pb, cs.w))
                        : __fadd_rn(__fmul_rn(b, cs.z), __fmul_rn(pb, cs.w));
    return __floats2half2_rn(oa, ob);
}

}  // namespace qasr
