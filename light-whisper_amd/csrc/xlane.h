// Cross-lane reductions on DPP (VALU; no LDS round trip like the ds_bpermute behind __shfl_xor), gfx950 wave64.
// xor 1 / xor 2 = quad_perm, the 8- and 16-lane halves = row_half_mirror / row_mirror (a mirror pairs lane i with a
// lane of the other half, which is all a symmetric reduction needs; semantics pinned by tools/micro/xlane_check.hip);
// the four 16-lane row totals are combined through v_readlane, so wave results are wave-uniform.  Every lane of the
// groups involved must be active.
#pragma once
#include <hip/hip_runtime.h>

namespace qasr {

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// over aligned groups of 8 / 16 lanes, result in every lane of the group
__device__ __forceinline__ float sum8(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    return v + dpp<0x141>(v);
}
__device__ __forceinline__ float max8(float v) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    return fmaxf(v, dpp<0x141>(v));
}
__device__ __forceinline__ float max16(float v) {
    v = max8(v);
    return fmaxf(v, dpp<0x140>(v));
}
// whole wave, wave-uniform result
__device__ __forceinline__ float wave_sum(float v) {
    v = sum8(v);
    v += dpp<0x140>(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
    v = max16(v);
    return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

}  // namespace qasr
