// Semantics check of cross-lane primitives for the decode attention (DPP quad_perm / mirrors used there; the
// v_permlane16/32_swap builtins, which returned the SAME row-swapped image in both results when given one source
// twice, are printed for reference and not used)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__global__ void k(const float* x, float* out) {
    const int l = threadIdx.x;
    const float v = x[l];
    out[0 * 64 + l] = dpp<0xB1>(v);
    out[1 * 64 + l] = dpp<0x4E>(v);
    out[2 * 64 + l] = dpp<0x141>(v);
    out[3 * 64 + l] = dpp<0x140>(v);
    const auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    out[4 * 64 + l] = __builtin_bit_cast(float, a[0]);
    out[5 * 64 + l] = __builtin_bit_cast(float, a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    out[6 * 64 + l] = __builtin_bit_cast(float, b[0]);
    out[7 * 64 + l] = __builtin_bit_cast(float, b[1]);
}
int main() {
    float h[64], o[8 * 64];
    for (int i = 0; i < 64; i++) h[i] = (float)i;
    float *dx, *dout;
    hipMalloc(&dx, sizeof h);
    hipMalloc(&dout, sizeof o);
    hipMemcpy(dx, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dx, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const char* names[] = {"qp_B1", "qp_4E", "half_mirror", "row_mirror", "pl16[0]", "pl16[1]", "pl32[0]", "pl32[1]"};
    for (int r = 0; r < 8; r++) {
        printf("%-12s", names[r]);
        for (int i = 0; i < 64; i++) printf(" %d", (int)o[r * 64 + i]);
        printf("\n");
    }
    return 0;
}
