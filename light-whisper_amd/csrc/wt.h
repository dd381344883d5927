// Write-through (sc1) loads and stores for data handed between workgroups of ONE launch (the xr launches' leaf
// split and fused-norm tail, kernels_xr.hip).  MI355X_MICROARCH.md, inter-workgroup visibility, table row 1: every store of the
// handed-off bytes `sc1` (write-through past the XCD's L2), the storing waves' `s_waitcnt vmcnt(0)`, then one lane's
// agent-scope add; the consumer polls with an `sc1` load, passes a workgroup barrier and reads every byte with `sc1`
// loads (L1 bypassed, so a line this CU read before the producer's store is never served stale).  Buffer
// instructions with cache policy 16 (= sc1, checked in the gfx950 disassembly) so the compiler tracks their vmcnt;
// the base pointer must be wave-uniform (it goes into the buffer descriptor's SGPRs), the offset is per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qasr {

typedef int wt_v4i __attribute__((ext_vector_type(4)));
typedef int wt_v2i __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
    // stride 0, 2 GiB of records, the gfx9 default format dword (CK_BUFFER_RESOURCE_3RD_DWORD)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
constexpr int kSc1 = 16;

__device__ __forceinline__ wt_v4i wt_ld16(const void* base, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(wt_rsrc(base), off, 0, kSc1);
}
__device__ __forceinline__ float2 wt_ldf2(const void* base, uint32_t off) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(wt_rsrc(base), off, 0, kSc1));
}
__device__ __forceinline__ float4 wt_ldf4(const void* base, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wt_rsrc(base), off, 0, kSc1));
}
__device__ __forceinline__ float wt_ldf(const void* base, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wt_rsrc(base), off, 0, kSc1));
}
__device__ __forceinline__ void wt_stf(void* base, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), wt_rsrc(base), off, 0, kSc1);
}
__device__ __forceinline__ void wt_st32(void* base, uint32_t off, int32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, wt_rsrc(base), off, 0, kSc1);
}
__device__ __forceinline__ void wt_st16(void* base, uint32_t off, uint16_t v) {
    __builtin_amdgcn_raw_buffer_store_b16(v, wt_rsrc(base), off, 0, kSc1);
}
__device__ __forceinline__ void wt_st128(void* base, uint32_t off, wt_v4i v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, wt_rsrc(base), off, 0, kSc1);
}

}  // namespace qasr
