// LDS-DMA staging helpers shared by the Q8 / MXFP8 GEMMs and the conv implicit GEMM (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qasr {

// LDS-DMA (global_load_lds): lane i's 16 (4) bytes from its own global address land at LDS byte m0 + 16·i (4·i).
// Issued from inline asm so the compiler does not treat the in-flight DMA as a pending LDS write and drain it
// (vmcnt(0)) before the next ds_read; the kernels count these loads in their own s_waitcnt vmcnt(N).
__device__ __forceinline__ void dma_lds16(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma_lds4(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
// wait until at most ahead·NPW of this wave's DMAs are outstanding (ahead ∈ [0, D))
template <int NPW, int D>
__device__ __forceinline__ void wait_stages(int ahead) {
    static_assert(D <= 8 && NPW * (D - 1) <= 63, "vmcnt range");
    switch (ahead) {
        case 0: wait_vm_lgkm0<0>(); break;
        case 1: wait_vm_lgkm0<NPW * (D > 1 ? 1 : 0)>(); break;
        case 2: wait_vm_lgkm0<NPW * (D > 2 ? 2 : 0)>(); break;
        case 3: wait_vm_lgkm0<NPW * (D > 3 ? 3 : 0)>(); break;
        case 4: wait_vm_lgkm0<NPW * (D > 4 ? 4 : 0)>(); break;
        case 5: wait_vm_lgkm0<NPW * (D > 5 ? 5 : 0)>(); break;
        case 6: wait_vm_lgkm0<NPW * (D > 6 ? 6 : 0)>(); break;
        default: wait_vm_lgkm0<NPW * (D > 7 ? 7 : 0)>(); break;
    }
}

}  // namespace qasr
