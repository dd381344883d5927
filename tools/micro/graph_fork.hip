// Does a hipGraph with two independent branches run them concurrently on gfx950 (ROCm 7.2)?  A chain of n dependent
// latency-bound kernels (each: G workgroups, each workgroup a dependent chain of L global loads — a decode-step
// launch in miniature) captured (a) as one chain of 2n, (b) as two forked chains of n (fork/join with events inside one
// capture).  If the branches overlap, (b) takes about half of (a).
//   hipcc --offload-arch=gfx950 -O3 -o graph_fork graph_fork.hip && ./graph_fork [n] [G] [L]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// a dependent chain of L loads per lane (pointer chasing through a small table), result stored so nothing is dead
__global__ void k_chain(const int* __restrict__ next, int L, int* __restrict__ out) {
    int p = (blockIdx.x * 64 + threadIdx.x) & 4095;
    for (int i = 0; i < L; i++) p = next[p];
    if (p < 0) out[blockIdx.x] = p;   // never true; keeps the chain alive
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 28, G = argc > 2 ? atoi(argv[2]) : 128, L = argc > 3 ? atoi(argv[3]) : 8;
    int *next, *out;
    CK(hipMalloc(&next, 4096 * sizeof(int)));
    CK(hipMalloc(&out, 65536 * sizeof(int)));
    int h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (i * 977 + 13) & 4095;
    CK(hipMemcpy(next, h, sizeof h, hipMemcpyHostToDevice));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t fork, join, t0, t1;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    hipGraphExec_t ex[3];
    for (int mode = 0; mode < 3; mode++) {   // 0: chain of 2n; 1: two forked chains of n; 2: chain of n (reference)
        hipGraph_t g;
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
        if (mode == 1) {
            CK(hipEventRecord(fork, s0));
            CK(hipStreamWaitEvent(s1, fork, 0));
            for (int i = 0; i < n; i++) {
                k_chain<<<G, 64, 0, s0>>>(next, L, out);
                k_chain<<<G, 64, 0, s1>>>(next, L, out + 32768);
            }
            CK(hipEventRecord(join, s1));
            CK(hipStreamWaitEvent(s0, join, 0));
        } else {
            for (int i = 0; i < (mode == 0 ? 2 * n : n); i++) k_chain<<<G, 64, 0, s0>>>(next, L, out);
        }
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&ex[mode], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    const char* name[3] = {"one chain of 2n", "two forked chains of n", "one chain of n"};
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 3; mode++) {
            for (int w = 0; w < 5; w++) CK(hipGraphLaunch(ex[mode], s0));
            CK(hipEventRecord(t0, s0));
            const int R = 50;
            for (int r = 0; r < R; r++) CK(hipGraphLaunch(ex[mode], s0));
            CK(hipEventRecord(t1, s0));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            printf("n=%d G=%d L=%d  %-24s %8.1f us per graph\n", n, G, L, name[mode], 1000.0 * ms / R);
        }
    return 0;
}
