// Per-kernel cost of a dependent chain of small kernels, eager vs hipGraph replay (decode-step shape question).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_tiny(int* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1;
}

static float time_chain(bool graph, int kernels, int wgs, int* buf, hipStream_t s) {
    hipGraphExec_t ex = nullptr;
    if (graph) {
        hipGraph_t g;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
        for (int k = 0; k < kernels; k++) k_tiny<<<wgs, 256, 0, s>>>(buf, wgs * 256);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        (void)hipGraphLaunch(ex, s);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int rep = 0; rep < 10; rep++) {
        if (graph) (void)hipGraphLaunch(ex, s);
        else
            for (int k = 0; k < kernels; k++) k_tiny<<<wgs, 256, 0, s>>>(buf, wgs * 256);
    }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ex) (void)hipGraphExecDestroy(ex);
    return ms * 1000.f / (10 * kernels);
}

int main() {
    int* buf;
    (void)hipMalloc(&buf, 64 << 20);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int wgs : {1, 64, 256, 1024, 4096})
        printf("wgs=%5d  eager %.2f us/kernel   graph %.2f us/kernel\n", wgs, time_chain(false, 200, wgs, buf, s),
               time_chain(true, 200, wgs, buf, s));
    return 0;
}
