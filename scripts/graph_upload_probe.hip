// graph_upload_probe.hip — diagnostic (not part of the product): device time
// of a captured graph's first launch against later ones, with and without
// hipGraphUpload after instantiation (HIP events around each launch).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gup scripts/graph_upload_probe.hip && /tmp/gup
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void busy(float *x, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] * 1.0001f + 1.0f;
}

int main() {
    const int n = 1 << 20, K = 20;
    float *x;
    (void)hipMalloc(&x, n * sizeof(float));
    hipStream_t s, cap;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    busy<<<n / 256, 256, 0, s>>>(x, n);              // the module is loaded
    (void)hipStreamSynchronize(s);
    for (int upload = 0; upload < 2; ++upload) {
        hipGraph_t g;
        hipGraphExec_t ex;
        (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < K; ++k) busy<<<n / 256, 256, 0, cap>>>(x, n);
        (void)hipStreamEndCapture(cap, &g);
        (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        if (upload) (void)hipGraphUpload(ex, s);
        (void)hipStreamSynchronize(s);
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a, s);
            (void)hipGraphLaunch(ex, s);
            (void)hipEventRecord(b, s);
            (void)hipStreamSynchronize(s);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("upload %d launch %d: %.1f us (%.2f us per node)\n", upload, rep, ms * 1e3, ms * 1e3 / K);
        }
        (void)hipGraphExecDestroy(ex);
        (void)hipGraphDestroy(g);
    }
    return 0;
}
