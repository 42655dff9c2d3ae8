// Diagnostic: does kernel-argument preloading (gfx950 user SGPRs filled at
// wave launch, -mllvm -amdgpu-kernarg-preload-count=N) shorten a kernel whose
// first loads depend on its arguments?  The probe mimics the step kernel's
// start: one wave per SIMD (1,024 waves), a by-value parameter block behind
// the leading scalar arguments, a first load that needs three of them, and a
// second, dependent load.  Build it twice (with and without the flag) and
// compare the kernel durations under rocprofv3 --kernel-trace --stats.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct Block { double pad[120]; const int *link; };

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void probe(const double *__restrict__ snap, double *__restrict__ out, const int *__restrict__ kind, int n, int lo,
           Block blk) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const double x = snap[lo + i];
    const int k = kind[lo + i];
    const int j = blk.link[(i * 7 + k) & (n - 1)];
    const double y = snap[j];
    out[i] = x + y + blk.pad[3];
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const int n = 65536, iters = argc > 1 ? atoi(argv[1]) : 2000;
    double *snap, *out;
    int *kind, *link;
    CK(hipMalloc(&snap, n * sizeof(double)));
    CK(hipMalloc(&out, n * sizeof(double)));
    CK(hipMalloc(&kind, n * sizeof(int)));
    CK(hipMalloc(&link, n * sizeof(int)));
    CK(hipMemset(snap, 0, n * sizeof(double)));
    CK(hipMemset(kind, 0, n * sizeof(int)));
    int *h = (int *)malloc(n * sizeof(int));
    for (int t = 0; t < n; ++t) h[t] = (int)((t * 2654435761u) & (n - 1));
    CK(hipMemcpy(link, h, n * sizeof(int), hipMemcpyHostToDevice));
    Block blk{};
    blk.link = link;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 50; ++w) probe<<<n / 64, 64>>>(snap, out, kind, n, 0, blk);
    CK(hipEventRecord(e0));
    for (int t = 0; t < iters; ++t) probe<<<n / 64, 64>>>(snap, out, kind, n, 0, blk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("probe: %d launches, %.3f us per launch (stream time)\n", iters, 1000.0 * ms / iters);
    free(h);
    return 0;
}
