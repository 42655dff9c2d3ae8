// Diagnostic: what does one round of random 16-byte gathers cost at the step
// kernel's launch shape (1,024 one-wave blocks, one wave per SIMD, every wave
// issuing at once, L2 cold at kernel start)?  Each lane issues L dwordx4
// loads (its "bucket heads") into a 256 MB table and sums them.
//   mode 0: L loads to L random 128-B lines
//   mode 1: L/2 random lines, two 16-B loads from each (the 32-B heads)
//   mode 2: L loads, lanes of a wave reading consecutive 16 B (coalesced)
// Reported: kernel time by HIP events, mean over launches; argv[1] = table MB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

static size_t TABLE = size_t(256) << 20;              // bytes (argv[1] MB)

__device__ __forceinline__ unsigned mix(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int L, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gather(const uint4 *__restrict__ tab, unsigned *__restrict__ out, unsigned seed, unsigned LINES) {
    const unsigned g = blockIdx.x * 64 + threadIdx.x;
    uint4 v[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        size_t idx;
        if (MODE == 0) idx = (size_t)(mix(g * 131u + k * 7919u + seed) % LINES) * 8;
        else if (MODE == 1) idx = (size_t)(mix(g * 131u + (k / 2) * 7919u + seed) % LINES) * 8 + (k & 1);
        else idx = ((size_t)(blockIdx.x * L + k) * 64 + threadIdx.x + seed * 64) % ((size_t)LINES * 8);
        v[k] = tab[idx];
    }
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < L; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x9e3779b9u) out[g] = acc;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

template <int L, int MODE> int run(const uint4 *tab, unsigned *out, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int t = 0; t < 20; ++t) gather<L, MODE><<<1024, 64>>>(tab, out, t, (unsigned)(TABLE / 128));
    CK(hipEventRecord(e0));
    for (int t = 0; t < iters; ++t) gather<L, MODE><<<1024, 64>>>(tab, out, 1000 + t, (unsigned)(TABLE / 128));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("table %4zu MB  L=%2d mode %d: %.2f us per launch\n", TABLE >> 20, L, MODE, 1000.0f * ms / iters);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1) TABLE = size_t(atoi(argv[1])) << 20;
    uint4 *tab;
    unsigned *out;
    CK(hipMalloc(&tab, TABLE));
    CK(hipMemset(tab, 1, TABLE));
    CK(hipMalloc(&out, 1024 * 64 * sizeof(unsigned)));
    const int it = 500;
    run<1, 0>(tab, out, it);
    run<8, 0>(tab, out, it);
    run<16, 0>(tab, out, it);
    run<16, 1>(tab, out, it);
    run<16, 2>(tab, out, it);
    return 0;
}
