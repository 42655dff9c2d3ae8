// Diagnostic: does an XCD's L2 keep what the previous kernel on the same
// stream wrote?  Kernel W writes 2 MB per XCD (block b writes slice b); kernel
// R then reads slice (b + shift) in block b.  Blocks are dealt to the XCDs
// round-robin (b % 8), so shift 0 reads what the same XCD wrote, shift 1
// what its neighbour wrote.  If the L2 survives the kernel boundary, shift 0
// reads hit it (rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum, and a shorter R).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int BLOCKS = 256, THREADS = 256, SLICE = 64 * 1024;   // bytes per block

__global__ __launch_bounds__(THREADS) void w_kernel(uint4 *buf, unsigned v) {
    uint4 *s = buf + (size_t)blockIdx.x * (SLICE / 16);
    for (int k = threadIdx.x; k < SLICE / 16; k += THREADS) s[k] = make_uint4(v, k, blockIdx.x, 1);
}

__global__ __launch_bounds__(THREADS) void r_kernel(const uint4 *buf, unsigned *out, int shift) {
    const int b = (blockIdx.x + shift) % BLOCKS;
    const uint4 *s = buf + (size_t)b * (SLICE / 16);
    unsigned acc = 0;
    for (int k = threadIdx.x; k < SLICE / 16; k += THREADS) { const uint4 t = s[k]; acc += t.x ^ t.y ^ t.z ^ t.w; }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;     // keeps the loads
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const int shift = argc > 1 ? atoi(argv[1]) : 0, iters = argc > 2 ? atoi(argv[2]) : 200;
    uint4 *buf;
    unsigned *out;
    CK(hipMalloc(&buf, (size_t)BLOCKS * SLICE));
    CK(hipMalloc(&out, BLOCKS * sizeof(unsigned)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0;
    for (int t = 0; t < iters; ++t) {
        w_kernel<<<BLOCKS, THREADS>>>(buf, t);
        CK(hipEventRecord(e0));
        r_kernel<<<BLOCKS, THREADS>>>(buf, out, shift);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (t >= 10) tot += ms;
    }
    printf("shift %d: read kernel %.2f us (event pair, mean of %d)\n", shift, 1000.0f * tot / (iters - 10), iters - 10);
    return 0;
}
