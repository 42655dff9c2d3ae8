// Probe (diagnostic, not product code): are workgroup-scope returning
// atomics executed in the XCD's L2 (so that the workgroups of ONE XCD see one
// counter), and what does a returning atomic cost at workgroup vs agent
// scope, with the line then read back by an sc1 load?
//   hipcc --offload-arch=gfx950 -O3 -o scripts/atomic_probe scripts/atomic_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

constexpr int NB = 256, NT = 64, M = 64;

template <int SCOPE>
__global__ void count_kernel(unsigned long long *ctr, int per_xcd) {
    // per_xcd: counter of group b % 8 (one XCD); else one counter for all
    unsigned long long *c = ctr + (per_xcd ? (blockIdx.x % 8) * 16 : 0);
    for (int k = 0; k < M; ++k) (void)__hip_atomic_fetch_add(c, 1ull, __ATOMIC_RELAXED, SCOPE);
}

// dependent chain: atomic add returning old, then an sc1 load of a word on
// the same line, k times; cycles per iteration
template <int SCOPE>
__global__ void chain_kernel(unsigned long long *base, long long *cyc) {
    unsigned long long *c = base + (size_t)(blockIdx.x * NT + threadIdx.x) * 16;
    unsigned long long v = 0;
    const long long t0 = clock64();
    for (int k = 0; k < M; ++k) {
        v += __hip_atomic_fetch_add(c + (v & 1), 1ull, __ATOMIC_RELAXED, SCOPE);
        v += __hip_atomic_load(c + 2 + (v & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) / M + (long long)(v & 0);
}

int main() {
    unsigned long long *ctr;
    long long *cyc;
    hipMalloc(&ctr, sizeof(unsigned long long) * 16 * NB * NT);
    hipMalloc(&cyc, sizeof(long long) * NB);
    const char *scopes[2] = {"workgroup", "agent"};
    for (int per = 1; per >= 0; --per)
        for (int sc = 0; sc < 2; ++sc) {
            hipMemset(ctr, 0, sizeof(unsigned long long) * 16 * 8);
            if (sc == 0) hipLaunchKernelGGL(count_kernel<__HIP_MEMORY_SCOPE_WORKGROUP>, dim3(NB), dim3(NT), 0, 0, ctr, per);
            else hipLaunchKernelGGL(count_kernel<__HIP_MEMORY_SCOPE_AGENT>, dim3(NB), dim3(NT), 0, 0, ctr, per);
            hipDeviceSynchronize();
            std::vector<unsigned long long> h(16 * 8);
            hipMemcpy(h.data(), ctr, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
            if (per) {
                int ok = 0;
                for (int g = 0; g < 8; ++g) ok += h[g * 16] == (unsigned long long)(NB / 8) * NT * M;
                printf("per-XCD counters, %s scope: %d of 8 exact (want %llu, got %llu ...)\n", scopes[sc], ok,
                       (unsigned long long)(NB / 8) * NT * M, h[0]);
            } else {
                printf("one counter for all XCDs, %s scope: got %llu of %llu\n", scopes[sc], h[0],
                       (unsigned long long)NB * NT * M);
            }
        }
    for (int sc = 0; sc < 2; ++sc) {
        hipMemset(ctr, 0, sizeof(unsigned long long) * 16 * NB * NT);
        if (sc == 0) hipLaunchKernelGGL(chain_kernel<__HIP_MEMORY_SCOPE_WORKGROUP>, dim3(NB), dim3(NT), 0, 0, ctr, cyc);
        else hipLaunchKernelGGL(chain_kernel<__HIP_MEMORY_SCOPE_AGENT>, dim3(NB), dim3(NT), 0, 0, ctr, cyc);
        hipDeviceSynchronize();
        std::vector<long long> c(NB);
        hipMemcpy(c.data(), cyc, sizeof(long long) * NB, hipMemcpyDeviceToHost);
        long long s = 0;
        for (long long v : c) s += v;
        printf("dependent (returning atomic + sc1 load of its line), %s scope: %lld cycles per iteration (mean over blocks)\n",
               scopes[sc], s / NB);
    }
    return 0;
}
