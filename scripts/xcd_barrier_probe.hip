// Diagnostic: a grid barrier among workgroups of ONE XCD.
//   1. Which XCD does block b run on?  (XCC_ID hardware register per block)
//   2. What does a barrier cost when every participant shares one L2
//      (device-scope atomic arrive, spin on an atomic load, then an L1
//      invalidate instead of the L2 writeback / invalidate an agent-scope
//      fence costs on a multi-XCD device)?
//   3. Do loads after it see the other workgroups' stores of the round?
// 8 x W one-wave blocks are launched; blocks on XCD 0 take worker slots, the
// others exit.  Every spin has a time limit (s_memrealtime, 100 MHz), so a
// wrong assumption ends in a reported timeout, not a hang.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15; }

__device__ __forceinline__ bool spin_until(unsigned *ctr, unsigned target, unsigned long long t0) {
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) return false;   // 100 ms
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

__global__ __launch_bounds__(64) void probe(unsigned *xcc, unsigned *ctl, unsigned *data, unsigned *errs, int W, int K,
                                            int inv) {
    const int tid = threadIdx.x;
    const unsigned x = xcc_id();
    if (tid == 0) xcc[blockIdx.x] = x;
    if (x != 0) return;
    __shared__ unsigned s_w;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) s_w = atomicAdd(&ctl[0], 1u);
    __syncthreads();
    const unsigned w = s_w;
    if (w >= (unsigned)W) return;                       // more XCD-0 blocks than workers
    // all workers present
    if (tid == 0 && !spin_until(&ctl[0], W, t0)) atomicOr(&ctl[2], 1u);
    __syncthreads();
    unsigned bad = 0;
    for (int it = 0; it < K; ++it) {
        data[(size_t)w * 64 + tid] = it * 1000003u + w * 64 + tid;
        if (inv == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_s_waitcnt(0);                  // (vmcnt, lgkmcnt, expcnt all 0) the stores reached L2
        __syncthreads();
        if (tid == 0) {
            atomicAdd(&ctl[1], 1u);
            if (!spin_until(&ctl[1], (unsigned)(it + 1) * W, t0)) atomicOr(&ctl[2], 2u);
        }
        __syncthreads();
        // inv 1: L1 invalidate; 2: the read is an agent-scope atomic load (bypasses L1);
        // 3: agent-scope acquire fence (what the memory model emits across XCDs)
        if (inv == 1) asm volatile("buffer_inv sc0" ::: "memory");
        if (inv == 3) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const unsigned v = (w + 1) % W;
        const unsigned got = inv == 2 ? __hip_atomic_load(&data[(size_t)v * 64 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : data[(size_t)v * 64 + tid];
        const unsigned want = it * 1000003u + v * 64 + tid;
        bad += got != want;
        if (it == 1 && w == 0 && tid == 1) { ctl[8] = got; ctl[9] = want; }
        __syncthreads();                                // (no worker overwrites before every read)
        if (tid == 0) {
            atomicAdd(&ctl[3], 1u);
            if (!spin_until(&ctl[3], (unsigned)(it + 1) * W, t0)) atomicOr(&ctl[2], 4u);
        }
        __syncthreads();
        if (ctl[2]) break;
    }
    if (bad) atomicAdd(errs, bad);
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const int W = argc > 1 ? atoi(argv[1]) : 64, K = argc > 2 ? atoi(argv[2]) : 1000, inv = argc > 3 ? atoi(argv[3]) : 1;
    const int B = 8 * W;
    unsigned *xcc, *ctl, *data, *errs;
    CK(hipMalloc(&xcc, B * 4));
    CK(hipMalloc(&ctl, 64));
    CK(hipMalloc(&data, (size_t)W * 64 * 4));
    CK(hipMalloc(&errs, 4));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(ctl, 0, 64));
        CK(hipMemset(errs, 0, 4));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        probe<<<B, 64>>>(xcc, ctl, data, errs, W, K, inv);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned h_ctl[16], h_err;
        CK(hipMemcpy(h_ctl, ctl, 64, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&h_err, errs, 4, hipMemcpyDeviceToHost));
        unsigned *hx = (unsigned *)malloc(B * 4);
        CK(hipMemcpy(hx, xcc, B * 4, hipMemcpyDeviceToHost));
        int on0 = 0, rr = 0;
        for (int b = 0; b < B; ++b) { on0 += hx[b] == 0; rr += hx[b] == (unsigned)(b % 8); }
        printf("W=%d K=%d inv=%d: %.3f us per round (2 barriers), blocks on XCD0 %d, round-robin %d/%d, "
               "flags %u, stale reads %u (worker 0 lane 1 round 1: read %u, expected %u)\n", W, K, inv,
               1000.0f * ms / K, on0, rr, B, h_ctl[2], h_err, h_ctl[8], h_ctl[9]);
        free(hx);
    }
    return 0;
}
