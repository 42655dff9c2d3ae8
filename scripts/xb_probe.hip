// Diagnostic probe for the XCD-resident K-step blocks (csrc/rb_xblock.hip):
//   1. placement: do blocks b and b + 8 share an XCD (XCC_ID register)?
//   2. group barrier among the 32 workgroups of one XCD (512 threads each,
//      one per CU, all 8 XCDs at once): plain stores, vmcnt(0), workgroup
//      barrier, one device-scope atomic arrive, a poll of sc1 loads — then
//      which load flavours see the other workgroups' stores (plain, nt,
//      8-byte sc1 atomic loads, 16-byte sc1 buffer loads)?
//   3. its cost per barrier.
//   4. a dependent chain of loads (pointer chase) over a buffer written in
//      the same launch: cycles per hop, plain vs sc1 vs nt, L2-resident.
// Every spin has a time limit (s_memrealtime, 100 MHz): a wrong assumption
// ends in a reported timeout, not a hang.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15; }

constexpr int NG = 8, WPG = 32, NT = 512;

struct Ctl {
    unsigned long long bar[NG][16];   // one line per group
    unsigned flags;
    unsigned stale[8];
    unsigned xcc[NG * WPG];
    unsigned long long t_bar[NG * WPG];
    unsigned long long t_chase[8];
};

__device__ __forceinline__ bool group_barrier(unsigned long long *ctr, unsigned long long t0, unsigned *flags) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long target = (old / WPG + 1) * WPG;
        int ok = 1;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { ok = 0; atomicOr(flags, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok;
}

using u4 = __attribute__((ext_vector_type(4))) unsigned;

template <int MODE>
__device__ __forceinline__ unsigned load_word(const unsigned *p, __amdgpu_buffer_rsrc_t r, unsigned off) {
    if (MODE == 0) return *p;
    if (MODE == 1) return __builtin_nontemporal_load(p);
    if (MODE == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_raw_buffer_load_b32(r, off * 4, 0, 16);   // sc1
}

// K rounds: every lane writes its word, group barrier, reads the word of the
// next workgroup in its group (load flavour MODE), group barrier.
template <int MODE>
__global__ __launch_bounds__(NT) void probe_handoff(Ctl *ctl, unsigned *data, int K) {
    const unsigned g = blockIdx.x % NG, r = blockIdx.x / NG, tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) __hip_atomic_store(&ctl->xcc[blockIdx.x], xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(data, 0, 0x7fffffff, 0x00020000);
    unsigned bad = 0;
    unsigned long long tb = 0;
    for (int it = 0; it < K; ++it) {
        const unsigned idx = (g * WPG + r) * NT + tid;
        data[idx] = it * 1000003u + idx;
        const unsigned long long a = __builtin_amdgcn_s_memtime();
        if (!group_barrier(&ctl->bar[g][0], t0, &ctl->flags)) break;
        tb += __builtin_amdgcn_s_memtime() - a;
        const unsigned v = (g * WPG + (r + 1) % WPG) * NT + tid;
        const unsigned got = load_word<MODE>(data + v, rs, v);
        bad += got != it * 1000003u + v;
        if (!group_barrier(&ctl->bar[g][0], t0, &ctl->flags)) break;
    }
    if (bad) atomicAdd(&ctl->stale[MODE], bad);
    if (tid == 0) ctl->t_bar[blockIdx.x] = tb / (K ? K : 1);
}

// Pointer chase in group 0's workgroup 0, lane 0, over a ring written by the
// group in this launch (after a barrier): cycles per dependent hop.
template <int MODE>
__global__ __launch_bounds__(NT) void probe_chase(Ctl *ctl, unsigned *ring, int n, int hops) {
    const unsigned g = blockIdx.x % NG, r = blockIdx.x / NG, tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // group 0 writes the ring (a random cycle with stride of a few KB)
    if (g == 0)
        for (int k = r * NT + tid; k < n; k += WPG * NT) ring[k] = (unsigned)(((unsigned long long)k * 2654435761ull + 7919) % n);
    if (!group_barrier(&ctl->bar[g][0], t0, &ctl->flags)) return;
    if (g != 0 || r != 0 || tid != 0) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ring, 0, 0x7fffffff, 0x00020000);
    unsigned p = 0;
    // warm pass (brings the ring's lines the chase touches into L2 via this path)
    for (int h = 0; h < hops; ++h) p = load_word<MODE>(ring + p, rs, p);
    const unsigned long long a = __builtin_amdgcn_s_memtime();
    for (int h = 0; h < hops; ++h) p = load_word<MODE>(ring + p, rs, p);
    const unsigned long long b = __builtin_amdgcn_s_memtime();
    ctl->t_chase[MODE] = (b - a) / hops + (p == 0xffffffffu ? 1 : 0);
}

// Atomic placement: every workgroup adds M times to its group's counter with
// workgroup (S=0) or agent (S=1) scope; totals checked by the host.
template <int S>
__global__ __launch_bounds__(NT) void probe_atomic(unsigned long long *cnt, int M) {
    const unsigned g = blockIdx.x % NG;
    for (int k = 0; k < M; ++k) {
        if (S == 0) __hip_atomic_fetch_add(&cnt[g * 16], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_fetch_add(&cnt[g * 16], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r_)); return 1; } } while (0)

template <int MODE> int run_handoff(Ctl *ctl, unsigned *data, int K, const char *name) {
    CK(hipMemset(ctl, 0, sizeof(Ctl)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    probe_handoff<MODE><<<NG * WPG, NT>>>(ctl, data, K);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    Ctl h; CK(hipMemcpy(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    int same = 1;
    for (int b = 0; b < NG * WPG; ++b) same &= h.xcc[b] == h.xcc[b % NG];
    unsigned long long tb = 0;
    for (int b = 0; b < NG * WPG; ++b) tb += h.t_bar[b];
    printf("handoff %-12s K=%d: %.3f us per round (2 group barriers), barrier %.0f cycles avg, "
           "b%%8 groups single-XCD %d, flags %u, stale %u of %u\n", name, K, 1000.0f * ms / K,
           (double)tb / (NG * WPG), same, h.flags, h.stale[MODE], (unsigned)K * NG * WPG * NT);
    return 0;
}

template <int MODE> int run_chase(Ctl *ctl, unsigned *ring, int n, const char *name) {
    CK(hipMemset(ctl, 0, sizeof(Ctl)));
    probe_chase<MODE><<<NG * WPG, NT>>>(ctl, ring, n, 2000);
    CK(hipDeviceSynchronize());
    Ctl h; CK(hipMemcpy(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    printf("chase %-12s ring %d KB: %llu cycles per dependent hop (flags %u)\n", name, n * 4 / 1024, h.t_chase[MODE], h.flags);
    return 0;
}

int main() {
    Ctl *ctl; unsigned *data, *ring; unsigned long long *cnt;
    CK(hipMalloc(&ctl, sizeof(Ctl)));
    CK(hipMalloc(&data, NG * WPG * NT * 4));
    CK(hipMalloc(&ring, 4 << 20));
    CK(hipMalloc(&cnt, NG * 16 * 8));
    for (int rep = 0; rep < 2; ++rep) {
        if (run_handoff<0>(ctl, data, 200, "plain")) return 1;
        if (run_handoff<1>(ctl, data, 200, "nt")) return 1;
        if (run_handoff<2>(ctl, data, 200, "sc1 atomic")) return 1;
        if (run_handoff<3>(ctl, data, 200, "sc1 buffer")) return 1;
    }
    for (int n : {1 << 16, 1 << 19}) {   // 256 KB, 2 MB
        if (run_chase<0>(ctl, ring, n, "plain")) return 1;
        if (run_chase<1>(ctl, ring, n, "nt")) return 1;
        if (run_chase<2>(ctl, ring, n, "sc1 atomic")) return 1;
        if (run_chase<3>(ctl, ring, n, "sc1 buffer")) return 1;
    }
    const int M = 64;
    for (int s = 0; s < 2; ++s) {
        CK(hipMemset(cnt, 0, NG * 16 * 8));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        if (s == 0) probe_atomic<0><<<NG * WPG, NT>>>(cnt, M); else probe_atomic<1><<<NG * WPG, NT>>>(cnt, M);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long h[NG * 16];
        CK(hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost));
        unsigned long long want = (unsigned long long)WPG * NT * M, worst = 0;
        for (int g = 0; g < NG; ++g) worst = h[g * 16] != want ? 1 : worst;
        printf("atomics %s scope: %d per lane into one counter per group, %.1f us, totals %s (group 0: %llu of %llu)\n",
               s ? "agent" : "workgroup", M, ms * 1000.0f, worst ? "WRONG" : "exact", h[0], want);
    }
    return 0;
}
