// solve_probe.hip — diagnostic (not part of the product): core cycles per
// sphere-sphere contact of one body's Gauss-Seidel loop (sphere_sphere +
// solve_contact, rb_device.hpp / rb_body.hpp), one wave per SIMD as in the
// C4 pile-ups, for variants of the loop's structure.  Every variant runs the
// same per-contact arithmetic in the same order; the final v, w of each lane
// are compared across variants (bit-identical or the probe says so).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//         -I rigidbody-simulation_amd/csrc -o /tmp/solve_probe scripts/solve_probe.hip
//   /tmp/solve_probe [partners=28] [blocks=1024]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <cmath>

#include "rb_body.hpp"

using namespace rb;
using T = double;
constexpr int NP_MAX = 32;

struct In {
    T x[3], v[3], w[3], q[4], m, I[3], r;
    T pj[NP_MAX][4];
};

// variant 0: as body_update (geometry, record-free, solve; partner by partner)
// variant 1: the next partner's geometry before this partner's solve
// variant 2: geometry of a batch of 4 first, then the 4 solves
template <int VAR>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void probe(const In *in, int np, StepParams<T> p, T *out, unsigned long long *cyc) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    const In &b = in[t];
    V3<T> x = {b.x[0], b.x[1], b.x[2]}, v = {b.v[0], b.v[1], b.v[2]}, w = {b.w[0], b.w[1], b.w[2]};
    LazyInvI<T> invI;
    invI.I = {b.I[0], b.I[1], b.I[2]};
    invI.q = {b.q[0], b.q[1], b.q[2], b.q[3]};
    invI.get();
    const T m = b.m, k = impulse_k(m), r = b.r;
    __shared__ T s_p[NP_MAX][4][64];
    for (int a = 0; a < np; ++a)
        for (int c = 0; c < 4; ++c) s_p[a][c][threadIdx.x] = b.pj[a][c];
    __syncthreads();
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    auto pos = [&](int a) { return V3<T>{s_p[a][0][threadIdx.x], s_p[a][1][threadIdx.x], s_p[a][2][threadIdx.x]}; };
    auto rad = [&](int a) { return s_p[a][3][threadIdx.x]; };
    if constexpr (VAR == 0) {
        for (int a = 0; a < np; ++a) {
            Contact<T> con;
            const V3<T> cj = pos(a);
            sphere_sphere(x, r, cj, rad(a), con);
            solve_contact(p, con, x, con.frame, m, k, invI, v, w);
        }
    } else if constexpr (VAR == 1) {
        Contact<T> cn;
        bool hn = np > 0 && sphere_sphere(x, r, pos(0), rad(0), cn);
        for (int a = 0; a < np; ++a) {
            const Contact<T> con = cn;
            const bool h = hn;
            if (a + 1 < np) hn = sphere_sphere(x, r, pos(a + 1), rad(a + 1), cn);
            if (h) solve_contact(p, con, x, con.frame, m, k, invI, v, w);
        }
    } else {
        for (int a0 = 0; a0 < np; a0 += 4) {
            Contact<T> con[4];
            bool h[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                h[u] = a0 + u < np && sphere_sphere(x, r, pos(a0 + u < np ? a0 + u : 0), rad(a0 + u < np ? a0 + u : 0), con[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (h[u]) solve_contact(p, con[u], x, con[u].frame, m, k, invI, v, w);
        }
    }
    unsigned long long t1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    T *o = out + (int64_t)t * 6;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = w.x; o[4] = w.y; o[5] = w.z;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
    const int np = argc > 1 ? atoi(argv[1]) : 28;
    const int blocks = argc > 2 ? atoi(argv[2]) : 1024;
    const int n = blocks * 64;
    std::vector<In> h(n);
    srand(1);
    auto U = [] { return (T)rand() / RAND_MAX; };
    for (auto &b : h) {
        for (int d = 0; d < 3; ++d) { b.x[d] = U(); b.v[d] = 2 * U() - 1; b.w[d] = 4 * U() - 2; }
        T qq[4] = {1 + U(), U() - 0.5, U() - 0.5, U() - 0.5}, nq = 0;
        for (T c : qq) nq += c * c;
        for (int d = 0; d < 4; ++d) b.q[d] = qq[d] / sqrt(nq);
        b.m = 4.18879; b.I[0] = b.I[1] = b.I[2] = 0.016755; b.r = 0.1;
        for (int a = 0; a < NP_MAX; ++a) {
            T dir[3] = {U() - 0.5, U() - 0.5, U() - 0.5}, nd = 0;
            for (T c : dir) nd += c * c;
            nd = sqrt(nd);
            const T d = 0.2 * (0.9 + 0.09 * U());      // penetrating partners
            for (int c = 0; c < 3; ++c) b.pj[a][c] = b.x[c] + dir[c] / nd * d;
            b.pj[a][3] = 0.1;
        }
    }
    In *din;
    T *dout;
    unsigned long long *dcyc;
    (void)hipMalloc(&din, sizeof(In) * n);
    (void)hipMalloc(&dout, sizeof(T) * 6 * n);
    (void)hipMalloc(&dcyc, sizeof(unsigned long long) * blocks);
    (void)hipMemcpy(din, h.data(), sizeof(In) * n, hipMemcpyHostToDevice);
    StepParams<T> p{};
    p.e = 0.2; p.mu = 0.6; p.thr = 0.0;
    std::vector<T> ref, res(6 * n);
    std::vector<unsigned long long> cyc(blocks);
    for (int rep = 0; rep < 2; ++rep)
        for (int var = 0; var < 3; ++var) {
            if (var == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(64), 0, 0, din, np, p, dout, dcyc);
            if (var == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(64), 0, 0, din, np, p, dout, dcyc);
            if (var == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(64), 0, 0, din, np, p, dout, dcyc);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(res.data(), dout, sizeof(T) * 6 * n, hipMemcpyDeviceToHost);
            (void)hipMemcpy(cyc.data(), dcyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
            if (ref.empty()) ref = res;
            const bool same = memcmp(ref.data(), res.data(), sizeof(T) * res.size()) == 0;
            std::vector<unsigned long long> c = cyc;
            std::sort(c.begin(), c.end());
            printf("variant %d (rep %d): median %llu cycles per body-loop, %.0f per contact, max %llu; %s\n", var, rep,
                   c[c.size() / 2], (double)c[c.size() / 2] / np, c.back(), same ? "bit-identical" : "DIFFERS");
        }
    return 0;
}
