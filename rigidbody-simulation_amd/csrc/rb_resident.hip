// rb_resident.hip — the resident form of the step (rb_internal.hpp ResParams;
// DESIGN §4.3): sphere worlds on one rank, K reference steps per launch.
//
// The step is the reference's: contacts from the step-start positions of
// every body (mj_forward, collision.py:57 / multi_sphere_bounce.py:43), then
// per body gravity, its plane contacts and its sphere partners in ascending
// id, each through compute_collision_impulse_friction (collision.py:7-48) and
// apply_impulse_friction (physics_utils.py:25-49), then the integration
// (collision.py:90-100) — Jacobi across bodies, Gauss-Seidel within one
// (collision.py:72-88).  The per-body arithmetic is rb_body.hpp's, shared
// with the hashed-cell and tile kernels, so every form steps a body
// bit-identically.  What differs is where the step-start data lives and who
// waits for whom:
//
//   hashed cells / tiles: one launch per step; every body's state goes
//     through HBM each step, and the launch boundary orders the steps;
//   here: one launch per window of K steps; a single-wave workgroup owns the
//     bodies of one slot (a square tile of the plane, mapped periodically)
//     and keeps their state in registers, their positions in LDS.  A body's
//     partners come from its candidate list (every body within rl in x, y
//     at the last list build, sorted by id — the reference's contact order);
//     the list names bodies of this slot (LDS) and of the 8 neighbouring
//     slots, whose positions the workgroup imports each step from the
//     neighbours' publication: 8-byte granules {tag = step, 32-bit half}
//     stored write-through (sc1), so the data is its own flag and a
//     workgroup waits only for its neighbours, never for the grid.
//
// Exactness: a pair missing from a list was >= rl apart in x, y at the build;
// every body is checked each step to have moved <= skin in x, y since then,
// and rl = 2 rmax + 2 skin, so a missing pair stays > r_i + r_j apart and is
// no contact.  The lists are rebuilt every M steps from all bodies of the 3 x
// 3 slots; that covers every body within rl while no body has left its home
// tile by more than `drift` (checked) and L >= rl + 2 drift.  Any violation,
// a full list or import table, a partner overflow, a bad position or a wait
// that times out raises ERR_TILE with a RES_WHY_* bit and sets the abort word
// (spinning workgroups see it and leave); the commit kernel then leaves the
// id-ordered state at the window start and the host replays the window with
// the hashed forms (rb_capi.hip tile_finish).
#include "rb_device.hpp"
#include "rb_grid.hpp"
#include "rb_internal.hpp"
#include "rb_body.hpp"

// diagnostic build only (RB_RES_STAMPS=1, scripts/res_stamps.py): per
// workgroup s_memrealtime (100 MHz, comparable across XCDs) at the start,
// after the setup, after steps 1 and K/2, and at the end; and the cycles the
// waits for the neighbours spun
#ifndef RB_RES_STAMPS
#define RB_RES_STAMPS 0
#endif
#if RB_RES_STAMPS
constexpr int RES_NSTAMP = 40;
__device__ unsigned long long rb_res_stamp_buf[1 << 12][RES_NSTAMP];
#define RSTAMP(k)                                                                                  \
    do {                                                                                           \
        unsigned long long r_;                                                                     \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");             \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 12) && (k) < RES_NSTAMP) rb_res_stamp_buf[blockIdx.x][k] = r_; \
    } while (0)
#else
#define RSTAMP(k) do {} while (0)
#endif

namespace rb {

static_assert(RES_CAP == 64, "one wave per slot: the kernel relies on the wave's lockstep between phases");
static_assert(RES_STAGE % RES_CAP == 0, "per-lane strides");
constexpr int32_t RES_IMPORT_BIT = 1 << 30;          // (ids < 2^30: rb_world_create)

typedef __attribute__((address_space(1))) unsigned long long res_gu64;
typedef __attribute__((address_space(1))) int32_t res_gi32;

// agent-scope relaxed accesses: global_store / global_load ... sc1 (write-
// through, L1-bypassing; MI355X_MICROARCH.md § visibility)
__device__ __forceinline__ void res_store(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store((res_gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long res_load(const unsigned long long *p) {
    return __hip_atomic_load((res_gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t res_load_i32(const int32_t *p) {
    return __hip_atomic_load((res_gi32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a position as G granule halves: fp64 x lo, x hi, y lo, y hi, z lo, z hi;
// fp32 x, y, z
template <typename T> constexpr int res_G() { return sizeof(T) == 8 ? 6 : 3; }
__device__ __forceinline__ uint32_t res_half(const V3<double> &x, int g) {
    const double v = g < 2 ? x.x : g < 4 ? x.y : x.z;
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (g & 1) ? (uint32_t)(u >> 32) : (uint32_t)u;
}
__device__ __forceinline__ uint32_t res_half(const V3<float> &x, int g) {
    return __float_as_uint(g == 0 ? x.x : g == 1 ? x.y : x.z);
}
__device__ __forceinline__ double res_join(unsigned long long lo, unsigned long long hi) {
    return __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
}
template <typename T> __device__ __forceinline__ V3<T> res_decode(const unsigned long long (&g)[res_G<T>()]) {
    if constexpr (sizeof(T) == 8) return V3<T>{res_join(g[0], g[1]), res_join(g[2], g[3]), res_join(g[4], g[5])};
    else return V3<T>{__uint_as_float((uint32_t)g[0]), __uint_as_float((uint32_t)g[1]), __uint_as_float((uint32_t)g[2])};
}

__device__ __forceinline__ int32_t res_pmod(int32_t a, int32_t m) {
    const int32_t r = a % m;
    return r < 0 ? r + m : r;
}

template <typename T> __device__ __forceinline__ void res_fail(const ResParams<T> &p, int why) {
    atomicOr(p.why, why);
    atomicOr(p.sp.err, ERR_TILE);
    __hip_atomic_store((res_gi32 *)p.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// inclusive scan over the wave's 64 lanes (DPP, as rb_tiles.hip)
__device__ __forceinline__ int res_wave_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

// Wait until every granule of the lane's needed requests carries `tag`:
// req[q] (bit q of `need`) is a granule offset from `base` (stride RES_CAP
// between a body's granules), NG granules each.  Returns false when the
// window is aborted or the wait timed out (raised here).  Every lane issues
// every load (requests not needed read offset 0) so the waits count them
// exactly.
template <typename T, int NQ, int NG>
__device__ __forceinline__ bool res_wait(const ResParams<T> &p, const unsigned long long *base, const int32_t (&req)[NQ],
                                         uint32_t need, uint32_t tag, unsigned long long (&g)[NQ][NG]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int k = 0; k < NG; ++k) g[q][k] = res_load(base + (((need >> q) & 1u) ? req[q] : 0) + k * RES_CAP);
    auto fresh = [&](int q) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NG; ++k) ok &= (uint32_t)(g[q][k] >> 32) == tag;
        return ok || !((need >> q) & 1u);
    };
    bool ok = true;
#pragma unroll
    for (int q = 0; q < NQ; ++q) ok &= fresh(q);
    if (__all(ok)) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (res_load_i32(p.abort)) return false;
        ok = true;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (!fresh(q)) {
#pragma unroll
                for (int k = 0; k < NG; ++k) g[q][k] = res_load(base + req[q] + k * RES_CAP);
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) ok &= fresh(q);
        if (__all(ok)) return true;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > p.timeout) {
            if (threadIdx.x == 0) res_fail(p, RES_WHY_TIMEOUT);
            return false;
        }
    }
}

template <typename T, int MAXP>
__global__ __launch_bounds__(RES_CAP) __attribute__((amdgpu_waves_per_eu(2, 2))) void res_step_kernel(const int32_t *err, const int32_t *cnt, ResParams<T> p) {
    constexpr int G = res_G<T>();
    constexpr int GXY = sizeof(T) == 8 ? 4 : 2;     // the granules of x and y
    constexpr int SPL = RES_STAGE / RES_CAP;        // staged bodies per lane
    constexpr int IPL = (RES_MMAX + RES_CAP - 1) / RES_CAP;   // imports per lane
    // unified candidate table: [0, RES_CAP) this slot's bodies (lane order),
    // [RES_CAP, RES_CAP + nimp) the imports; positions of the current step
    __shared__ T s_px[RES_NU], s_py[RES_NU], s_pz[RES_NU], s_r[RES_NU];
    __shared__ int32_t s_gid[RES_NU];
    __shared__ int32_t s_ioff[RES_MMAX];            // an import's granule offset in a parity's publication
    __shared__ uint16_t s_list[RES_LMAX][RES_CAP];  // candidate lists (unified indices, ascending id)
    // list builds: the 3 x 3 slots' bodies, x and y relative to the origin (fp32)
    __shared__ float s_sx[RES_STAGE], s_sy[RES_STAGE];
    // their ids; after the lists are built, bit 30 marks an import, and then
    // the entry holds the staged body's unified index (LDS: 8 slots per CU)
    __shared__ int32_t s_sgid[RES_STAGE];
    __shared__ int32_t s_ko[10];                    // staging offsets of the 3 x 3 slots
    __shared__ int32_t s_kslot[9];
    __shared__ T s_m[RES_CAP], s_I[3][RES_CAP], s_home[2][RES_CAP], s_xref[2][RES_CAP];

    RSTAMP(0);
    const int tid = threadIdx.x;
    const int nslots = p.ntx * p.nty;
    // XCD-aware: blocks b and b + 8 share an XCD; each XCD takes a contiguous
    // band of slot rows, so most neighbours share its L2 (speed only)
    const int b = (int)blockIdx.x, xq = nslots / (int)N_XCD, xr = nslots % (int)N_XCD, xx = b % (int)N_XCD;
    const int slot = xx * xq + (xx < xr ? xx : xr) + b / (int)N_XCD;
    if (*err & ERR_TILE) return;                    // a window after a failed one: replayed anyway
    const int n = cnt[slot];
    if (n <= 0) return;
    if (n > RES_CAP) {                              // (the bin kernel raised it)
        if (tid == 0) res_fail(p, TILE_WHY_CAP);
        return;
    }
    const int sxs = slot % p.ntx, sys = slot / p.ntx;
    if (tid < 9) s_kslot[tid] = res_pmod(sys + tid / 3 - 1, p.nty) * p.ntx + res_pmod(sxs + tid % 3 - 1, p.ntx);
    // the 3 x 3 slots' counts and staging offsets (slot k at [s_ko[k], s_ko[k + 1]))
    {
        const int kc = tid < 9 ? cnt[res_pmod(sys + tid / 3 - 1, p.nty) * p.ntx + res_pmod(sxs + tid % 3 - 1, p.ntx)] : 0;
        const int kcc = kc < 0 ? 0 : kc > RES_CAP ? RES_CAP : kc;
        const int inc = res_wave_scan(kcc);
        if (tid < 10) s_ko[tid] = inc - kcc;       // (lane 9: the total)
    }

    // ---- the own body ----------------------------------------------------------
    const bool own = tid < n;
    const int32_t id = p.ids[(int64_t)slot * RES_CAP + (own ? tid : 0)];
    const StepParams<T> &sp = p.sp;
    const Snap<T> s0 = p.snap[id];
    V3<T> x = {s0.x, s0.y, s0.z};
    const T rad = s0.r;
    Q4<T> q = {sp.st.qw()[id], sp.st.qx()[id], sp.st.qy()[id], sp.st.qz()[id]};
    V3<T> v = {sp.st.vx()[id], sp.st.vy()[id], sp.st.vz()[id]};
    V3<T> w = {sp.st.wx()[id], sp.st.wy()[id], sp.st.wz()[id]};
    // per-lane constants and reference positions live in LDS (registers are
    // the step's: two waves per SIMD keep a CU's 8 slots resident)
    s_m[tid] = sp.cs.mass()[id];
    s_I[0][tid] = sp.cs.ix()[id]; s_I[1][tid] = sp.cs.iy()[id]; s_I[2][tid] = sp.cs.iz()[id];
    // the home tile (drift checks) and the staging origin (lane 0's tile)
    const T htx = (T)__builtin_floor((double)(x.x * p.inv_L)), hty = (T)__builtin_floor((double)(x.y * p.inv_L));
    const T ox = __shfl(htx, 0) * p.L, oy = __shfl(hty, 0) * p.L;
    s_home[0][tid] = htx * p.L - p.drift;
    s_home[1][tid] = hty * p.L - p.drift;
    s_px[tid] = x.x; s_py[tid] = x.y; s_pz[tid] = x.z; s_r[tid] = rad; s_gid[tid] = id;
    s_xref[0][tid] = x.x; s_xref[1][tid] = x.y;      // position at the last list build
    int ne = 0;                                      // this body's list length
    int nimp = 0;                                    // imports of the slot
    bool bail = false;
    const uint32_t base = *p.epoch;
    __syncthreads();

    // ---- list build at step t (0: the window start, from the snapshot;
    // later: from the neighbours' publication of step t) -------------------
    auto build = [&](int t) -> bool {
        const int ns = s_ko[9];
        const unsigned long long *pb = p.pub + (size_t)(t & 1) * nslots * G * RES_CAP;
        // 1. stage the 3 x 3 slots' bodies (x, y, id), SPC per lane at a time
        constexpr int SPC = 3;
        float fm = 0.f;
#pragma unroll
        for (int s0 = 0; s0 < SPL; s0 += SPC) {
            int32_t req[SPC];
            int kq[SPC], iq[SPC];
            uint32_t need = 0;                       // staged bodies of the neighbours (not in LDS)
#pragma unroll
            for (int s = 0; s < SPC; ++s) {
                const int u = tid + (s0 + s) * RES_CAP;
                int k = 0;
#pragma unroll
                for (int kk = 1; kk < 9; ++kk) k = u >= s_ko[kk] ? kk : k;
                kq[s] = k;
                iq[s] = u - s_ko[k];
                req[s] = (s_kslot[k] * G) * RES_CAP + iq[s];
                if (u < ns && k != 4) need |= 1u << s;
            }
            if (__all(tid + s0 * RES_CAP >= ns)) continue;
            unsigned long long g[SPC][GXY];
            if (t > 0 && !res_wait<T, SPC, GXY>(p, pb, req, need, base + (uint32_t)t, g)) return false;
#pragma unroll
            for (int s = 0; s < SPC; ++s) {
                const int u = tid + (s0 + s) * RES_CAP;
                if (u >= ns) break;
                T px, py;
                int32_t gid;
                if (kq[s] == 4) {
                    px = s_px[iq[s]]; py = s_py[iq[s]]; gid = s_gid[iq[s]];
                } else {
                    gid = p.ids[(int64_t)s_kslot[kq[s]] * RES_CAP + iq[s]];
                    if (t == 0) {
                        const Snap<T> sn = p.snap[gid];
                        px = sn.x; py = sn.y;
                    } else if constexpr (sizeof(T) == 8) {
                        px = res_join(g[s][0], g[s][1]); py = res_join(g[s][2], g[s][3]);
                    } else {
                        px = __uint_as_float((uint32_t)g[s][0]); py = __uint_as_float((uint32_t)g[s][1]);
                    }
                }
                const float fx = (float)(px - ox), fy = (float)(py - oy);
                s_sx[u] = fx;
                s_sy[u] = fy;
                s_sgid[u] = gid;
                fm = fmaxf(fm, fmaxf(fabsf(fx), fabsf(fy)));
            }
        }
        // the largest staged coordinate bounds the fp32 rounding of the test
        for (int o = 32; o > 0; o >>= 1) fm = fmaxf(fm, __shfl_xor(fm, o));
        __syncthreads();
        // 2. each body's candidates: staged bodies within rl (+ a bound on the
        // fp32 rounding of coordinates up to fm) in x, y, itself excluded,
        // kept sorted by id (insertion into the lane's LDS column)
        const float eps = 8.0f * 5.96e-8f * (2.0f * fm + (float)p.rl) + 1e-30f;
        const float rlf = (float)p.rl + eps;
        const float rl2 = rlf * rlf * (1.0f + 1e-6f);
        ne = 0;
        bool bad = false;
        if (own) {
            const int me = s_ko[4] + tid;
            const float xi = s_sx[me], yi = s_sy[me];
            for (int u = 0; u < ns; ++u) {
                const float dx = s_sx[u] - xi, dy = s_sy[u] - yi;
                if (u != me && dx * dx + dy * dy < rl2) {
                    if (ne < RES_LMAX) {
                        const int32_t key = s_sgid[u];
                        int f = ne - 1;
                        while (f >= 0 && s_sgid[s_list[f][tid]] > key) {
                            s_list[f + 1][tid] = s_list[f][tid];
                            --f;
                        }
                        s_list[f + 1][tid] = (uint16_t)u;
                    }
                    ++ne;
                }
            }
        }
        if (ne > RES_LMAX) {
            res_fail(p, RES_WHY_LIST);
            bad = true;
            ne = RES_LMAX;
        }
        for (int e = 0; e < ne; ++e) {
            const int u = s_list[e][tid];
            if (u < s_ko[4] || u >= s_ko[5]) s_sgid[u] |= RES_IMPORT_BIT;   // an import
        }
        if (__any(bad)) return false;
        __syncthreads();
        // 3. number the imports (ascending staging index) and record them
        uint32_t mk = 0;
        int cntl = 0;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const int u = tid * SPL + s;
            if (u < ns && (s_sgid[u] & RES_IMPORT_BIT)) { mk |= 1u << s; ++cntl; }
        }
        const int incl = res_wave_scan(cntl);
        nimp = __shfl(incl, 63);
        int j = incl - cntl;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
            const int u = tid * SPL + s;
            if (u >= ns) continue;
            int k = 0;
#pragma unroll
            for (int kk = 1; kk < 9; ++kk) k = u >= s_ko[kk] ? kk : k;
            const int idx = u - s_ko[k];
            if (k == 4) { s_sgid[u] = idx; continue; }
            if (!((mk >> s) & 1u)) continue;
            if (j < RES_MMAX) {
                const int32_t gid = s_sgid[u] & ~RES_IMPORT_BIT;
                s_sgid[u] = RES_CAP + j;
                s_ioff[j] = (s_kslot[k] * G) * RES_CAP + idx;
                s_gid[RES_CAP + j] = gid;
                s_r[RES_CAP + j] = sp.cs.bound()[gid];
            }
            ++j;
        }
        if (nimp > RES_MMAX) {
            if (tid == 0) res_fail(p, RES_WHY_IMPORT);
            return false;
        }
        __syncthreads();
        for (int e = 0; e < ne; ++e) s_list[e][tid] = (uint16_t)s_sgid[s_list[e][tid]];
        s_xref[0][tid] = x.x;
        s_xref[1][tid] = x.y;
        return true;
    };

    // the imports' positions of step t (0: the snapshot; later: granules)
    auto import = [&](int t) -> bool {
        if (t == 0) {
#pragma unroll
            for (int s = 0; s < IPL; ++s) {
                const int jj = tid + s * RES_CAP;
                if (jj < nimp) {
                    const Snap<T> sn = p.snap[s_gid[RES_CAP + jj]];
                    s_px[RES_CAP + jj] = sn.x; s_py[RES_CAP + jj] = sn.y; s_pz[RES_CAP + jj] = sn.z;
                }
            }
            return true;
        }
        const unsigned long long *pb = p.pub + (size_t)(t & 1) * nslots * G * RES_CAP;
        int32_t req[IPL];
        int nr = 0;
#pragma unroll
        for (int s = 0; s < IPL; ++s) {
            const int jj = tid + s * RES_CAP;
            req[s] = jj < nimp ? s_ioff[jj] : 0;
            if (jj < nimp) nr = s + 1;
        }
        unsigned long long g[IPL][G];
        if (!res_wait<T, IPL, G>(p, pb, req, (1u << nr) - 1u, base + (uint32_t)t, g)) return false;
#pragma unroll
        for (int s = 0; s < IPL; ++s) {
            const int jj = tid + s * RES_CAP;
            if (jj < nimp) {
                const V3<T> c = res_decode<T>(g[s]);
                s_px[RES_CAP + jj] = c.x; s_py[RES_CAP + jj] = c.y; s_pz[RES_CAP + jj] = c.z;
            }
        }
        return true;
    };

    if (!build(0) || !import(0)) bail = true;
    __syncthreads();
    RSTAMP(1);

    // ---- the steps -----------------------------------------------------------------
    for (int t = 0; t < p.K && !bail; ++t) {
        // (keeps the list builds' LDS tables out of registers across steps)
        asm volatile("" ::: "memory");
        if (t > 0) {
            const bool rebuild = p.M > 0 && t % p.M == 0;
            if (rebuild && !build(t)) { bail = true; break; }
            if (!import(t)) { bail = true; break; }
            __syncthreads();
        }
        if (t < 16) RSTAMP(4 + 2 * t);
        const bool last = t + 1 == p.K;
        const bool rec = last && p.rec && sp.rec_count;
        bool bad = false;                            // this lane raised a failure
        if (own) {
            const T m = s_m[tid];
            const T kimp = impulse_k(m);
            LazyInvI<T> invI;
            invI.I = V3<T>{s_I[0][tid], s_I[1][tid], s_I[2][tid]};
            invI.q = q;
            int32_t nrec = 0;
            auto rcd = [&](int32_t partner, int32_t kind, T dist) {
                if (!rec) return;
                if (nrec < sp.maxrec) {
                    const int64_t o = (int64_t)id * sp.maxrec + nrec;
                    sp.rec_partner[o] = partner;
                    sp.rec_kind[o] = kind;
                    sp.rec_dist[o] = dist;
                }
                ++nrec;
            };
            // a4 gravity, K2 plane contacts, then the
            // partners in ascending id: the list order
            apply_force<T, false>(sp, id, m, invI, v, w);   // (no xfrc: res_eligible)
            for (int pl = 0; pl < sp.n_planes; ++pl) {
                const V3<T> pn = {sp.pn[pl][0], sp.pn[pl][1], sp.pn[pl][2]};
                const V3<T> pp = {sp.pp[pl][0], sp.pp[pl][1], sp.pp[pl][2]};
                Contact<T> con;
                if (!plane_sphere(pn, pp, x, rad, con)) continue;
                rcd(-1 - pl, 0, con.dist);
                solve_contact(sp, con, x, con.frame, m, kimp, invI, v, w);
            }
            int np_ = 0;
            for (int e = 0; e < ne; ++e) {
                const int c = s_list[e][tid];
                const V3<T> cj = {s_px[c], s_py[c], s_pz[c]};
                const T rj = s_r[c];
                if (!sphere_sphere_hit(x, rad, cj, rj)) continue;
                if (++np_ > MAXP) {
                    res_fail(p, TILE_WHY_PARTNERS);
                    bad = true;
                    break;
                }
                const int32_t j = s_gid[c];
                Contact<T> con;
                V3<T> nrm;
                if (id < j) {                        // this body is geom1
                    sphere_sphere(x, rad, cj, rj, con);
                    nrm = sp.oriented ? V3<T>{-con.frame.x, -con.frame.y, -con.frame.z} : con.frame;
                } else {
                    sphere_sphere(cj, rj, x, rad, con);
                    nrm = con.frame;
                }
                rcd(j, 16, con.dist);
                solve_contact(sp, con, x, nrm, m, kimp, invI, v, w);
            }
            if (rec) sp.rec_count[id] = nrec;
            Q4<T> qn;
            integrate_pose(x, qn, q, v, w, sp.dt);
            q = qn;
            // the checks that keep the lists exact for the next step
            int why = 0;
            if (!(absval(x.x) < T(1e12) && absval(x.y) < T(1e12) && absval(x.z) < T(1e12))) {
                why = TILE_WHY_DOMAIN;
            } else if (!last) {
                const bool next_rebuild = p.M > 0 && (t + 1) % p.M == 0;
                if (next_rebuild) {
                    const T lx = s_home[0][tid], ly = s_home[1][tid], hx = lx + p.L + T(2) * p.drift,
                            hy = ly + p.L + T(2) * p.drift;
                    if (!(x.x >= lx && x.x < hx && x.y >= ly && x.y < hy)) why = RES_WHY_DRIFT;
                } else {
                    const T dx = x.x - s_xref[0][tid], dy = x.y - s_xref[1][tid];
                    if (!(dx * dx + dy * dy <= p.skin2)) why = RES_WHY_SKIN;
                }
            }
            if (why) {
                res_fail(p, why);
                bad = true;
            }
        }
        // a failed slot stops here (its neighbours see the abort word)
        if (__any(bad)) { bail = true; break; }
        __syncthreads();
        if (!last) {
            // publish: this slot's positions of step t + 1, to LDS and (tag t + 1) to
            // the neighbours
            if (own) {
                s_px[tid] = x.x; s_py[tid] = x.y; s_pz[tid] = x.z;
                unsigned long long *dst = p.pub + ((size_t)((t + 1) & 1) * nslots + slot) * G * RES_CAP + tid;
                const unsigned long long tg = (unsigned long long)(base + (uint32_t)(t + 1)) << 32;
#pragma unroll
                for (int k = 0; k < G; ++k) res_store(dst + k * RES_CAP, tg | res_half(x, k));
            }
            __syncthreads();
        }
        if (t < 16) RSTAMP(5 + 2 * t);
    }
    RSTAMP(2);
    if (bail || !own) return;
    // the window's end state (committed by res_commit_kernel if no slot failed)
    p.out_snap[id] = Snap<T>{x.x, x.y, x.z, rad};
    T *o = p.out_st;
    const int64_t S = sp.st.S;
    o[0 * S + id] = q.w; o[1 * S + id] = q.x; o[2 * S + id] = q.y; o[3 * S + id] = q.z;
    o[4 * S + id] = v.x; o[5 * S + id] = v.y; o[6 * S + id] = v.z;
    o[7 * S + id] = w.x; o[8 * S + id] = w.y; o[9 * S + id] = w.z;
}

// ---- binning and commit ----------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void res_bin_kernel(ResParams<T> p, int64_t n) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= n) return;
    const Snap<T> sn = p.snap[b];
    const T fx = sn.x * p.inv_L, fy = sn.y * p.inv_L;
    if (!(absval(fx) < T(1 << 29) && absval(fy) < T(1 << 29))) {
        atomicOr(p.why, TILE_WHY_DOMAIN);
        atomicOr(p.sp.err, ERR_TILE);
        return;
    }
    const int32_t tx = (int32_t)__builtin_floor((double)fx), ty = (int32_t)__builtin_floor((double)fy);
    const int64_t slot = (int64_t)res_pmod(ty, p.nty) * p.ntx + res_pmod(tx, p.ntx);
    const int32_t k = atomicAdd(const_cast<int32_t *>(p.cnt) + slot, 1);
    if (k < RES_CAP) {
        const_cast<int32_t *>(p.ids)[slot * RES_CAP + k] = (int32_t)b;
    } else if (k == RES_CAP) {
        atomicOr(p.why, TILE_WHY_CAP);
        atomicOr(p.sp.err, ERR_TILE);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void res_commit_kernel(ResCommit<T> p) {
    const bool ok = !(*p.err & ERR_TILE);
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (ok) {
        for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < p.n; b += stride) {
            p.snap[b] = p.out_snap[b];
#pragma unroll
            for (int d = 0; d < 10; ++d) p.st.row(d)[b] = p.out_st[d * p.S + b];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *p.epoch += (uint32_t)p.K + 1u;
        *p.abort = 0;
        if (ok) *p.commits += 1;
    }
}

// ---- launchers ----------------------------------------------------------------
template <typename T> hipError_t launch_res_bin(const ResParams<T> &p, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((res_bin_kernel<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
    return hipGetLastError();
}
template <typename T> hipError_t launch_res_step(const ResParams<T> &p, int maxp, hipStream_t s) {
    if (p.ntx < 3 || p.nty < 3 || p.K < 1 || !(p.L > 0)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(p.ntx * p.nty)), block(RES_CAP);
    if (maxp > 16) hipLaunchKernelGGL((res_step_kernel<T, 32>), grid, block, 0, s, p.sp.err, p.cnt, p);
    else hipLaunchKernelGGL((res_step_kernel<T, 16>), grid, block, 0, s, p.sp.err, p.cnt, p);
    return hipGetLastError();
}
template <typename T> hipError_t launch_res_commit(const ResCommit<T> &p, hipStream_t s) {
    const int64_t nb = (p.n + 255) / 256;
    hipLaunchKernelGGL((res_commit_kernel<T>), dim3((unsigned)(nb < 1024 ? (nb > 0 ? nb : 1) : 1024)), dim3(256), 0, s, p);
    return hipGetLastError();
}

int res_blocks_per_cu(int f64, int maxp) {
    int nb = 0;
    hipError_t r;
    if (f64) r = maxp > 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<double, 32>, RES_CAP, 0)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<double, 16>, RES_CAP, 0);
    else r = maxp > 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<float, 32>, RES_CAP, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, res_step_kernel<float, 16>, RES_CAP, 0);
    return r == hipSuccess ? nb : 0;
}

#if RB_RES_STAMPS
extern "C" int rb_diag_res_stamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_res_stamp_buf), sizeof(unsigned long long) * RES_NSTAMP * nblocks);
}
#endif

template hipError_t launch_res_bin<double>(const ResParams<double> &, int64_t, hipStream_t);
template hipError_t launch_res_bin<float>(const ResParams<float> &, int64_t, hipStream_t);
template hipError_t launch_res_step<double>(const ResParams<double> &, int, hipStream_t);
template hipError_t launch_res_step<float>(const ResParams<float> &, int, hipStream_t);
template hipError_t launch_res_commit<double>(const ResCommit<double> &, hipStream_t);
template hipError_t launch_res_commit<float>(const ResCommit<float> &, hipStream_t);

}  // namespace rb
