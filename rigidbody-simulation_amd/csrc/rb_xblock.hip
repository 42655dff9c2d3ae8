// rb_xblock.hip — XCD-resident K-step blocks.
//
// The reference step is Jacobi across bodies: one contact pass
// (multi_sphere_bounce.py:43), then every body's update from step-start data
// (:46-90).  So K steps of a body depend only on bodies that reach it through
// a chain of contacts within those K steps.  A launch here runs K steps:
//
//   groups    the workgroups b, b + 8, b + 16, ... (one XCD under the
//             hardware's round-robin dealing; checked with the XCC_ID
//             register, and the block is abandoned if a group spans XCDs,
//             since its hand-offs rely on one shared L2);
//   slabs     group g owns the bodies whose coordinate along the scene's
//             widest horizontal axis lies in [cut[g], cut[g+1]) at the start;
//   copy      it copies its slab plus a ghost band of width
//               W = K reach + 2 (K - 1) V dt
//             (V bounds every body's speed over the K steps) into buffers of
//             its own, ids compacted in ascending order — so sorting partners
//             by local index is sorting them by global id, the reference's
//             contact order;
//   steps     it steps the whole copy K times with the per-step kernel's own
//             body code (rb_kernels.hip body_step: the wide one-lane form),
//             on a broadphase table of its own rebuilt every step, with a
//             barrier among its workgroups between steps.  Loads of data
//             another workgroup wrote in this launch bypass the L1 (xld,
//             rb_grid.hpp); the copy, its snapshots and its table stay in
//             the XCD's L2 across steps;
//   commit    it writes its owned bodies back in place, once every group has
//             finished copying (a launch-wide counter).
//
// Exactness: a body's step-K state depends on step-0 positions within
// K reach + 2 (K - 1) V dt (a chain of K contacts, each between bodies
// within `reach` at that step, each body moving at most V dt per step), so the
// owned bodies' results are exactly those of K per-step launches — provided
// every body keeps |v| <= V.  Every group checks that for its owned bodies at
// every step (the union covers every body); a violation, a copy larger than
// the buffers, a group spread over two XCDs or a wait that times out raises
// ERR_XB, and the host rolls the chunk back and replays it step by step
// (rb_capi.hip xb_finish).  V = valpha max|v| + vbeta + K |g| dt, max|v| taken
// over every body at the launch's start (each group scans all of them).
#define RB_XB 1
#undef RB_STAMPS
#if RB_XB_STAMPS                 // diagnostic build: the body code's phase stamps, this unit's own buffer
#define RB_STAMPS 1
#else
#define RB_STAMPS 0              // (stamp builds of the per-step kernels: their buffer lives in their own unit)
#endif
#define RB_STEP_BLOCK 512        // (rb_internal.hpp XB_THREADS): the wide form's LDS columns
#define RB_WIDE_LDSPOS 0         // partner snapshots re-read in the solve (L2-resident here)
#define RB_WIDE_QBATCH 8         // candidates per round trip: two waves per SIMD must fit in 256 registers
#define RB_INST 0                // none of rb_kernels.hip's own kernels
#include "rb_kernels.hip"

namespace rb {

static_assert(STEP_BLOCK == XB_THREADS, "one body per lane of the block");
constexpr int XB_CHUNK = 16384;        // ids a workgroup scans at most (the host checks N <= XB_CHUNK x wpg)

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15; }

__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A barrier among the workgroups of group g: every storing wave's stores are
// complete (vmcnt 0: they reached the L2 the group shares), one device-scope
// arrival per workgroup, a poll of sc1 loads.  Arrivals are never skipped,
// waits are once a wait has timed out anywhere (poison), so the group never
// deadlocks; the counters are monotone (a launch adds wpg per barrier).
__device__ __forceinline__ void xb_barrier(XbCtl *C, int g, int wpg, unsigned long long t0, int64_t tmo, int32_t *err) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long *ctr = &C->bar[g][0];
        const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long target = (old / (unsigned)wpg + 1ull) * (unsigned)wpg;
        while (ld_sc1(ctr) < target) {
            if (__hip_atomic_load(&C->poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
                __hip_atomic_store(&C->poison, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicOr(&C->why, XB_WHY_TIMEOUT);
                atomicOr(err, ERR_XB);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#if RB_XB_LD == 0
        // plain (L1-cached) loads in the steps: this CU's L1 may hold lines
        // other CUs of the XCD have since rewritten in the L2
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    }
    __syncthreads();
}

// block-wide exclusive prefix of one flag per thread (512 threads); returns
// the thread's offset, total in *tot
__device__ __forceinline__ int block_scan(int f, int *s_w, int *tot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(f);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    int off = 0, t = 0;
#pragma unroll
    for (int k = 0; k < XB_THREADS / 64; ++k) {
        const int c = s_w[k];
        off += k < wave ? c : 0;
        t += c;
    }
    __syncthreads();
    *tot = t;
    return off + pre;
}

template <typename T>
__device__ __forceinline__ T axis_of(const Snap<T> &s, int axis) { return axis == 0 ? s.x : s.y; }

// sharded worlds: the mailbox's pushed rows (written by the peers over
// xGMI into this rank's uncached mailbox), read past the caches
template <typename T> __device__ __forceinline__ T ld_sys(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sc1_ull(const unsigned long long *p) { return ld_sc1(p); }

template <typename T, int MAXP, bool SH>
__global__ __launch_bounds__(XB_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
void xblock_kernel(XbParams<T> P) {
    __shared__ int32_t s_id[MAXP * XB_THREADS];
    __shared__ uint32_t s_cand[WIDE_MAXC * XB_THREADS];
    __shared__ uint8_t s_didx[1];
    __shared__ int s_w[XB_THREADS / 64];
    __shared__ unsigned long long s_flag[XB_CHUNK / 64 + 32];   // the chunk's ids in the copy (one bit each)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = (int)(blockIdx.x % XB_GROUPS), r = (int)(blockIdx.x / XB_GROUPS), wpg = P.wpg;
    XbCtl *C = P.ctl;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    auto stamp = [&](int k) {
        if (tid == 0) C->stamp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    const int64_t tmo = P.timeout_ticks;
    const int cap = P.cap;
    if (tid == 0) __hip_atomic_store(&C->xcc[blockIdx.x], xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ---- 1. the launch's speed bound V and band W.  One rank: every group
    // scans every body for max |v|, each workgroup a contiguous id chunk.
    // Sharded (SH): the push kernel made them from every rank's header; the
    // group instead indexes the ghosts the peers pushed (gidx: id -> inbox
    // slot, tagged with the push's epoch)
    const int chunk = (P.n + wpg - 1) / wpg;
    const int c0 = r * chunk, c1 = min(P.n, c0 + chunk);
    T V, W;
    float vmax = 0.f;
    [[maybe_unused]] int64_t e = 0, G = 0;
    [[maybe_unused]] const uint32_t *in_ids = nullptr;
    [[maybe_unused]] const T *in_pay = nullptr;
    [[maybe_unused]] unsigned long long *gx = nullptr;
    if constexpr (SH) {
        e = *P.xs_epoch;
        G = P.lay.xg;
        const int par = (int)(e & 1);
        in_ids = reinterpret_cast<const uint32_t *>(P.mail + P.lay.o_xids) + (int64_t)par * P.P * G;
        in_pay = reinterpret_cast<const T *>(P.mail + P.lay.o_xpay) + (int64_t)par * P.P * XS_PAY * G;
        gx = P.gidx + (int64_t)g * P.Npad;
        int tot = 0;
        for (int q = 0; q < P.P; ++q) tot += P.in_cnt[q];
        for (int k = r * XB_THREADS + tid; k < tot; k += wpg * XB_THREADS) {
            int q = 0, o = k;
            while (o >= P.in_cnt[q]) { o -= P.in_cnt[q]; ++q; }
            const uint32_t id = ld_sys(in_ids + (int64_t)q * G + o);
            if ((int64_t)id < (int64_t)q * P.S || (int64_t)id >= (int64_t)(q + 1) * P.S || (int64_t)id >= P.n) {
                atomicOr(P.err, ERR_XB);
                continue;
            }
            gx[id] = ((unsigned long long)e << 32) | (unsigned long long)(q * G + o);
        }
        V = P.vw[0];
        W = P.vw[1];
    } else {
        for (int b0 = c0; b0 < c1; b0 += 4 * XB_THREADS) {
            T vv[4][3];                                  // four bodies' loads in flight together
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int id = min(b0 + q * XB_THREADS + tid, c1 - 1);
                vv[q][0] = P.st_base[4 * P.S + id]; vv[q][1] = P.st_base[5 * P.S + id]; vv[q][2] = P.st_base[6 * P.S + id];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = (float)sqroot(vv[q][0] * vv[q][0] + vv[q][1] * vv[q][1] + vv[q][2] * vv[q][2]);
                vmax = (v > vmax || v != v) ? v : vmax;       // a NaN poisons the bound (the check then fails)
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) { const float o = __shfl_xor(vmax, off); vmax = (o > vmax || o != o) ? o : vmax; }
        if (lane == 0) s_w[wave] = (int)__float_as_uint(vmax);
        __syncthreads();
        if (tid == 0) {
            float m = 0.f;
            for (int k = 0; k < XB_THREADS / 64; ++k) { const float o = __uint_as_float((uint32_t)s_w[k]); m = (o > m || o != o) ? o : m; }
            C->vpart[g][r] = __float_as_uint(m);
        }
    }
    xb_barrier(C, g, wpg, t0, tmo, P.err);
    stamp(1);
    // the placement check: every workgroup of the group on one XCD
    if (tid < wpg && __hip_atomic_load(&C->xcc[g + XB_GROUPS * tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                         __hip_atomic_load(&C->xcc[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        atomicOr(&C->why, XB_WHY_PLACEMENT);
        atomicOr(P.err, ERR_XB);
    }
    if constexpr (!SH) {
        vmax = 0.f;
        for (int k = 0; k < wpg; ++k) {
            const float o = __uint_as_float(__hip_atomic_load(&C->vpart[g][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            vmax = (o > vmax || o != o) ? o : vmax;
        }
        V = P.valpha * (T)vmax + P.vbeta + (T)P.K * P.gdt;
        W = (T)P.K * P.reach + T(2) * (T)(P.K - 1) * V * P.sp[0].dt + T(1e-3) * P.reach;
        if (g == 0 && r == 0 && tid == 0) C->vmax_bits = __float_as_uint(vmax);
    }
    const T V2 = V * V;
    const T lo = g == 0 ? -INFINITY : P.cut[g] - W, hi = g == XB_GROUPS - 1 ? INFINITY : P.cut[g + 1] + W;
    const T olo = g == 0 ? -INFINITY : P.cut[g], ohi = g == XB_GROUPS - 1 ? INFINITY : P.cut[g + 1];
    // sharded: where body id's step-start position comes from (own rows, a
    // ghost's inbox slot, or absent: -1)
    [[maybe_unused]] auto ghost_slot = [&](int id) -> int64_t {
        const unsigned long long t = xld(gx + id);
        return (int64_t)(t >> 32) == e ? (int64_t)(uint32_t)t : -1;
    };
    [[maybe_unused]] auto own = [&](int id) { return id >= P.lo && id < P.lo + P.n_local; };

    // ---- 2. the copy: this chunk's bodies within [lo, hi), flagged in LDS
    // (one bit per id of the chunk) and counted
    int cnt = 0;
    for (int b0 = c0; b0 < c1; b0 += 4 * XB_THREADS) {
        T u[4];                                      // four independent loads, then the flags
        [[maybe_unused]] bool have[4] = {true, true, true, true};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int id = b0 + q * XB_THREADS + tid;
            if constexpr (SH) {
                u[q] = T(0);
                have[q] = false;
                if (id < c1) {
                    if (own(id)) {
                        u[q] = axis_of(P.snap_in[id], P.axis);
                        have[q] = true;
                    } else {
                        const int64_t sl = ghost_slot(id);
                        if (sl >= 0) {
                            u[q] = ld_sys(in_pay + ((sl / G) * XS_PAY + P.axis) * G + sl % G);
                            have[q] = true;
                        }
                    }
                }
            } else {
                u[q] = id < c1 ? axis_of(P.snap_in[id], P.axis) : T(0);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int id = b0 + q * XB_THREADS + tid;
            bool in = false;
            if (id < c1 && have[q]) {
                if (!(u[q] == u[q])) atomicOr(P.err, ERR_DOMAIN);
                in = u[q] >= lo && u[q] < hi;
            }
            const unsigned long long m = __ballot(in);
            if (lane == 0) s_flag[(b0 + q * XB_THREADS - c0) / 64 + wave] = m;
            cnt += in ? 1 : 0;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0) s_w[wave] = cnt;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int k = 0; k < XB_THREADS / 64; ++k) t += s_w[k];
        C->cnt[g][r] = t;
    }
    xb_barrier(C, g, wpg, t0, tmo, P.err);
    stamp(2);
    // offsets of this chunk's bodies in the copy (ascending ids)
    int off = 0, total = 0;
    for (int k = 0; k < wpg; ++k) {
        const int c = __hip_atomic_load(&C->cnt[g][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        off += k < r ? c : 0;
        total += c;
    }
    const bool fits = total <= cap;                  // the same decision in every workgroup of the group
    if (!fits && r == 0 && tid == 0) { atomicOr(&C->why, XB_WHY_CAP); atomicOr(P.err, ERR_XB); }
    int32_t *map = P.map + (int64_t)g * cap;
    if (fits) {
        for (int b0 = c0; b0 < c1; b0 += XB_THREADS) {
            const int id = b0 + tid;
            const unsigned long long m = s_flag[(b0 - c0) / 64 + wave];
            const bool in = (m >> lane) & 1ull;
            int t;
            const int o = block_scan(in ? 1 : 0, s_w, &t);
            if (in) map[off + o] = id;
            off += t;
        }
    }
    if (r == 0 && tid == 0) C->nload[g] = total;
    xb_barrier(C, g, wpg, t0, tmo, P.err);
    stamp(3);

    // ---- 3. each lane gathers the bodies it steps (waves dealt over the
    // group's workgroups in turn) and inserts them into step 0's table
    const int n = fits ? total : 0;
    const int passes = (n + wpg * XB_THREADS - 1) / (wpg * XB_THREADS);
    Snap<T> *ls0 = P.lsnap + (int64_t)g * 2 * cap;
    T *lst = P.lstate + (int64_t)g * 13 * cap;
    T *lcs = P.lconst + (int64_t)g * 8 * cap;
    int32_t *lkd = P.lkind + (int64_t)g * cap;
    const uint32_t gen0 = C->gen[g][0];
    const StepParams<T> *SP = P.sp + 4 * g;
    uint32_t owned = 0;                              // bit p: the lane's body of pass p is owned
    for (int p = 0; p < passes; ++p) {
        const int l = ((p * (XB_THREADS / 64) + wave) * wpg + r) * 64 + lane;
        if (l >= n) continue;
        const int id = xld(map + l);
        Snap<T> s;
        if (!SH || own(id)) {
            s = P.snap_in[id];
            const int64_t row = SH ? id - P.lo : id;
#pragma unroll
            for (int k = 0; k < 13; ++k) lst[(int64_t)k * cap + l] = P.st_base[(int64_t)k * P.S + row];
            const T u = axis_of(s, P.axis);
            if (u >= olo && u < ohi) owned |= 1u << p;
        } else if constexpr (SH) {
            int64_t sl = ghost_slot(id);             // (present: it was copied)
            if (sl < 0) { atomicOr(P.err, ERR_XB); sl = 0; }
            const T *src = in_pay + (sl / G) * XS_PAY * G + sl % G;
            s.x = ld_sys(src); s.y = ld_sys(src + G); s.z = ld_sys(src + 2 * G); s.r = ld_sys(src + 3 * G);
#pragma unroll
            for (int k = 0; k < 13; ++k) lst[(int64_t)k * cap + l] = ld_sys(src + (4 + k) * G);
        }
        ls0[l] = s;
#pragma unroll
        for (int k = 0; k < 8; ++k) lcs[(int64_t)k * cap + l] = P.cs.base[(int64_t)k * P.cs.Npad + id];
        lkd[l] = P.cs.kind[id];
        insert_id(SP[0].grid, SP[0].cur, P.err, s, (uint32_t)l, gen0);
    }
    // every group has read the global state it needs once every workgroup
    // has arrived here (the commit below writes it in place)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    unsigned long long gtarget = 0;
    if (tid == 0) {
        const unsigned long long tot = (unsigned long long)XB_GROUPS * (unsigned)wpg;
        const unsigned long long old = __hip_atomic_fetch_add(&C->gathered[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gtarget = (old / tot + 1ull) * tot;
    }
    xb_barrier(C, g, wpg, t0, tmo, P.err);
    stamp(4);

    // ---- 4. K steps of the copy
    for (int s = 0; s < P.K; ++s) {
        const StepParams<T> &sp = SP[(s & 1) + (s == P.K - 1 ? 2 : 0)];
        const Lead<T> ld{sp.snap_cur, BodyState<T>{lst, cap}, BodyConsts<T>{lcs, cap, lkd}, n, 0};
        bool bad = false;
        for (int p = 0; p < passes; ++p) {
            const int l = ((p * (XB_THREADS / 64) + wave) * wpg + r) * 64 + lane;
            if (l >= n) continue;
            int32_t cell[3] = {INT32_MAX, 0, 0};
            body_step<T, MAXP, 1, true, false, false, false>(sp, ld, true, l, tid, 0, tid, s_id, nullptr, nullptr,
                                                             nullptr, s_cand, cell, gen0 + (uint32_t)s, nullptr, s_didx,
                                                             nullptr, nullptr);
            if ((owned >> p) & 1u) {
                const T vx = lst[4 * (int64_t)cap + l], vy = lst[5 * (int64_t)cap + l], vz = lst[6 * (int64_t)cap + l];
                bad |= !(vx * vx + vy * vy + vz * vz <= V2);
            }
        }
        if (bad) { atomicOr(&C->why, XB_WHY_SPEED); atomicOr(P.err, ERR_XB); }
        if (s == 0) stamp(5);
        if (s + 1 < P.K) xb_barrier(C, g, wpg, t0, tmo, P.err);
    }

    stamp(6);
    // ---- 5. commit the owned bodies, once every group has its copy
    if (tid == 0) {
        while (ld_sc1(&C->gathered[0]) < gtarget) {
            if (__hip_atomic_load(&C->poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > tmo) {
                __hip_atomic_store(&C->poison, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicOr(&C->why, XB_WHY_TIMEOUT);
                atomicOr(P.err, ERR_XB);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    const Snap<T> *lsK = ls0 + (int64_t)(P.K & 1) * cap;
    for (int p = 0; p < passes; ++p) {
        const int l = ((p * (XB_THREADS / 64) + wave) * wpg + r) * 64 + lane;
        if (l >= n || !((owned >> p) & 1u)) continue;
        const int id = xld(map + l);
        P.snap_out[id] = lsK[l];                     // (written by this lane)
        const int64_t row = SH ? id - P.lo : id;
#pragma unroll
        for (int k = 0; k < 13; ++k) P.st_base[(int64_t)k * P.S + row] = lst[(int64_t)k * cap + l];
    }
    // the group's next table generation (read by the next launch only)
    if (r == 0 && tid == 0) C->gen[g][0] = gen0 + (uint32_t)P.K + 1u;
    stamp(7);
}

template <typename T> hipError_t launch_xblock(const XbParams<T> &p, int maxp, hipStream_t s) {
    if (p.wpg < 1 || p.wpg > XB_MAX_WPG || p.K < 1 || !p.sp || !p.ctl) return hipErrorInvalidValue;
    if (maxp > 16) return hipErrorInvalidValue;   // 32 partners: the LDS lists do not fit (per-step kernels)
    const dim3 grid((unsigned)(XB_GROUPS * p.wpg));
    if (p.xs) {
        if (!p.mail || !p.in_cnt || !p.vw || !p.xs_epoch || !p.gidx || p.lay.o_xpay < 0 || p.P < 2) return hipErrorInvalidValue;
        hipLaunchKernelGGL((xblock_kernel<T, 16, true>), grid, dim3(XB_THREADS), 0, s, p);
    } else {
        hipLaunchKernelGGL((xblock_kernel<T, 16, false>), grid, dim3(XB_THREADS), 0, s, p);
    }
    return hipGetLastError();
}

#if RB_XB_STAMPS
// the last step's stamps of wave 0 of every workgroup (scripts/stamps_c4.py reads 16 per block)
extern "C" int rb_diag_stamps(unsigned long long *out, int nblocks) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rb_stamp_buf), sizeof(unsigned long long) * 16 * nblocks);
}
#endif

template hipError_t launch_xblock<double>(const XbParams<double> &, int, hipStream_t);
template hipError_t launch_xblock<float>(const XbParams<float> &, int, hipStream_t);

}  // namespace rb
